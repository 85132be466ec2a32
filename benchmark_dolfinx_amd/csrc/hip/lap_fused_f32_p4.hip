// Fused operator kernels, float, degree 4 (nq = 5, 6).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 4)
