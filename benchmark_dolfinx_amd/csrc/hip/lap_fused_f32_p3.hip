// Fused operator kernels, float, degree 3 (nq = 4, 5).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 3)
