// Fused operator kernels, float, degree 5 (nq = 6, 7).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 5)
