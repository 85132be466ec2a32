// Fused operator kernels, float, degree 1 (nq = 2, 3).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 1)
