// Fused operator kernels, float, degree 7 (nq = 8, 9).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 7)
