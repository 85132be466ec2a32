// Fused operator kernels, float, degree 6 (nq = 7, 8).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 6)
