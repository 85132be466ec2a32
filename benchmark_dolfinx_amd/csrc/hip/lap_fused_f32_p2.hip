// Fused operator kernels, float, degree 2 (nq = 3, 4).
#include "lap_fused_api.h"
BDX_FUSED_TU(float, f32, 2)
