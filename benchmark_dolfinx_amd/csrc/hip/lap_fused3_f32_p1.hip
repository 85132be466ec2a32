// Fused v3 operator kernels, float, degree 1 (nq = 3).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 1)
