// Fused v3 operator kernels, float, degree 5 (nq = 7).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 5)
