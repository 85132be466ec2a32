// Fused v3 operator kernels, float, degree 7 (nq = 9).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 7)
