// Fused v3 operator kernels, float, degree 6 (nq = 8).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 6)
