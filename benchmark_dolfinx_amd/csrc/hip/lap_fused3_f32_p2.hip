// Fused v3 operator kernels, float, degree 2 (nq = 4).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 2)
