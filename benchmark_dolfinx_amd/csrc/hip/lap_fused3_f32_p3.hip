// Fused v3 operator kernels, float, degree 3 (nq = 5).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 3)
