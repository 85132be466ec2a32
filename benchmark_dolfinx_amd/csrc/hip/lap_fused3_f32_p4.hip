// Fused v3 operator kernels, float, degree 4 (nq = 6).
#include "lap_fused3.h"
BDX_FUSED3_TU(float, f32, 4)
