// Fused v2 operator kernels, float, degree 1 (nq = 2, 3).
#include "lap_fused2.h"
BDX_FUSED2_TU(float, f32, 1)
