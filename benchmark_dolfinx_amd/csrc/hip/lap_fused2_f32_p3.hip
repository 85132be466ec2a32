// Fused v2 operator kernels, float, degree 3 (nq = 4, 5).
#include "lap_fused2.h"
BDX_FUSED2_TU(float, f32, 3)
