// Fused v2 operator kernels, float, degree 5 (nq = 6, 7).
#include "lap_fused2.h"
BDX_FUSED2_TU(float, f32, 5)
