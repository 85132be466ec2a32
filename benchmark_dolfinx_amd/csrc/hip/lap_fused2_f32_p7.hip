// Fused v2 operator kernels, float, degree 7 (nq = 8, 9).
#include "lap_fused2.h"
BDX_FUSED2_TU(float, f32, 7)
