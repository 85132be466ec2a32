// Fused v2 operator kernels, float, degree 4 (nq = 5, 6).
#include "lap_fused2.h"
BDX_FUSED2_TU(float, f32, 4)
