// Fused v2 operator kernels, double, degree 1 (nq = 2, 3).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 1)
