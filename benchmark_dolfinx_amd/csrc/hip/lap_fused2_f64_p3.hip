// Fused v2 operator kernels, double, degree 3 (nq = 4, 5).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 3)
