// Fused v2 operator kernels, double, degree 2 (nq = 3, 4).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 2)
