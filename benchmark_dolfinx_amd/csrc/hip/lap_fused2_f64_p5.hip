// Fused v2 operator kernels, double, degree 5 (nq = 6, 7).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 5)
