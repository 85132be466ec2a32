// Fused v2 operator kernels, double, degree 6 (nq = 7, 8).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 6)
