// Fused v2 operator kernels, double, degree 7 (nq = 8, 9).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 7)
