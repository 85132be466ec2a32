// Fused v2 operator kernels, double, degree 4 (nq = 5, 6).
#include "lap_fused2.h"
BDX_FUSED2_TU(double, f64, 4)
