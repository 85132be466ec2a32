// Fused v3 operator kernels, double, degree 1 (nq = 3).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 1)
