// Fused v3 operator kernels, double, degree 5 (nq = 7).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 5)
