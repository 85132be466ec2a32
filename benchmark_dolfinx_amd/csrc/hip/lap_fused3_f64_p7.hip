// Fused v3 operator kernels, double, degree 7 (nq = 9).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 7)
