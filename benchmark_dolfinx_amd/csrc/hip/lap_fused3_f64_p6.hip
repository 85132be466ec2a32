// Fused v3 operator kernels, double, degree 6 (nq = 8).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 6)
