// Fused v3 operator kernels, double, degree 2 (nq = 4).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 2)
