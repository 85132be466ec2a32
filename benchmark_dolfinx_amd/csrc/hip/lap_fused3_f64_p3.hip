// Fused v3 operator kernels, double, degree 3 (nq = 5).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 3)
