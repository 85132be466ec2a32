// Fused v3 operator kernels, double, degree 4 (nq = 6).
#include "lap_fused3.h"
BDX_FUSED3_TU(double, f64, 4)
