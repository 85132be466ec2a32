// Fused operator kernels, double, degree 1 (nq = 2, 3).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 1)
