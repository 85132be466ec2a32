// Fused operator kernels, double, degree 2 (nq = 3, 4).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 2)
