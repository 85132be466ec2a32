// Fused operator kernels, double, degree 5 (nq = 6, 7).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 5)
