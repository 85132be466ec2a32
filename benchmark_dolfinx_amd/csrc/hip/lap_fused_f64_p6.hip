// Fused operator kernels, double, degree 6 (nq = 7, 8).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 6)
