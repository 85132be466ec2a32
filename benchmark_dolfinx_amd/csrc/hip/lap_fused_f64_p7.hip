// Fused operator kernels, double, degree 7 (nq = 8, 9).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 7)
