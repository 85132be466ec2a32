// Fused operator kernels, double, degree 4 (nq = 5, 6).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 4)
