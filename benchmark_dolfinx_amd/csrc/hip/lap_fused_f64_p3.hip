// Fused operator kernels, double, degree 3 (nq = 4, 5).
#include "lap_fused_api.h"
BDX_FUSED_TU(double, f64, 3)
