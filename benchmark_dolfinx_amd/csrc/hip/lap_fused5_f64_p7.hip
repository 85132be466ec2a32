// Fused v5 operator kernels (nodal Kronecker core), double, degree 7.
#include "lap_fused5.h"
BDX_FUSED5_TU(double, f64, 7)
