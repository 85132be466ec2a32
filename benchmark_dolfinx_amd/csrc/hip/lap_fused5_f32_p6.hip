// Fused v5 operator kernels (nodal Kronecker core), float, degree 6.
#include "lap_fused5.h"
BDX_FUSED5_TU(float, f32, 6)
