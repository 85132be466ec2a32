// v1 operator kernels, float64 instantiations.
#include "lap_v1_api.h"
BDX_V1_API(double, f64)
