// v1 operator kernels, float32 instantiations.
#include "lap_v1_api.h"
BDX_V1_API(float, f32)
