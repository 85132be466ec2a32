// dofmap (unstructured data model) operator, float instantiations.
#include "lap_dofmap.h"
BDX_DOFMAP_API(float, f32)
