// dofmap (unstructured data model) operator, double instantiations.
#include "lap_dofmap.h"
BDX_DOFMAP_API(double, f64)
