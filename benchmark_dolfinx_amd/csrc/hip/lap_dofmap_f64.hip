// dofmap (unstructured data model) operator, double instantiations.
#include "lap_dofmap.h"
BDX_DOFMAP_API(double, f64)

// Writer designation of the dofmap CG (type independent): the first
// occurrence of every dof over the launch order [cells_a..., cells_b...]
// gets the sign bit in cdofs, every other occurrence loses it.  first:
// scratch of ndofs unsigned.
extern "C" int bdx_dofmap_mark_writers(const int* cells_a, int na, const int* cells_b, int nb,
                                       int* cdofs, int nd3, unsigned* first, int64_t ndofs,
                                       hipStream_t st) {
  if ((static_cast<int64_t>(na) + nb) * nd3 >= 0xffffffffLL)
    return static_cast<int>(hipErrorInvalidValue);
  BDX_CHECK(hipMemsetAsync(first, 0xff, ndofs * sizeof(unsigned), st));
  // launch positions are unsigned 32-bit (< 2^32 - 1 by the guard above)
  const unsigned pos_b = static_cast<unsigned>(static_cast<int64_t>(na) * nd3);
  auto grid = [&](int n) {
    return static_cast<unsigned>((static_cast<int64_t>(n) * nd3 + 255) / 256);
  };
  if (na > 0) dofmap_first_kernel<<<grid(na), 256, 0, st>>>(cells_a, na, cdofs, nd3, 0u, first);
  if (nb > 0) dofmap_first_kernel<<<grid(nb), 256, 0, st>>>(cells_b, nb, cdofs, nd3, pos_b, first);
  if (na > 0) dofmap_mark_kernel<<<grid(na), 256, 0, st>>>(cells_a, na, cdofs, nd3, 0u, first);
  if (nb > 0) dofmap_mark_kernel<<<grid(nb), 256, 0, st>>>(cells_b, nb, cdofs, nd3, pos_b, first);
  return static_cast<int>(hipGetLastError());
}
