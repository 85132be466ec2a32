// dofmap (unstructured data model) operator, double instantiations.
#include <cstdlib>

#include "lap_dofmap.h"
BDX_DOFMAP_API(double, f64)

// kernel choice of the FP64 dofmap launches (lap_dofmap.h): -1 = environment
// (BDX_DOFMAP_MFMA) / default, 0 = VALU kernel, 1 = MFMA kernel
static int g_dofmap_mfma = -1;
// Select the FP64 dofmap operator kernel for later launches (tests, A/B).
extern "C" int bdx_dofmap_set_mfma(int mode) {
  g_dofmap_mfma = mode < 0 ? -1 : (mode ? 1 : 0);
  return 0;
}
int bdx_dofmap_mfma_mode() {
  if (g_dofmap_mfma >= 0) return g_dofmap_mfma;
  const char* e = std::getenv("BDX_DOFMAP_MFMA");
  if (e && *e) return std::atoi(e) ? 1 : 0;
  return -1;
}
// Which kernel an FP64 dofmap launch of this element takes right now (the
// selection of launch_dofmap): 1 = lap_dofmfma_kernel, 0 = lap_dofmap_kernel.
extern "C" int bdx_dofmap_uses_mfma(int nd, int nq) {
  if (nd > 8 || nq > 8) return 0;
  const int mm = bdx_dofmap_mfma_mode();
  return (mm == 1 || (mm < 0 && kDofMfmaDefault(nq))) ? 1 : 0;
}

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

// p.Ap partials (blocks) of a CG launch over ncl cells at this rule (the
// native runtime places the boundary launch's partials after the interior's)
extern "C" int bdx_dofmap_nblocks(int nq, int ncl) {
  int cpb = 0;
  if (ncl <= 0) return 0;
  switch (nq) {
    case 2: return dofmap_blocks<2>(ncl, &cpb);
    case 3: return dofmap_blocks<3>(ncl, &cpb);
    case 4: return dofmap_blocks<4>(ncl, &cpb);
    case 5: return dofmap_blocks<5>(ncl, &cpb);
    case 6: return dofmap_blocks<6>(ncl, &cpb);
    case 7: return dofmap_blocks<7>(ncl, &cpb);
    case 8: return dofmap_blocks<8>(ncl, &cpb);
    case 9: return dofmap_blocks<9>(ncl, &cpb);
  }
  return -1;
}
