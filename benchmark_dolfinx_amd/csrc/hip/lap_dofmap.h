// Unstructured-data-model operator ("dofmap"): the reference's general mesh
// representation instead of lattice index arithmetic.
//
// Inputs are the arrays a DOLFINx mesh carries (reference src/laplacian.hpp:
// 105-114 and src/laplacian_gpu.hpp:153-170, built in src/mesh.cpp:87-102):
//   cell_dofs  [ncells][ND^3]  cell -> dof map (tensor-product order i, j, k)
//   cell_verts [ncells][8]     cell -> geometry-node map (v = 4a + 2b + c)
//   coords     [nverts][3]     geometry nodes
//   dof_flags  [ndofs]         bit 0: Dirichlet dof, bit 1: owned by this rank
//   cells      [ncl]           the cells of this launch (interior or boundary
//                              list, so the halo exchange can overlap the
//                              interior cells as in src/laplacian.hpp:281-349)
// and optionally stored G [ncells][6][nq^3] (the reference layout) and a
// per-cell coefficient.  Any hexahedral mesh, any cell order and any dof
// numbering work: nothing is derived from a lattice.  The per-cell core is
// v1's (lap_v1.h: one thread per quadrature point, sum factorisation through
// LDS); the element vectors are scattered with float atomics like the
// reference's kernel.  This path measures what the dofmap indirection costs;
// the structured kernels (lap_fused*.h) are the performance path.
#pragma once
#include "lap_v1.h"

// dofmap: v1 core on an explicit cell->dof / cell->vertex map (any hex mesh).
template <typename T, int ND, int NQ, int GEOM>
__global__ void __launch_bounds__(V1Shape<NQ>::threads)
    lap_dofmap_kernel(const int* __restrict__ cells, int ncl, const int* __restrict__ cdofs,
                      const int* __restrict__ cverts, const T* __restrict__ coords,
                      const unsigned char* __restrict__ flags, OpTables<T> tb,
                      const T* __restrict__ G, T kappa, const T* __restrict__ kc,
                      const T* __restrict__ u, T* __restrict__ y) {
  constexpr int nq3 = NQ * NQ * NQ, ND3 = ND * ND * ND;
  constexpr int CPB = V1Shape<NQ>::cpb;
  __shared__ V1Smem<T, ND, NQ> sm;
  const int tid = threadIdx.x;
  for (int i = tid; i < NQ * ND; i += blockDim.x) sm.phi0[i] = tb.phi0[i];
  for (int i = tid; i < NQ * NQ; i += blockDim.x) sm.dphi[i] = tb.dphi1[i];

  const int cs = tid / nq3;
  const int q = tid - cs * nq3;
  const int qx = q / (NQ * NQ), qy = (q / NQ) % NQ, qz = q % NQ;
  const bool active = cs < CPB;
  const int64_t li = static_cast<int64_t>(blockIdx.x) * CPB + cs;
  const bool valid = active && li < ncl;
  const int64_t cell = valid ? cells[li] : 0;
  const bool is_dof = valid && qx < ND && qy < ND && qz < ND;
  int dof = -1;
  unsigned f = 0;
  if (is_dof) {
    dof = cdofs[cell * ND3 + (qx * ND + qy) * ND + qz];
    BDX_DASSERT(dof >= 0);
    f = flags[dof];
  }
  const bool bc = f & 1u;
  if (active) sm.s0[cs][q] = (is_dof && !bc) ? u[dof] : T(0);
  if constexpr (GEOM == kGeomOTF) {
    if (active && q < 24 && valid) {
      const int v = q / 3, d = q % 3;
      sm.X[cs][v][d] = coords[3 * static_cast<int64_t>(cverts[cell * 8 + v]) + d];
    }
  }
  __syncthreads();
  const T* Gc = (GEOM == kGeomStored && valid) ? G + cell * 6 * nq3 : G;
  const T kap = (kc && valid) ? kc[cell] : kappa;
  const T ye = v1_core<T, ND, NQ, kModeStiffness, GEOM>(sm, tb, cs, q, active, valid, Gc, kap);
  if (is_dof) {
    if (!bc)
      atomicAdd(y + dof, ye);
    else if (f & 2u)
      y[dof] = u[dof];  // Dirichlet identity row (owned copy only)
  }
}

// Stored G in the reference layout for a cell list (geometry_computation_gpu,
// src/geometry_gpu.hpp:26-132): one thread per (cell, quadrature point).
template <typename T, int NQ>
__global__ void __launch_bounds__(256)
    dofmap_geometry_kernel(int ncells, const int* __restrict__ cverts, const T* __restrict__ coords,
                           OpTables<T> tb, T* __restrict__ G) {
  constexpr int nq3 = NQ * NQ * NQ;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(ncells) * nq3) return;
  const int64_t cell = t / nq3;
  const int q = static_cast<int>(t - cell * nq3);
  const int qx = q / (NQ * NQ), qy = (q / NQ) % NQ, qz = q % NQ;
  T X[8][3];
#pragma unroll
  for (int v = 0; v < 8; ++v)
#pragma unroll
    for (int d = 0; d < 3; ++d) X[v][d] = coords[3 * static_cast<int64_t>(cverts[cell * 8 + v]) + d];
  T Gd[6];
  geometry_G<T>(X, tb.qpts[qx], tb.qpts[qy], tb.qpts[qz], tb.wts[qx] * tb.wts[qy] * tb.wts[qz], Gd);
#pragma unroll
  for (int k = 0; k < 6; ++k) G[(cell * 6 + k) * nq3 + q] = Gd[k];
}

template <typename T, int ND, int NQ>
int launch_dofmap(int geom, const int* cells, int ncl, const int* cdofs, const int* cverts,
                  const T* coords, const unsigned char* flags, const OpTables<T>& tb, const T* G,
                  T kappa, const T* kc, const T* u, T* y, hipStream_t st) {
  if (ncl <= 0) return 0;
  constexpr int cpb = V1Shape<NQ>::cpb;
  const int nblk = (ncl + cpb - 1) / cpb;
  if (geom == kGeomStored)
    lap_dofmap_kernel<T, ND, NQ, kGeomStored><<<nblk, V1Shape<NQ>::threads, 0, st>>>(
        cells, ncl, cdofs, cverts, coords, flags, tb, G, kappa, kc, u, y);
  else
    lap_dofmap_kernel<T, ND, NQ, kGeomOTF><<<nblk, V1Shape<NQ>::threads, 0, st>>>(
        cells, ncl, cdofs, cverts, coords, flags, tb, G, kappa, kc, u, y);
  return static_cast<int>(hipGetLastError());
}

template <typename T, int NQ>
int launch_dofmap_geometry(int ncells, const int* cverts, const T* coords, const OpTables<T>& tb,
                           T* G, hipStream_t st) {
  constexpr int nq3 = NQ * NQ * NQ;
  const int64_t n = static_cast<int64_t>(ncells) * nq3;
  if (n <= 0) return 0;
  const int64_t nblk = (n + 255) / 256;
  if (nblk > 0x7fffffffLL) return static_cast<int>(hipErrorInvalidValue);
  dofmap_geometry_kernel<T, NQ><<<static_cast<unsigned>(nblk), 256, 0, st>>>(ncells, cverts, coords,
                                                                             tb, G);
  return static_cast<int>(hipGetLastError());
}

#define BDX_DOFMAP_API(T, SUF)                                                                    \
  extern "C" int bdx_dofmap_apply_##SUF(int P, int nq, int geom, const double* phi0,             \
                                        const double* dphi1, const double* wts,                   \
                                        const double* qpts, int identity, const int* cells,       \
                                        int ncl, const int* cdofs, const int* cverts,             \
                                        const T* coords, const unsigned char* flags, const T* G,  \
                                        double kappa, const T* kc, const T* u, T* y,              \
                                        hipStream_t st) {                                         \
    const OpTables<T> tb = make_op_tables<T>(P + 1, nq, phi0, dphi1, wts, qpts, identity);       \
    const T k = static_cast<T>(kappa);                                                            \
    switch (P * 16 + nq) {                                                                        \
      BDX_DOFMAP_CASE(T, 1)                                                                       \
      BDX_DOFMAP_CASE(T, 2)                                                                       \
      BDX_DOFMAP_CASE(T, 3)                                                                       \
      BDX_DOFMAP_CASE(T, 4)                                                                       \
      BDX_DOFMAP_CASE(T, 5)                                                                       \
      BDX_DOFMAP_CASE(T, 6)                                                                       \
      BDX_DOFMAP_CASE(T, 7)                                                                       \
    }                                                                                             \
    return static_cast<int>(hipErrorInvalidValue);                                                \
  }                                                                                               \
  extern "C" int bdx_dofmap_geometry_##SUF(int P, int nq, const double* phi0, const double* dphi1, \
                                           const double* wts, const double* qpts, int ncells,     \
                                           const int* cverts, const T* coords, T* G,              \
                                           hipStream_t st) {                                      \
    const OpTables<T> tb = make_op_tables<T>(P + 1, nq, phi0, dphi1, wts, qpts, 0);               \
    switch (nq) {                                                                                 \
      case 2: return launch_dofmap_geometry<T, 2>(ncells, cverts, coords, tb, G, st);             \
      case 3: return launch_dofmap_geometry<T, 3>(ncells, cverts, coords, tb, G, st);             \
      case 4: return launch_dofmap_geometry<T, 4>(ncells, cverts, coords, tb, G, st);             \
      case 5: return launch_dofmap_geometry<T, 5>(ncells, cverts, coords, tb, G, st);             \
      case 6: return launch_dofmap_geometry<T, 6>(ncells, cverts, coords, tb, G, st);             \
      case 7: return launch_dofmap_geometry<T, 7>(ncells, cverts, coords, tb, G, st);             \
      case 8: return launch_dofmap_geometry<T, 8>(ncells, cverts, coords, tb, G, st);             \
      case 9: return launch_dofmap_geometry<T, 9>(ncells, cverts, coords, tb, G, st);             \
    }                                                                                             \
    return static_cast<int>(hipErrorInvalidValue);                                                \
  }

#define BDX_DOFMAP_CASE(T, PP)                                                                    \
  case PP * 16 + PP + 1:                                                                          \
    return launch_dofmap<T, PP + 1, PP + 1>(geom, cells, ncl, cdofs, cverts, coords, flags, tb,   \
                                            G, k, kc, u, y, st);                                  \
  case PP * 16 + PP + 2:                                                                          \
    return launch_dofmap<T, PP + 1, PP + 2>(geom, cells, ncl, cdofs, cverts, coords, flags, tb,   \
                                            G, k, kc, u, y, st);
