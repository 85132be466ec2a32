// Host (CPU) runtime of benchmark_dolfinx_amd.
//
// Native replacements for the DOLFINx/Basix machinery the reference leans on
//  plus its CPU operator:
//   * stiffness action, sum-factorised, any P in 1..7 and qmode 0/1
//     (the reference CPU kernel supports only qmode 0: src/laplacian_cpu.hpp:73,
//     quirk Q4; here both work);
//   * mass action (RHS b = M f; replaces fem::assemble_vector + the FFCx
//     kernel, src/laplacian_solver.cpp:100-105);
//   * interpolation of f at the physical dof nodes (src/main.cpp:81-92);
//   * CSR assembly of the local stiffness matrix with Dirichlet rows/cols
//     replaced by the identity (replaces create_sparsity_pattern +
//     assemble_matrix + set_diagonal, src/laplacian_solver.cpp:161-184);
//   * CSR SpMV (CPUMatrixOperator, src/laplacian_solver.cpp:247-262).
// Geometry factors are computed on the fly per cell with 64-bit offsets
// everywhere (reference quirk Q6: int offset in src/geometry_cpu.hpp:91).
//
// Parallelism: OpenMP over the cells of one of 8 parity colours at a time, so
// no two concurrently processed cells share a dof: the scatter is race-free
// and deterministic.

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "../include/bdx_lattice.h"
#include "../include/bdx_watchdog.h"

namespace {

template <typename T>
struct Tables {
  const T* phi0;   // nq x nd
  const T* dphi1;  // nq x nq
  const T* wts;    // nq
  const T* qpts;   // nq
  const T* nodes;  // nd
  bool identity;
};

// Geometry factor G = w * adj(J) adj(J)^T / det(J) at one point of a
// trilinear cell with vertices X[8][3] (v = 4a+2b+c), reference point (s,t,u).
template <typename T>
inline T geometry_point(const T X[8][3], T s, T t, T u, T w, T G[6]) {
  T J[3][3];
  for (int i = 0; i < 3; ++i) {
    T d0 = 0, d1 = 0, d2 = 0;
    for (int a = 0; a < 2; ++a)
      for (int b = 0; b < 2; ++b)
        for (int c = 0; c < 2; ++c) {
          const T x = X[4 * a + 2 * b + c][i];
          const T fx = a ? s : 1 - s, fy = b ? t : 1 - t, fz = c ? u : 1 - u;
          const T sx = a ? 1 : -1, sy = b ? 1 : -1, sz = c ? 1 : -1;
          d0 += x * sx * fy * fz;
          d1 += x * fx * sy * fz;
          d2 += x * fx * fy * sz;
        }
    J[i][0] = d0;
    J[i][1] = d1;
    J[i][2] = d2;
  }
  // K = adj(J) = det(J) J^{-1}
  const T K[3][3] = {{J[1][1] * J[2][2] - J[1][2] * J[2][1],
                      J[0][2] * J[2][1] - J[0][1] * J[2][2],
                      J[0][1] * J[1][2] - J[0][2] * J[1][1]},
                     {J[1][2] * J[2][0] - J[1][0] * J[2][2],
                      J[0][0] * J[2][2] - J[0][2] * J[2][0],
                      J[0][2] * J[1][0] - J[0][0] * J[1][2]},
                     {J[1][0] * J[2][1] - J[1][1] * J[2][0],
                      J[0][1] * J[2][0] - J[0][0] * J[2][1],
                      J[0][0] * J[1][1] - J[0][1] * J[1][0]}};
  const T det = J[0][0] * K[0][0] + J[0][1] * K[1][0] + J[0][2] * K[2][0];
  const T sc = w / det;
  G[0] = (K[0][0] * K[0][0] + K[0][1] * K[0][1] + K[0][2] * K[0][2]) * sc;
  G[1] = (K[1][0] * K[0][0] + K[1][1] * K[0][1] + K[1][2] * K[0][2]) * sc;
  G[2] = (K[2][0] * K[0][0] + K[2][1] * K[0][1] + K[2][2] * K[0][2]) * sc;
  G[3] = (K[1][0] * K[1][0] + K[1][1] * K[1][1] + K[1][2] * K[1][2]) * sc;
  G[4] = (K[2][0] * K[1][0] + K[2][1] * K[1][1] + K[2][2] * K[1][2]) * sc;
  G[5] = (K[2][0] * K[2][0] + K[2][1] * K[2][1] + K[2][2] * K[2][2]) * sc;
  return det;
}

template <typename T>
inline void cell_vertices(const BdxLattice& lat, const T* xv, int64_t cx,
                          int64_t cy, int64_t cz, T X[8][3]) {
  for (int a = 0; a < 2; ++a)
    for (int b = 0; b < 2; ++b)
      for (int c = 0; c < 2; ++c) {
        const int64_t v = lat.vidx(cx + a, cy + b, cz + c);
        for (int d = 0; d < 3; ++d) X[4 * a + 2 * b + c][d] = xv[3 * v + d];
      }
}

// out = A applied along axis `ax` of `in` (extents e), A is M x K row-major
// (or K x M used transposed).
template <typename T>
inline void contract(const T* A, int M, int K, bool transpose, const T* in,
                     const int e[3], int ax, T* out) {
  int eo[3] = {e[0], e[1], e[2]};
  eo[ax] = M;
  const int s_in[3] = {e[1] * e[2], e[2], 1};
  const int s_out[3] = {eo[1] * eo[2], eo[2], 1};
  for (int i = 0; i < eo[0]; ++i)
    for (int j = 0; j < eo[1]; ++j)
      for (int k = 0; k < eo[2]; ++k) {
        int o[3] = {i, j, k};
        const int m = o[ax];
        T acc = 0;
        for (int q = 0; q < K; ++q) {
          o[ax] = q;
          const T a = transpose ? A[q * M + m] : A[m * K + q];
          acc += a * in[o[0] * s_in[0] + o[1] * s_in[1] + o[2] * s_in[2]];
        }
        out[i * s_out[0] + j * s_out[1] + k * s_out[2]] = acc;
      }
}

// Interpolate element dofs (nd^3) to quadrature points (nq^3).
template <typename T, int ND, int NQ>
inline void interp(const Tables<T>& tb, const T* ue, T* U, T* t1, T* t2) {
  if (tb.identity) {
    std::memcpy(U, ue, sizeof(T) * NQ * NQ * NQ);
    return;
  }
  const int e0[3] = {ND, ND, ND};
  contract(tb.phi0, NQ, ND, false, ue, e0, 0, t1);
  const int e1[3] = {NQ, ND, ND};
  contract(tb.phi0, NQ, ND, false, t1, e1, 1, t2);
  const int e2[3] = {NQ, NQ, ND};
  contract(tb.phi0, NQ, ND, false, t2, e2, 2, U);
}

// Transposed interpolation (nq^3 -> nd^3).
template <typename T, int ND, int NQ>
inline void interp_t(const Tables<T>& tb, const T* r, T* ye, T* t1, T* t2) {
  if (tb.identity) {
    std::memcpy(ye, r, sizeof(T) * ND * ND * ND);
    return;
  }
  const int e0[3] = {NQ, NQ, NQ};
  contract(tb.phi0, ND, NQ, true, r, e0, 2, t1);
  const int e1[3] = {NQ, NQ, ND};
  contract(tb.phi0, ND, NQ, true, t1, e1, 1, t2);
  const int e2[3] = {NQ, ND, ND};
  contract(tb.phi0, ND, NQ, true, t2, e2, 0, ye);
}

// y += kappa * A_cell u for one cell, BC semantics of the reference
// (src/laplacian_gpu.hpp:153-170, 424-425): BC inputs are zeroed, BC outputs
// get y = u (only on the owning rank).
// Compile-time extents (the loops unroll and the innermost axis -- contiguous
// qz or the NQ^2 plane -- vectorises) and, when the caller precomputed them,
// the geometry factors G[6][nq^3] of the cell in the reference layout
// (src/geometry_cpu.hpp; computed once per operator by bdx_cpu_geometry, as
// the reference's MatFreeLaplacianCPU does, src/laplacian.hpp:515-541).
// Gc == nullptr: per-point trilinear geometry.  Round 6: this replaced a
// runtime-extent version (generic contract() with index arrays, geometry per
// point): 1 M DoF Q3 CG on 8 cores 0.0093 -> see docs/PARITY.md.
template <typename T, int ND, int NQ>
struct CellTables {
  T B[NQ][ND], D[NQ][NQ], w[NQ], q[NQ];
  bool ident;
  explicit CellTables(const Tables<T>& tb) : ident(tb.identity) {
    for (int a = 0; a < NQ; ++a) {
      for (int i = 0; i < ND; ++i) B[a][i] = tb.phi0[a * ND + i];
      for (int m = 0; m < NQ; ++m) D[a][m] = tb.dphi1[a * NQ + m];
      w[a] = tb.wts[a];
      q[a] = tb.qpts[a];
    }
  }
};

// ye = A_e ue for one cell (no BC handling): geometry factors from Gc
// (reference layout [6][nq^3]) or, when Gc is null, per point from the
// cell's vertices X.
template <typename T, int ND, int NQ>
inline void cell_core(const CellTables<T, ND, NQ>& tb, const T (&ue)[ND][ND][ND], const T* Gc,
                      const T (*X)[3], T kappa, T (&ye)[ND][ND][ND]) {
  constexpr int nd3 = ND * ND * ND, NQ2 = NQ * NQ, nq3 = NQ * NQ2;
  // interpolation to the quadrature points (z, y, x)
  T U[NQ][NQ][NQ];
  if (tb.ident && ND == NQ) {
    std::memcpy(U, ue, sizeof(T) * nq3);
  } else {
    T t1[ND][ND][NQ], t2[ND][NQ][NQ];
    for (int i = 0; i < ND; ++i)
      for (int j = 0; j < ND; ++j)
        for (int qz = 0; qz < NQ; ++qz) {
          T s = 0;
          for (int k = 0; k < ND; ++k) s += tb.B[qz][k] * ue[i][j][k];
          t1[i][j][qz] = s;
        }
    for (int i = 0; i < ND; ++i)
      for (int qy = 0; qy < NQ; ++qy) {
        T acc[NQ] = {};
        for (int j = 0; j < ND; ++j)
          for (int qz = 0; qz < NQ; ++qz) acc[qz] += tb.B[qy][j] * t1[i][j][qz];
        for (int qz = 0; qz < NQ; ++qz) t2[i][qy][qz] = acc[qz];
      }
    for (int qx = 0; qx < NQ; ++qx) {
      T acc[NQ2] = {};
      for (int i = 0; i < ND; ++i)
        for (int p = 0; p < NQ2; ++p) acc[p] += tb.B[qx][i] * (&t2[i][0][0])[p];
      std::memcpy(&U[qx][0][0], acc, sizeof(acc));
    }
  }
  // reference gradient
  T gx[NQ][NQ][NQ], gy[NQ][NQ][NQ], gz[NQ][NQ][NQ];
  for (int qx = 0; qx < NQ; ++qx) {
    T acc[NQ2] = {};
    for (int m = 0; m < NQ; ++m)
      for (int p = 0; p < NQ2; ++p) acc[p] += tb.D[qx][m] * (&U[m][0][0])[p];
    std::memcpy(&gx[qx][0][0], acc, sizeof(acc));
  }
  for (int qx = 0; qx < NQ; ++qx)
    for (int qy = 0; qy < NQ; ++qy) {
      T acc[NQ] = {};
      for (int m = 0; m < NQ; ++m)
        for (int qz = 0; qz < NQ; ++qz) acc[qz] += tb.D[qy][m] * U[qx][m][qz];
      for (int qz = 0; qz < NQ; ++qz) gy[qx][qy][qz] = acc[qz];
      for (int qz = 0; qz < NQ; ++qz) {
        T s = 0;
        for (int m = 0; m < NQ; ++m) s += tb.D[qz][m] * U[qx][qy][m];
        gz[qx][qy][qz] = s;
      }
    }
  // kappa G grad u
  for (int qx = 0; qx < NQ; ++qx)
    for (int qy = 0; qy < NQ; ++qy)
      for (int qz = 0; qz < NQ; ++qz) {
        const int q = (qx * NQ + qy) * NQ + qz;
        T G[6];
        if (Gc) {
          for (int c = 0; c < 6; ++c) G[c] = Gc[c * nq3 + q];
        } else {
          geometry_point<T>(X, tb.q[qx], tb.q[qy], tb.q[qz], tb.w[qx] * tb.w[qy] * tb.w[qz], G);
        }
        const T a = gx[qx][qy][qz], b = gy[qx][qy][qz], c = gz[qx][qy][qz];
        gx[qx][qy][qz] = kappa * (G[0] * a + G[1] * b + G[2] * c);
        gy[qx][qy][qz] = kappa * (G[1] * a + G[3] * b + G[4] * c);
        gz[qx][qy][qz] = kappa * (G[2] * a + G[4] * b + G[5] * c);
      }
  // transposed gradient: r = Dx^T gx + Dy^T gy + Dz^T gz
  T r[NQ][NQ][NQ];
  for (int m = 0; m < NQ; ++m) {
    T acc[NQ2] = {};
    for (int qx = 0; qx < NQ; ++qx)
      for (int p = 0; p < NQ2; ++p) acc[p] += tb.D[qx][m] * (&gx[qx][0][0])[p];
    std::memcpy(&r[m][0][0], acc, sizeof(acc));
  }
  for (int qx = 0; qx < NQ; ++qx)
    for (int m = 0; m < NQ; ++m) {
      T acc[NQ] = {};
      for (int qy = 0; qy < NQ; ++qy)
        for (int qz = 0; qz < NQ; ++qz) acc[qz] += tb.D[qy][m] * gy[qx][qy][qz];
      for (int qz = 0; qz < NQ; ++qz) r[qx][m][qz] += acc[qz];
    }
  for (int qx = 0; qx < NQ; ++qx)
    for (int qy = 0; qy < NQ; ++qy) {
      T acc[NQ] = {};
      for (int qz = 0; qz < NQ; ++qz)
        for (int m = 0; m < NQ; ++m) acc[m] += tb.D[qz][m] * gz[qx][qy][qz];
      for (int m = 0; m < NQ; ++m) r[qx][qy][m] += acc[m];
    }
  // transposed interpolation (x, y, z)
  if (tb.ident && ND == NQ) {
    std::memcpy(ye, r, sizeof(T) * nd3);
  } else {
    T t2[ND][NQ][NQ], t1[ND][ND][NQ];
    for (int i = 0; i < ND; ++i) {
      T acc[NQ2] = {};
      for (int qx = 0; qx < NQ; ++qx)
        for (int p = 0; p < NQ2; ++p) acc[p] += tb.B[qx][i] * (&r[qx][0][0])[p];
      std::memcpy(&t2[i][0][0], acc, sizeof(acc));
    }
    for (int i = 0; i < ND; ++i)
      for (int j = 0; j < ND; ++j) {
        T acc[NQ] = {};
        for (int qy = 0; qy < NQ; ++qy)
          for (int qz = 0; qz < NQ; ++qz) acc[qz] += tb.B[qy][j] * t2[i][qy][qz];
        for (int qz = 0; qz < NQ; ++qz) t1[i][j][qz] = acc[qz];
      }
    for (int i = 0; i < ND; ++i)
      for (int j = 0; j < ND; ++j)
        for (int k = 0; k < ND; ++k) {
          T s = 0;
          for (int qz = 0; qz < NQ; ++qz) s += tb.B[qz][k] * t1[i][j][qz];
          ye[i][j][k] = s;
        }
  }
}

template <typename T, int ND, int NQ>
void stiffness_cell_fast(const BdxLattice& lat, const CellTables<T, ND, NQ>& tb, const T* xv,
                         const T* Gc, T kappa, const T* kc, const T* u, T* y, int64_t cx,
                         int64_t cy, int64_t cz) {
  if (kc) kappa = kc[(cx * lat.n[1] + cy) * lat.n[2] + cz];
  constexpr int nd3 = ND * ND * ND;
  const int64_t P = lat.P;
  T ue[ND][ND][ND];
  int64_t dof[nd3];
  bool bc[nd3];
  for (int i = 0; i < ND; ++i)
    for (int j = 0; j < ND; ++j)
      for (int k = 0; k < ND; ++k) {
        const int a = (i * ND + j) * ND + k;
        const int64_t li = cx * P + i, lj = cy * P + j, lk = cz * P + k;
        dof[a] = lat.idx(li, lj, lk);
        bc[a] = lat.is_bc(li, lj, lk);
        ue[i][j][k] = bc[a] ? T(0) : u[dof[a]];
      }
  T X[8][3];
  if (!Gc) cell_vertices(lat, xv, cx, cy, cz, X);
  T ye[ND][ND][ND];
  cell_core<T, ND, NQ>(tb, ue, Gc, X, kappa, ye);
  const T* yf = &ye[0][0][0];
  for (int a = 0; a < nd3; ++a) {
    if (!bc[a]) {
      y[dof[a]] += yf[a];
    } else {
      const int i = a / (ND * ND), j = (a / ND) % ND, k = a % ND;
      if (lat.is_owned(cx * P + i, cy * P + j, cz * P + k)) y[dof[a]] = u[dof[a]];
    }
  }
}

// The reference data model on the CPU (its MatFreeLaplacianCPU gathers
// through the cell -> dof map with G stored per cell, src/laplacian.hpp:
// 592-631): y += A u over the listed cells, cell_dofs (sign bit = writer,
// ignored here), per-dof flags (bit 0 Dirichlet, bit 1 owned), stored G
// [cell][6][nq^3] or per-point geometry from cell_verts / coords.  Cells run
// in parallel; the scatter uses atomic adds (any mesh, any cell order), the
// Dirichlet identity rows an atomic write of u (every writer writes the
// same value).
template <typename T, int ND, int NQ>
void dofmap_cells(const CellTables<T, ND, NQ>& tb, const int* cells, int ncl, const int* cdofs,
                  const int* cverts, const T* coords, const T* G,
                  const unsigned char* flags, T kappa, const T* kc, const T* u, T* y) {
  constexpr int nd3 = ND * ND * ND, nq3 = NQ * NQ * NQ;
#pragma omp parallel for schedule(dynamic, 16)
  for (int li = 0; li < ncl; ++li) {
    const int64_t c = cells[li];
    T ue[ND][ND][ND];
    T* uf = &ue[0][0][0];
    int64_t dof[nd3];
    unsigned char fl[nd3];
    for (int a = 0; a < nd3; ++a) {
      dof[a] = cdofs[c * nd3 + a] & 0x7fffffff;
      fl[a] = flags[dof[a]];
      uf[a] = (fl[a] & 1u) ? T(0) : u[dof[a]];
    }
    T X[8][3];
    if (!G)
      for (int v = 0; v < 8; ++v)
        for (int d = 0; d < 3; ++d) X[v][d] = coords[3 * int64_t{cverts[c * 8 + v]} + d];
    T ye[ND][ND][ND];
    cell_core<T, ND, NQ>(tb, ue, G ? G + c * 6 * nq3 : nullptr, X, kc ? kc[c] : kappa, ye);
    const T* yf = &ye[0][0][0];
    for (int a = 0; a < nd3; ++a) {
      if (!(fl[a] & 1u)) {
#pragma omp atomic
        y[dof[a]] += yf[a];
      } else if (fl[a] & 2u) {
#pragma omp atomic write
        y[dof[a]] = u[dof[a]];
      }
    }
  }
}

template <typename T>
struct DofArgsCPU {
  Tables<T> tb;
  const int *cells, *cdofs, *cverts;
  int ncl;
  const T *coords, *G;
  const unsigned char* flags;
  T kappa;
  const T *kc, *u;
  T* y;
};

template <typename T>
struct DofmapCPU {
  template <int ND, int NQ>
  struct K {
    static void run(const DofArgsCPU<T>& a) {
      const CellTables<T, ND, NQ> tb(a.tb);
      dofmap_cells<T, ND, NQ>(tb, a.cells, a.ncl, a.cdofs, a.cverts, a.coords, a.G, a.flags,
                              a.kappa, a.kc, a.u, a.y);
    }
  };
};

// Stored G of explicit cells (cell_verts / coords): the reference's
// geometry_computation_cpu on the dofmap data model.
template <typename T, int NQ>
void dofmap_geometry_cpu(int ncells, const int* cverts, const T* coords, const T* wts,
                         const T* qpts, T* G) {
  constexpr int nq3 = NQ * NQ * NQ;
#pragma omp parallel for schedule(static)
  for (int c = 0; c < ncells; ++c) {
    T X[8][3];
    for (int v = 0; v < 8; ++v)
      for (int d = 0; d < 3; ++d) X[v][d] = coords[3 * int64_t{cverts[int64_t{c} * 8 + v]} + d];
    T* Gc = G + int64_t{c} * 6 * nq3;
    for (int qx = 0; qx < NQ; ++qx)
      for (int qy = 0; qy < NQ; ++qy)
        for (int qz = 0; qz < NQ; ++qz) {
          const int q = (qx * NQ + qy) * NQ + qz;
          T g[6];
          geometry_point<T>(X, qpts[qx], qpts[qy], qpts[qz], wts[qx] * wts[qy] * wts[qz], g);
          for (int k = 0; k < 6; ++k) Gc[k * nq3 + q] = g[k];
        }
  }
}

template <typename T>
struct DofGeomArgs {
  int ncells;
  const int* cverts;
  const T *coords, *wts, *qpts;
  T* G;
};

template <typename T>
struct DofGeomCPU {
  template <int ND, int NQ>
  struct K {
    static void run(const DofGeomArgs<T>& a) {
      dofmap_geometry_cpu<T, NQ>(a.ncells, a.cverts, a.coords, a.wts, a.qpts, a.G);
    }
  };
};

// Geometry factors of every local cell in the reference layout
// G[c][6][nq^3], c = (cx n1 + cy) n2 + cz (geometry_computation_cpu,
// src/geometry_cpu.hpp:25-112, with 64-bit offsets: quirk Q6).
template <typename T, int NQ>
void geometry_all(const BdxLattice& lat, const T* wts, const T* qpts, const T* xv, T* G) {
  constexpr int nq3 = NQ * NQ * NQ;
#pragma omp parallel for collapse(3) schedule(static)
  for (int64_t cx = 0; cx < lat.n[0]; ++cx)
    for (int64_t cy = 0; cy < lat.n[1]; ++cy)
      for (int64_t cz = 0; cz < lat.n[2]; ++cz) {
        T X[8][3];
        cell_vertices(lat, xv, cx, cy, cz, X);
        T* Gc = G + ((cx * lat.n[1] + cy) * lat.n[2] + cz) * int64_t{6} * nq3;
        for (int qx = 0; qx < NQ; ++qx)
          for (int qy = 0; qy < NQ; ++qy)
            for (int qz = 0; qz < NQ; ++qz) {
              const int q = (qx * NQ + qy) * NQ + qz;
              T g[6];
              geometry_point<T>(X, qpts[qx], qpts[qy], qpts[qz], wts[qx] * wts[qy] * wts[qz], g);
              for (int c = 0; c < 6; ++c) Gc[c * nq3 + q] = g[c];
            }
      }
}

// b += M_cell f (no BC handling; the caller zeroes BC rows afterwards).
template <typename T, int ND, int NQ>
void mass_cell(const BdxLattice& lat, const Tables<T>& tb, const T* xv,
               const T* f, T* b, int64_t cx, int64_t cy, int64_t cz) {
  constexpr int nd3 = ND * ND * ND, nq3 = NQ * NQ * NQ;
  const int64_t P = lat.P;
  T fe[nd3];
  int64_t dof[nd3];
  for (int i = 0; i < ND; ++i)
    for (int j = 0; j < ND; ++j)
      for (int k = 0; k < ND; ++k) {
        const int a = (i * ND + j) * ND + k;
        dof[a] = lat.idx(cx * P + i, cy * P + j, cz * P + k);
        fe[a] = f[dof[a]];
      }
  T F[nq3], t1[nq3], t2[nq3];
  interp<T, ND, NQ>(tb, fe, F, t1, t2);
  T X[8][3];
  cell_vertices(lat, xv, cx, cy, cz, X);
  for (int qx = 0; qx < NQ; ++qx)
    for (int qy = 0; qy < NQ; ++qy)
      for (int qz = 0; qz < NQ; ++qz) {
        const int q = (qx * NQ + qy) * NQ + qz;
        T G[6];
        const T w = tb.wts[qx] * tb.wts[qy] * tb.wts[qz];
        const T det =
            geometry_point<T>(X, tb.qpts[qx], tb.qpts[qy], tb.qpts[qz], T(1), G);
        F[q] *= w * det;
      }
  T be[nd3];
  interp_t<T, ND, NQ>(tb, F, be, t1, t2);
  for (int a = 0; a < nd3; ++a) b[dof[a]] += be[a];
}

// Loop over a box of cells in 8 colour phases (parity of cx, cy, cz): cells
// of one colour share no dof, so the scatter-add is race-free and the
// summation order is deterministic.
template <typename F>
void for_cells(const int64_t lo[3], const int64_t hi[3], F&& fn) {
  for (int colour = 0; colour < 8; ++colour) {
    const int64_t ox = (colour >> 2) & 1, oy = (colour >> 1) & 1, oz = colour & 1;
#pragma omp parallel for schedule(dynamic, 4) collapse(3)
    for (int64_t cx = lo[0] + ox; cx < hi[0]; cx += 2)
      for (int64_t cy = lo[1] + oy; cy < hi[1]; cy += 2)
        for (int64_t cz = lo[2] + oz; cz < hi[2]; cz += 2) fn(cx, cy, cz);
  }
}

// Compile-time (P, nq) dispatch: P in 1..7, nq in {P+1, P+2}.
template <template <int, int> class Fn, typename... Args>
void dispatch(int P, int nq, Args&&... args) {
#define BDX_CASE(PP)                                      \
  case PP:                                                \
    if (nq == PP + 1)                                     \
      return Fn<PP + 1, PP + 1>::run(args...);            \
    if (nq == PP + 2)                                     \
      return Fn<PP + 1, PP + 2>::run(args...);            \
    break;
  switch (P) {
    BDX_CASE(1)
    BDX_CASE(2)
    BDX_CASE(3)
    BDX_CASE(4)
    BDX_CASE(5)
    BDX_CASE(6)
    BDX_CASE(7)
  }
#undef BDX_CASE
  throw std::runtime_error("unsupported (degree, nq)");
}

template <typename T>
struct StiffArgs {
  BdxLattice lat;
  Tables<T> tb;
  const T* xv;
  T kappa;
  const T* kc;
  const T* u;
  T* y;
  int64_t lo[3], hi[3];
  const T* G = nullptr;  // precomputed geometry factors (bdx_cpu_geometry) or null
};

template <typename T>
struct Stiff {
  template <int ND, int NQ>
  struct K {
    static void run(const StiffArgs<T>& a) {
      const CellTables<T, ND, NQ> tb(a.tb);
      constexpr int64_t gsz = 6 * NQ * NQ * NQ;
      for_cells(a.lo, a.hi, [&](int64_t cx, int64_t cy, int64_t cz) {
        const T* Gc = a.G ? a.G + ((cx * a.lat.n[1] + cy) * a.lat.n[2] + cz) * gsz : nullptr;
        stiffness_cell_fast<T, ND, NQ>(a.lat, tb, a.xv, Gc, a.kappa, a.kc, a.u, a.y, cx, cy,
                                       cz);
      });
    }
  };
};

template <typename T>
struct GeomArgs {
  BdxLattice lat;
  const T *wts, *qpts, *xv;
  T* G;
};

template <typename T>
struct Geom {
  template <int ND, int NQ>
  struct K {
    static void run(const GeomArgs<T>& a) { geometry_all<T, NQ>(a.lat, a.wts, a.qpts, a.xv, a.G); }
  };
};

template <typename T>
struct MassArgs {
  BdxLattice lat;
  Tables<T> tb;
  const T* xv;
  const T* f;
  T* b;
  int64_t lo[3], hi[3];
};

template <typename T>
struct Mass {
  template <int ND, int NQ>
  struct K {
    static void run(const MassArgs<T>& a) {
      for_cells(a.lo, a.hi, [&](int64_t cx, int64_t cy, int64_t cz) {
        mass_cell<T, ND, NQ>(a.lat, a.tb, a.xv, a.f, a.b, cx, cy, cz);
      });
    }
  };
};

template <typename T>
Tables<T> make_tables(const T* phi0, const T* dphi1, const T* wts,
                      const T* qpts, const T* nodes, int identity) {
  return Tables<T>{phi0, dphi1, wts, qpts, nodes, identity != 0};
}

// ---------------------------------------------------------------- CSR
// Column range of local lattice index i along an axis with n cells: the
// union of the dof ranges of the cells containing it.
inline void col_range(int64_t i, int64_t P, int64_t n, int64_t& lo,
                      int64_t& hi) {
  int64_t c_hi = std::min(i / P, n - 1);
  int64_t c_lo = (i % P == 0 && i > 0) ? i / P - 1 : c_hi;
  lo = c_lo * P;
  hi = c_hi * P + P;  // inclusive
}

template <typename T>
int64_t csr_build(const int64_t* latd, int nq, const T* B, const T* Dd,
                  const T* wts, const T* qpts, const T* xv, T kappa, const T* kc,
                  int64_t* row_ptr, int32_t* cols, T* vals, int count_only) {
  const BdxLattice lat = BdxLattice::from(latd);
  const int64_t P = lat.P, nd = P + 1;
  const int64_t nrows = lat.size();
  // pattern (row_ptr must be zero-initialised by the caller: padding rows
  // of the pitched storage stay empty)
  row_ptr[0] = 0;
  for (int64_t i = 0; i < lat.L[0]; ++i)
    for (int64_t j = 0; j < lat.L[1]; ++j)
      for (int64_t k = 0; k < lat.L[2]; ++k) {
        int64_t lo[3], hi[3];
        const int64_t ijk[3] = {i, j, k};
        int64_t cnt = 1;
        for (int d = 0; d < 3; ++d) {
          col_range(ijk[d], P, lat.n[d], lo[d], hi[d]);
          cnt *= hi[d] - lo[d] + 1;
        }
        row_ptr[lat.idx(i, j, k) + 1] = cnt;
      }
  for (int64_t r = 0; r < nrows; ++r) row_ptr[r + 1] += row_ptr[r];
  const int64_t nnz = row_ptr[nrows];
  if (count_only) return nnz;
  if (lat.size() > INT32_MAX) throw std::runtime_error("local size > int32");
#pragma omp parallel for collapse(2)
  for (int64_t i = 0; i < lat.L[0]; ++i)
    for (int64_t j = 0; j < lat.L[1]; ++j)
      for (int64_t k = 0; k < lat.L[2]; ++k) {
        int64_t lo[3], hi[3];
        const int64_t ijk[3] = {i, j, k};
        for (int d = 0; d < 3; ++d) col_range(ijk[d], P, lat.n[d], lo[d], hi[d]);
        int64_t p = row_ptr[lat.idx(i, j, k)];
        for (int64_t a = lo[0]; a <= hi[0]; ++a)
          for (int64_t b = lo[1]; b <= hi[1]; ++b)
            for (int64_t c = lo[2]; c <= hi[2]; ++c) {
              cols[p] = static_cast<int32_t>(lat.idx(a, b, c));
              vals[p] = 0;
              ++p;
            }
      }
  // reference gradients gref[a][q][3]
  const int nd3 = static_cast<int>(nd * nd * nd), nq3 = nq * nq * nq;
  std::vector<T> gref(static_cast<size_t>(nd3) * nq3 * 3);
  for (int ia = 0; ia < nd; ++ia)
    for (int ja = 0; ja < nd; ++ja)
      for (int ka = 0; ka < nd; ++ka)
        for (int qx = 0; qx < nq; ++qx)
          for (int qy = 0; qy < nq; ++qy)
            for (int qz = 0; qz < nq; ++qz) {
              const int a = (ia * nd + ja) * nd + ka;
              const int q = (qx * nq + qy) * nq + qz;
              T* g = &gref[(static_cast<size_t>(a) * nq3 + q) * 3];
              g[0] = Dd[qx * nd + ia] * B[qy * nd + ja] * B[qz * nd + ka];
              g[1] = B[qx * nd + ia] * Dd[qy * nd + ja] * B[qz * nd + ka];
              g[2] = B[qx * nd + ia] * B[qy * nd + ja] * Dd[qz * nd + ka];
            }
  const int64_t lo0[3] = {0, 0, 0};
  const int64_t hi0[3] = {lat.n[0], lat.n[1], lat.n[2]};
  for_cells(lo0, hi0, [&](int64_t cx, int64_t cy, int64_t cz) {
    T X[8][3];
    cell_vertices(lat, xv, cx, cy, cz, X);
    const T kap = kc ? kc[(cx * lat.n[1] + cy) * lat.n[2] + cz] : kappa;
    std::vector<T> Gq(static_cast<size_t>(nq3) * 6);
    for (int qx = 0; qx < nq; ++qx)
      for (int qy = 0; qy < nq; ++qy)
        for (int qz = 0; qz < nq; ++qz) {
          const int q = (qx * nq + qy) * nq + qz;
          geometry_point<T>(X, qpts[qx], qpts[qy], qpts[qz],
                            wts[qx] * wts[qy] * wts[qz], &Gq[6 * q]);
        }
    std::vector<T> tmp(static_cast<size_t>(nd3) * nq3 * 3);
    for (int b = 0; b < nd3; ++b)
      for (int q = 0; q < nq3; ++q) {
        const T* g = &gref[(static_cast<size_t>(b) * nq3 + q) * 3];
        const T* G = &Gq[6 * q];
        T* t = &tmp[(static_cast<size_t>(b) * nq3 + q) * 3];
        t[0] = kap * (G[0] * g[0] + G[1] * g[1] + G[2] * g[2]);
        t[1] = kap * (G[1] * g[0] + G[3] * g[1] + G[4] * g[2]);
        t[2] = kap * (G[2] * g[0] + G[4] * g[1] + G[5] * g[2]);
      }
    for (int a = 0; a < nd3; ++a) {
      const int ia = a / static_cast<int>(nd * nd),
                ja = (a / static_cast<int>(nd)) % nd, ka = a % nd;
      const int64_t ri = cx * P + ia, rj = cy * P + ja, rk = cz * P + ka;
      if (lat.is_bc(ri, rj, rk)) continue;
      const int64_t row = lat.idx(ri, rj, rk);
      int64_t lo[3], hi[3];
      const int64_t rijk[3] = {ri, rj, rk};
      for (int d = 0; d < 3; ++d) col_range(rijk[d], P, lat.n[d], lo[d], hi[d]);
      const int64_t w1 = hi[1] - lo[1] + 1, w2 = hi[2] - lo[2] + 1;
      for (int b = 0; b < nd3; ++b) {
        const int ib = b / static_cast<int>(nd * nd),
                  jb = (b / static_cast<int>(nd)) % nd, kb = b % nd;
        const int64_t ci = cx * P + ib, cj = cy * P + jb, ck = cz * P + kb;
        if (lat.is_bc(ci, cj, ck)) continue;
        T s = 0;
        const T* ga = &gref[static_cast<size_t>(a) * nq3 * 3];
        const T* tb = &tmp[static_cast<size_t>(b) * nq3 * 3];
        for (int q = 0; q < nq3 * 3; ++q) s += ga[q] * tb[q];
        const int64_t off = ((ci - lo[0]) * w1 + (cj - lo[1])) * w2 + (ck - lo[2]);
        vals[row_ptr[row] + off] += s;
      }
    }
  });
  // identity rows for owned BC dofs
  for (int64_t i = 0; i < lat.L[0]; ++i)
    for (int64_t j = 0; j < lat.L[1]; ++j)
      for (int64_t k = 0; k < lat.L[2]; ++k) {
        if (!lat.is_bc(i, j, k) || !lat.is_owned(i, j, k)) continue;
        int64_t lo[3], hi[3];
        const int64_t ijk[3] = {i, j, k};
        for (int d = 0; d < 3; ++d) col_range(ijk[d], P, lat.n[d], lo[d], hi[d]);
        const int64_t w1 = hi[1] - lo[1] + 1, w2 = hi[2] - lo[2] + 1;
        const int64_t off = ((i - lo[0]) * w1 + (j - lo[1])) * w2 + (k - lo[2]);
        vals[row_ptr[lat.idx(i, j, k)] + off] = 1;
      }
  return nnz;
}

}  // namespace

extern "C" {

int bdx_host_version() { return 1; }

#define BDX_HOST_API(T, SUF)                                                  \
  void bdx_cpu_stiffness_##SUF(const int64_t* latd, int nq, const T* phi0,    \
                               const T* dphi1, const T* wts, const T* qpts,   \
                               const T* nodes, int identity, const T* xv,     \
                               T kappa, const T* kc, const T* u, T* y,        \
                               const int64_t* lo, const int64_t* hi) {        \
    StiffArgs<T> a;                                                           \
    a.lat = BdxLattice::from(latd);                                           \
    a.tb = make_tables<T>(phi0, dphi1, wts, qpts, nodes, identity);           \
    a.xv = xv;                                                                \
    a.kappa = kappa;                                                          \
    a.kc = kc;                                                                \
    a.u = u;                                                                  \
    a.y = y;                                                                  \
    for (int d = 0; d < 3; ++d) {                                             \
      a.lo[d] = lo[d];                                                        \
      a.hi[d] = hi[d];                                                        \
    }                                                                         \
    dispatch<Stiff<T>::template K>(static_cast<int>(a.lat.P), nq, a);         \
  }                                                                           \
  /* the same with precomputed geometry factors G (null: on the fly) */       \
  void bdx_cpu_stiffness_g_##SUF(const int64_t* latd, int nq, const T* phi0,  \
                                 const T* dphi1, const T* wts, const T* qpts, \
                                 const T* nodes, int identity, const T* xv,   \
                                 const T* G, T kappa, const T* kc,            \
                                 const T* u, T* y, const int64_t* lo,         \
                                 const int64_t* hi) {                         \
    StiffArgs<T> a;                                                           \
    a.lat = BdxLattice::from(latd);                                           \
    a.tb = make_tables<T>(phi0, dphi1, wts, qpts, nodes, identity);           \
    a.xv = xv;                                                                \
    a.G = G;                                                                  \
    a.kappa = kappa;                                                          \
    a.kc = kc;                                                                \
    a.u = u;                                                                  \
    a.y = y;                                                                  \
    for (int d = 0; d < 3; ++d) {                                             \
      a.lo[d] = lo[d];                                                        \
      a.hi[d] = hi[d];                                                        \
    }                                                                         \
    dispatch<Stiff<T>::template K>(static_cast<int>(a.lat.P), nq, a);         \
  }                                                                           \
  /* the reference data model on the CPU (dofmap_cells) */                   \
  void bdx_cpu_dofmap_##SUF(int P, int nq, const T* phi0, const T* dphi1,     \
                            const T* wts, const T* qpts, int identity,        \
                            const int* cells, int ncl, const int* cdofs,      \
                            const int* cverts, const T* coords, const T* G,   \
                            const unsigned char* flags, T kappa, const T* kc, \
                            const T* u, T* y) {                               \
    DofArgsCPU<T> a{make_tables<T>(phi0, dphi1, wts, qpts, nullptr, identity), \
                    cells, cdofs, cverts, ncl, coords, G, flags, kappa, kc,  \
                    u, y};                                                    \
    dispatch<DofmapCPU<T>::template K>(P, nq, a);                             \
  }                                                                           \
  void bdx_cpu_dofmap_geometry_##SUF(int P, int nq, const T* wts,             \
                                     const T* qpts, int ncells,               \
                                     const int* cverts, const T* coords,      \
                                     T* G) {                                  \
    DofGeomArgs<T> a{ncells, cverts, coords, wts, qpts, G};                   \
    dispatch<DofGeomCPU<T>::template K>(P, nq, a);                            \
  }                                                                           \
  /* geometry factors of every local cell, reference layout [c][6][nq^3] */  \
  void bdx_cpu_geometry_##SUF(const int64_t* latd, int nq, const T* wts,      \
                              const T* qpts, const T* xv, T* G) {             \
    GeomArgs<T> a{BdxLattice::from(latd), wts, qpts, xv, G};                  \
    dispatch<Geom<T>::template K>(static_cast<int>(a.lat.P), nq, a);          \
  }                                                                           \
  void bdx_cpu_mass_##SUF(const int64_t* latd, int nq, const T* phi0,         \
                          const T* dphi1, const T* wts, const T* qpts,        \
                          const T* nodes, int identity, const T* xv,          \
                          const T* f, T* b, const int64_t* lo,                \
                          const int64_t* hi) {                                \
    MassArgs<T> a;                                                            \
    a.lat = BdxLattice::from(latd);                                           \
    a.tb = make_tables<T>(phi0, dphi1, wts, qpts, nodes, identity);           \
    a.xv = xv;                                                                \
    a.f = f;                                                                  \
    a.b = b;                                                                  \
    for (int d = 0; d < 3; ++d) {                                             \
      a.lo[d] = lo[d];                                                        \
      a.hi[d] = hi[d];                                                        \
    }                                                                         \
    dispatch<Mass<T>::template K>(static_cast<int>(a.lat.P), nq, a);          \
  }                                                                           \
  int64_t bdx_cpu_csr_##SUF(const int64_t* latd, int nq, const T* B,          \
                            const T* Dd, const T* wts, const T* qpts,         \
                            const T* xv, T kappa, const T* kc,                \
                            int64_t* row_ptr, int32_t* cols, T* vals,         \
                            int count_only) {                                 \
    return csr_build<T>(latd, nq, B, Dd, wts, qpts, xv, kappa, kc, row_ptr,   \
                        cols, vals, count_only);                              \
  }                                                                           \
  void bdx_cpu_spmv_##SUF(int64_t nrows, const int64_t* beg, const int64_t* end, \
                          const int32_t* cols, const T* vals, const T* x,     \
                          T* y, int acc) {                                    \
    _Pragma("omp parallel for schedule(static)") for (int64_t r = 0;          \
                                                      r < nrows; ++r) {       \
      T s = 0;                                                                \
      for (int64_t p = beg[r]; p < end[r]; ++p) s += vals[p] * x[cols[p]];    \
      y[r] = acc ? y[r] + s : s;                                              \
    }                                                                         \
  }                                                                           \
  /* f = 1000 exp(-((x-1/2)^2 + (y-1/2)^2)/0.02) at the physical dof nodes */ \
  void bdx_cpu_interp_f_##SUF(const int64_t* latd, const T* nodes,            \
                              const T* xv, T* f) {                            \
    const BdxLattice lat = BdxLattice::from(latd);                            \
    const int64_t P = lat.P;                                                  \
    _Pragma("omp parallel for collapse(2)") for (int64_t i = 0;               \
                                                 i < lat.L[0]; ++i) {         \
      for (int64_t j = 0; j < lat.L[1]; ++j) {                                \
        for (int64_t k = 0; k < lat.L[2]; ++k) {                              \
          const int64_t ijk[3] = {i, j, k};                                   \
          int64_t c[3];                                                       \
          T s[3];                                                             \
          for (int d = 0; d < 3; ++d) {                                       \
            c[d] = std::min<int64_t>(ijk[d] / P, lat.n[d] - 1);               \
            s[d] = nodes[ijk[d] - c[d] * P];                                  \
          }                                                                   \
          T X[8][3];                                                          \
          cell_vertices(lat, xv, c[0], c[1], c[2], X);                        \
          T x[3] = {0, 0, 0};                                                 \
          for (int a = 0; a < 2; ++a)                                         \
            for (int b = 0; b < 2; ++b)                                       \
              for (int cc = 0; cc < 2; ++cc) {                                \
                const T wgt = (a ? s[0] : 1 - s[0]) * (b ? s[1] : 1 - s[1]) * \
                              (cc ? s[2] : 1 - s[2]);                         \
                for (int d = 0; d < 3; ++d)                                   \
                  x[d] += wgt * X[4 * a + 2 * b + cc][d];                     \
              }                                                               \
          const T dx = x[0] - T(0.5), dy = x[1] - T(0.5);                     \
          f[lat.idx(i, j, k)] =                                               \
              T(1000) * std::exp(-(dx * dx + dy * dy) / T(0.02));             \
        }                                                                     \
      }                                                                       \
    }                                                                         \
  }

BDX_HOST_API(double, f64)
BDX_HOST_API(float, f32)

// CPU unit test of the RCCL deadline policy (csrc/include/bdx_watchdog.h, used
// by the native runtime around every blocking RCCL call and host wait): a
// busy scope of `busy_s` under a `timeout_s` deadline, with the communicator
// reporting an asynchronous error from `err_after_s` on (< 0: never).
// Returns 1 if the watchdog fired (0 if not); *fire_s = seconds from the
// start of the scope to the abort callback (-1 if it never ran), *reason =
// 1 deadline / 2 async error.
int bdx_watchdog_selftest(double timeout_s, double busy_s, double err_after_s, double* fire_s,
                          int* reason) {
  const int64_t t0 = bdx::Watchdog::now_ns();
  std::atomic<int64_t> fired_at{0};
  bdx::Watchdog w(
      timeout_s,
      [&] { return err_after_s >= 0 && (bdx::Watchdog::now_ns() - t0) * 1e-9 >= err_after_s; },
      [&] { fired_at.store(bdx::Watchdog::now_ns()); });
  w.start(0.005);
  {
    bdx::Watchdog::Busy scope(&w);
    const int64_t end = t0 + static_cast<int64_t>(busy_s * 1e9);
    // the "blocked call": returns early once the abort has run, like an
    // RCCL call unblocked by ncclCommAbort
    while (bdx::Watchdog::now_ns() < end && !w.fired())
      std::this_thread::sleep_for(std::chrono::milliseconds(1));
  }
  w.stop();
  *fire_s = fired_at.load() ? (fired_at.load() - t0) * 1e-9 : -1.0;
  *reason = w.reason();
  return w.fired() ? 1 : 0;
}

}  // extern "C"
