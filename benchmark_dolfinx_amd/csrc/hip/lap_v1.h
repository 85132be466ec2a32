// Generic cell-wise sum-factorised operator kernel ("v1").
//
// Reference-equivalent algorithm (stiffness_operator_gpu,
// src/laplacian_gpu.hpp:91-426; geometry_computation_gpu,
// src/geometry_gpu.hpp:26-132): one thread per quadrature point, 1D tables in
// LDS, the three interpolation / gradient contractions through LDS, and an
// atomic scatter-add of the element vector.  Differences:
//   * CPB cells per workgroup so every launch uses >= 4 full waves
//     (Q=5: 2 cells x 125 points in 256 threads);
//   * lattice-derived dof indices and BC flags (no dofmap / marker arrays);
//   * geometry either read from the precomputed G array (reference layout
//     G[cell][6][nq^3]) or computed on the fly from the 8 cell vertices;
//   * the same template also computes the mass action for the RHS.
// This kernel is the correctness baseline and the path for MODE=mass; the
// fused structured kernel (lap_fused.h) is the performance path.
#pragma once
#include "bdx_common.h"

enum { kModeStiffness = 0, kModeMass = 1 };


// Cell index of the reference-layout G array: lexicographic over the local box.
__device__ __forceinline__ int64_t cell_index(const BdxLattice& lat, int64_t cx,
                                              int64_t cy, int64_t cz) {
  return (cx * lat.n[1] + cy) * lat.n[2] + cz;
}

template <int NQ>
struct V1Shape {
  static constexpr int nq3 = NQ * NQ * NQ;
  static constexpr int cpb = nq3 >= 256 ? 1 : 256 / nq3;
  static constexpr int threads = ((cpb * nq3 + 63) / 64) * 64;
};

// Shared-memory image of one v1 workgroup (CPB cells x nq^3 points).
template <typename T, int ND, int NQ>
struct V1Smem {
  static constexpr int nq3 = NQ * NQ * NQ, CPB = V1Shape<NQ>::cpb;
  T phi0[NQ * ND];
  T dphi[NQ * NQ];
  T s0[CPB][nq3];
  T s1[CPB][nq3];
  T s2[CPB][nq3];
  T s3[CPB][nq3];
  T X[CPB][8][3];
};

// The per-cell sum-factorised core shared by the lattice (v1) and dofmap
// kernels: on entry s0[cs] holds the element input (nd^3 embedded in the
// nq^3 grid) and X[cs] the 8 vertices (OTF geometry / mass); returns the
// element-vector entry of this thread's point (meaningful where qx, qy,
// qz < ND).  Gc: this cell's stored G (GEOM == kGeomStored), kap: the
// cell's coefficient.  Every thread of the block must call it (barriers).
template <typename T, int ND, int NQ, int MODE, int GEOM>
__device__ __forceinline__ T v1_core(V1Smem<T, ND, NQ>& sm, const OpTables<T>& tb, int cs,
                                     int q, bool active, bool valid, const T* __restrict__ Gc,
                                     T kap) {
  constexpr int nq3 = NQ * NQ * NQ;
  const int qx = q / (NQ * NQ), qy = (q / NQ) % NQ, qz = q % NQ;
  T(&s0)[V1Shape<NQ>::cpb][nq3] = sm.s0;
  T(&s1)[V1Shape<NQ>::cpb][nq3] = sm.s1;
  T(&s2)[V1Shape<NQ>::cpb][nq3] = sm.s2;
  T(&s3)[V1Shape<NQ>::cpb][nq3] = sm.s3;
  const T* s_phi0 = sm.phi0;
  const T* s_dphi = sm.dphi;
  T U = 0;
  if (!tb.identity) {
    // x: t[qx][j][k] = sum_i phi0[qx][i] u[i][j][k]   (j, k < ND)
    if (active && qy < ND && qz < ND) {
      T acc = 0;
#pragma unroll
      for (int i = 0; i < ND; ++i) acc += s_phi0[qx * ND + i] * s0[cs][(i * NQ + qy) * NQ + qz];
      s1[cs][q] = acc;
    }
    __syncthreads();
    if (active && qz < ND) {
      T acc = 0;
#pragma unroll
      for (int j = 0; j < ND; ++j) acc += s_phi0[qy * ND + j] * s1[cs][(qx * NQ + j) * NQ + qz];
      s2[cs][q] = acc;
    }
    __syncthreads();
    if (active) {
      T acc = 0;
#pragma unroll
      for (int k = 0; k < ND; ++k) acc += s_phi0[qz * ND + k] * s2[cs][(qx * NQ + qy) * NQ + k];
      U = acc;
    }
    __syncthreads();
    if (active) s0[cs][q] = U;
    __syncthreads();
  } else {
    if (active) U = s0[cs][q];
  }

  T r = 0;
  if constexpr (MODE == kModeMass) {
    T Gd[6];
    const T w = tb.wts[qx] * tb.wts[qy] * tb.wts[qz];
    T det = 1;
    if (valid) det = geometry_G<T>(sm.X[cs], tb.qpts[qx], tb.qpts[qy], tb.qpts[qz], T(1), Gd);
    r = U * w * det;
  } else {
    T gx = 0, gy = 0, gz = 0;
    if (active) {
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        gx += s_dphi[qx * NQ + i] * s0[cs][(i * NQ + qy) * NQ + qz];
        gy += s_dphi[qy * NQ + i] * s0[cs][(qx * NQ + i) * NQ + qz];
        gz += s_dphi[qz * NQ + i] * s0[cs][(qx * NQ + qy) * NQ + i];
      }
    }
    T Gd[6] = {0, 0, 0, 0, 0, 0};
    if (valid) {
      if constexpr (GEOM == kGeomStored) {
        const T* g = Gc + q;
#pragma unroll
        for (int k = 0; k < 6; ++k) Gd[k] = __builtin_nontemporal_load(g + k * nq3);
      } else {
        const T w = tb.wts[qx] * tb.wts[qy] * tb.wts[qz];
        geometry_G<T>(sm.X[cs], tb.qpts[qx], tb.qpts[qy], tb.qpts[qz], w, Gd);
      }
    }
    const T fx = kap * (Gd[0] * gx + Gd[1] * gy + Gd[2] * gz);
    const T fy = kap * (Gd[1] * gx + Gd[3] * gy + Gd[4] * gz);
    const T fz = kap * (Gd[2] * gx + Gd[4] * gy + Gd[5] * gz);
    if (active) {
      s1[cs][q] = fx;
      s2[cs][q] = fy;
      s3[cs][q] = fz;
    }
    __syncthreads();
    if (active) {
#pragma unroll
      for (int i = 0; i < NQ; ++i) {
        r += s_dphi[i * NQ + qx] * s1[cs][(i * NQ + qy) * NQ + qz];
        r += s_dphi[i * NQ + qy] * s2[cs][(qx * NQ + i) * NQ + qz];
        r += s_dphi[i * NQ + qz] * s3[cs][(qx * NQ + qy) * NQ + i];
      }
    }
  }

  T ye = r;
  if (!tb.identity) {
    __syncthreads();
    if (active) s0[cs][q] = r;
    __syncthreads();
    if (active && qz < ND) {
      T acc = 0;
#pragma unroll
      for (int k = 0; k < NQ; ++k) acc += s_phi0[k * ND + qz] * s0[cs][(qx * NQ + qy) * NQ + k];
      s1[cs][q] = acc;
    }
    __syncthreads();
    if (active && qy < ND && qz < ND) {
      T acc = 0;
#pragma unroll
      for (int j = 0; j < NQ; ++j) acc += s_phi0[j * ND + qy] * s1[cs][(qx * NQ + j) * NQ + qz];
      s2[cs][q] = acc;
    }
    __syncthreads();
    if (active && qx < ND && qy < ND && qz < ND) {
      T acc = 0;
#pragma unroll
      for (int i = 0; i < NQ; ++i) acc += s_phi0[i * ND + qx] * s2[cs][(i * NQ + qy) * NQ + qz];
      ye = acc;
    }
  }
  return ye;
}

// v1: the reference algorithm (one cell per workgroup slot, quadrature-point arrays).
template <typename T, int ND, int NQ, int MODE, int GEOM>
__global__ void __launch_bounds__(V1Shape<NQ>::threads)
    lap_v1_kernel(BdxLattice lat, OpTables<T> tb, const T* __restrict__ G,
                  const T* __restrict__ xv, T kappa, const T* __restrict__ kc,
                  const T* __restrict__ u,
                  T* __restrict__ y, int64_t lo0, int64_t lo1, int64_t lo2,
                  int64_t e0, int64_t e1, int64_t e2) {
  constexpr int nq3 = NQ * NQ * NQ;
  constexpr int CPB = V1Shape<NQ>::cpb;
  __shared__ V1Smem<T, ND, NQ> sm;
  T* const s_phi0 = sm.phi0;
  T* const s_dphi = sm.dphi;
  T(&s0)[CPB][nq3] = sm.s0;
  T(&s_X)[CPB][8][3] = sm.X;

  const int tid = threadIdx.x;
  for (int i = tid; i < NQ * ND; i += blockDim.x) s_phi0[i] = tb.phi0[i];
  for (int i = tid; i < NQ * NQ; i += blockDim.x) s_dphi[i] = tb.dphi1[i];

  const int cs = tid / nq3;
  const int q = tid - cs * nq3;
  const int qx = q / (NQ * NQ), qy = (q / NQ) % NQ, qz = q % NQ;
  const bool active = cs < CPB;
  const int64_t ncell = e0 * e1 * e2;
  const int64_t cell_lin = static_cast<int64_t>(blockIdx.x) * CPB + cs;
  const bool valid = active && cell_lin < ncell;
  int64_t cx = 0, cy = 0, cz = 0;
  if (valid) {
    cz = lo2 + cell_lin % e2;
    cy = lo1 + (cell_lin / e2) % e1;
    cx = lo0 + cell_lin / (e1 * e2);
  }
  const int64_t P = lat.P;
  const bool is_dof = valid && qx < ND && qy < ND && qz < ND;
  int64_t dof = -1;
  bool bc = false;
  int64_t li = cx * P + qx, lj = cy * P + qy, lk = cz * P + qz;
  if (is_dof) {
    dof = lat.idx(li, lj, lk);
    bc = (MODE == kModeStiffness) && lat.is_bc(li, lj, lk);
  }
  // Stage element input into s0 (nd^3 embedded in the nq^3 grid).
  if (active) s0[cs][q] = (is_dof && !bc) ? u[dof] : T(0);
  if (GEOM == kGeomOTF || MODE == kModeMass) {
    if (active && q < 24 && valid) {
      const int v = q / 3, d = q % 3;
      const int a = v >> 2, b = (v >> 1) & 1, c = v & 1;
      s_X[cs][v][d] = xv[3 * lat.vidx(cx + a, cy + b, cz + c) + d];
    }
  }
  __syncthreads();

  const T* Gc = (GEOM == kGeomStored && valid) ? G + cell_index(lat, cx, cy, cz) * 6 * nq3 : G;
  // per-cell coefficient (random-coefficient runs) or the constant kappa
  const T kap = (kc && valid) ? kc[cell_index(lat, cx, cy, cz)] : kappa;
  const T ye = v1_core<T, ND, NQ, MODE, GEOM>(sm, tb, cs, q, active, valid, Gc, kap);
  if (is_dof) {
    if (!bc) {
      atomicAdd(y + dof, ye);
    } else if (lat.is_owned(li, lj, lk)) {
      y[dof] = u[dof];
    }
  }
}

