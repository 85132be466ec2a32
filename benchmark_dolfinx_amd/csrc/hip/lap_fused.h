// Fused, atomic-free structured operator kernel ("fused", the fast path).
//
// Same operator as the reference's stiffness_operator_gpu
// (src/laplacian_gpu.hpp:91-426) + geometry_computation_gpu
// (src/geometry_gpu.hpp:26-132), re-designed for CDNA4:
//
// * Tiling.  A workgroup owns a tile of TY x TZ cells in the (y, z) plane and
//   marches through all local cells along x.  Threads map to the tile's
//   (cell, qy, qz) quadrature columns (TY*TZ*NQ^2 <= 256 lanes); each thread
//   keeps its column's NQ values along x in registers, so every x-contraction
//   is register-only and only the y/z contractions go through LDS.
// * No atomics.  Cells of a layer scatter into an LDS dof slab in 4 parity
//   phases (deterministic).  The x-shared dof plane is carried in LDS from one
//   layer to the next.  Dofs on the tile's upper y/z faces (owned by the
//   neighbouring tile) go to small interface buffers (YB, ZB, CB) that a light
//   finalize kernel folds into y.  Every other dof is written exactly once,
//   with a plain store, so y needs no zero fill.
// * Geometry.  GEOM=otf recomputes J per quadrature point from the cell's 8
//   vertices, exploiting the trilinear structure: dX/ds is constant along the
//   thread's x column and dX/dt, dX/du are linear in s (6 FMAs per point),
//   then F = kappa w/det adj(J) (adj(J)^T grad) without forming G.  GEOM=stored
//   reads the reference-layout G[cell][6][nq^3] array (coalesced along z).
// * CG fusion (MODE=1).  The input is formed on the fly as p = r + beta p_old
//   (double-buffered p), written back once for tile-owned dofs, and the
//   reduction p.(A p) is accumulated per cell (sum over the cell's dofs of
//   p_i (A_c p)_i, exact because every cell is computed by exactly one
//   rank/tile) plus p_i^2 for owned Dirichlet dofs (A has identity rows).
//   So one CG iteration = this kernel + finalize + one fused x/r/r.r update.
#pragma once
#include "bdx_common.h"

enum { kFusedAction = 0, kFusedCG = 1 };


// 1/x from the hardware reciprocal estimate + two Newton steps (full
// precision for the normal, positive Jacobian determinants seen here) instead
// of the IEEE division sequence (div_scale x2, rcp, 5 fma, div_fmas, div_fixup).
__device__ __forceinline__ double fast_rcp(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = __builtin_fma(-x, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-x, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ float fast_rcp(float x) {
  float r = __builtin_amdgcn_rcpf(x);
  const float e = __builtin_fmaf(-x, r, 1.0f);
  return __builtin_fmaf(r, e, r);
}

// Scheduling fence between unrolled iterations: keeps the scheduler from
// hoisting every LDS read of a fully unrolled stage to its top (which costs
// hundreds of registers and occupancy).
// Pin values computed in an unrolled iteration before the next iteration's
// LDS reads (the register operands keep this iteration's FMAs above the
// fence; the scheduling barrier keeps the next reads below it).  Without it
// the scheduler issues every read of a stage first and spills the results.
// No memory clobber: the per-thread table rows stay CSE'd in registers.
#define BDX_PIN1(x)                    \
  do {                                 \
    asm volatile("" : "+v"(x));        \
    __builtin_amdgcn_sched_barrier(0); \
  } while (0)
#define BDX_PIN3(x, y, z)                              \
  do {                                                 \
    asm volatile("" : "+v"(x), "+v"(y), "+v"(z));      \
    __builtin_amdgcn_sched_barrier(0);                 \
  } while (0)

#define BDX_SCHED_FENCE()               \
  do {                                  \
    asm volatile("" ::: "memory");      \
    __builtin_amdgcn_sched_barrier(0);  \
  } while (0)

// Minimum waves per SIMD requested from the register allocator (the LDS
// footprint allows 3 workgroups/CU up to nq=6 and 2 beyond).
template <int NQ>
struct FusedWaves {
  static constexpr int value = NQ <= 6 ? 3 : 2;
};

template <typename T> struct VecOf;
template <> struct VecOf<double> {
  typedef double __attribute__((ext_vector_type(2))) type;
  static constexpr int W = 2;
};
template <> struct VecOf<float> {
  typedef float __attribute__((ext_vector_type(4))) type;
  static constexpr int W = 4;
};

template <typename T, int ND, int NQ, int TY, int TZ>
struct FusedShape {
  static constexpr int P = ND - 1;
  static constexpr int cells = TY * TZ;
  static constexpr int lanes = cells * NQ * NQ;
  static constexpr int threads = ((lanes + 63) / 64) * 64;
  static constexpr int DY = TY * P + 1;
  static constexpr int DZ = TZ * P + 1;
  static constexpr int DZP = DZ | 1;  // odd LDS row pitch of the input slab (bank spread)
  static constexpr int VW = VecOf<T>::W;
  static constexpr int XP = (NQ + VW - 1) / VW * VW;  // 16-byte aligned row pitch (x axis)
  static constexpr int NP = (ND + VW - 1) / VW * VW;
  static constexpr int work = cells * NQ * NQ * XP;   // [c][a][b][x] scratch
  // packed 1D tables (host: bdx_fused_tables): rows padded for vector reads
  static constexpr int OFF_DR = 0;                  // Dr[q][m] = dphi1[q][m]
  static constexpr int OFF_DC = NQ * XP;            // Dc[m][q] = dphi1[q][m]
  static constexpr int OFF_PR = 2 * NQ * XP;        // Pr[q][i] = phi0[q][i]   (pitch NP)
  static constexpr int OFF_PC = 2 * NQ * XP + NQ * NP;  // Pc[i][q] = phi0[q][i]
  static constexpr int TAB = OFF_PC + ND * XP;
};

// 16-byte vector row load / store (p 16-byte aligned, row padded to the
// vector width; the tail of the last vector reads/writes padding).
template <int N, typename T>
__device__ __forceinline__ void ldrow(const T* __restrict__ p, T (&o)[N]) {
  using V = typename VecOf<T>::type;
  constexpr int W = VecOf<T>::W;
#pragma unroll
  for (int k = 0; k < N; k += W) {
    const V v = *reinterpret_cast<const V*>(p + k);
#pragma unroll
    for (int e = 0; e < W; ++e)
      if (k + e < N) o[k + e] = v[e];
  }
}
template <int N, typename T>
__device__ __forceinline__ void strow(T* __restrict__ p, const T (&x)[N]) {
  using V = typename VecOf<T>::type;
  constexpr int W = VecOf<T>::W;
#pragma unroll
  for (int k = 0; k < N; k += W) {
    V v;
#pragma unroll
    for (int e = 0; e < W; ++e) v[e] = (k + e < N) ? x[k + e] : T(0);
    *reinterpret_cast<V*>(p + k) = v;
  }
}

// Tile selection per (ND, NQ): as many whole cells as fit in 256 lanes.
template <int NQ> struct TileFor;
template <> struct TileFor<2> { static constexpr int TY = 8, TZ = 8; };
template <> struct TileFor<3> { static constexpr int TY = 4, TZ = 7; };
template <> struct TileFor<4> { static constexpr int TY = 4, TZ = 4; };
template <> struct TileFor<5> { static constexpr int TY = 2, TZ = 5; };
template <> struct TileFor<6> { static constexpr int TY = 1, TZ = 7; };
template <> struct TileFor<7> { static constexpr int TY = 1, TZ = 5; };
template <> struct TileFor<8> { static constexpr int TY = 2, TZ = 2; };
template <> struct TileFor<9> { static constexpr int TY = 1, TZ = 3; };

// Packed 1D tables + quadrature, passed by value in the kernarg segment
// (constant address space: wave-uniform reads become scalar loads).
template <typename T>
struct FusedTables {
  T tab[kFusedTabMax];
  T qpts[kMaxNq];
  T wts[kMaxNq];
};

template <typename T>
struct FusedArgs {
  BdxLattice lat;
  const T* __restrict__ u;      // action: input; CG: r
  const T* __restrict__ pold;   // CG: previous p (read)
  T* __restrict__ pnew;         // CG: new p (written, tile-owned dofs)
  T* __restrict__ y;            // output (tile-owned dofs)
  T* __restrict__ yb;           // [Lx][nty-1][Lz]   upper-y face partials
  T* __restrict__ zb;           // [Lx][ntz-1][Ly]   upper-z face partials (a tile face contiguous)
  T* __restrict__ cb;           // [Lx][nty-1][ntz-1] upper corner partials
  const T* __restrict__ G;      // stored geometry (GEOM=stored)
  const T* __restrict__ xv;     // vertex coordinates (GEOM=otf)
  const double* __restrict__ scal;
  double* __restrict__ partials;  // per-block p.Ap
  int beta_num, beta_den;       // CG: beta = scal[num]/scal[den]; num<0 -> beta=0
  int nty, ntz;
  T kappa;
};

// fused (v1 family): stored or on-the-fly geometry, quadrature-point arrays in LDS.
template <typename T, int ND, int NQ, int TY, int TZ, int GEOM, int MODE>
__global__ void __launch_bounds__((FusedShape<T, ND, NQ, TY, TZ>::threads), FusedWaves<NQ>::value)
    lap_fused_kernel(FusedArgs<T> A, FusedTables<T> tb) {
  using S = FusedShape<T, ND, NQ, TY, TZ>;
  constexpr int P = S::P, DY = S::DY, DZ = S::DZ, PL = DY * DZ;
  constexpr int DZP = S::DZP, PLP = DY * DZP;  // padded LDS pitches of the input slab
  constexpr int NQ2 = NQ * NQ;
  constexpr bool IDENT = (ND == NQ);
  constexpr int NT = S::threads;
  constexpr int NPF = (P * PL + NT - 1) / NT;          // prefetched dofs per thread
  constexpr int NV = (TY + 1) * (TZ + 1) * 3;          // vertex values per plane
  constexpr int NPV = (NV + NT - 1) / NT;

  constexpr int XP = S::XP, NP = S::NP;
  __shared__ __attribute__((aligned(16))) T s_tab[S::TAB];  // per-thread table rows
  __shared__ T s_qw[2 * NQ];          // quadrature points, weights
  __shared__ T s_u[2][ND * PLP];      // input slab [pl][ly][lz] (BC dofs zeroed), double-buffered
  __shared__ T s_c[2][PL];            // x-carried output plane, ping-pong
  __shared__ __attribute__((aligned(16))) T s_w1[S::work];  // [c][a][b][x] scratch, pitch XP
  __shared__ __attribute__((aligned(16))) T s_w2[S::work];
  __shared__ __attribute__((aligned(16))) T s_w3[S::work];
  __shared__ T s_X[2][2 * NV];        // vertex planes (cx, cx+1) of the tile, double-buffered
  __shared__ double s_red[16];

  const BdxLattice& lat = A.lat;
  const int tid = threadIdx.x;
  static_assert(S::TAB <= kFusedTabMax, "table too large");
  for (int i = tid; i < S::TAB; i += NT) s_tab[i] = tb.tab[i];
  if (tid < NQ) {
    s_qw[tid] = tb.qpts[tid];
    s_qw[NQ + tid] = tb.wts[tid];
  }

  // XCD-aware bijective remap of the block id (tiles adjacent in z share an
  // XCD's L2: cdna_hip_programming.md T1).
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  const int ty = bid / A.ntz, tz = bid % A.ntz;
  const int64_t y0 = static_cast<int64_t>(ty) * TY * P, z0 = static_cast<int64_t>(tz) * TZ * P;
  const int64_t Ly = lat.L[1], Lz = lat.L[2];
  const int64_t ncx = lat.n[0];
  const bool top_y = (ty == A.nty - 1), top_z = (tz == A.ntz - 1);
  // local dof extent of this tile's slab (clipped at the lattice end)
  const int ey = static_cast<int>(y0 + DY <= Ly ? DY : Ly - y0);
  const int ez = static_cast<int>(z0 + DZ <= Lz ? DZ : Lz - z0);
  // tile-owned dof extents in y/z (the top tile owns the last plane)
  const int oy = top_y ? ey : TY * P;
  const int oz = top_z ? ez : TZ * P;

  // thread -> (cell c = (cy, cz), a, b); idle lanes alias the last cell
  const int c = (tid / NQ2 < S::cells) ? tid / NQ2 : S::cells - 1;
  const int a = (tid / NQ) % NQ, b = tid % NQ;
  const int cy = c / TZ, cz = c % TZ;
  const bool lane_on = tid < S::lanes;
  const bool cell_on = lane_on && (static_cast<int64_t>(ty) * TY + cy < lat.n[1]) &&
                       (static_cast<int64_t>(tz) * TZ + cz < lat.n[2]);
  const int yb = cy * P, zb = cz * P;
  T* w1c = s_w1 + c * NQ2 * XP;
  T* w2c = s_w2 + c * NQ2 * XP;
  T* w3c = s_w3 + c * NQ2 * XP;

  T beta = T(0);
  if constexpr (MODE == kFusedCG) {
    if (A.beta_num >= 0) beta = static_cast<T>(A.scal[A.beta_num] / A.scal[A.beta_den]);
  }
  double pap = 0.0;

  // Input value of dof (gx, ly, lz) for the slab; side effects for CG (write
  // p) and for Dirichlet dofs (y = p on the owner, p^2 into p.Ap).
  auto stage = [&](int64_t gx, int ly, int lz, T r, T po) -> T {
    const int64_t gy = y0 + ly, gz = z0 + lz;
    const int64_t id = lat.idx(gx, gy, gz);
    T v;
    if constexpr (MODE == kFusedCG) {
      v = r + beta * po;
    } else {
      v = r;
      (void)po;
    }
    const bool owned_tile = ly < oy && lz < oz;
    if constexpr (MODE == kFusedCG) {
      if (owned_tile) A.pnew[id] = v;
    }
    if (lat.is_bc(gx, gy, gz)) {
      if (owned_tile) {
        const bool rank_owned = lat.is_owned(gx, gy, gz);
        A.y[id] = rank_owned ? v : T(0);
        if constexpr (MODE == kFusedCG) {
          if (rank_owned) pap += static_cast<double>(v) * static_cast<double>(v);
        }
      }
      v = T(0);
    }
    return v;
  };
  auto vertex = [&](int64_t vx, int e) -> T {
    const int d = e % 3, r = e / 3;
    const int vz = r % (TZ + 1), vy = r / (TZ + 1);
    const int64_t gy = static_cast<int64_t>(ty) * TY + vy, gz = static_cast<int64_t>(tz) * TZ + vz;
    if (gy > lat.n[1] || gz > lat.n[2]) return T(0);
    return A.xv[3 * lat.vidx(vx, gy, gz) + d];
  };

  // ---- prologue: layer 0 input planes, vertex planes 0/1, zero carry
  for (int e = tid; e < ND * PL; e += NT) {
    const int pl = e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
    T v = T(0);
    if (ly < ey && lz < ez) {
      const int64_t id = lat.idx(pl, y0 + ly, z0 + lz);
      v = stage(pl, ly, lz, A.u[id], MODE == kFusedCG ? A.pold[id] : T(0));
    }
    s_u[0][pl * PLP + ly * DZP + lz] = v;
  }
  if constexpr (GEOM == kGeomOTF) {
    for (int e = tid; e < 2 * NV; e += NT) s_X[0][e] = vertex(e / NV, e % NV);
  }
  for (int e = tid; e < PL; e += NT) s_c[0][e] = T(0);

  // Per-thread vertex-derived geometry coefficients for the current layer.
  T Js[3] = {0, 0, 0};                        // dX/ds at (t_a, u_b): constant in s
  T Jt0[3] = {0, 0, 0}, Jt1[3] = {0, 0, 0};   // dX/dt = Jt0 + s Jt1
  T Ju0[3] = {0, 0, 0}, Ju1[3] = {0, 0, 0};   // dX/du = Ju0 + s Ju1

  for (int64_t cx = 0; cx < ncx; ++cx) {
    const int cur = static_cast<int>(cx & 1), nxt = cur ^ 1;
    const bool last = (cx == ncx - 1);
    __syncthreads();  // staged buffers of this layer complete

    // ---- prefetch the next layer (planes 1..P of x-layer cx+1, vertex plane cx+2)
    T pf_r[NPF], pf_p[NPF];
    T pf_v[NPV];
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      pf_r[k] = T(0);
      pf_p[k] = T(0);
      const int e = tid + k * NT;
      if (!last && e < P * PL) {
        const int pl = 1 + e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
        if (ly < ey && lz < ez) {
          const int64_t id = lat.idx((cx + 1) * P + pl, y0 + ly, z0 + lz);
          pf_r[k] = A.u[id];
          if constexpr (MODE == kFusedCG) pf_p[k] = A.pold[id];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NPV; ++k) {
      pf_v[k] = T(0);
      if constexpr (GEOM == kGeomOTF) {
        const int e = tid + k * NT;
        if (!last && e < NV) pf_v[k] = vertex(cx + 2, e);
      }
    }

    // Opaque zero: keeps the uniform table reads (scalar loads into SGPRs)
    // inside the layer instead of pinning them for the whole x-march.
    int toff = 0;
    asm volatile("" : "+s"(toff));
    const T* __restrict__ gt = tb.tab + toff;  // wave-uniform rows -> SMEM (kernarg)
    const T* __restrict__ su = s_u[cur];
    const T* __restrict__ sX = s_X[cur];

    // per-thread LDS bases (rows of pitch XP, 16-byte aligned)
    const T* __restrict__ ua = su + (yb + a) * DZP + zb;
    T* __restrict__ w1ab = w1c + (a * NQ + b) * XP;
    T* __restrict__ w2ab = w2c + (a * NQ + b) * XP;
    T* __restrict__ w3ab = w3c + (a * NQ + b) * XP;
    const T* __restrict__ w1b = w1c + b * XP;        // + m * NQ * XP : [c][m][b][.]
    const T* __restrict__ w2b = w2c + b * XP;
    const T* __restrict__ w1a = w1c + a * NQ * XP;   // + m * XP      : [c][a][m][.]
    const T* __restrict__ w2a = w2c + a * NQ * XP;
    const T* __restrict__ w3a = w3c + a * NQ * XP;

    // ------------------------------------------------ interpolate to qpts
    T U[NQ];
    if constexpr (IDENT) {
#pragma unroll
      for (int i = 0; i < NQ; ++i) U[i] = lane_on ? ua[i * PLP + b] : T(0);
    } else {
      // S1: z-interp, thread (c, a=j<ND, b=qz): w1[c][j][qz][i]
      if (lane_on && a < ND) {
        const T* __restrict__ ph = s_tab + S::OFF_PR + b * NP;
        T o[ND];
#pragma unroll
        for (int i = 0; i < ND; ++i) o[i] = 0;
#pragma unroll 1
        for (int k = 0; k < ND; ++k) {
          const T c = ph[k];
#pragma unroll
          for (int i = 0; i < ND; ++i) o[i] += c * ua[i * PLP + k];
        }
        strow<ND>(w1ab, o);
      }
      __syncthreads();
      // S2: y-interp, thread (c, a=qy, b=qz): t2[i] = sum_j phi0[a][j] w1[c][j][b][i]
      const T* __restrict__ pa = s_tab + S::OFF_PR + a * NP;
      T t2[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) t2[i] = 0;
#pragma unroll 1
      for (int j = 0; j < ND; ++j) {
        T row[ND];
        ldrow<ND>(w1b + j * NQ * XP, row);
        const T c = pa[j];
#pragma unroll
        for (int i = 0; i < ND; ++i) t2[i] += c * row[i];
      }
      // S3: x-interp in registers, uniform rows of phi0^T
#pragma unroll
      for (int q = 0; q < NQ; ++q) U[q] = 0;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
#pragma unroll
        for (int q = 0; q < NQ; ++q) U[q] += gt[S::OFF_PC + i * XP + q] * t2[i];
      }
    }

    // ------------------------------------------------ reference gradient (m-outer)
    if (lane_on) strow<NQ>(w2ab, U);
    __syncthreads();
    T gx[NQ], gy[NQ], gz[NQ];
    {
      const T* __restrict__ dra = s_tab + S::OFF_DR + a * XP;   // dphi1[a][.]
      const T* __restrict__ drb = s_tab + S::OFF_DR + b * XP;   // dphi1[b][.]
#pragma unroll
      for (int q = 0; q < NQ; ++q) gx[q] = gy[q] = gz[q] = 0;
#pragma unroll 1
      for (int m = 0; m < NQ; ++m) {
        T ry[NQ], rz[NQ];
        ldrow<NQ>(w2b + m * NQ * XP, ry);   // U[c][m][b][.]
        ldrow<NQ>(w2a + m * XP, rz);        // U[c][a][m][.]
        const T um = w2ab[m], cy_ = dra[m], cz_ = drb[m];
        const T* __restrict__ dc = gt + S::OFF_DC + m * XP;
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          gx[q] += dc[q] * um;
          gy[q] += cy_ * ry[q];
          gz[q] += cz_ * rz[q];
        }
      }
    }

    // ------------------------------------------------ geometry coefficients
    if constexpr (GEOM == kGeomOTF) {
      const T t = s_qw[a], u = s_qw[b];
      const T* X0 = sX;        // plane cx
      const T* X1 = sX + NV;   // plane cx+1
      const int v00 = (cy * (TZ + 1) + cz) * 3, v01 = v00 + 3;
      const int v10 = v00 + (TZ + 1) * 3, v11 = v10 + 3;
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const T X000 = X0[v00 + d], X001 = X0[v01 + d], X010 = X0[v10 + d], X011 = X0[v11 + d];
        const T X100 = X1[v00 + d], X101 = X1[v01 + d], X110 = X1[v10 + d], X111 = X1[v11 + d];
        Js[d] = (1 - t) * ((1 - u) * (X100 - X000) + u * (X101 - X001)) +
                t * ((1 - u) * (X110 - X010) + u * (X111 - X011));
        Jt0[d] = (1 - u) * (X010 - X000) + u * (X011 - X001);
        Jt1[d] = (1 - u) * (X110 - X100) + u * (X111 - X101) - Jt0[d];
        Ju0[d] = (1 - t) * (X001 - X000) + t * (X011 - X010);
        Ju1[d] = (1 - t) * (X101 - X100) + t * (X111 - X110) - Ju0[d];
      }
    }
    const T kwyz = A.kappa * s_qw[NQ + a] * s_qw[NQ + b];
    int64_t gcell = 0;
    if constexpr (GEOM == kGeomStored) {
      gcell = ((cx * lat.n[1] + static_cast<int64_t>(ty) * TY + cy) * lat.n[2] +
               static_cast<int64_t>(tz) * TZ + cz) * 6 * (NQ * NQ2) + a * NQ + b;
    }

    // ------------------------------------------------ F = kappa G grad
    T Fx[NQ];
    using V = typename VecOf<T>::type;
    constexpr int VW = VecOf<T>::W;
    V vy, vz;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      T fx, fy, fz;
      if constexpr (GEOM == kGeomOTF) {
        const T s = s_qw[q];
        const T J00 = Js[0], J10 = Js[1], J20 = Js[2];
        const T J01 = Jt0[0] + s * Jt1[0], J11 = Jt0[1] + s * Jt1[1], J21 = Jt0[2] + s * Jt1[2];
        const T J02 = Ju0[0] + s * Ju1[0], J12 = Ju0[1] + s * Ju1[1], J22 = Ju0[2] + s * Ju1[2];
        // K = adj(J)
        const T K00 = J11 * J22 - J12 * J21, K01 = J02 * J21 - J01 * J22, K02 = J01 * J12 - J02 * J11;
        const T K10 = J12 * J20 - J10 * J22, K11 = J00 * J22 - J02 * J20, K12 = J02 * J10 - J00 * J12;
        const T K20 = J10 * J21 - J11 * J20, K21 = J01 * J20 - J00 * J21, K22 = J00 * J11 - J01 * J10;
        const T det = J00 * K00 + J01 * K10 + J02 * K20;
        const T sc = kwyz * s_qw[NQ + q] / det;
        // h = K^T g, F = sc K h  (= kappa w det J^-1 J^-T g)
        const T h0 = K00 * gx[q] + K10 * gy[q] + K20 * gz[q];
        const T h1 = K01 * gx[q] + K11 * gy[q] + K21 * gz[q];
        const T h2 = K02 * gx[q] + K12 * gy[q] + K22 * gz[q];
        fx = sc * (K00 * h0 + K01 * h1 + K02 * h2);
        fy = sc * (K10 * h0 + K11 * h1 + K12 * h2);
        fz = sc * (K20 * h0 + K21 * h1 + K22 * h2);
      } else {
        T Gd[6] = {0, 0, 0, 0, 0, 0};
        if (cell_on) {
          const T* g = A.G + gcell + q * NQ2;
#pragma unroll
          for (int k = 0; k < 6; ++k) Gd[k] = __builtin_nontemporal_load(g + k * NQ * NQ2);
        }
        fx = A.kappa * (Gd[0] * gx[q] + Gd[1] * gy[q] + Gd[2] * gz[q]);
        fy = A.kappa * (Gd[1] * gx[q] + Gd[3] * gy[q] + Gd[4] * gz[q]);
        fz = A.kappa * (Gd[2] * gx[q] + Gd[4] * gy[q] + Gd[5] * gz[q]);
      }
      BDX_PIN3(fx, fy, fz);
      Fx[q] = fx;
      vy[q % VW] = fy;
      vz[q % VW] = fz;
      if (q % VW == VW - 1 || q == NQ - 1) {
        if (q % VW != VW - 1) {
#pragma unroll
          for (int e = q % VW + 1; e < VW; ++e) vy[e] = vz[e] = T(0);
        }
        if (lane_on) {
          *reinterpret_cast<V*>(w1ab + (q / VW) * VW) = vy;
          *reinterpret_cast<V*>(w3ab + (q / VW) * VW) = vz;
        }
      }
    }
    __syncthreads();

    // ------------------------------------------------ transposed gradient (m-outer)
    T r[NQ];
    {
      // Fx goes to this thread's own w2 row (all U reads finished at the
      // barrier above; only this lane reads it back: no further barrier).
      if (lane_on) strow<NQ>(w2ab, Fx);
      const T* __restrict__ dca = s_tab + S::OFF_DC + a * XP;   // dphi1[.][a]
      const T* __restrict__ dcb = s_tab + S::OFF_DC + b * XP;   // dphi1[.][b]
#pragma unroll
      for (int q = 0; q < NQ; ++q) r[q] = 0;
#pragma unroll 1
      for (int m = 0; m < NQ; ++m) {
        T r1[NQ], r3[NQ];
        ldrow<NQ>(w1b + m * NQ * XP, r1);   // Fy[c][m][b][.]
        ldrow<NQ>(w3a + m * XP, r3);        // Fz[c][a][m][.]
        const T fm = w2ab[m], ca = dca[m], cb = dcb[m];
        const T* __restrict__ dr = gt + S::OFF_DR + m * XP;
#pragma unroll
        for (int q = 0; q < NQ; ++q) r[q] += dr[q] * fm + ca * r1[q] + cb * r3[q];
      }
    }
    // S7: x interp^T in registers, uniform rows of phi0^T
    T sx[ND];
    if constexpr (IDENT) {
#pragma unroll
      for (int i = 0; i < ND; ++i) sx[i] = r[i];
    } else {
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        T acc = 0;
#pragma unroll
        for (int q = 0; q < NQ; ++q) acc += gt[S::OFF_PC + i * XP + q] * r[q];
        sx[i] = acc;
      }
    }

    // ------------------------------------------------ back to the dofs
    T ye[ND];
    if constexpr (IDENT) {
#pragma unroll
      for (int i = 0; i < ND; ++i) ye[i] = sx[i];
    } else {
      __syncthreads();  // reads of w1/w3 done
      if (lane_on) strow<ND>(w2ab, sx);
      __syncthreads();
      // S8: y, thread (c, a=j<ND, b=qz): w1[c][j][qz][i] = sum_q phi0[q][j] w2[c][q][qz][i]
      if (lane_on && a < ND) {
        const T* __restrict__ pca = s_tab + S::OFF_PC + a * XP;
        T o[ND];
#pragma unroll
        for (int i = 0; i < ND; ++i) o[i] = 0;
#pragma unroll 1
        for (int q = 0; q < NQ; ++q) {
          T row[ND];
          ldrow<ND>(w2b + q * NQ * XP, row);
          const T c = pca[q];
#pragma unroll
          for (int i = 0; i < ND; ++i) o[i] += c * row[i];
        }
        strow<ND>(w1ab, o);
      }
      __syncthreads();
      // S9: z, thread (c, a=j<ND, b=k<ND): ye[i] = sum_q phi0[q][k] w1[c][j][q][i]
#pragma unroll
      for (int i = 0; i < ND; ++i) ye[i] = 0;
      if (a < ND && b < ND) {
        const T* __restrict__ pcb = s_tab + S::OFF_PC + b * XP;
#pragma unroll 1
        for (int q = 0; q < NQ; ++q) {
          T row[ND];
          ldrow<ND>(w1a + q * XP, row);
          const T c = pcb[q];
#pragma unroll
          for (int i = 0; i < ND; ++i) ye[i] += c * row[i];
        }
      }
    }

    // ------------------------------------------------ element vectors -> LDS
    const bool dof_lane = cell_on && a < ND && b < ND;
    if constexpr (MODE == kFusedCG) {
      if (dof_lane) {
#pragma unroll
        for (int i = 0; i < ND; ++i)
          pap += static_cast<double>(ua[i * PLP + b]) * static_cast<double>(ye[i]);
      }
    }
    if constexpr (IDENT) {
      __syncthreads();  // all reads of w2 (the gradient stage) done
    }
    if (lane_on && a < ND && b < ND) {
      if (!dof_lane) {
#pragma unroll
        for (int i = 0; i < ND; ++i) ye[i] = T(0);
      }
      strow<ND>(w2ab, ye);
    }
    __syncthreads();

    // ------------------------------------------------ gather-sum, write out, stage next layer
    for (int e = tid; e < ND * PL; e += NT) {
      const int pl = e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
      if (ly >= ey || lz >= ez) continue;
      const int cyh = (ly / P < TY - 1) ? ly / P : TY - 1;
      const int cyl = (ly % P == 0 && ly > 0 && ly / P - 1 < cyh) ? ly / P - 1 : cyh;
      const int czh = (lz / P < TZ - 1) ? lz / P : TZ - 1;
      const int czl = (lz % P == 0 && lz > 0 && lz / P - 1 < czh) ? lz / P - 1 : czh;
      T v = (pl == 0) ? s_c[cur][rem] : T(0);
      for (int ccy = cyl; ccy <= cyh; ++ccy)
        for (int ccz = czl; ccz <= czh; ++ccz)
          v += s_w2[(((ccy * TZ + ccz) * NQ + (ly - ccy * P)) * NQ + (lz - ccz * P)) * XP + pl];
      if (pl == P && !last) {
        s_c[nxt][rem] = v;
        continue;
      }
      const int64_t gx = cx * P + pl, gy = y0 + ly, gz = z0 + lz;
      const bool bc = lat.is_bc(gx, gy, gz);
      if (bc) v = T(0);
      const bool iy = ly < oy, iz = lz < oz;
      if (iy && iz) {
        if (!bc) A.y[lat.idx(gx, gy, gz)] = v;
      } else if (!iy && iz) {
        A.yb[(gx * (A.nty - 1) + ty) * Lz + gz] = v;
      } else if (iy && !iz) {
        A.zb[(gx * (A.ntz - 1) + tz) * Ly + gy] = v;
      } else {
        A.cb[(gx * (A.nty - 1) + ty) * (A.ntz - 1) + tz] = v;
      }
    }
    if (!last) {
      T* __restrict__ un = s_u[nxt];
      for (int e = tid; e < PL; e += NT) {
        const int o = (e / DZ) * DZP + e % DZ;
        un[o] = su[P * PLP + o];
      }
#pragma unroll
      for (int k = 0; k < NPF; ++k) {
        const int e = tid + k * NT;
        if (e < P * PL) {
          const int pl = 1 + e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
          T v = T(0);
          if (ly < ey && lz < ez) v = stage((cx + 1) * P + pl, ly, lz, pf_r[k], pf_p[k]);
          un[pl * PLP + ly * DZP + lz] = v;
        }
      }
      if constexpr (GEOM == kGeomOTF) {
        for (int e = tid; e < NV; e += NT) s_X[nxt][e] = sX[NV + e];
#pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int e = tid + k * NT;
          if (e < NV) s_X[nxt][NV + e] = pf_v[k];
        }
      }
    }
  }
  if constexpr (MODE == kFusedCG) {
    const double t = block_sum(pap, s_red);
    if (tid == 0) A.partials[blockIdx.x] = t;
  }
}

// Fold the interface partials into y (all local dofs incl. ghost planes).
// Index space: [YB rows: Lx * (nty-1) * Lz] ++ [ZB columns not on a YB row:
// Lx * Ly * (ntz-1)].  The two dof sets are disjoint, so no races.
// ghost_only: fold only dofs on this rank's ghost planes (the CG path folds
// the owned dofs inside the CG update, fused_common.hip; the ghost planes must
// be complete before the reverse halo exchange packs them).
template <typename T>
__global__ void __launch_bounds__(256)
    fused_finalize_kernel(BdxLattice lat, T* __restrict__ y, const T* __restrict__ yb,
                          const T* __restrict__ zb, const T* __restrict__ cb, int nty,
                          int ntz, int sy, int sz, int ghost_only) {
  const int64_t Lx = lat.L[0], Ly = lat.L[1], Lz = lat.L[2];
  const int64_t n1 = Lx * (nty - 1) * Lz;
  const int64_t n2 = Lx * Ly * (ntz - 1);
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n1 + n2;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (t < n1) {
      const int64_t z = t % Lz;
      const int64_t r = t / Lz;
      const int64_t tym1 = r % (nty - 1), x = r / (nty - 1);
      const int64_t yy = (tym1 + 1) * sy;
      if (ghost_only && lat.is_owned(x, yy, z)) continue;
      T add = yb[t];
      const int64_t tzz = z / sz;
      if (z % sz == 0 && tzz >= 1 && tzz < ntz) {
        add += zb[(x * (ntz - 1) + (tzz - 1)) * Ly + yy];
        add += cb[(x * (nty - 1) + tym1) * (ntz - 1) + (tzz - 1)];
      }
      y[lat.sidx(x, yy, z)] += add;
    } else {
      const int64_t s = t - n1;
      const int64_t yy = s % Ly;
      const int64_t r = s / Ly;
      const int64_t tzm1 = r % (ntz - 1), x = r / (ntz - 1);
      const int64_t tyy = yy / sy;
      if (yy % sy == 0 && tyy >= 1 && tyy < nty) continue;  // handled by the YB pass
      const int64_t z = (tzm1 + 1) * sz;
      if (ghost_only && lat.is_owned(x, yy, z)) continue;
      y[lat.sidx(x, yy, z)] += zb[s];
    }
  }
}

// Ghost-plane-only finalize (multi-rank CG path): the same sums as
// fused_finalize_kernel, restricted to the interface entries whose dof lies on
// one of this rank's ghost planes (x = Lx-1, y = Ly-1, z = Lz-1 when that
// plane is a ghost plane).  Interface rows/columns are never on the y/z ghost
// planes themselves ((nt-1)*TP < n*P), so three compact index ranges cover it:
//   A: x = Lx-1: every YB row (with its ZB/CB crossings) and every ZB column
//      not on a YB row;  B: y = Ly-1, ZB columns (x < Lx-1 if A ran);
//   C: z = Lz-1, YB rows (x < Lx-1 if A ran).
template <typename T>
__global__ void __launch_bounds__(256)
    fused_finalize_ghost_kernel(BdxLattice lat, T* __restrict__ y, const T* __restrict__ yb,
                                const T* __restrict__ zb, const T* __restrict__ cb, int nty,
                                int ntz, int sy, int sz) {
  const int64_t Lx = lat.L[0], Ly = lat.L[1], Lz = lat.L[2];
  const bool gx = lat.gh[0], gy = lat.gh[1], gz = lat.gh[2];
  const int64_t xB = gx ? Lx - 1 : Lx;  // x range of parts B, C
  const int64_t nA1 = gx ? (nty - 1) * Lz : 0, nA2 = gx ? Ly * (ntz - 1) : 0;
  const int64_t nB = gy ? xB * (ntz - 1) : 0;
  const int64_t nC = gz ? xB * (nty - 1) : 0;
  const int64_t ntot = nA1 + nA2 + nB + nC;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < ntot;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    if (t < nA1) {  // YB row entry on the x ghost plane
      const int64_t x = Lx - 1, z = t % Lz, tym1 = t / Lz;
      const int64_t yy = (tym1 + 1) * sy;
      T add = yb[(x * (nty - 1) + tym1) * Lz + z];
      const int64_t tzz = z / sz;
      if (z % sz == 0 && tzz >= 1 && tzz < ntz) {
        add += zb[(x * (ntz - 1) + (tzz - 1)) * Ly + yy];
        add += cb[(x * (nty - 1) + tym1) * (ntz - 1) + (tzz - 1)];
      }
      y[lat.sidx(x, yy, z)] += add;
    } else if (t < nA1 + nA2) {  // ZB column entry on the x ghost plane
      const int64_t s = t - nA1, x = Lx - 1;
      const int64_t yy = s % Ly, tzm1 = s / Ly;
      const int64_t tyy = yy / sy;
      if (yy % sy == 0 && tyy >= 1 && tyy < nty) continue;  // on a YB row: done above
      y[lat.sidx(x, yy, (tzm1 + 1) * sz)] += zb[(x * (ntz - 1) + tzm1) * Ly + yy];
    } else if (t < nA1 + nA2 + nB) {  // ZB column entry on the y ghost plane
      const int64_t s = t - nA1 - nA2, yy = Ly - 1;
      const int64_t tzm1 = s % (ntz - 1), x = s / (ntz - 1);
      y[lat.sidx(x, yy, (tzm1 + 1) * sz)] += zb[(x * (ntz - 1) + tzm1) * Ly + yy];
    } else {  // YB row entry on the z ghost plane
      const int64_t s = t - nA1 - nA2 - nB, z = Lz - 1;
      const int64_t tym1 = s % (nty - 1), x = s / (nty - 1);
      y[lat.sidx(x, (tym1 + 1) * sy, z)] += yb[(x * (nty - 1) + tym1) * Lz + z];
    }
  }
}
