// Fused structured operator kernel, v3 ("fused3"): fused2's x-march,
// (y, z) tiles, precomputed addressing, interface buffers and CG fusion, with
// a re-designed contraction core (qmode=1 / Gauss, i.e. phi0 != I):
//
// * The reference gradient is taken directly from the dofs with the
//   (nq x nd) table Dd = dphi1 phi0 (sum factorisation shares the B/Dd
//   passes: z then y through LDS, x in registers), instead of interpolating
//   to the quadrature points and differentiating there (reference
//   src/laplacian_gpu.hpp:188-251).  The transposed path mirrors it:
//   x in registers, then y and z through LDS.  Per cell layer this saves two
//   workgroup barriers and about a quarter of the LDS traffic of fused2, and
//   the x-direction passes are fused per quadrature point with the geometry
//   (no gx/gy/gz/F arrays are kept live).
// * When a tile cell's NQ^2 quadrature columns fill whole waves (NQ = 2, 4,
//   8: Q6 qmode=1 is one cell per wave), the y/z contraction stages only
//   exchange data inside a wave, so their barriers become wave-local syncs;
//   only the dof staging and the gather keep workgroup barriers.
// The math is the reference operator's (tests compare against the C++ CPU
// operator and the numpy oracle); results differ only by rounding order.
#pragma once
#include <type_traits>

#include "lap_fused2.h"

// Unroll of the per-quadrature-point x/F loop.  Parallelepiped instances:
// full unroll up to NQ = 5, 2-way beyond (full unroll hoists 2*ND*NQ uniform
// table values into SGPRs, which spills beyond NQ = 5).  General-geometry
// instances (AFF = 0; FP32 only up to NQ = 5) and the x-trilinear FP64
// instances (AFF = 2) keep the loop rolled, so the per-point geometry of one
// point at a time is live, not NQ: general Q3 18.5 -> 21.4 GDoF/s (with 3
// waves, below), x-trilinear Q3 25.0 -> 26.2, Q6 neutral; FP32 at NQ > 5
// keeps the 2-way unroll (Q6 34.4 vs 33.9).  profiles/r2_launder.md,
// r2_xtrilinear.md.
template <int NQ> struct QUnroll3 { static constexpr int value = NQ <= 5 ? NQ : 2; };
template <typename T, int NQ, int AFF> struct QUnroll3G {
  static constexpr bool rolled =
      (AFF == 0 && (sizeof(T) == 8 || NQ <= 5)) || (AFF == 2 && sizeof(T) == 8);
  static constexpr int value = rolled ? 1 : QUnroll3<NQ>::value;
};
// Waves per SIMD the instances are compiled for.  General (AFF = 0) and
// x-trilinear (AFF = 2) cells: 3.  With the rolled per-point x loop the NQ = 5
// general instance is 175 VGPRs at 2 waves and fits 3 waves with an 8-dword
// spill (Q3 general 18.5 -> 21.4 GDoF/s, job_r2af.sh).  LDS caps the P >= 4
// instances at 2 workgroups per CU anyway, and there the compiler keeps its
// 2-wave allocation (no spill).
template <int NQ, int AFF> struct Fused3Waves {
  static constexpr int value = AFF == 1 ? FusedWaves<NQ>::value : 3;
};
// The gather and staging descriptors are re-materialised every layer through
// an empty asm (the descriptor laundering of lap_fused5.h).

// y / z contraction stages of the FP64 Q6 (NQ = 8, one cell per wave)
// instances on the matrix pipe (v_mfma_f64_16x16x4f64, [B; Dd] stacked into
// the 16-row operand) instead of the VALU.  Same-box A/B, Q6 500 M perturbed
// (x-trilinear), 3 interleaved runs each, GDoF/s (profiles/r4_fused3_mfma.md):
// VALU 30.2; front z 30.4; back z 30.1; front + back z 30.6; front z + back y
// + back z 30.9 (adopted); all four 30.2 (the front-y stage's lane exchange
// stalls on its MFMA results).
constexpr bool kF3MfmaFrontZ = true;
// 16-byte staging loads / stores (the VEC instance, as lap_fused5.h)
constexpr bool kF3Vec = true;
constexpr bool kF3MfmaFrontY = false;
constexpr bool kF3MfmaBackY = true;
constexpr bool kF3MfmaBackZ = true;
// the same three stages in FP32 (v_mfma_f32_16x16x4_f32; bdx_mfma_row maps
// the FP32 accumulator rows onto the FP64 layout the stages are written for)
constexpr bool kF3MfmaF32 = true;
// Dirichlet-free copies of the staging and the gather for the tiles / layers
// without a boundary node (the split of lap_fused5.h)
constexpr bool kF3DirSplit = true;

// fused3: fused2's march with direct collocation gradients and wave-local x passes.
template <typename T, int ND, int NQ, int TY, int TZ, int MODE, int AFF, bool VEC = false>
__global__ void __launch_bounds__((FusedShape<T, ND, NQ, TY, TZ>::threads),
                                  (VEC && NQ == 8 && sizeof(T) == 8 ? 2 : Fused3Waves<NQ, AFF>::value))
    lap_fused3_kernel(Fused2Args<T> A, FusedTables<T> tb) {
  using S = FusedShape<T, ND, NQ, TY, TZ>;
  constexpr int P = S::P, DY = S::DY, DZ = S::DZ, PL = DY * DZ;
  constexpr int DZP = S::DZP, PLP = DY * DZP;
  constexpr int NQ2 = NQ * NQ;
  constexpr bool IDENT = (ND == NQ);
  constexpr int NT = S::threads;
  constexpr int NPF = (P * PL + NT - 1) / NT;     // staged input dofs per thread and layer
  constexpr int NOUT = (ND * PL + NT - 1) / NT;   // output dofs per thread and layer
  constexpr int NCP = (PL + NT - 1) / NT;         // carried-plane copies per thread
  constexpr int NV = (TY + 1) * (TZ + 1) * 3;
  constexpr int NPV = (NV + NT - 1) / NT;
  constexpr int XP = S::XP, NP = S::NP;
  // VEC: the staging's loads and p / x stores in 16-byte vectors (items of V
  // z-nodes of a tile row, the z-neighbour's column as single items), as in
  // lap_fused5.h; the host selects it when every tile row is 16-byte aligned
  constexpr int V = 16 / static_cast<int>(sizeof(T));
  constexpr int OWNZ = TZ * P;
  static_assert(!VEC || (OWNZ % V == 0 && (OWNZ * static_cast<int>(sizeof(T))) % 16 == 0),
                "VEC: whole 16-byte vectors per tile row");
  constexpr int NIV = OWNZ / V;
  constexpr int NITV = P * DY * NIV, NPI = VEC ? (NITV + NT - 1) / NT : 1;
  constexpr int NITS = P * DY, NPS = VEC ? (NITS + NT - 1) / NT : 1;
  typedef T VT __attribute__((ext_vector_type(V)));
  // intra-cell stages only exchange data inside a wave when a cell's NQ^2
  // columns tile whole waves
  constexpr bool WAVELOCAL = (64 % NQ2 == 0) && (S::lanes % 64 == 0);
  // front z on the matrix pipe: FP64 cells that are one wave each (Q6 qmode=1)
  // y / z contraction stages on the matrix pipe (see kF3Mfma*): FP64 cells
  // that are one wave each (Q6 qmode=1), x-trilinear and parallelepiped
  // instances (the general trilinear instance measured 1.3 % slower with them)
  constexpr bool MFOK = (sizeof(T) == 8 || kF3MfmaF32) && NQ == 8 && ND == 7 && WAVELOCAL &&
                       AFF != 0;
  constexpr bool MFZ = kF3MfmaFrontZ && MFOK;
  constexpr bool MFY = kF3MfmaFrontY && MFOK && sizeof(T) == 8;  // FP64 map only
  using MAcc = typename BdxMfmaAcc<T>::type;
  constexpr bool MFBY = kF3MfmaBackY && MFOK;
  constexpr bool MFBZ = kF3MfmaBackZ && MFOK;
  // LDS work buffers of the contraction core: NBUFS buffers W[k][cell][i1][i2]
  // of rows of ND values.  Padded for conflict-free 16-byte LDS access
  // (scripts/lds_bank_sim.py; measured: unpadded Q6 lost 56 % of its LDS
  // cycles to bank conflicts): the row pitch RP, the i1 pitch P1 and the cell
  // pitch PC are odd numbers of 16-byte slots, so the rows one ds_read_b128 /
  // ds_write_b128 touches (varying i2, or varying i1) start on distinct banks.
  //  block layout (cells straddle waves), 3 buffers:
  //    W0: B_z u -> A1 -> C1      W1: Dd_z u -> A2 -> C3      W2: A3 -> E
  //  wave-local layout, 2 buffers updated in place (a wave's LDS reads all
  //  issue before its later writes):
  //    W0: B_z u -> A1 -> C1 -> E  W1: Dd_z u -> A2 -> A3 -> C3
  constexpr int VW = VecOf<T>::W;
  constexpr int odd_slots_rp = (NP / VW) % 2 ? NP / VW : NP / VW + 1;
  constexpr int RP = odd_slots_rp * VW;
  constexpr int P1 = ((NQ * RP / VW) % 2 ? NQ * RP / VW : NQ * RP / VW + 1) * VW;
  constexpr int PC = ((NQ * P1 / VW) % 2 ? NQ * P1 / VW : NQ * P1 / VW + 1) * VW;
  constexpr int NBUFS = WAVELOCAL ? 2 : 3;
  constexpr int NWBUF = S::cells * PC;            // one buffer
  constexpr int EBUF = WAVELOCAL ? 0 : 2;         // buffer holding the element vectors
  constexpr int ZSLOT = NBUFS * NWBUF;            // zero row after the pool
  static_assert(ZSLOT + NP < 32768, "16-bit LDS source offsets");
  static_assert(!IDENT, "fused3 is the phi0 != I core (qmode=1 or Gauss)");
  constexpr int OFF_BR = 0, OFF_DR = NQ * NP, OFF_BC = 2 * NQ * NP, OFF_DC = 2 * NQ * NP + ND * XP;
  constexpr int TAB3 = 2 * NQ * NP + 2 * ND * XP;
  static_assert(TAB3 <= kFusedTabMax, "table too large");
  static_assert(PL < 256, "8-bit plane index");

  __shared__ __attribute__((aligned(16))) T s_tab[TAB3];
  __shared__ T s_qw[2 * NQ];
  __shared__ T s_u[2][ND * PLP + V];  // + dummy slots (VEC padding items)
  __shared__ T s_c[2][PL];
  __shared__ __attribute__((aligned(16))) T s_wa[NBUFS * NWBUF + RP];
  __shared__ T s_X[2][2 * NV];
  __shared__ double s_red[16];

  const int tid = threadIdx.x;
  for (int i = tid; i < TAB3; i += NT) s_tab[i] = tb.tab[i];
  if (tid < NQ) {
    s_qw[tid] = tb.qpts[tid];
    s_qw[NQ + tid] = tb.wts[tid];
  }
  if (tid < RP) s_wa[ZSLOT + tid] = T(0);

  // XCD-aware bijective remap of the block id (cdna_hip_programming.md T1).
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  // work item = (tile of the launch rectangle, x segment); see fused_set_segments
  const int tix = bid % A.rtiles, seg = bid / A.rtiles;
  const int ty = A.ty0 + tix / A.rwz, tz = A.tz0 + tix % A.rwz;
  // own cell layers [sa, cend); the march starts one layer early (redundant)
  // in every segment but the first
  const int sa = seg * A.seglen;
  const int cend = (sa + A.seglen < A.ncx) ? sa + A.seglen : A.ncx;
  const int cbeg = sa > 0 ? sa - 1 : 0;
  const int y0 = ty * TY * P, z0 = tz * TZ * P;
  const int Ly = A.Ly, Lz = A.Lz;
  const int ncx = A.ncx;
  const bool top_y = (ty == A.nty - 1), top_z = (tz == A.ntz - 1);
  const int ey = (y0 + DY <= Ly) ? DY : Ly - y0;
  const int ez = (z0 + DZ <= Lz) ? DZ : Lz - z0;
  const int oy = top_y ? ey : TY * P;
  const int oz = top_z ? ez : TZ * P;
  // Dirichlet work only where a tile holds a y / z boundary node or a layer
  // an x boundary plane (workgroup-uniform; see lap_fused5.h)
  auto in_rng = [](int v, int lo, int n) { return v >= lo && v < lo + n; };
  const bool tile_bc = in_rng(A.bcy_lo, y0, ey) || in_rng(A.bcy_hi, y0, ey) ||
                       in_rng(A.bcz_lo, z0, ez) || in_rng(A.bcz_hi, z0, ez);
  auto xbc_in = [&](int gx0, int n) { return in_rng(A.bcx_lo, gx0, n) || in_rng(A.bcx_hi, gx0, n); };

  const int c = (tid / NQ2 < S::cells) ? tid / NQ2 : S::cells - 1;
  const int a = (tid / NQ) % NQ, b = tid % NQ;
  const int cy = c / TZ, cz = c % TZ;
  const bool lane_on = tid < S::lanes;
  const bool cell_on = lane_on && (ty * TY + cy < A.n1) && (tz * TZ + cz < A.n2);
  const int ycell = cy * P, zcell = cz * P;

  T beta = T(0), xalpha = T(0);
  const bool xupd = MODE == kFusedCG && A.xa_num >= 0;
  if constexpr (MODE == kFusedCG) {
    if (A.beta_num >= 0) beta = static_cast<T>(A.scal[A.beta_num] / A.scal[A.beta_den]);
    if (xupd) xalpha = static_cast<T>(A.scal[A.xa_num] / A.scal[A.xa_den]);
  }
  double pap = 0.0;

  // y/z classification of a slab position (layer invariant)
  enum { kValid = 1, kOwnT = 2, kBcYZ = 4, kRownYZ = 8 };
  auto yz_flags = [&](int ly, int lz) -> int {
    if (ly >= ey || lz >= ez) return 0;
    const int gy = y0 + ly, gz = z0 + lz;
    int f = kValid;
    if (ly < oy && lz < oz) f |= kOwnT;
    if (gy == A.bcy_lo || gy == A.bcy_hi || gz == A.bcz_lo || gz == A.bcz_hi) f |= kBcYZ;
    if (gy < A.owny && gz < A.ownz) f |= kRownYZ;
    return f;
  };
  // Input value of a staged dof + its CG / Dirichlet side effects.
  // (wr = false: a redundant layer, whose planes the previous segment owns:
  // the value only, no side effects)
  auto stage = [&](int f, int gx, const T* __restrict__ ul, T* __restrict__ pn, T* __restrict__ yl,
                   int goff, bool wr) -> T {
    T v;
    if (!wr) f &= ~kOwnT;
    if constexpr (MODE == kFusedCG) {
      const T po = A.pold[(ul - A.u) + goff];
      v = ul[goff] + beta * po;
      if (xupd && (f & kOwnT)) {
        T* __restrict__ xl = A.x + (ul - A.u);
        xl[goff] += xalpha * po;
      }
    } else {
      v = ul[goff];
    }
    (void)pn;
    if constexpr (MODE == kFusedCG) {
      if (f & kOwnT) pn[goff] = v;
    }
    if ((f & kBcYZ) || gx == A.bcx_lo || gx == A.bcx_hi) {
      if (f & kOwnT) {
        const bool rown = (f & kRownYZ) && gx < A.ownx;
        yl[goff] = rown ? v : T(0);
        if constexpr (MODE == kFusedCG) {
          if (rown) pap += static_cast<double>(v) * static_cast<double>(v);
        }
      }
      v = T(0);
    }
    return v;
  };

  // ---- per-thread staging descriptors (planes 1..P of a layer)
  int st_goff[NPF], st_meta[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int e = tid + k * NT;
    st_goff[k] = 0;
    st_meta[k] = 0;
    if (e < P * PL) {
      const int pl = 1 + e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
      const int f = yz_flags(ly, lz);
      st_goff[k] = static_cast<int>(pl * A.ps + fused_yzoff(A, y0 + ly, z0 + lz));
      st_meta[k] = f | (pl << 4) | ((pl * PLP + ly * DZP + lz) << 8);
    }
  }
  // ---- VEC staging items (lap_fused5.h): meta = 4 flag bits per node at
  // 4 e, the plane at bits 16-19, any node valid at 21, every node owned at
  // 22, any node owned at 23
  unsigned it_goff[NPI], is_goff[NPS];
  int it_meta[NPI], it_lds[NPI], is_meta[NPS], is_lds[NPS];
  auto item_desc = [&](int pl, int ly, int lz0, int nel, unsigned& goff, int& meta, int& lds) {
    int m = pl << 16, allown = 1, anyown = 0, anyv = 0;
    for (int e = 0; e < nel; ++e) {
      const int f = yz_flags(ly, lz0 + e);
      m |= f << (4 * e);
      anyv |= f & kValid;
      allown &= (f & kOwnT) ? 1 : 0;
      anyown |= (f & kOwnT) ? 1 : 0;
    }
    meta = m | (anyv ? 1 << 21 : 0) | (allown ? 1 << 22 : 0) | (anyown ? 1 << 23 : 0);
    goff = anyv ? static_cast<unsigned>(pl * A.ps + fused_yzoff(A, y0 + ly, z0 + lz0)) : 0u;
    lds = pl * PLP + ly * DZP + lz0;
  };
#pragma unroll
  for (int k = 0; k < NPI; ++k) {
    it_goff[k] = 0;
    it_meta[k] = 0;
    it_lds[k] = ND * PLP;  // padding items: the dummy LDS slots
    const int it = tid + k * NT;
    if (VEC && it < NITV) {
      const int pl = 1 + it / (DY * NIV), rem = it % (DY * NIV);
      item_desc(pl, rem / NIV, (rem % NIV) * V, V, it_goff[k], it_meta[k], it_lds[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < NPS; ++k) {
    is_goff[k] = 0;
    is_meta[k] = 0;
    is_lds[k] = ND * PLP;
    const int it = tid + k * NT;
    if (VEC && it < NITS) item_desc(1 + it / DY, it % DY, OWNZ, 1, is_goff[k], is_meta[k], is_lds[k]);
  }
  // ---- per-thread output descriptors (planes 0..P of a layer): slot e's
  // <= 4 LDS sources (packed 16-bit pairs), destination offset and meta
  auto out_desc = [&](int e, int& s0, int& s1, int& off_o, int& meta_o) {
    s0 = s1 = ZSLOT | (ZSLOT << 16);
    off_o = 0;
    meta_o = 0;
    if (e < ND * PL) {
      const int pl = e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
      const int f = yz_flags(ly, lz);
      if (f & kValid) {
        const int cyh = (ly / P < TY - 1) ? ly / P : TY - 1;
        const int cyl = (ly % P == 0 && ly > 0 && ly / P - 1 < cyh) ? ly / P - 1 : cyh;
        const int czh = (lz / P < TZ - 1) ? lz / P : TZ - 1;
        const int czl = (lz % P == 0 && lz > 0 && lz / P - 1 < czh) ? lz / P - 1 : czh;
        int src[4] = {ZSLOT, ZSLOT, ZSLOT, ZSLOT};
        int ns = 0;
        for (int ccy = cyl; ccy <= cyh; ++ccy)
          for (int ccz = czl; ccz <= czh; ++ccz)
            src[ns++] = EBUF * NWBUF + (ccy * TZ + ccz) * PC + (ly - ccy * P) * P1 +
                        (lz - ccz * P) * RP + pl;
        s0 = src[0] | (src[1] << 16);
        s1 = src[2] | (src[3] << 16);
        const int gy = y0 + ly, gz = z0 + lz;
        const bool iy = ly < oy, iz = lz < oz;
        int kind, off;
        if (iy && iz) {
          kind = 0;
          off = static_cast<int>(pl * A.ps + fused_yzoff(A, gy, gz));
        } else if (!iy && iz) {
          kind = 1;
          off = static_cast<int>(pl * A.ybps) + ty * Lz + gz;
        } else if (iy && !iz) {
          kind = 2;
          off = static_cast<int>(pl * A.zbps) + tz * Ly + gy;
        } else {
          kind = 3;
          off = static_cast<int>(pl * A.cbps) + ty * (A.ntz - 1) + tz;
        }
        off_o = off;
        meta_o = f | (kind << 4) | (pl << 8) | (rem << 12);
      }
    }
  };
  // General instances at NQ >= 7 recompute them per layer in the gather
  // (frees 4 NOUT VGPRs: the Q6 general CG instance spilled 34 dwords with them
  // resident; same-box Q6 general 18.8 -> 22.0 GDoF/s, while Q3 general, which
  // did not spill, drops 18.2 -> 14.0 with the recomputation)
  constexpr bool ORECOMP = AFF == 0 && NQ >= 7;
  int o_src[ORECOMP ? 1 : NOUT][2], o_off[ORECOMP ? 1 : NOUT], o_meta[ORECOMP ? 1 : NOUT];
  if constexpr (!ORECOMP) {
#pragma unroll
    for (int k = 0; k < NOUT; ++k)
      out_desc(tid + k * NT, o_src[k][0], o_src[k][1], o_off[k], o_meta[k]);
  }
  // ---- carried-plane copy descriptors (plane P of a slab -> plane 0 of the next)
  int cp_lds[NCP];
#pragma unroll
  for (int k = 0; k < NCP; ++k) {
    const int e = tid + k * NT;
    cp_lds[k] = (e < PL) ? (e / DZ) * DZP + e % DZ : -1;
  }
  // ---- vertex descriptors
  int v_off[NPV];
#pragma unroll
  for (int k = 0; k < NPV; ++k) {
    const int e = tid + k * NT;
    v_off[k] = -1;
    if (e < NV) {
      const int d = e % 3, r = e / 3;
      const int vz = r % (TZ + 1), vy = r / (TZ + 1);
      const int gy = ty * TY + vy, gz = tz * TZ + vz;
      if (gy <= A.n1 && gz <= A.n2) v_off[k] = (gy * (A.n2 + 1) + gz) * 3 + d;
    }
  }

  // ---- prologue: layer cbeg (planes 0..P), vertex planes cbeg/cbeg+1, zero carry
  {
    const int64_t l0 = static_cast<int64_t>(cbeg) * P * A.ps;
    const bool wr = cbeg == sa;  // not a redundant layer
    for (int e = tid; e < ND * PL; e += NT) {
      const int pl = e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
      const int f = yz_flags(ly, lz);
      T v = T(0);
      if (f & kValid)
        v = stage(f, cbeg * P + pl, A.u + l0, A.pnew + l0, A.y + l0,
                  static_cast<int>(pl * A.ps + fused_yzoff(A, y0 + ly, z0 + lz)), wr);
      s_u[0][pl * PLP + ly * DZP + lz] = v;
    }
  }
  for (int e = tid; e < 2 * NV; e += NT) {
    const int k = e % NV;
    int off = -1;
    {
      const int d = k % 3, r = k / 3;
      const int vz = r % (TZ + 1), vy = r / (TZ + 1);
      const int gy = ty * TY + vy, gz = tz * TZ + vz;
      if (gy <= A.n1 && gz <= A.n2) off = (gy * (A.n2 + 1) + gz) * 3 + d;
    }
    s_X[0][e] = off >= 0 ? A.xv[static_cast<int64_t>(cbeg + e / NV) * A.vps + off] : T(0);
  }
  for (int e = tid; e < PL; e += NT) s_c[0][e] = T(0);

  T Js[3] = {0, 0, 0};                        // AFF = 0 only
  T Jt0[3] = {0, 0, 0}, Jt1[3] = {0, 0, 0};
  T Ju0[3] = {0, 0, 0}, Ju1[3] = {0, 0, 0};
  // AFF = 2 only: 1/x_s, 1/hy, 1/hz, x_t/hy = bt0 + s bt1, x_u/hz = cu0 + s cu1,
  // kappa w_t w_u det J / w_s
  T xia = 0, xihy = 0, xihz = 0, xbt0 = 0, xbt1 = 0, xcu0 = 0, xcu1 = 0, xcs = 0;

  // per-cell coefficient: the next layer's value rides with the prefetch
  // batch (consumed in the same layer, its load made the waitcnt pass drain
  // the whole batch with a vmcnt(0) in the geometry phase, even with
  // constant kappa, where the load itself is skipped)
  const int64_t kc_ps = static_cast<int64_t>(A.n1) * A.n2;
  const int64_t kc_cell = static_cast<int64_t>(ty * TY + cy) * A.n2 + tz * TZ + cz;
  T kc_cur = A.kc ? (cell_on ? A.kc[cbeg * kc_ps + kc_cell] : T(0)) : A.kappa;
  for (int cx = cbeg; cx < cend; ++cx) {
    const int cur = (cx - cbeg) & 1, nxt = cur ^ 1;
    const bool last = (cx == cend - 1);   // end of this segment
    const bool glast = (cx == ncx - 1);   // end of the march
    const bool red = (cx < sa);           // redundant layer: carry only
    __syncthreads();

    // ---- prefetch the next layer (planes 1..P of layer cx+1, vertex plane cx+2)
    const int64_t lnext = static_cast<int64_t>(cx + 1) * P * A.ps;
    T pf_r[VEC ? 1 : NPF], pf_p[VEC ? 1 : NPF], pf_x[VEC ? 1 : NPF];
    VT vf_r[NPI], vf_p[NPI], vf_x[NPI];
    T sf_r[NPS], sf_p[NPS], sf_x[NPS];
    T pf_v[NPV];
    // vertex plane and coefficient first: the loads whose addresses may come
    // back from a register spill (and its vmcnt wait) go before the vector
    // batch, so such a wait cannot drain it
    T kc_nxt = kc_cur;
    if (A.kc && !last && cell_on) kc_nxt = A.kc[static_cast<int64_t>(cx + 1) * kc_ps + kc_cell];
#pragma unroll
    for (int k = 0; k < NPV; ++k) {
      pf_v[k] = T(0);
      if (!last && v_off[k] >= 0) pf_v[k] = A.xv[static_cast<int64_t>(cx + 2) * A.vps + v_off[k]];
    }
    const T* __restrict__ un_r = A.u + lnext;
    const T* __restrict__ un_p = A.pold + lnext;
    T* __restrict__ un_x = A.x + lnext;
#pragma unroll
    for (int k = 0; k < NPI; ++k) {
      vf_r[k] = vf_p[k] = vf_x[k] = VT{};
      if constexpr (VEC) {
        const int m = it_meta[k];
        if (last || !(m & (1 << 21))) continue;
        vf_r[k] = *reinterpret_cast<const VT*>(un_r + it_goff[k]);
        if constexpr (MODE == kFusedCG) {
          vf_p[k] = *reinterpret_cast<const VT*>(un_p + it_goff[k]);
          if (xupd && (m & (1 << 23))) vf_x[k] = *reinterpret_cast<const VT*>(un_x + it_goff[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NPS; ++k) {
      sf_r[k] = sf_p[k] = sf_x[k] = T(0);
      if constexpr (VEC) {
        const int m = is_meta[k];
        if (last || !(m & (1 << 21))) continue;
        sf_r[k] = un_r[is_goff[k]];
        if constexpr (MODE == kFusedCG) {
          sf_p[k] = un_p[is_goff[k]];
          if (xupd && (m & (1 << 23))) sf_x[k] = un_x[is_goff[k]];
        }
      }
    }
#pragma unroll
    for (int k = 0; k < (VEC ? 0 : NPF); ++k) {
      pf_r[k] = T(0);
      pf_p[k] = T(0);
      pf_x[k] = T(0);
      if (!last && (st_meta[k] & kValid)) {
        pf_r[k] = A.u[lnext + st_goff[k]];
        if constexpr (MODE == kFusedCG) {
          pf_p[k] = A.pold[lnext + st_goff[k]];
          if (xupd && (st_meta[k] & kOwnT)) pf_x[k] = A.x[lnext + st_goff[k]];
        }
      }
    }

    int toff = 0;
    asm volatile("" : "+s"(toff));
    const T* __restrict__ gt = tb.tab + toff;
    const T* __restrict__ su = s_u[cur];
    const T* __restrict__ sX = s_X[cur];

    const T* __restrict__ ua = su + (ycell + a) * DZP + zcell;
    // (no __restrict__: the wave-local layout rewrites rows in place, so the
    // compiler must keep each stage's LDS reads ahead of its writes)
    T* const W0 = s_wa;
    T* const W1 = s_wa + NWBUF;
    T* const W2 = s_wa + 2 * NWBUF;  // block layout only
    auto offA = [&](int cc, int i1, int i2) { return cc * PC + i1 * P1 + i2 * RP; };
    // sync between intra-cell stages: wave-local when cells tile whole waves
    auto cell_sync = [&]() {
      if constexpr (WAVELOCAL) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      } else {
        __syncthreads();
      }
    };
    // compiler-level ordering of a wave's in-place LDS rewrite
    auto wave_order = [&]() {
      if constexpr (WAVELOCAL) {
        __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
    };

    // ------------------------------------------------ front z: (B_z u, Dd_z u)
    if constexpr (MFZ) {
      // matrix pipe (one cell per wave, FP64, NQ = 8):
      //   C[(B | Dd, qz)][(i, j)] = [B; Dd] (16 x 8, k = 7 zero) . u[k][(i, j)]
      // 4 column tiles of 16 (i, j) pairs x 2 k-steps of v_mfma_f64_16x16x4f64;
      // the stacked table is the constant A operand (lane: row n, k = g), the
      // u column the B operand (lane: k = g, column n), one scalar LDS read
      // per MFMA instead of the VALU form's ND^2 reads and 2 ND^2 FMAs per lane.
      // Result rows g + 4r: r = 0, 1 -> B_z u at qz = g, g + 4; r = 2, 3 -> Dd_z u.
      int ltid = tid;
      asm volatile("" : "+v"(ltid));  // lane roles and operands re-derived per layer, not hoisted
      const int mg = (ltid & 63) >> 4, mn = ltid & 15;
      const int mr = bdx_mfma_row<T>(mn);  // the table row this lane carries
      const T* __restrict__ arow = s_tab + (mr < NQ ? OFF_BR + mr * NP : OFF_DR + (mr - NQ) * NP);
      const T a0 = arow[mg];
      const T a1 = mg + 4 < ND ? arow[mg + 4] : T(0);
      const int kb = mg + 4 < ND ? mg + 4 : ND - 1;  // k = 7: finite operand, zero row of A
      const T* __restrict__ ub = su + ycell * DZP + zcell;
      constexpr int NTL = (ND * ND + 15) / 16;
      MAcc acc[NTL];
#pragma unroll
      for (int t = 0; t < NTL; ++t) {  // first k-step of every tile, then the second
        const int cc = t * 16 + mn < ND * ND ? t * 16 + mn : ND * ND - 1;
        acc[t] = bdx_mfma16x4(a0, ub[(cc / ND) * PLP + (cc % ND) * DZP + mg], MAcc{0, 0, 0, 0});
      }
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int cc = t * 16 + mn < ND * ND ? t * 16 + mn : ND * ND - 1;
        acc[t] = bdx_mfma16x4(a1, ub[(cc / ND) * PLP + (cc % ND) * DZP + kb], acc[t]);
      }
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int col = t * 16 + mn;
        if (col < ND * ND) {
          const int ii = col / ND, jj = col - (col / ND) * ND;
          W0[offA(c, jj, mg) + ii] = acc[t][0];
          W0[offA(c, jj, mg + 4) + ii] = acc[t][1];
          W1[offA(c, jj, mg) + ii] = acc[t][2];
          W1[offA(c, jj, mg + 4) + ii] = acc[t][3];
        }
      }
    } else if (lane_on && a < ND) {
      // lanes (c, j = a < ND, qz = b): rows over the cell's x dofs i
      const T* __restrict__ br = s_tab + OFF_BR + b * NP;
      const T* __restrict__ dr = s_tab + OFF_DR + b * NP;
      T ob[ND], od[ND];
#pragma unroll
      for (int i = 0; i < ND; ++i) ob[i] = od[i] = T(0);
#pragma unroll
      for (int k = 0; k < ND; ++k) {
        const T cb_ = br[k], cd_ = dr[k];
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          const T uv = ua[i * PLP + k];
          ob[i] += cb_ * uv;
          od[i] += cd_ * uv;
        }
      }
      const int o = offA(c, a, b);
      strow<ND>(W0 + o, ob);
      strow<ND>(W1 + o, od);
    }
    cell_sync();

    // ------------------------------------------------ front y
    // lanes (c, qy = a, qz = b): tBB = B_y B_z u, tDB = Dd_y B_z u, tBD = B_y Dd_z u
    // PEEL: each contraction's first term initialises its accumulators (no
    // zeroing moves before the rolled loops): x-trilinear Q3 26.1 -> 27.3
    // GDoF/s, Q6 neutral (scripts/r3_flushx.sh); the general instance would
    // spill (61 VGPRs), so it keeps the zeroed accumulators.
    constexpr bool PEEL = AFF != 0;
    T tBB[ND], tDB[ND], tBD[ND];
    // lane roles (qy, qz) = (xa, xb) of the geometry and x stages
    int xa = a, xb = b;
    if constexpr (MFY) {
      // matrix pipe: [tBB | tDB](qz, i; qy) = E[(qz, i)][j] . [B | Dd]^T[j][qy] (E = B_z u,
      // W0) and tBD from F = Dd_z u (W1) the same way (its Dd half unused).
      // Row tiles (s, h): row m = (qz = (m & 3) + 4 s, i = (m >> 2) + 4 h), so lane
      // (g, n) ends with the i-lines at qz = g + 4 s of column n: B rows (qy = n)
      // in lanes n < 8, Dd rows (qy = n - 8) in lanes n >= 8.  Lane n < 8 takes
      // (qy, qz) = (n, g), lane n >= 8 (n - 8, g + 4); the halves of each
      // 16-lane row swap the line the partner needs (DPP row rotate by 8).
      int ltid = tid;
      asm volatile("" : "+v"(ltid));
      const int mg = (ltid & 63) >> 4, mn = ltid & 15;
      const bool lo = mn < NQ;
      xa = mn & (NQ - 1);
      xb = mg + (lo ? 0 : 4);
      const T* __restrict__ brow = s_tab + (lo ? OFF_BR + mn * NP : OFF_DR + (mn - NQ) * NP);
      const double by0 = brow[mg];
      const double by1 = mg + 4 < ND ? brow[mg + 4] : 0.0;
      const int kb = mg + 4 < ND ? mg + 4 : ND - 1;
      auto tiles = [&](const T* __restrict__ Wsrc, int sq, T (&out)[ND]) __attribute__((always_inline)) {
        const int qz = (mn & 3) + 4 * sq;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int ii = (mn >> 2) + 4 * h < ND ? (mn >> 2) + 4 * h : ND - 1;
          bdx_f64x4 acc = {0, 0, 0, 0};
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Wsrc[offA(c, mg, qz) + ii], by0, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(Wsrc[offA(c, kb, qz) + ii], by1, acc, 0, 0, 0);
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (r + 4 * h < ND) out[r + 4 * h] = acc[r];
        }
      };
      T e1[ND], f1[ND], f0[ND], e0[ND];
      tiles(W1, 1, f1);  // F at qz = g + 4: the lower half's tBD, sent up
      tiles(W1, 0, f0);
      tiles(W0, 1, e1);
      tiles(W0, 0, e0);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const T rcv = dpp_row_ror8(f1[i]);
        tBD[i] = lo ? f0[i] : rcv;
      }
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const T rcv = dpp_row_ror8(lo ? e1[i] : e0[i]);
        tBB[i] = lo ? e0[i] : rcv;
        tDB[i] = lo ? rcv : e1[i];
      }
    } else {
      const T* __restrict__ bra = s_tab + OFF_BR + a * NP;
      const T* __restrict__ dra = s_tab + OFF_DR + a * NP;
      auto row = [&](int j, bool first) __attribute__((always_inline)) {
        T rb[ND], rd[ND];
        const int o = offA(c, j, b);
        ldrow<ND>(W0 + o, rb);
        ldrow<ND>(W1 + o, rd);
        const T cb_ = bra[j], cd_ = dra[j];
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          tBB[i] = first ? cb_ * rb[i] : tBB[i] + cb_ * rb[i];
          tDB[i] = first ? cd_ * rb[i] : tDB[i] + cd_ * rb[i];
          tBD[i] = first ? cb_ * rd[i] : tBD[i] + cb_ * rd[i];
        }
      };
      if constexpr (PEEL) {
        row(0, true);
      } else {
#pragma unroll
        for (int i = 0; i < ND; ++i) tBB[i] = tDB[i] = tBD[i] = T(0);
      }
BDX_PRAGMA_UNROLL((PEEL ? 3 : 2))
      for (int j = PEEL ? 1 : 0; j < ND; ++j) row(j, false);
    }

    // ------------------------------------------------ geometry coefficients
    // AFF = 0: general trilinear map, dX/ds = Js (constant along the thread's
    // x column), dX/dt = Jt0 + s Jt1, dX/du = Ju0 + s Ju1, G formed per point.
    // AFF = 1: every cell of the launch is a parallelepiped (host-verified by
    // bitwise edge equality, models/fused.py), so J is constant per cell and
    // G = kappa w_a w_b adj(J) adj(J)^T / det J is formed once per thread and
    // layer; per point only the weight w_q remains (same operator, same maths).
    T Gc[6] = {0, 0, 0, 0, 0, 0};
    const T kwyz = kc_cur * s_qw[NQ + xa] * s_qw[NQ + xb];
    {
      const T* X0 = sX;
      const T* X1 = sX + NV;
      const int v00 = (cy * (TZ + 1) + cz) * 3, v01 = v00 + 3;
      const int v10 = v00 + (TZ + 1) * 3;
      if constexpr (AFF == 1) {
        T E[3], F[3], G[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const T X000 = X0[v00 + d];
          E[d] = X1[v00 + d] - X000;
          F[d] = X0[v10 + d] - X000;
          G[d] = X0[v01 + d] - X000;
        }
        const T J00 = E[0], J10 = E[1], J20 = E[2];
        const T J01 = F[0], J11 = F[1], J21 = F[2];
        const T J02 = G[0], J12 = G[1], J22 = G[2];
        const T K00 = J11 * J22 - J12 * J21, K01 = J02 * J21 - J01 * J22, K02 = J01 * J12 - J02 * J11;
        const T K10 = J12 * J20 - J10 * J22, K11 = J00 * J22 - J02 * J20, K12 = J02 * J10 - J00 * J12;
        const T K20 = J10 * J21 - J11 * J20, K21 = J01 * J20 - J00 * J21, K22 = J00 * J11 - J01 * J10;
        const T det = J00 * K00 + J01 * K10 + J02 * K20;
        const T sc = kwyz * fast_rcp(det);
        Gc[0] = sc * (K00 * K00 + K01 * K01 + K02 * K02);
        Gc[1] = sc * (K00 * K10 + K01 * K11 + K02 * K12);
        Gc[2] = sc * (K00 * K20 + K01 * K21 + K02 * K22);
        Gc[3] = sc * (K10 * K10 + K11 * K11 + K12 * K12);
        Gc[4] = sc * (K10 * K20 + K11 * K21 + K12 * K22);
        Gc[5] = sc * (K20 * K20 + K21 * K21 + K22 * K22);
      } else if constexpr (AFF == 2) {
        // x-trilinear cells: the vertex y (z) coordinates depend on the y (z)
        // lattice index only (host-verified bitwise, models/poisson.py
        // cells_x_trilinear), the class src/mesh.cpp:199-207's perturbation
        // produces.  J = [[x_s, x_t, x_u], [0, hy, 0], [0, 0, hz]] with x_s
        // constant along the thread's x column and x_t, x_u linear in s; the
        // zero entries of the trilinear form below are dropped.
        const T t = s_qw[xa], uu = s_qw[xb];
        const int v11 = v10 + 3;
        const T X000 = X0[v00], X001 = X0[v01], X010 = X0[v10], X011 = X0[v11];
        const T X100 = X1[v00], X101 = X1[v01], X110 = X1[v10], X111 = X1[v11];
        const T xs = (1 - t) * ((1 - uu) * (X100 - X000) + uu * (X101 - X001)) +
                     t * ((1 - uu) * (X110 - X010) + uu * (X111 - X011));
        const T xt0 = (1 - uu) * (X010 - X000) + uu * (X011 - X001);
        const T xt1 = (1 - uu) * (X110 - X100) + uu * (X111 - X101) - xt0;
        const T xu0 = (1 - t) * (X001 - X000) + t * (X011 - X010);
        const T xu1 = (1 - t) * (X101 - X100) + t * (X111 - X110) - xu0;
        const T hy = X0[v10 + 1] - X0[v00 + 1], hz = X0[v01 + 2] - X0[v00 + 2];
        xia = fast_rcp(xs);
        xihy = fast_rcp(hy);
        xihz = fast_rcp(hz);
        xbt0 = xt0 * xihy;
        xbt1 = xt1 * xihy;
        xcu0 = xu0 * xihz;
        xcu1 = xu1 * xihz;
        xcs = kwyz * xs * hy * hz;
      } else {
        const T t = s_qw[xa], uu = s_qw[xb];
        const int v11 = v10 + 3;
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const T X000 = X0[v00 + d], X001 = X0[v01 + d], X010 = X0[v10 + d], X011 = X0[v11 + d];
          const T X100 = X1[v00 + d], X101 = X1[v01 + d], X110 = X1[v10 + d], X111 = X1[v11 + d];
          Js[d] = (1 - t) * ((1 - uu) * (X100 - X000) + uu * (X101 - X001)) +
                  t * ((1 - uu) * (X110 - X010) + uu * (X111 - X011));
          Jt0[d] = (1 - uu) * (X010 - X000) + uu * (X011 - X001);
          Jt1[d] = (1 - uu) * (X110 - X100) + uu * (X111 - X101) - Jt0[d];
          Ju0[d] = (1 - t) * (X001 - X000) + t * (X011 - X010);
          Ju1[d] = (1 - t) * (X101 - X100) + t * (X111 - X110) - Ju0[d];
        }
      }
    }

    // ------------------------------------------------ x front + F + x back
    // per quadrature point q along the thread's x column (uniform table rows):
    //   g = (Dd_x tBB, B_x tDB, B_x tBD)(q),  F = kappa G g,
    //   a1 += Dd_x^T Fx, a2 += B_x^T Fy, a3 += B_x^T Fz
    T a1[ND], a2[ND], a3[ND];
    auto xpoint = [&](int q, bool first) __attribute__((always_inline)) {
      T gxq = 0, gyq = 0, gzq = 0;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const T dq = gt[OFF_DC + i * XP + q], bq = gt[OFF_BC + i * XP + q];
        gxq += dq * tBB[i];
        gyq += bq * tDB[i];
        gzq += bq * tBD[i];
      }
      T fx, fy, fz;
      if constexpr (AFF == 1) {
        const T w = s_qw[NQ + q];
        const T t0 = w * gxq, t1 = w * gyq, t2 = w * gzq;
        fx = Gc[0] * t0 + Gc[1] * t1 + Gc[2] * t2;
        fy = Gc[1] * t0 + Gc[3] * t1 + Gc[4] * t2;
        fz = Gc[2] * t0 + Gc[4] * t1 + Gc[5] * t2;
      } else if constexpr (AFF == 2) {
        // grad_X u = (p, gy/hy - bb p, gz/hz - cc p) with p = gx / x_s;
        // F = kappa w det J^-1 grad_X u (16 operations per point)
        const T s = s_qw[q];
        const T bb = xbt0 + s * xbt1, cc = xcu0 + s * xcu1;
        const T p = gxq * xia;
        const T q1 = gyq * xihy - bb * p, q2 = gzq * xihz - cc * p;
        const T sq = xcs * s_qw[NQ + q];
        const T m0 = sq * p, m1 = sq * q1, m2 = sq * q2;
        fy = m1 * xihy;
        fz = m2 * xihz;
        fx = (m0 - bb * m1 - cc * m2) * xia;
      } else {
        const T s = s_qw[q];
        const T J00 = Js[0], J10 = Js[1], J20 = Js[2];
        const T J01 = Jt0[0] + s * Jt1[0], J11 = Jt0[1] + s * Jt1[1], J21 = Jt0[2] + s * Jt1[2];
        const T J02 = Ju0[0] + s * Ju1[0], J12 = Ju0[1] + s * Ju1[1], J22 = Ju0[2] + s * Ju1[2];
        const T K00 = J11 * J22 - J12 * J21, K01 = J02 * J21 - J01 * J22, K02 = J01 * J12 - J02 * J11;
        const T K10 = J12 * J20 - J10 * J22, K11 = J00 * J22 - J02 * J20, K12 = J02 * J10 - J00 * J12;
        const T K20 = J10 * J21 - J11 * J20, K21 = J01 * J20 - J00 * J21, K22 = J00 * J11 - J01 * J10;
        const T det = J00 * K00 + J01 * K10 + J02 * K20;
        const T sc = kwyz * s_qw[NQ + q] * fast_rcp(det);
        const T h0 = K00 * gxq + K10 * gyq + K20 * gzq;
        const T h1 = K01 * gxq + K11 * gyq + K21 * gzq;
        const T h2 = K02 * gxq + K12 * gyq + K22 * gzq;
        fx = sc * (K00 * h0 + K01 * h1 + K02 * h2);
        fy = sc * (K10 * h0 + K11 * h1 + K12 * h2);
        fz = sc * (K20 * h0 + K21 * h1 + K22 * h2);
      }
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        const T dq = gt[OFF_DC + i * XP + q], bq = gt[OFF_BC + i * XP + q];
        a1[i] = first ? dq * fx : a1[i] + dq * fx;
        a2[i] = first ? bq * fy : a2[i] + bq * fy;
        a3[i] = first ? bq * fz : a3[i] + bq * fz;
      }
    };
    if constexpr (PEEL) {
      xpoint(0, true);
    } else {
#pragma unroll
      for (int i = 0; i < ND; ++i) a1[i] = a2[i] = a3[i] = T(0);
    }
BDX_PRAGMA_UNROLL((QUnroll3G<T, NQ, AFF>::value))
    for (int q = PEEL ? 1 : 0; q < NQ; ++q) xpoint(q, false);
    if constexpr (WAVELOCAL) {
      // W0 <- A1, W1 <- A2 (the front-y reads of this wave are already issued)
      wave_order();
      if (lane_on) {
        strow<ND>(W0 + offA(c, xa, xb), a1);
        strow<ND>(W1 + offA(c, xa, xb), a2);
      }
      cell_sync();
      if constexpr (MFBY) {
        // back y on the matrix pipe: C[(qz, i)][j] = A[(qz, i)][(src, qy)] . [B; Dd][(src, qy)][j]
        // (column tiles of 16 (qz, i) pairs, e = 7 qz + i; the table is the
        // constant B operand, zero for j >= ND).  Pass 1: C1 from A1 (W0) and
        // A2 (W1), 4 k-steps, in place into W0; then A3 -> W1; pass 2: C3 from
        // A3, 2 k-steps, in place into W1.  Lane (g, n) ends with
        // C[(qz, i) = 16 t + g + 4 r][j = n].
        int ltid = tid;
        asm volatile("" : "+v"(ltid));
        const int mg = (ltid & 63) >> 4, mn = ltid & 15;
        constexpr int NE = NQ * ND, NTL = (NE + 15) / 16;
        auto pass = [&](int nks, const T* __restrict__ Wk0, const T* __restrict__ Wk1, T* __restrict__ Wout)
            __attribute__((always_inline)) {
          T bk[4];
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            const int qy = (ks & 1) * 4 + mg;
            bk[ks] = (ks < nks && mn < ND) ? s_tab[(ks < 2 ? OFF_BR : OFF_DR) + qy * NP + mn] : T(0);
          }
          // k-step outer: the NTL independent accumulators interleave, so no
          // MFMA waits on the previous one's result
          MAcc acc[NTL];
          int aoff[NTL];
#pragma unroll
          for (int t = 0; t < NTL; ++t) {
            const int m = t * 16 + bdx_mfma_row<T>(mn);
            const int e = m < NE ? m : NE - 1;
            aoff[t] = offA(c, mg, e / ND) + (e - (e / ND) * ND);
            acc[t] = MAcc{0, 0, 0, 0};
          }
#pragma unroll
          for (int ks = 0; ks < 4; ++ks) {
            if (ks >= nks) break;
#pragma unroll
            for (int t = 0; t < NTL; ++t) {
              const T av = (ks < 2 ? Wk0 : Wk1)[aoff[t] + (ks & 1) * 4 * P1];
              acc[t] = bdx_mfma16x4(av, bk[ks], acc[t]);
            }
          }
          wave_order();  // every lane's reads are issued before the in-place writes
          if (mn < ND) {
#pragma unroll
            for (int t = 0; t < NTL; ++t)
#pragma unroll
              for (int r = 0; r < 4; ++r) {
                const int e = t * 16 + mg + 4 * r;
                if (e >= NE) continue;
                const int qz = e / ND, ii = e - (e / ND) * ND;
                Wout[offA(c, mn, qz) + ii] = acc[t][r];
              }
          }
        };
        pass(4, W0, W1, W0);
        if (lane_on) strow<ND>(W1 + offA(c, xa, xb), a3);
        cell_sync();
        pass(2, W1, W1, W1);
        cell_sync();
      } else {
        // back y, pass 1: C1 = B_y^T A1 + Dd_y^T A2 -> W0; then A3 -> W1
        T c1[ND];
  #pragma unroll
        for (int i = 0; i < ND; ++i) c1[i] = T(0);
        if (lane_on && a < ND) {
          const T* bcj = s_tab + OFF_BC + a * XP;
          const T* dcj = s_tab + OFF_DC + a * XP;
  BDX_PRAGMA_UNROLL(2)
          for (int qy = 0; qy < NQ; ++qy) {
            T r1[ND], r2[ND];
            ldrow<ND>(W0 + offA(c, qy, b), r1);
            ldrow<ND>(W1 + offA(c, qy, b), r2);
            const T bq = bcj[qy], dq = dcj[qy];
  #pragma unroll
            for (int i = 0; i < ND; ++i) c1[i] += bq * r1[i] + dq * r2[i];
          }
        }
        wave_order();
        if (lane_on && a < ND) strow<ND>(W0 + offA(c, a, b), c1);
        if (lane_on) strow<ND>(W1 + offA(c, xa, xb), a3);
        cell_sync();
        // pass 2: C3 = B_y^T A3 -> W1
        T c3[ND];
  #pragma unroll
        for (int i = 0; i < ND; ++i) c3[i] = T(0);
        if (lane_on && a < ND) {
          const T* bcj = s_tab + OFF_BC + a * XP;
  BDX_PRAGMA_UNROLL(2)
          for (int qy = 0; qy < NQ; ++qy) {
            T r3[ND];
            ldrow<ND>(W1 + offA(c, qy, b), r3);
            const T bq = bcj[qy];
  #pragma unroll
            for (int i = 0; i < ND; ++i) c3[i] += bq * r3[i];
          }
        }
        wave_order();
        if (lane_on && a < ND) strow<ND>(W1 + offA(c, a, b), c3);
        cell_sync();
      }
    } else {
      // A3 -> W2 (free since the previous layer's gather); A1, A2 -> W0, W1
      // once every wave finished its front-y reads of them
      if (lane_on) strow<ND>(W2 + offA(c, xa, xb), a3);
      cell_sync();
      if (lane_on) {
        strow<ND>(W0 + offA(c, xa, xb), a1);
        strow<ND>(W1 + offA(c, xa, xb), a2);
      }
      cell_sync();
      // back y: lanes (c, j = a < ND, qz = b): C1 = B_y^T A1 + Dd_y^T A2, C3 = B_y^T A3
      T c1[ND], c3[ND];
      if (lane_on && a < ND) {
        const T* bcj = s_tab + OFF_BC + a * XP;
        const T* dcj = s_tab + OFF_DC + a * XP;
        auto row = [&](int qy, bool first) __attribute__((always_inline)) {
          const int o = offA(c, qy, b);
          T r1[ND], r2[ND], r3[ND];
          ldrow<ND>(W0 + o, r1);
          ldrow<ND>(W1 + o, r2);
          ldrow<ND>(W2 + o, r3);
          const T bq = bcj[qy], dq = dcj[qy];
#pragma unroll
          for (int i = 0; i < ND; ++i) {
            c1[i] = first ? bq * r1[i] + dq * r2[i] : c1[i] + bq * r1[i] + dq * r2[i];
            c3[i] = first ? bq * r3[i] : c3[i] + bq * r3[i];
          }
        };
        if constexpr (PEEL) {
          row(0, true);
        } else {
#pragma unroll
          for (int i = 0; i < ND; ++i) c1[i] = c3[i] = T(0);
        }
BDX_PRAGMA_UNROLL(2)
        for (int qy = PEEL ? 1 : 0; qy < NQ; ++qy) row(qy, false);
      } else {
#pragma unroll
        for (int i = 0; i < ND; ++i) c1[i] = c3[i] = T(0);
      }
      cell_sync();  // every wave's back-y reads done before C overwrites A1/A2
      if (lane_on && a < ND) {
        strow<ND>(W0 + offA(c, a, b), c1);
        strow<ND>(W1 + offA(c, a, b), c3);
      }
      cell_sync();
    }

    // ------------------------------------------------ back z
    if constexpr (MFBZ) {
      // matrix pipe: y_e[(j, i)][k] = [C1 | C3][(j, i)][(src, qz)] . [B; Dd][(src, qz)][k]
      // 4 row tiles of 16 (j, i) pairs x 4 k-steps (C1 at qz = g, g + 4, then
      // C3); the table is the constant B operand (lane: k-row g, column n = z
      // dof, zero for n >= ND).  Lane (g, n) ends with y_e[(j, i) = 16 t + g + 4 r][k = n].
      int ltid = tid;
      asm volatile("" : "+v"(ltid));
      const int mg = (ltid & 63) >> 4, mn = ltid & 15;
      T bk[4];
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const int qz = (ks & 1) * 4 + mg;
        bk[ks] = mn < ND ? s_tab[(ks < 2 ? OFF_BR : OFF_DR) + qz * NP + mn] : T(0);
      }
      constexpr int NTL = (ND * ND + 15) / 16;
      MAcc acc[NTL];
      int aoff[NTL];
#pragma unroll
      for (int t = 0; t < NTL; ++t) {
        const int col = t * 16 + bdx_mfma_row<T>(mn);  // the (j, i) row this lane carries
        const int cc = col < ND * ND ? col : ND * ND - 1;
        aoff[t] = offA(c, cc / ND, mg) + (cc - (cc / ND) * ND);
        acc[t] = MAcc{0, 0, 0, 0};
      }
#pragma unroll
      for (int ks = 0; ks < 4; ++ks)  // k-step outer: independent accumulators interleave
#pragma unroll
        for (int t = 0; t < NTL; ++t) {
          const T av = (ks < 2 ? W0 : W1)[aoff[t] + (ks & 1) * 4 * RP];
          acc[t] = bdx_mfma16x4(av, bk[ks], acc[t]);
        }
      wave_order();  // every lane's C1 / C3 reads are issued before E overwrites W0
      if (mn < ND) {
#pragma unroll
        for (int t = 0; t < NTL; ++t)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int e = t * 16 + mg + 4 * r;
            if (e >= ND * ND) continue;
            const int jj = e / ND, ii = e - (e / ND) * ND;
            const T v = cell_on ? acc[t][r] : T(0);
            if constexpr (MODE == kFusedCG) {
              if (!red)
                pap += static_cast<double>(su[ii * PLP + (ycell + jj) * DZP + zcell + mn]) *
                       static_cast<double>(v);
            }
            W0[offA(c, jj, mn) + ii] = v;
          }
      }
    }
    T ye[ND];
    if constexpr (MFBZ) {
    } else if (lane_on && a < ND && b < ND) {
      // lanes (c, j = a < ND, k = b < ND): y_e = B_z^T C1 + Dd_z^T C3
      const T* bck = s_tab + OFF_BC + b * XP;
      const T* dck = s_tab + OFF_DC + b * XP;
      auto row = [&](int qz, bool first) __attribute__((always_inline)) {
        const int o = offA(c, a, qz);
        T r1[ND], r3[ND];
        ldrow<ND>(W0 + o, r1);
        ldrow<ND>(W1 + o, r3);
        const T bq = bck[qz], dq = dck[qz];
#pragma unroll
        for (int i = 0; i < ND; ++i)
          ye[i] = first ? bq * r1[i] + dq * r3[i] : ye[i] + bq * r1[i] + dq * r3[i];
      };
      if constexpr (PEEL) {
        row(0, true);
      } else {
#pragma unroll
        for (int i = 0; i < ND; ++i) ye[i] = T(0);
      }
BDX_PRAGMA_UNROLL(2)
      for (int qz = PEEL ? 1 : 0; qz < NQ; ++qz) row(qz, false);
    } else {
#pragma unroll
      for (int i = 0; i < ND; ++i) ye[i] = T(0);
    }

    // ------------------------------------------------ element vectors -> A1 of the cell
    const bool dof_lane = cell_on && a < ND && b < ND;
    if constexpr (MODE == kFusedCG && !MFBZ) {
      if (dof_lane && !red) {
#pragma unroll
        for (int i = 0; i < ND; ++i)
          pap += static_cast<double>(ua[i * PLP + b]) * static_cast<double>(ye[i]);
      }
    }
    if constexpr (!MFBZ) {
      wave_order();
      if (lane_on && a < ND && b < ND) {
        if (!dof_lane) {
#pragma unroll
          for (int i = 0; i < ND; ++i) ye[i] = T(0);
        }
        strow<ND>((WAVELOCAL ? W0 : W2) + offA(c, a, b), ye);
      }
    }
    __syncthreads();

    auto do_gather = [&](auto DIRC) __attribute__((always_inline)) {
      constexpr bool DIR = decltype(DIRC)::value;
      // ------------------------------------------------ gather-sum and write out
      {
        const int64_t lbase = static_cast<int64_t>(cx) * P;
        T* __restrict__ ybase[4] = {A.y + lbase * A.ps, A.yb + lbase * A.ybps,
                                    A.zb + lbase * A.zbps, A.cb + lbase * A.cbps};
  #pragma unroll
        for (int k = 0; k < NOUT; ++k) {
          int os0, os1, ooff, m;
          if constexpr (ORECOMP) {
            int e = tid + k * NT;
            asm volatile("" : "+v"(e));  // recompute here, not hoisted out of the march
            out_desc(e, os0, os1, ooff, m);
          } else {
            asm volatile("" : "+v"(o_src[k][0]), "+v"(o_src[k][1]), "+v"(o_off[k]), "+v"(o_meta[k]));
            os0 = o_src[k][0];
            os1 = o_src[k][1];
            ooff = o_off[k];
            m = o_meta[k];
          }
          if (!(m & kValid)) continue;
          const int pl = (m >> 8) & 15, rem = m >> 12;
          T v = s_wa[os0 & 0xffff] + s_wa[os0 >> 16] + s_wa[os1 & 0xffff] + s_wa[os1 >> 16];
          if (pl == 0) v += s_c[cur][rem];
          if (pl == P && !last) {
            s_c[nxt][rem] = v;
            continue;
          }
          // a redundant layer only carries; a segment's end plane is completed
          // (and written) by the next segment
          if (red || (pl == P && !glast)) continue;
          const int gxx = cx * P + pl;
          const bool bc = DIR && ((m & kBcYZ) || gxx == A.bcx_lo || gxx == A.bcx_hi);
          const int kind = (m >> 4) & 3;
          if (bc) {
            if (kind == 0) continue;  // Dirichlet y was written at staging
            v = T(0);
          }
          if (BDX_OOB(lbase * (kind == 0 ? A.ps : kind == 1 ? A.ybps : kind == 2 ? A.zbps : A.cbps) +
                          ooff, kind == 0 ? A.vsize : A.ibsize, "f3 gather store"))
            continue;
          T* __restrict__ dst = kind == 0 ? ybase[0] : kind == 1 ? ybase[1] : kind == 2 ? ybase[2] : ybase[3];
          dst[ooff] = v;
        }
      }

    };
    auto do_stage_vec = [&](auto DIRC) __attribute__((always_inline)) {
      constexpr bool DIR = decltype(DIRC)::value;
      // ------------------------------------------------ stage the next layer (VEC items)
      if (!last) {
#pragma unroll
        for (int k = 0; k < NPI; ++k)
          asm volatile("" : "+v"(it_goff[k]), "+v"(it_meta[k]), "+v"(it_lds[k]));
#pragma unroll
        for (int k = 0; k < NPS; ++k)
          asm volatile("" : "+v"(is_goff[k]), "+v"(is_meta[k]), "+v"(is_lds[k]));
        T* __restrict__ un = s_u[nxt];
#pragma unroll
        for (int k = 0; k < NCP; ++k)
          if (cp_lds[k] >= 0) un[cp_lds[k]] = su[P * PLP + cp_lds[k]];
        T* __restrict__ pnl = A.pnew + lnext;
        T* __restrict__ yl = A.y + lnext;
        // node e of an item: Dirichlet identity row (plane 0 of the march is
        // the prologue's); returns the value staged into LDS
        auto dirichlet = [&](int m, int e, unsigned goff, T v) __attribute__((always_inline)) -> T {
          const int f = (m >> (4 * e)) & 15;
          const int gxx = (cx + 1) * P + ((m >> 16) & 15);
          if constexpr (!DIR) return (f & kValid) ? v : T(0);
          if (!(f & kValid)) return T(0);
          if ((f & kBcYZ) || gxx == A.bcx_hi) {
            if (f & kOwnT) {
              const bool rown = (f & kRownYZ) && gxx < A.ownx;
              yl[goff + e] = rown ? v : T(0);
              if constexpr (MODE == kFusedCG) {
                if (rown) pap += static_cast<double>(v) * static_cast<double>(v);
              }
            }
            return T(0);
          }
          return v;
        };
#pragma unroll
        for (int k = 0; k < NPI; ++k) {
          const int m = it_meta[k];
          VT val;
          if constexpr (MODE == kFusedCG) {
            val = vf_r[k] + beta * vf_p[k];
            const VT xn = vf_x[k] + xalpha * vf_p[k];
            if (m & (1 << 22)) {  // every node owned: whole vectors
              *reinterpret_cast<VT*>(pnl + it_goff[k]) = val;
              if (xupd) *reinterpret_cast<VT*>(un_x + it_goff[k]) = xn;
            } else if (m & (1 << 23)) {  // some owned (a tile at the domain's edge)
#pragma unroll
              for (int e = 0; e < V; ++e) {
                if (!((m >> (4 * e)) & kOwnT)) continue;
                pnl[it_goff[k] + e] = val[e];
                if (xupd) un_x[it_goff[k] + e] = xn[e];
              }
            }
          } else {
            val = vf_r[k];
          }
#pragma unroll
          for (int e = 0; e < V; ++e) un[it_lds[k] + e] = dirichlet(m, e, it_goff[k], val[e]);
        }
#pragma unroll
        for (int k = 0; k < NPS; ++k) {
          const int m = is_meta[k];
          T val;
          if constexpr (MODE == kFusedCG) {
            val = sf_r[k] + beta * sf_p[k];
            if (m & (1 << 23)) {
              pnl[is_goff[k]] = val;
              if (xupd) un_x[is_goff[k]] = sf_x[k] + xalpha * sf_p[k];
            }
          } else {
            val = sf_r[k];
          }
          if (tid + k * NT < NITS) un[is_lds[k]] = dirichlet(m, 0, is_goff[k], val);
        }
#pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int e = tid + k * NT;
          if (e < NV) s_X[nxt][e] = sX[NV + e];
        }
#pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int e = tid + k * NT;
          if (e < NV) s_X[nxt][NV + e] = pf_v[k];
        }
      }
    };
    auto do_stage = [&](auto DIRC) __attribute__((always_inline)) {
      constexpr bool DIR = decltype(DIRC)::value;
      // ------------------------------------------------ stage the next layer
      if (!last) {
        #pragma unroll
        for (int k = 0; k < NPF; ++k) asm volatile("" : "+v"(st_goff[k]), "+v"(st_meta[k]));
        T* __restrict__ un = s_u[nxt];
  #pragma unroll
        for (int k = 0; k < NCP; ++k)
          if (cp_lds[k] >= 0) un[cp_lds[k]] = su[P * PLP + cp_lds[k]];
        T* __restrict__ pnl = A.pnew + lnext;
        T* __restrict__ yl = A.y + lnext;
  #pragma unroll
        for (int k = 0; k < NPF; ++k) {
          const int m = st_meta[k];
          if (tid + k * NT < P * PL) {
            T v = T(0);
            if (m & kValid) {
              const int gxx = (cx + 1) * P + ((m >> 4) & 15);
              T val;
              if constexpr (MODE == kFusedCG) {
                val = pf_r[k] + beta * pf_p[k];
              } else {
                val = pf_r[k];
              }
              if constexpr (MODE == kFusedCG) {
                if (m & kOwnT) {
                  pnl[st_goff[k]] = val;
                  if (xupd) A.x[lnext + st_goff[k]] = pf_x[k] + xalpha * pf_p[k];
                }
              }
              if (DIR && ((m & kBcYZ) || gxx == A.bcx_hi)) {
                if (m & kOwnT) {
                  const bool rown = (m & kRownYZ) && gxx < A.ownx;
                  yl[st_goff[k]] = rown ? val : T(0);
                  if constexpr (MODE == kFusedCG) {
                    if (rown) pap += static_cast<double>(val) * static_cast<double>(val);
                  }
                }
                val = T(0);
              }
              v = val;
            }
            un[m >> 8] = v;
          }
        }
  #pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int e = tid + k * NT;
          if (e < NV) s_X[nxt][e] = sX[NV + e];
        }
  #pragma unroll
        for (int k = 0; k < NPV; ++k) {
          const int e = tid + k * NT;
          if (e < NV) s_X[nxt][NV + e] = pf_v[k];
        }
      }
    };
    // Consume the prefetch before the gather stores,
    // behind one explicit vmcnt(0) (as in lap_fused5.h)
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // staging: planes 1..P of layer cx + 1; gather: planes 0..P of layer cx.
    // As in lap_fused5.h the Q3 (ND = 4) instances keep the single copy (the
    // split lost 1.5 % on the x-trilinear one; Q6 +0.3 %, profiles/r5_kernel_ab.md)
    constexpr bool SPLIT = kF3DirSplit && (ND >= 6 || sizeof(T) == 4);
    const bool dir_s = !SPLIT || tile_bc || xbc_in((cx + 1) * P + 1, P);
    const bool dir_g = !SPLIT || tile_bc || xbc_in(cx * P, P + 1);
    if constexpr (VEC) {
      if (dir_s)
        do_stage_vec(std::true_type{});
      else
        do_stage_vec(std::false_type{});
    } else {
      if (dir_s)
        do_stage(std::true_type{});
      else
        do_stage(std::false_type{});
    }
    if (dir_g)
      do_gather(std::true_type{});
    else
      do_gather(std::false_type{});
    kc_cur = kc_nxt;
  }
  if constexpr (MODE == kFusedCG) {
    const double t = block_sum(pap, s_red);
    // indexed by (tile, segment): invariant under any launch split
    if (tid == 0) A.partials[(ty * A.ntz + tz) * A.nseg + seg] = t;
  }
}

// Host-side launch: build the argument block from the packed lattice
// descriptor (fem/mesh.py LocalLattice.as_int64) and launch one workgroup per
// (y, z) tile.
// Does a tile row's own part split into whole 16-byte vectors (the VEC
// instance)?  Shape (compile time) and layout / alignment (launch time).
template <typename T, int ND, int NQ>
constexpr bool f3_vec_shape() {
  constexpr int V = 16 / static_cast<int>(sizeof(T)), OWNZ = TileFor<NQ>::TZ * (ND - 1);
  return kF3Vec && OWNZ % V == 0 && (OWNZ * static_cast<int>(sizeof(T))) % 16 == 0;
}
template <typename T, int ND, int NQ>
bool f3_vec_ok(const Fused2Args<T>& a) {
  constexpr int V = 16 / static_cast<int>(sizeof(T)), P = ND - 1;
  constexpr int OWNY = TileFor<NQ>::TY * P, OWNZ = TileFor<NQ>::TZ * P;
  const bool lay = a.tsy ? (a.tsy == OWNY && a.tsz == OWNZ)
                         : (a.ld % V == 0 && a.ps % V == 0 && static_cast<int64_t>(a.ntz) * OWNZ <= a.ld);
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return lay && al(a.u) && al(a.pold) && al(a.pnew) && al(a.x);
}

template <typename T, int ND, int NQ, int MODE>
int launch_fused3(int affine, const Fused2Args<T>& a, const FusedTables<T>& tb, hipStream_t st) {
  using TF = TileFor<NQ>;
  using S = FusedShape<T, ND, NQ, TF::TY, TF::TZ>;
  const int nblk = a.nblk;
  if (nblk <= 0) return 0;
  if constexpr (MODE == kFusedCG && f3_vec_shape<T, ND, NQ>()) {
    if (affine != 1 && f3_vec_ok<T, ND, NQ>(a)) {
      if (affine == 2)
        lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, MODE, 2, true><<<nblk, S::threads, 0, st>>>(a, tb);
      else
        lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, MODE, 0, true><<<nblk, S::threads, 0, st>>>(a, tb);
      return static_cast<int>(hipGetLastError());
    }
  }
  // affine: 1 = parallelepipeds, 2 = x-trilinear (y/z lattice), 0 = trilinear
  if (affine == 1)
    lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, MODE, 1><<<nblk, S::threads, 0, st>>>(a, tb);
  else if (affine == 2)
    lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, MODE, 2><<<nblk, S::threads, 0, st>>>(a, tb);
  else
    lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, MODE, 0><<<nblk, S::threads, 0, st>>>(a, tb);
  return static_cast<int>(hipGetLastError());
}

// Workgroups of a fused3 CG instance the chip holds at once (segment sizing).
template <typename T, int ND, int NQ>
int fused3_resident(int affine) {
  using TF = TileFor<NQ>;
  using S = FusedShape<T, ND, NQ, TF::TY, TF::TZ>;
  int per_cu = 0, dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return 0;
  const hipError_t e =
      affine == 1 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                        &per_cu, lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, kFusedCG, 1>, S::threads, 0)
      : affine == 2 ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                          &per_cu, lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, kFusedCG, 2,
                                                     f3_vec_shape<T, ND, NQ>()>, S::threads, 0)
                    : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                          &per_cu, lap_fused3_kernel<T, ND, NQ, TF::TY, TF::TZ, kFusedCG, 0,
                                                     f3_vec_shape<T, ND, NQ>()>, S::threads, 0);
  return e == hipSuccess ? per_cu * cus : 0;
}

#define BDX_FUSED3_TU(T, SUF, PP)                                                   \
  extern "C" int bdx_fused3_apply_##SUF##_p##PP(                                   \
      int mode, int affine_ok, const int64_t* latd, int nq, const double* wts,     \
      const double* qpts,                                                          \
      const T* u, const T* pold, T* pnew, T* x, T* y, T* yb, T* zb, T* cb,         \
      const T* xv, const T* kc, const T* tabs, double kappa, const double* scal,   \
      double* partials, int beta_num, int beta_den, int xa_num, int xa_den,        \
      int nty, int ntz, const int* rect, hipStream_t st) {                                          \
    Fused2Args<T> a;                                                               \
    BDX_CHECK(static_cast<hipError_t>(make_fused2_args(a, latd, nty, ntz)));  \
    BDX_CHECK(static_cast<hipError_t>(fused_set_rect(a, rect)));       \
    BDX_CHECK(static_cast<hipError_t>(fused_set_segments(a, (mode >> 8) & 0xff))); \
    mode &= 0xff;                                                                  \
    a.u = u;                                                                       \
    a.pold = pold;                                                                 \
    a.pnew = pnew;                                                                 \
    a.x = x;                                                                       \
    a.y = y;                                                                       \
    a.yb = yb;                                                                     \
    a.zb = zb;                                                                     \
    a.cb = cb;                                                                     \
    a.xv = xv;                                                                     \
    a.kc = kc;                                                                     \
    a.scal = scal;                                                                 \
    a.partials = partials;                                                         \
    a.beta_num = beta_num;                                                         \
    a.beta_den = beta_den;                                                         \
    a.xa_num = xa_num;                                                             \
    a.xa_den = xa_den;                                                             \
    a.kappa = static_cast<T>(kappa);                                               \
    if (!tabs) return static_cast<int>(hipErrorInvalidValue);                      \
    FusedTables<T> tb;                                                             \
    for (int i = 0; i < kFusedTabMax; ++i) tb.tab[i] = tabs[i];                    \
    for (int q = 0; q < kMaxNq; ++q) {                                             \
      tb.qpts[q] = q < nq ? static_cast<T>(qpts[q]) : T(0);                        \
      tb.wts[q] = q < nq ? static_cast<T>(wts[q]) : T(0);                          \
    }                                                                              \
    if (nq == PP + 2)                                                              \
      return mode == kFusedCG ? launch_fused3<T, PP + 1, PP + 2, kFusedCG>(affine_ok, a, tb, st) \
                              : launch_fused3<T, PP + 1, PP + 2, kFusedAction>(affine_ok, a, tb, st); \
    return static_cast<int>(hipErrorInvalidValue);                                 \
  }                                                                                \
  extern "C" int bdx_fused3_segments_##SUF##_p##PP(int affine_ok, int nq, int tiles, int ncx) { \
    if (nq != PP + 2) return 1;                                                    \
    const int s = fused_choose_segments(tiles, ncx, fused3_resident<T, PP + 1, PP + 2>(affine_ok)); \
    /* x-trilinear: at least 2 segments (measured 1 -> 2: Q3 +1.5 %, Q6 +3.7 %, \
       Q6 FP32 +4.0 %, profiles/r2_xtrilinear.md) */                              \
    return (affine_ok == 2 && s < 2 && ncx >= 8) ? 2 : s;                           \
  }

// Packed tables of the fused3 core (layout: OFF_BR/OFF_DR rows of B = phi0 and
// Dd = dphi1 phi0 with pitch NP, OFF_BC/OFF_DC their transposes with pitch XP).
template <typename T, int ND, int NQ>
int pack_tables3(const double* phi0, const double* Dd, T* out) {
  using S = FusedShape<T, ND, NQ, 1, 1>;
  constexpr int NP = S::NP, XP = S::XP;
  constexpr int OFF_BR = 0, OFF_DR = NQ * NP, OFF_BC = 2 * NQ * NP, OFF_DC = 2 * NQ * NP + ND * XP;
  if (!out) return kFusedTabMax;
  for (int i = 0; i < kFusedTabMax; ++i) out[i] = T(0);
  for (int q = 0; q < NQ; ++q)
    for (int i = 0; i < ND; ++i) {
      out[OFF_BR + q * NP + i] = static_cast<T>(phi0[q * ND + i]);
      out[OFF_DR + q * NP + i] = static_cast<T>(Dd[q * ND + i]);
      out[OFF_BC + i * XP + q] = static_cast<T>(phi0[q * ND + i]);
      out[OFF_DC + i * XP + q] = static_cast<T>(Dd[q * ND + i]);
    }
  return kFusedTabMax;
}
