// Fused structured operator kernel, v5 ("fused5"): nodal Kronecker sum
// factorisation for axis-aligned box cells, any degree P = 3..7, FP64 / FP32.
//
// For a cell with a constant Jacobian the quadrature sum of the reference
// stiffness operator (src/laplacian_gpu.hpp:91-426 with
// src/geometry_gpu.hpp:26-132) factorises exactly into 1D matrices of the
// same quadrature rule:
//   M = B^T W B,  K = Dd^T W Dd,  C = Dd^T W B   (B = phi0, Dd = dphi1 phi0),
//   A_e = G00 K.M.M + G11 M.K.M + G22 M.M.K + G12 M.(C.Ct + Ct.C)
//       + G01 (C.Ct.M + Ct.C.M) + G02 (C.M.Ct + Ct.M.C)      (x . y . z).
// On an axis-aligned box G01 = G02 = G12 = 0.  (An earlier core, fused4,
// contracted the (y, z) factor as one 16 x 16 MFMA operand, which only paid
// at ND = 4 and lost to this one; removed in round 5.)  Here the three
// directions are applied one after another
// on ND x ND nodal matrices -- no quadrature-point arrays at all (ND^3 instead
// of NQ^3 values per cell, 343 vs 512 at Q6) -- with every pass reading its
// input line once:
//   x pass   lane (j, k) holds the x-line u[.][j][k] (slab LDS -> registers),
//            forms Kx u, Mx u;
//   z pass   lane (i, j) reads its z-lines (one 16-byte vector row each) and
//            forms the y-factor groups
//              zM  = G00 Mz(Kx u) + G22 Kz(Mx u)
//              zK  = G11 Mz(Mx u);
//   y pass   lane (i, k) reads its y-lines and forms
//              y_e = My zM + Ky zK.
// A cell is one wave for ND >= 6 (ND^2 lanes of 64) and 2 / 4 cells share a
// wave at ND = 5 / 4, so the passes exchange data only inside a wave:
// wave-local syncs, in-place rewrites of one per-wave buffer, two workgroup
// barriers per cell layer (gather and staging).  The 1D matrices are
// wave-uniform scalar loads from a device buffer that each operator owns
// (allocated at construction, passed by pointer: a captured hipGraph keeps
// reading its own operator's tables).  The kernel runs on axis-aligned
// boxes only (diagonal Jacobians, the benchmark mesh; exact host check):
// two arrays of line rows, 7 ND^2 FMAs per lane and cell.  Parallelepipeds
// with a full Jacobian (G01, G02, G12 != 0) take fused3's affine instance
// (driver.py): the four-array form of this core for them was reachable only
// from a test-only shear map and was removed in round 5.
//
// Everything around the core -- the x-march over (y, z) tiles, the double
// buffered slab staging with the CG fusion (p = r + beta p_old, lagged
// x update, Dirichlet identity rows, p.Ap partials as element dots) and the
// atomic-free gather with tile-interface buffers -- is shared with fused3's
// x-march design (lap_fused2.h / lap_fused3.h).
#pragma once
#include <cmath>
#include <cstdlib>
#include <type_traits>

#include "lap_fused2.h"

// Resident waves per SIMD the kernel is compiled for (__launch_bounds__):
// the FP64 Q6 CG instance is 170 VGPRs, so 2; a 3-wave build spills and
// measured 9 % slower (profiles/r2_launder.md).
constexpr int kF5Waves = 2;

// 16-byte staging loads / stores (the VEC instance, lap_fused5_kernel)
constexpr bool kF5Vec = true;

// Slab pitches of the FP64 ND = 7 (Q6) instance congruent to 7 mod 16 words
// (switch): the x-pass and p.Ap reads put 7 lanes on each slab row, so a
// 16-lane group of a ds_read2_b64 then covers 16 consecutive banks instead of
// colliding on the next row's first ones (scripts/lds_bank_f5.py: 168 of the
// 546 modelled conflict cycles per layer and workgroup).  Measured off: bank
// conflicts -10 %, no fewer LDS waits, 0.4 % slower (the larger pitch breaks
// ds_read2_b64 pairing, +4 % LDS instructions; profiles/r5_kernel_ab.md).
constexpr bool kF5Pad7 = false;

// Late prefetch (switch): issue the next layer's loads after the z pass
// instead of at the top of the layer, so their registers are not live during
// the x and z passes; with it the FP64 ND = 7 (Q6) CG instance is compiled
// for 3 waves / SIMD (LDS admits 3 workgroups per CU).
constexpr bool kF5Late = false;
template <typename T, int ND, int MODE>
constexpr bool f5_late() { return kF5Late && sizeof(T) == 8 && ND == 7 && MODE == 1; }
template <typename T, int ND, int MODE>
constexpr int f5_waves() { return f5_late<T, ND, MODE>() ? 3 : kF5Waves; }
constexpr int f5_pad7(int n) { return n + ((7 - n % 16) + 16) % 16; }

// table layout: M, K, C, C^T as 8 x 8 row-major blocks, then the even-odd
// forms of M and K (4 x 4 blocks at kF5EO + 32 id: E, then O at + 16)
constexpr int kF5Stride = 8;
constexpr int kF5EO = 4 * 64;
constexpr int kF5Tab = kF5EO + 2 * 32;
// Even-odd decomposition of the centrosymmetric M and K (M[i][j] =
// M[nd-1-i][nd-1-j] for the symmetric GLL / Gauss rules; checked on the
// host): out = M in costs ceil(nd/2) x ceil(nd/2) + floor(nd/2)^2 FMAs
// instead of nd^2 (31 instead of 49 at nd = 7) and half the scalar table
// loads.  Used on all three passes in both precisions (FP32 +11 % at Q6,
// FP64 spill-free at 188 VGPRs with the descriptor laundering below).
//
// Register-pressure measures that the production kernel relies on (each an
// A/B on the box, profiles/r2_launder.md):
//  * descriptor laundering: the per-thread gather / staging descriptors are
//    re-materialised every layer through an empty asm, so the compiler cannot
//    hoist their unpacked fields and flag masks out of the x-march (hoisted,
//    they cost ~20 VGPRs and the SGPR masks spill to VGPR lanes);
//  * one laundered table base pointer per matrix row, rows addressed by a
//    constant offset (folded into the scalar load's immediate);
//  * the z pass writes zK back before forming zM (one output row live, not
//    two: Q6 FP64 188 -> 170 VGPRs, +0.9 %);
//  * the prefetch is consumed (LDS staging, p / x stores) before the
//    gather's stores, behind one explicit vmcnt(0) (Q3 +4.1 %, Q6 +1.1 %).
static_assert(kF5Tab <= kFusedTabMax, "fused5 tables exceed the kernarg table");

// cells per wave and (y, z) tile per degree.  Tile shapes: same-box A/Bs of 4x4 vs 4x2 at ND = 4 and 2x2 vs 2x1 at
// ND = 7 kept these (profiles/r2_fused5_evenodd.md).
template <int ND> struct F5Tile;
template <> struct F5Tile<4> { static constexpr int CPW = 4, TY = 4, TZ = 4; };
template <> struct F5Tile<5> { static constexpr int CPW = 2, TY = 2, TZ = 4; };
template <> struct F5Tile<6> { static constexpr int CPW = 1, TY = 2, TZ = 2; };
template <> struct F5Tile<7> { static constexpr int CPW = 1, TY = 2, TZ = 2; };
template <> struct F5Tile<8> { static constexpr int CPW = 1, TY = 2, TZ = 2; };

template <typename T, int ND>
struct F5Shape {
  static constexpr int P = ND - 1;
  static constexpr int CPW = F5Tile<ND>::CPW, TY = F5Tile<ND>::TY, TZ = F5Tile<ND>::TZ;
  static constexpr int CELLS = TY * TZ;
  static_assert(CELLS % CPW == 0, "whole waves of cells");
  static constexpr int WAVES = CELLS / CPW;
  static constexpr int NT = WAVES * 64;
  static constexpr int VW = VecOf<T>::W;
  // line pitch: an odd number of 16-byte slots (conflict-free b128 rows)
  static constexpr int SLOTS = (ND + VW - 1) / VW;
  static constexpr int NDP = (SLOTS % 2 ? SLOTS : SLOTS + 1) * VW;
  static constexpr int ARR = CPW * ND * ND * NDP;  // one array of line rows
  // element vectors for the gather: E[cell][j][k][i]
  static constexpr int RP = ND, P1 = ND * ND, PC = ND * ND * ND;
  static constexpr int WB0 = 2 * ARR;  // arrays 0 (Kx u / zM) and 1 (Mx u / zK)
  static constexpr int WB = WB0 > CPW * PC ? WB0 : CPW * PC;  // per-wave buffer
  static constexpr int DY = TY * P + 1, DZ = TZ * P + 1, PL = DY * DZ;
  static constexpr bool PAD7 = kF5Pad7 && sizeof(T) == 8 && ND == 7;
  static constexpr int DZP = PAD7 ? f5_pad7(DZ) : (DZ | 1);
  static constexpr int PLP = PAD7 ? f5_pad7(DY * DZP) : DY * DZP;
};

// Does a tile row's own part split into whole 16-byte vectors (the VEC instance)?
template <typename T, int ND>
constexpr bool f5_vec_shape() {
  using S = F5Shape<T, ND>;
  constexpr int V = 16 / static_cast<int>(sizeof(T)), OWNZ = S::TZ * S::P;
  return kF5Vec && OWNZ % V == 0 && (OWNZ * static_cast<int>(sizeof(T))) % 16 == 0;
}

// fused5: nodal x / z / y Kronecker passes for parallelepiped cells, P = 3..7.
// (An MFMA form of the three passes lost to this VALU core at Q6 in both
// precisions: profiles/r2_fused5_mfma.md, profiles/r3_mfma.md.)
template <typename T, int ND, int MODE, bool VEC = false>
__global__ void __launch_bounds__((F5Shape<T, ND>::NT), (f5_waves<T, ND, MODE>()))
    lap_fused5_kernel(Fused2Args<T> A, const T* __restrict__ tabd) {
  using S = F5Shape<T, ND>;
  constexpr int P = S::P, CPW = S::CPW, TY = S::TY, TZ = S::TZ;
  constexpr int DY = S::DY, DZ = S::DZ, PL = S::PL, DZP = S::DZP, PLP = S::PLP;
  constexpr int NT = S::NT, ND2 = ND * ND, NDP = S::NDP, ARR = S::ARR, WB = S::WB;
  constexpr int RP = S::RP, P1 = S::P1, PC = S::PC;
  // VEC: the next layer's loads and the staging's p / x stores move 16 bytes
  // per lane -- items of V consecutive z-nodes of a tile row (its OWNZ own
  // nodes) plus one single node (the z-neighbour's first column); the host
  // selects this instance only when every row of a tile is 16-byte aligned
  // (launch_fused5)
  constexpr int V = 16 / static_cast<int>(sizeof(T));
  constexpr int OWNZ = TZ * P;
  static_assert(!VEC || (OWNZ % V == 0 && (OWNZ * static_cast<int>(sizeof(T))) % 16 == 0),
                "VEC: whole 16-byte vectors per tile row");
  constexpr int NIV = OWNZ / V;
  constexpr int NITV = P * DY * NIV, NPI = VEC ? (NITV + NT - 1) / NT : 1;  // vector items
  constexpr int NITS = P * DY, NPS = VEC ? (NITS + NT - 1) / NT : 1;         // single items
  typedef T VT __attribute__((ext_vector_type(V)));
  constexpr int NPF = (P * PL + NT - 1) / NT;
  constexpr int NOUT = (ND * PL + NT - 1) / NT;
  constexpr int NCP = (PL + NT - 1) / NT;
  constexpr int NV = (TY + 1) * (TZ + 1) * 3;
  constexpr int NPV = (NV + NT - 1) / NT;
  constexpr int ZSLOT = S::WAVES * WB;
  static_assert(ZSLOT < 32768, "16-bit LDS source offsets");
  static_assert(PL < (1 << 19), "plane index field");
  static_assert(ND * PLP < (1 << 23), "staging offset field");

  __shared__ __attribute__((aligned(16))) T s_w[ZSLOT + 1];
  __shared__ T s_u[2][ND * PLP + V];  // + dummy slots (VEC padding items)
  __shared__ T s_c[2][PL];
  __shared__ T s_X[2][2 * NV];
  __shared__ double s_red[16];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_w[ZSLOT] = T(0);

  // XCD-aware bijective remap of the block id (cdna_hip_programming.md T1).
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  // work item = (tile of the launch rectangle, x segment); see fused_set_segments
  const int tix = bid % A.rtiles, seg = bid / A.rtiles;
  const int ty = A.ty0 + tix / A.rwz, tz = A.tz0 + tix % A.rwz;
  const int y0 = ty * TY * P, z0 = tz * TZ * P;
  const int Ly = A.Ly, Lz = A.Lz, ld = A.ld;
  const int ncx = A.ncx;
  // own cell layers [sa, cend); the march starts one layer early (redundant)
  // in every segment but the first
  const int sa = seg * A.seglen;
  const int cend = (sa + A.seglen < ncx) ? sa + A.seglen : ncx;
  const int cbeg = sa > 0 ? sa - 1 : 0;
  const bool top_y = (ty == A.nty - 1), top_z = (tz == A.ntz - 1);
  const int ey = (y0 + DY <= Ly) ? DY : Ly - y0;
  const int ez = (z0 + DZ <= Lz) ? DZ : Lz - z0;
  const int oy = top_y ? ey : TY * P;
  const int oz = top_z ? ez : TZ * P;
  // Dirichlet nodes: the staging and the gather carry the identity-row work
  // (y = r at Dirichlet dofs, zero columns) only where a tile holds a y / z
  // boundary node or a layer an x boundary plane; both decisions are
  // workgroup-uniform, so every other tile and layer runs a Dirichlet-free
  // copy of the code, without the per-node branches (their exec-mask
  // bookkeeping cost Q6 FP64 7 %, Q6 FP32 6 %, Q3 3 %: profiles/r5_kernel_ab.md)
  auto in_rng = [](int v, int lo, int n) { return v >= lo && v < lo + n; };
  const bool tile_bc = in_rng(A.bcy_lo, y0, ey) || in_rng(A.bcy_hi, y0, ey) ||
                       in_rng(A.bcz_lo, z0, ez) || in_rng(A.bcz_hi, z0, ez);
  auto xbc_in = [&](int gx0, int n) { return in_rng(A.bcx_lo, gx0, n) || in_rng(A.bcx_hi, gx0, n); };

  // lane roles: (cell of the wave, a, b); pass-dependent meaning of (a, b)
  const bool lane_on = lane < CPW * ND2;
  const int cw = lane_on ? lane / ND2 : 0;
  const int ab = lane_on ? lane % ND2 : 0;
  const int la = ab / ND, lb = ab % ND;
  const int c = wv * CPW + cw;
  const int cy = c / TZ, cz = c % TZ;
  const bool cell_on = lane_on && (ty * TY + cy < A.n1) && (tz * TZ + cz < A.n2);
  T* const Wb = s_w + wv * WB;             // this wave's buffer
  T* const Wc = Wb + cw * ND2 * NDP;       // this cell's rows of array 0

  // lagged x update: x += alpha_prev p_old (kXSingle), nothing but saving
  // alpha_prev (kXSave), or two terms: + alpha_prev2 p_prev2 read from pnew
  // before this iteration overwrites it (kXPair; saves the x read / write of
  // every other iteration, runtime.hip)
  // staggered pairing: the odd tiles run xmode1 (they pair when the even
  // ones save, so every iteration carries half of the x stream)
  T beta = T(0), xalpha = T(0), xalpha2 = T(0);
  const int xm = (A.xmode1 >= 0 && ((ty + tz) & 1)) ? A.xmode1 : A.xmode;
  const bool xupd = MODE == kFusedCG && A.xa_num >= 0 && xm != kXSave;
  const bool xpair = xupd && xm == kXPair;
  if constexpr (MODE == kFusedCG) {
    if (A.beta_num >= 0) beta = static_cast<T>(A.scal[A.beta_num] / A.scal[A.beta_den]);
    if (xupd) xalpha = static_cast<T>(A.scal[A.xa_num] / A.scal[A.xa_den]);
    if (xpair) xalpha2 = static_cast<T>(A.scal[A.xslot_r]);
    // every saving block writes the same value (any block of the saving
    // colour may be the first of a launch rectangle)
    if (xm == kXSave && A.xa_num >= 0 && threadIdx.x == 0 && (A.xmode1 >= 0 || blockIdx.x == 0))
      const_cast<double*>(A.scal)[A.xslot_w] = A.scal[A.xa_num] / A.scal[A.xa_den];
  }
  double pap = 0.0;

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
  // stage one input node of the prologue layer; wr = false (a redundant
  // layer: the previous segment owns these planes) computes the value only
  auto stage = [&](int f, int gx, const T* __restrict__ ul, T* __restrict__ pn, T* __restrict__ yl,
                   int goff, bool wr) -> T {
    T v;
    if (!wr) f &= ~kOwnT;
    if constexpr (MODE == kFusedCG) {
      if (BDX_OOB((ul - A.u) + goff, A.vsize, "stage")) return T(0);
      const T po = A.pold[(ul - A.u) + goff];
      v = ul[goff] + beta * po;
      if (xupd && (f & kOwnT)) {
        T* __restrict__ xl = A.x + (ul - A.u);
        T dx = xalpha * po;
        if (xpair) dx += xalpha2 * pn[goff];  // p_prev2, before p_new replaces it
        xl[goff] += dx;
      }
      if (f & kOwnT) pn[goff] = v;
    } else {
      if (BDX_OOB((ul - A.u) + goff, A.vsize, "stage")) return T(0);
      v = ul[goff];
    }
    (void)pn;
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
  // 32-bit unsigned per-layer offsets: uniform base + zero-extended VGPR
  // offset (SADDR addressing, no 64-bit address VGPRs per element)
  unsigned st_goff[NPF];
  int st_meta[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int e = tid + k * NT;
    st_goff[k] = 0;
    st_meta[k] = 0;
    if (e < P * PL) {
      const int pl = 1 + e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
      const int f = yz_flags(ly, lz);
      st_goff[k] = static_cast<unsigned>(pl * A.ps + fused_yzoff(A, y0 + ly, z0 + lz));
      st_meta[k] = f | (pl << 4) | ((pl * PLP + ly * DZP + lz) << 8);
    }
  }
  // ---- VEC: per-thread staging items (planes 1..P).  Vector item = (plane,
  // tile row ly, iz < NIV): the V own nodes lz = V iz .. V iz + V - 1; single
  // item = (plane, ly): the node lz = OWNZ (the z-neighbour's first column).
  // meta: 4 flag bits per node (kValid, kOwnT, kBcYZ, kRownYZ) at 4 e, the
  // plane at bits 16-19, any node valid at 21, every node owned at 22, any
  // node owned at 23
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
    if (VEC && it < NITS)
      item_desc(1 + it / DY, it % DY, OWNZ, 1, is_goff[k], is_meta[k], is_lds[k]);
  }
  // ---- per-thread output descriptors (planes 0..P of a layer)
  int o_src[NOUT][2], o_off[NOUT], o_meta[NOUT];
  auto ebase = [&](int cc) { return (cc / CPW) * WB + (cc % CPW) * PC; };
#pragma unroll
  for (int k = 0; k < NOUT; ++k) {
    const int e = tid + k * NT;
    o_src[k][0] = o_src[k][1] = ZSLOT | (ZSLOT << 16);
    o_off[k] = 0;
    o_meta[k] = 0;
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
            src[ns++] = ebase(ccy * TZ + ccz) + (ly - ccy * P) * P1 + (lz - ccz * P) * RP + pl;
        o_src[k][0] = src[0] | (src[1] << 16);
        o_src[k][1] = src[2] | (src[3] << 16);
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
        o_off[k] = off;
        o_meta[k] = f | (kind << 4) | (pl << 8) | (rem << 12);
      }
    }
  }
  int cp_lds[NCP];
#pragma unroll
  for (int k = 0; k < NCP; ++k) {
    const int e = tid + k * NT;
    cp_lds[k] = (e < PL) ? (e / DZ) * DZP + e % DZ : -1;
  }
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

  // wave-local LDS exchange between passes (a wave's lanes run in lockstep)
  auto wave_sync = [&]() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
  };
  // 1D matrices (kernarg: wave-uniform scalar loads): id 0 = M, 1 = K, 2 = C
  // The tables (a device copy, see f5_tables_on_device) are read through a
  // constant-address-space pointer that is laundered per matrix row, so the
  // scalar loads stream with the FMAs instead of being hoisted out of the
  // x-march (4 ND^2 doubles would not fit the SGPR file).
  typedef const __attribute__((address_space(4))) T CT;
  CT* const tab0 = (CT*)tabd;
  // One base pointer is laundered per row and the row is addressed by a
  // constant offset (folded into the scalar load's immediate) -- otherwise
  // the compiler hoists every row pointer out of the x-march and the ~40
  // SGPR pairs spill to VGPR lanes (v_readlane per use in the loop).
  CT* tabl = tab0;
  // out[a] (+)= s * sum_b Mat[a][b] in[b]; id 0 = M, 1 = K, 2 = C, 3 = C^T.
  // The base is laundered through an asm that consumes the result of row
  // a - 2 (d2): the scalar loads run one row ahead of the FMAs and at most
  // two rows are live in SGPRs.
  T d1 = T(0), d2 = T(0);
  auto matvec = [&](int id, const T (&in)[ND], T (&out)[ND], T s, bool acc) {
    if (id < 2) {  // M or K: even-odd form (compile-time after inlining)
      constexpr int H = ND / 2, ODD = ND % 2;
      T ev[H], od[H];
#pragma unroll
      for (int b = 0; b < H; ++b) {
        ev[b] = in[b] + in[ND - 1 - b];
        od[b] = in[b] - in[ND - 1 - b];
      }
#pragma unroll
      for (int a = 0; a < H + ODD; ++a) {
        asm volatile("" : "+s"(tabl) : "v"(d2));
        CT* re = tabl + kF5EO + id * 32 + a * 4;
        T te = T(0);
#pragma unroll
        for (int b = 0; b < H; ++b) te += re[b] * ev[b];
        if constexpr (ODD) te += re[H] * in[H];
        if (a < H) {
          CT* ro = tabl + kF5EO + id * 32 + 16 + a * 4;
          T to = T(0);
#pragma unroll
          for (int b = 0; b < H; ++b) to += ro[b] * od[b];
          const T r1 = te + to, r2 = te - to;
          out[a] = acc ? out[a] + s * r1 : s * r1;
          out[ND - 1 - a] = acc ? out[ND - 1 - a] + s * r2 : s * r2;
          d2 = d1;
          d1 = r1;
        } else {
          out[a] = acc ? out[a] + s * te : s * te;
          d2 = d1;
          d1 = te;
        }
      }
      return;
    }
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      asm volatile("" : "+s"(tabl) : "v"(d2));
      CT* row = tabl + id * 64 + a * kF5Stride;
      T t = T(0);
#pragma unroll
      for (int b = 0; b < ND; ++b) t += row[b] * in[b];
      d2 = d1;
      d1 = t;
      out[a] = acc ? out[a] + s * t : s * t;
    }
  };

  const int64_t kc_ps = static_cast<int64_t>(A.n1) * A.n2;
  const int64_t kc_cell = static_cast<int64_t>(ty * TY + cy) * A.n2 + tz * TZ + cz;
  T kc_cur = (A.kc && cell_on) ? A.kc[cbeg * kc_ps + kc_cell] : A.kappa;
  for (int cx = cbeg; cx < cend; ++cx) {
    const int cur = (cx - cbeg) & 1, nxt = cur ^ 1;
    const bool last = (cx == cend - 1);   // end of this segment
    const bool glast = (cx == ncx - 1);   // end of the march
    const bool red = (cx < sa);           // redundant layer: carry only
    __syncthreads();

    // ---- prefetch the next layer (planes 1..P of layer cx+1, vertex plane cx+2)
    constexpr bool LATE = f5_late<T, ND, MODE>();
    const int64_t lnext = static_cast<int64_t>(cx + 1) * P * A.ps;
    const T* __restrict__ un_r = A.u + lnext;
    const T* __restrict__ un_p = A.pold + lnext;
    T* __restrict__ un_x = A.x + lnext;
    const T* un_q = A.pnew + lnext;  // p_prev2 (kXPair), read before the staging store
    T pf_r[VEC ? 1 : NPF], pf_p[VEC ? 1 : NPF], pf_x[VEC ? 1 : NPF], pf_q[VEC ? 1 : NPF];
    VT vf_r[NPI], vf_p[NPI], vf_x[NPI], vf_q[NPI];
    T sf_r[NPS], sf_p[NPS], sf_x[NPS], sf_q[NPS];
    T pf_v[NPV];
    // next layer's cell coefficient rides with the prefetch: a load consumed
    // in the same layer would make the wave wait for the whole batch
    T kc_nxt = kc_cur;
    auto issue_prefetch = [&]() __attribute__((always_inline)) {
    if (A.kc && !last && cell_on) kc_nxt = A.kc[static_cast<int64_t>(cx + 1) * kc_ps + kc_cell];
#pragma unroll
    for (int k = 0; k < NPI; ++k) {
      vf_r[k] = vf_p[k] = vf_x[k] = vf_q[k] = VT{};
      if constexpr (VEC) {
        const int m = it_meta[k];
        if (last || !(m & (1 << 21))) continue;
        vf_r[k] = *reinterpret_cast<const VT*>(un_r + it_goff[k]);
        if constexpr (MODE == kFusedCG) {
          vf_p[k] = *reinterpret_cast<const VT*>(un_p + it_goff[k]);
          // x and p_prev2 are read by this tile only (own nodes): streamed
          // non-temporally, Q3 +2.1 % same box (profiles/r4_fused5_nt_ab.txt)
          if (xupd && (m & (1 << 23)))
            vf_x[k] = __builtin_nontemporal_load(reinterpret_cast<const VT*>(un_x + it_goff[k]));
          if (xpair && (m & (1 << 23)))
            vf_q[k] = __builtin_nontemporal_load(reinterpret_cast<const VT*>(un_q + it_goff[k]));
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NPS; ++k) {
      sf_r[k] = sf_p[k] = sf_x[k] = sf_q[k] = T(0);
      if constexpr (VEC) {
        const int m = is_meta[k];
        if (last || !(m & (1 << 21))) continue;
        sf_r[k] = ld_stream(un_r + is_goff[k]);
        if constexpr (MODE == kFusedCG) {
          sf_p[k] = ld_stream(un_p + is_goff[k]);
          if (xupd && (m & (1 << 23))) sf_x[k] = ld_stream(un_x + is_goff[k]);
          if (xpair && (m & (1 << 23))) sf_q[k] = ld_stream(un_q + is_goff[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < (VEC ? 0 : NPF); ++k) {
      pf_r[k] = T(0);
      pf_p[k] = T(0);
      pf_x[k] = T(0);
      pf_q[k] = T(0);
      if (!last && (st_meta[k] & kValid)) {
        if (BDX_OOB(lnext + st_goff[k], A.vsize, "f5 prefetch")) continue;
        pf_r[k] = ld_stream(un_r + st_goff[k]);
        if constexpr (MODE == kFusedCG) {
          pf_p[k] = ld_stream(un_p + st_goff[k]);
          if (xupd && (st_meta[k] & kOwnT)) pf_x[k] = ld_stream(un_x + st_goff[k]);
          if (xpair && (st_meta[k] & kOwnT)) pf_q[k] = ld_stream(un_q + st_goff[k]);
        }
      }
    }
#pragma unroll
    for (int k = 0; k < NPV; ++k) {
      pf_v[k] = T(0);
      if (!last && v_off[k] >= 0) pf_v[k] = A.xv[static_cast<int64_t>(cx + 2) * A.vps + v_off[k]];
    }
    };
    if constexpr (!LATE) issue_prefetch();

    const T* __restrict__ su = s_u[cur];
    const T* __restrict__ sX = s_X[cur];

    // ------------------------------------------------ geometry (constant J)
    T G00, G01, G02, G11, G12, G22;
    {
      const T* X0 = sX;
      const T* X1 = sX + NV;
      const int v00 = (cy * (TZ + 1) + cz) * 3, v01 = v00 + 3;
      const int v10 = v00 + (TZ + 1) * 3;
      T E[3], F[3], Gv[3];
#pragma unroll
      for (int d = 0; d < 3; ++d) {
        const T X000 = X0[v00 + d];
        E[d] = X1[v00 + d] - X000;
        F[d] = X0[v10 + d] - X000;
        Gv[d] = X0[v01 + d] - X000;
      }
      const T J00 = E[0], J10 = E[1], J20 = E[2];
      const T J01 = F[0], J11 = F[1], J21 = F[2];
      const T J02 = Gv[0], J12 = Gv[1], J22 = Gv[2];
      const T K00 = J11 * J22 - J12 * J21, K01 = J02 * J21 - J01 * J22, K02 = J01 * J12 - J02 * J11;
      const T K10 = J12 * J20 - J10 * J22, K11 = J00 * J22 - J02 * J20, K12 = J02 * J10 - J00 * J12;
      const T K20 = J10 * J21 - J11 * J20, K21 = J01 * J20 - J00 * J21, K22 = J00 * J11 - J01 * J10;
      const T det = J00 * K00 + J01 * K10 + J02 * K20;
      const T sc = cell_on ? kc_cur * fast_rcp(det) : T(0);
      G00 = sc * (K00 * K00 + K01 * K01 + K02 * K02);
      G01 = sc * (K00 * K10 + K01 * K11 + K02 * K12);
      G02 = sc * (K00 * K20 + K01 * K21 + K02 * K22);
      G11 = sc * (K10 * K10 + K11 * K11 + K12 * K12);
      G12 = sc * (K10 * K20 + K11 * K21 + K12 * K22);
      G22 = sc * (K20 * K20 + K21 * K21 + K22 * K22);
    }
    (void)G01;
    (void)G02;
    (void)G12;

    const T* __restrict__ ucell = su + (cy * P) * DZP + cz * P;
    // ------------------------------------------------ x pass: lane (j, k) = (la, lb)
    {
      T u[ND];
#pragma unroll
      for (int l = 0; l < ND; ++l) u[l] = ucell[l * PLP + la * DZP + lb];
      T o[ND];
      // array 0: Kx u, array 1: Mx u; rows [i][j][k]
      auto put = [&](int arr) {
        T* w = Wc + arr * ARR + la * NDP + lb;
        if (lane_on) {
#pragma unroll
          for (int i = 0; i < ND; ++i) w[i * ND * NDP] = o[i];
        }
      };
      matvec(1, u, o, T(1), false);
      put(0);
      matvec(0, u, o, T(1), false);
      put(1);
    }
    wave_sync();

    // ------------------------------------------------ z pass: lane (i, j) = (la, lb)
    {
      // both input rows of every lane are in registers once the loads have
      // returned (one ds_read per row for the whole wave), so zK can be
      // written back before zM is formed: one output row live, not two
      const T* r = Wc + ab * NDP;
      T ak[ND], am[ND];
      ldrow<ND>(r, ak);
      ldrow<ND>(r + ARR, am);
      T* w = Wc + la * ND * NDP + lb;
      {
        T zK[ND];
        matvec(0, am, zK, G11, false);
        wave_sync();
        if (lane_on) {
#pragma unroll
          for (int k = 0; k < ND; ++k) w[ARR + k * NDP] = zK[k];
        }
      }
      T zM[ND];
      matvec(0, ak, zM, G00, false);
      matvec(1, am, zM, G22, true);
      if (lane_on) {
#pragma unroll
        for (int k = 0; k < ND; ++k) w[k * NDP] = zM[k];
      }
      wave_sync();
    }

    if constexpr (LATE) issue_prefetch();

    // ------------------------------------------------ y pass: lane (i, k) = (la, lb)
    T ye[ND];
    {
      const T* r = Wc + ab * NDP;
      T sM[ND], sK[ND];
      ldrow<ND>(r, sM);
      ldrow<ND>(r + ARR, sK);
      matvec(0, sM, ye, T(1), false);
      matvec(1, sK, ye, T(1), true);
    }
    // element dot p_e . (A_e p_e): lane holds y_e[i = la][j][k = lb]
    if constexpr (MODE == kFusedCG) {
      if (cell_on && !red) {
#pragma unroll
        for (int j = 0; j < ND; ++j)
          pap += static_cast<double>(ucell[la * PLP + j * DZP + lb]) * static_cast<double>(ye[j]);
      }
    }
    wave_sync();
    if (lane_on) {
      T* eo = Wb + cw * PC + lb * RP + la;
#pragma unroll
      for (int j = 0; j < ND; ++j) eo[j * P1] = cell_on ? ye[j] : T(0);
    }
    __syncthreads();

    auto do_gather = [&](auto DIRC) __attribute__((always_inline)) {
      constexpr bool DIR = decltype(DIRC)::value;
      // ------------------------------------------------ gather-sum and write out
      {
  #pragma unroll
        for (int k = 0; k < NOUT; ++k)  // descriptor laundering (see the file head)
          asm volatile("" : "+v"(o_src[k][0]), "+v"(o_src[k][1]), "+v"(o_off[k]), "+v"(o_meta[k]));
        const int64_t lbase = static_cast<int64_t>(cx) * P;
        T* __restrict__ ybase[4] = {A.y + lbase * A.ps, A.yb + lbase * A.ybps,
                                    A.zb + lbase * A.zbps, A.cb + lbase * A.cbps};
  #pragma unroll
        for (int k = 0; k < NOUT; ++k) {
          const int m = o_meta[k];
          if (!(m & kValid)) continue;
          const int pl = (m >> 8) & 15, rem = m >> 12;
          BDX_DASSERT((o_src[k][0] & 0xffff) <= ZSLOT && (o_src[k][0] >> 16) <= ZSLOT &&
                      (o_src[k][1] & 0xffff) <= ZSLOT && (o_src[k][1] >> 16) <= ZSLOT && rem < PL);
          T v = s_w[o_src[k][0] & 0xffff] + s_w[o_src[k][0] >> 16] +
                s_w[o_src[k][1] & 0xffff] + s_w[o_src[k][1] >> 16];
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
                          o_off[k], kind == 0 ? A.vsize : A.ibsize, "f5 gather store"))
            continue;
          if (kind == 0)
            st_stream(ybase[0] + o_off[k], v);
          else
            (kind == 1 ? ybase[1] : kind == 2 ? ybase[2] : ybase[3])[o_off[k]] = v;
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
            VT xn = vf_x[k] + xalpha * vf_p[k];
            if (xpair) xn += xalpha2 * vf_q[k];
            if (m & (1 << 22)) {  // every node owned: whole vectors
              // non-temporal: whole 16-byte vectors of contiguous tile rows,
              // not read again before the next iteration (Q3 +1.5 %, Q6 FP32
              // +2.1 % same box, profiles/r4_fused5_nt_ab.txt)
              __builtin_nontemporal_store(val, reinterpret_cast<VT*>(pnl + it_goff[k]));
              if (xupd) __builtin_nontemporal_store(xn, reinterpret_cast<VT*>(un_x + it_goff[k]));
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
              if (xupd) {
                T xn = sf_x[k] + xalpha * sf_p[k];
                if (xpair) xn += xalpha2 * sf_q[k];
                un_x[is_goff[k]] = xn;
              }
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
            bool m_skip = false;
            T v = T(0);
            if ((m & kValid) && BDX_OOB(lnext + st_goff[k], A.vsize, "f5 staging store")) m_skip = true;
            if ((m & kValid) && !m_skip) {
              const int gxx = (cx + 1) * P + ((m >> 4) & 15);
              T val;
              if constexpr (MODE == kFusedCG) {
                val = pf_r[k] + beta * pf_p[k];
              } else {
                val = pf_r[k];
              }
              if constexpr (MODE == kFusedCG) {
                if (m & kOwnT) {
                  st_stream(pnl + st_goff[k], val);
                  if (xupd) {
                    T xn = pf_x[k] + xalpha * pf_p[k];
                    if (xpair) xn += xalpha2 * pf_q[k];
                    st_stream(un_x + st_goff[k], xn);
                  }
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
            BDX_DASSERT((m >> 8) >= 0 && (m >> 8) < ND * PLP);
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
    // Consume the prefetch (wait for the loads) before the gather issues its
    // stores, so the wait does not drain them: one explicit, unconditional
    // vmcnt(0) (gfx9 encoding; expcnt and lgkmcnt untouched).  The prefetch
    // has landed and no store of this layer is pending yet, so the waitcnt
    // pass sees nothing outstanding and does not put a draining wait before
    // each slot's stores.
    __builtin_amdgcn_s_waitcnt(0x0F70);
    // staging: planes 1..P of layer cx + 1; gather: planes 0..P of layer cx.
    // Q3 (ND = 4) keeps the single Dirichlet-aware copy: the split measured
    // 1.4 % slower there (profiles/r5_kernel_ab.md)
    constexpr bool SPLIT = ND >= 6 || sizeof(T) == 4;
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

// 1D matrices of the quadrature rule (host, double, cast to T): M = B^T W B,
// K = Dd^T W Dd, C = Dd^T W B with B = phi0 (nq x nd), Dd = dphi1 phi0.
template <typename T>
inline int pack_tables5(int nd, int nq, const double* phi0, const double* Dd, const double* wts,
                        T* out) {
  if (nd < 2 || nd > kF5Stride || nq < 1 || nq > kMaxNq) return -1;
  if (!out) return kFusedTabMax;
  for (int i = 0; i < kFusedTabMax; ++i) out[i] = T(0);
  for (int i = 0; i < nd; ++i)
    for (int l = 0; l < nd; ++l) {
      double m = 0, k = 0, c = 0;
      for (int q = 0; q < nq; ++q) {
        m += wts[q] * phi0[q * nd + i] * phi0[q * nd + l];
        k += wts[q] * Dd[q * nd + i] * Dd[q * nd + l];
        c += wts[q] * Dd[q * nd + i] * phi0[q * nd + l];
      }
      out[i * kF5Stride + l] = static_cast<T>(m);
      out[64 + i * kF5Stride + l] = static_cast<T>(k);
      out[128 + i * kF5Stride + l] = static_cast<T>(c);
      out[192 + l * kF5Stride + i] = static_cast<T>(c);
    }
  // even-odd forms of M and K (computed in double from the double matrices)
  for (int id = 0; id < 2; ++id) {
    double Mx[kF5Stride][kF5Stride];
    double mx = 0.0;
    for (int i = 0; i < nd; ++i)
      for (int l = 0; l < nd; ++l) {
        double v = 0;
        for (int q = 0; q < nq; ++q)
          v += id == 0 ? wts[q] * phi0[q * nd + i] * phi0[q * nd + l]
                       : wts[q] * Dd[q * nd + i] * Dd[q * nd + l];
        Mx[i][l] = v;
        mx = std::fabs(v) > mx ? std::fabs(v) : mx;
      }
    for (int i = 0; i < nd; ++i)  // centrosymmetry (symmetric rules): else refuse
      for (int l = 0; l < nd; ++l)
        if (std::fabs(Mx[i][l] - Mx[nd - 1 - i][nd - 1 - l]) > 1e-12 * mx) return -2;
    const int h = nd / 2, odd = nd % 2;
    T* E = out + kF5EO + id * 32;
    T* O = E + 16;
    for (int a = 0; a < h + odd; ++a) {
      for (int b = 0; b < h; ++b) {
        E[a * 4 + b] = static_cast<T>(0.5 * (Mx[a][b] + Mx[a][nd - 1 - b]));
        if (a < h) O[a * 4 + b] = static_cast<T>(0.5 * (Mx[a][b] - Mx[a][nd - 1 - b]));
      }
      if (odd) E[a * 4 + h] = static_cast<T>(Mx[a][h]);
    }
  }
  return kFusedTabMax;
}

// affine_ok: 2 = axis-aligned boxes (diagonal Jacobians); anything else is
// refused (general parallelepipeds run fused3's affine instance)
// Can the VEC instance run on this launch?  Every tile row's own nodes must
// start on a 16-byte boundary: the tiled storage's tiles are the kernel's
// (y, z) tiles, or the lattice rows are padded to whole vectors, and the
// vectors themselves are 16-byte aligned.
template <typename T, int ND>
bool f5_vec_ok(const Fused2Args<T>& a) {
  using S = F5Shape<T, ND>;
  constexpr int V = 16 / static_cast<int>(sizeof(T)), OWNZ = S::TZ * S::P;
  if (OWNZ % V || (OWNZ * static_cast<int>(sizeof(T))) % 16) return false;
  // lattice layout: the padded row pitch holds every tile's vectors (the top
  // tile's run past the domain but not past the row)
  const bool lay = a.tsy ? (a.tsy == S::TY * S::P && a.tsz == OWNZ)
                         : (a.ld % V == 0 && a.ps % V == 0 && static_cast<int64_t>(a.ntz) * OWNZ <= a.ld);
  auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  return lay && al(a.u) && al(a.pold) && al(a.pnew) && al(a.x);
}

template <typename T, int ND, int MODE>
int launch_fused5(int affine_ok, const Fused2Args<T>& a, const T* tabd, hipStream_t st) {
  if (affine_ok != 2) return static_cast<int>(hipErrorInvalidValue);
  const int nblk = a.nblk;
  if (nblk <= 0) return 0;
  if constexpr (MODE == kFusedCG && f5_vec_shape<T, ND>()) {
    if (f5_vec_ok<T, ND>(a)) {
      lap_fused5_kernel<T, ND, MODE, true><<<nblk, F5Shape<T, ND>::NT, 0, st>>>(a, tabd);
      return static_cast<int>(hipGetLastError());
    }
  }
  lap_fused5_kernel<T, ND, MODE><<<nblk, F5Shape<T, ND>::NT, 0, st>>>(a, tabd);
  return static_cast<int>(hipGetLastError());
}

#define BDX_FUSED5_TU(T, SUF, PP)                                                   \
  extern "C" int bdx_fused5_apply_##SUF##_p##PP(                                   \
      int mode, int affine_ok, const int64_t* latd, int nq, const double* wts,     \
      const double* qpts, const T* u, const T* pold, T* pnew, T* x, T* y, T* yb,   \
      T* zb, T* cb, const T* xv, const T* kc, const T* tabs, double kappa,         \
      const double* scal, double* partials, int beta_num, int beta_den,            \
      int xa_num, int xa_den, int nty, int ntz, const int* rect, hipStream_t st) {                  \
    (void)wts;                                                                     \
    (void)qpts;                                                                    \
    (void)nq;                                                                      \
    if (!affine_ok || !tabs) return static_cast<int>(hipErrorInvalidValue);        \
    Fused2Args<T> a;                                                               \
    BDX_CHECK(static_cast<hipError_t>(make_fused2_args(a, latd, nty, ntz)));  \
    BDX_CHECK(static_cast<hipError_t>(fused_set_rect(a, rect)));       \
    BDX_CHECK(static_cast<hipError_t>(fused_set_segments(a, (mode >> 8) & 0xff))); \
    a.xmode = (mode >> 4) & 3;                                                     \
    a.xmode1 = ((mode >> 6) & 3) - 1;                                              \
    a.xslot_w = kScalXSave + ((mode >> 16) & 1);                                   \
    a.xslot_r = kScalXSave + ((mode >> 17) & 1);                                   \
    mode &= 0xf;                                                                   \
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
    const T* tabd = tabs; /* device pointer: the operator's own table buffer */   \
    return mode == kFusedCG ? launch_fused5<T, PP + 1, kFusedCG>(affine_ok, a, tabd, st) \
                            : launch_fused5<T, PP + 1, kFusedAction>(affine_ok, a, tabd, st); \
  }                                                                                \
  extern "C" int bdx_fused5_tables_##SUF##_p##PP(int nd, int nq, const double* phi0, \
                                                  const double* Dd, const double* wts, \
                                                  T* out) {                        \
    return pack_tables5<T>(nd, nq, phi0, Dd, wts, out);                            \
  }                                                                                \
  extern "C" int bdx_fused5_segments_##SUF##_p##PP(int affine_ok, int tiles, int ncx) { \
    int per_cu = 0, dev = 0, cus = 0;                                              \
    hipError_t e = hipGetDevice(&dev);                                             \
    if (e == hipSuccess)                                                           \
      e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev); \
    if (affine_ok != 2) return 1;                                                  \
    if (e == hipSuccess)                                                           \
      e = hipOccupancyMaxActiveBlocksPerMultiprocessor(                            \
          &per_cu, lap_fused5_kernel<T, PP + 1, kFusedCG, f5_vec_shape<T, PP + 1>()>, \
          F5Shape<T, PP + 1>::NT, 0);                                              \
    return e == hipSuccess ? fused_choose_segments(tiles, ncx, per_cu * cus) : 1;  \
  }                                                                                \
  extern "C" int bdx_fused5_tile_p##PP##_##SUF(int affine_ok, int* ty, int* tz) {  \
    (void)affine_ok;                                                               \
    *ty = F5Tile<PP + 1>::TY;                                                      \
    *tz = F5Tile<PP + 1>::TZ;                                                      \
    return 0;                                                                      \
  }
