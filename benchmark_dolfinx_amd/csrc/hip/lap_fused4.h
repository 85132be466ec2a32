// Fused structured operator kernel, v4 ("fused4"): the y/z sum factorisation
// of an affine Q3 cell layer as an MFMA GEMM (v_mfma_f64_16x16x4_f64).
//
// For a parallelepiped cell the geometry factor G = kappa adj(J) adj(J)^T /
// det J is constant, so the quadrature sum of the reference stiffness
// operator (src/laplacian_gpu.hpp:91-426 with src/geometry_gpu.hpp:26-132)
// factorises exactly into 1D matrices of the same quadrature rule,
//   M1 = B^T W B,  K1 = Dd^T W Dd,  C1 = Dd^T W B     (B = phi0, Dd = dphi1 phi0),
// and the element operator is a sum of 8 Kronecker blocks (x (X) y (X) z):
//   G00 K.M.M + G11 M.K.M + G22 M.M.K + G12 M.(C.Ct + Ct.C)
//   + G01 (C.Ct.M + Ct.C.M) + G02 (C.M.Ct + Ct.M.C).
// With ND = 4 the (y, z) factor of a block is one 16 x 16 matrix, so per
// wave of 4 cells the operator is
//   Y[(j',k')][(i,cell)] = sum_t (Y_t (X) Z_t)[(j',k')][(j,k)] * G_t(cell) V_t[(j,k)][(i,cell)],
//   V_t = X_t along x (a 4x4 register contraction per lane),
// i.e. a 16 x 128 x 16 GEMM = 32 MFMAs with a constant A operand (LDS) and
// the B operand formed in registers: no LDS round trips between contraction
// stages, no quadrature-point arrays, two workgroup barriers per layer.
// MFMA f64 16x16x4 lane maps (cdna_hip_programming.md §3): A[m][k] at lane
// m + 16k, B[k][n] at lane n + 16k, D[m][n] at lane n + 16(m % 4), reg m / 4.
//
// Everything around the core -- the x-march over (y, z) tiles, the double
// buffered slab staging with the CG fusion (p = r + beta p_old, lagged x
// update, Dirichlet identity rows, p.Ap partials) and the atomic-free gather
// with tile-interface buffers -- is fused3's (lap_fused3.h).
#pragma once
#include <cstdlib>

#include "lap_fused2.h"

// Fixed design choices (same-box A/Bs in profiles/r1_kernel_ab.md,
// r2_launder.md, r2_fused4_attribution.md):
//  * 4 x 4 cell tile, 3 waves/SIMD (LDS-limited to 3 workgroups per CU);
//  * the per-lane x-factor rows and the gather-source descriptors (4 packed
//    LDS offsets per output slot) live in LDS, not registers (32 + 16 VGPRs);
//  * no descriptor laundering (it removes 111 v_readlane and 19 VGPRs, but
//    the kernel is LDS-limited and the A/B was neutral, 52.3 vs 52.6 GDoF/s).

constexpr int kF4TY = 4, kF4TZ = 4;  // cell tile

// kernarg table layout: M1, K1, C1 (4 x 4 row-major each)
constexpr int kF4Tab = 48;

// The 8 Kronecker blocks: (x factor, y factor, z factor) as matrix ids
// 0 = M1, 1 = K1, 2 = C1, 3 = C1^T; block 3's (y, z) factor is the sum
// C.Ct + Ct.C.
__host__ __device__ constexpr int f4_blk_y(int t) {
  return t == 0 ? 0 : t == 1 ? 1 : t == 2 ? 0 : t == 3 ? 2 : t == 4 ? 3 : t == 5 ? 2 : 0;
}
__host__ __device__ constexpr int f4_blk_z(int t) {
  return t == 0 ? 0 : t == 1 ? 0 : t == 2 ? 1 : t == 3 ? 3 : t == 4 ? 0 : t == 5 ? 0 : t == 6 ? 3 : 2;
}

__device__ __forceinline__ double f4_mat(const double* tab, int id, int r, int c) {
  return id == 3 ? tab[32 + c * 4 + r] : tab[id * 16 + r * 4 + c];
}

// fused4: MFMA (y, z) Kronecker core on parallelepiped Q3 cells, x-marching CG fusion.
template <int TY, int TZ, int MODE>
__global__ void __launch_bounds__(TY * TZ * 16, 3)
    lap_fused4_kernel(Fused2Args<double> A, FusedTables<double> tb) {
  using T = double;
  constexpr int ND = 4, P = 3;
  constexpr int DY = TY * P + 1, DZ = TZ * P + 1, PL = DY * DZ;
  constexpr int DZP = DZ | 1, PLP = DY * DZP;
  constexpr int CELLS = TY * TZ;
  static_assert(CELLS % 4 == 0, "4 cells per wave");
  constexpr int NT = CELLS * 16;
  constexpr int NPF = (P * PL + NT - 1) / NT;
  constexpr int NOUT = (ND * PL + NT - 1) / NT;
  constexpr int NCP = (PL + NT - 1) / NT;
  constexpr int NV = (TY + 1) * (TZ + 1) * 3;
  constexpr int NPV = (NV + NT - 1) / NT;
  // element-vector scratch [cell][j][k][i]; pitches from an exhaustive search
  // of the gather reads + element-vector writes with the gfx950 bank model
  // (b64: 2 x 32 lanes, 64 banks; scripts/lds_bank_f4.py): 135 LDS cycles per
  // workgroup layer vs 257 for the earlier odd pitches (5, 21, 85), ideal 112; the
  // same-box A/B is neutral (38.50 vs 38.47 GDoF/s): LDS is not the limiter
  constexpr int RP = 4, P1 = 17, PC = 72;
  constexpr int EB = CELLS * PC;
  constexpr int ZSLOT = EB;
  static_assert(ZSLOT < 32768, "16-bit LDS source offsets");
  static_assert(PL < 4096, "12-bit plane index");
  constexpr int NCH = 32;  // MFMA K chunks (8 blocks x 4)

  __shared__ __attribute__((aligned(16))) T s_A[NCH * 64];  // [chunk/2][lane][2]
  __shared__ T s_u[2][ND * PLP];
  __shared__ T s_c[2][PL];
  __shared__ T s_e[EB + 1];
  __shared__ T s_X[2][2 * NV];
  __shared__ T s_kc[2][CELLS];  // per-cell coefficient, double buffered
  __shared__ __attribute__((aligned(16))) T s_Xr[4 * 4 * ND];  // [m][xi][l]
  __shared__ __attribute__((aligned(8))) int s_osrc[NOUT][NT][2];
  __shared__ double s_red[16];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const double* tab = tb.tab;
  // ---- constant A operand of every chunk, lane-major pairs for b128 reads
  if (tid < 64) {
    const int jp = (lane & 15) >> 2, kp = lane & 3, kk = lane >> 4;
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int t = ch >> 2, cc = ch & 3;
      T v = f4_mat(tab, f4_blk_y(t), jp, cc) * f4_mat(tab, f4_blk_z(t), kp, kk);
      if (t == 3) v += f4_mat(tab, 3, jp, cc) * f4_mat(tab, 2, kp, kk);
      s_A[((ch >> 1) * 64 + lane) * 2 + (ch & 1)] = v;
    }
  }
  if (tid == 0) s_e[ZSLOT] = T(0);

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

  // MFMA lane roles: g = k (input z dof) = output row group, n = (i, cell)
  const int g = lane >> 4, n = lane & 15, xi = n & 3, cs = n >> 2;
  const int c = 4 * wv + cs;
  const int cy = c / TZ, cz = c % TZ;
  const bool cell_on = (ty * TY + cy < A.n1) && (tz * TZ + cz < A.n2);
  // this lane's rows X[xi][.] of the four x factors
  if (tid < 64) s_Xr[tid] = f4_mat(tab, tid >> 4, (tid >> 2) & 3, tid & 3);
  const T* __restrict__ XrL = s_Xr + xi * ND;

  T beta = T(0), xalpha = T(0);
  const bool xupd = MODE == kFusedCG && A.xa_num >= 0;
  if constexpr (MODE == kFusedCG) {
    if (A.beta_num >= 0) beta = static_cast<T>(A.scal[A.beta_num] / A.scal[A.beta_den]);
    if (xupd) xalpha = static_cast<T>(A.scal[A.xa_num] / A.scal[A.xa_den]);
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
        xl[goff] += xalpha * po;
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
  int st_goff[NPF], st_meta[NPF];
#pragma unroll
  for (int k = 0; k < NPF; ++k) {
    const int e = tid + k * NT;
    st_goff[k] = 0;
    st_meta[k] = 0;
    if (e < P * PL) {
      const int pl = 1 + e / PL, rem = e % PL, ly = rem / DZ, lz = rem % DZ;
      const int f = yz_flags(ly, lz);
      // invalid (off-lattice) slots keep offset 0: the prefetch loads them
      // unconditionally (in bounds, value unused)
      if (f & kValid) st_goff[k] = static_cast<int>(pl * A.ps + fused_yzoff(A, y0 + ly, z0 + lz));
      st_meta[k] = f | (pl << 4) | ((pl * PLP + ly * DZP + lz) << 8);
    }
  }
  // ---- per-thread output descriptors (planes 0..P of a layer)
  int(*o_src)[NT][2] = s_osrc;
  int o_off[NOUT], o_meta[NOUT];
#pragma unroll
  for (int k = 0; k < NOUT; ++k) {
    const int e = tid + k * NT;
    o_src[k][tid][0] = o_src[k][tid][1] = ZSLOT | (ZSLOT << 16);
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
            src[ns++] = (ccy * TZ + ccz) * PC + (ly - ccy * P) * P1 + (lz - ccz * P) * RP + pl;
        o_src[k][tid][0] = src[0] | (src[1] << 16);
        o_src[k][tid][1] = src[2] | (src[3] << 16);
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
          off = static_cast<int>(pl * A.zbps) + gy * (A.ntz - 1) + tz;
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

  const T* __restrict__ s_Al = s_A + lane * 2;

  const int64_t kc_ps = static_cast<int64_t>(A.n1) * A.n2;
  const int64_t kc_cell = static_cast<int64_t>(ty * TY + cy) * A.n2 + tz * TZ + cz;
  if (A.kc) s_kc[0][c] = cell_on ? A.kc[cbeg * kc_ps + kc_cell] : T(0);  // read after the loop-top barrier
  // Everything loaded so far (the per-lane x matrices Xr, the prologue
  // layer) has landed before the march starts: without this explicit wait the
  // waitcnt pass carries the Xr loads as pending around the loop and makes
  // their uses inside the MFMA core wait for each layer's prefetch batch.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  // Prefetch of layer cx + 1 (its planes 1..P, vertex plane cx + 2 and cell
  // coefficient) into one register set (a second set, two layers ahead,
  // measured 1.2-1.5 % slower: it costs occupancy headroom).  Every load is
  // issued unconditionally (past the segment it re-reads layer 0, unused).
  struct PF {
    T r[NPF], p[NPF], x[NPF];
    T v[NPV];
    T kc;
  };
  const T* __restrict__ kcp = A.kc ? A.kc : A.xv;
  auto issue = [&](PF& f, int cl) __attribute__((always_inline)) {
    const bool in = cl < cend;
    const int64_t lpf = in ? static_cast<int64_t>(cl) * P * A.ps : 0;
#pragma unroll
    for (int k = 0; k < NPF; ++k) {
      f.r[k] = T(0);
      f.p[k] = T(0);
      f.x[k] = T(0);
      if (BDX_OOB(lpf + st_goff[k], A.vsize, "f4 prefetch")) continue;
      f.r[k] = ld_stream(A.u + lpf + st_goff[k]);
      if constexpr (MODE == kFusedCG) {
        f.p[k] = ld_stream(A.pold + lpf + st_goff[k]);
        f.x[k] = ld_stream(A.x + lpf + st_goff[k]);
      }
    }
    const int64_t lv = (in && cl + 1 <= ncx) ? static_cast<int64_t>(cl + 1) * A.vps : 0;
#pragma unroll
    for (int k = 0; k < NPV; ++k) f.v[k] = A.xv[lv + (v_off[k] >= 0 ? v_off[k] : 0)];
    f.kc = kcp[(A.kc && in) ? static_cast<int64_t>(cl) * kc_ps + kc_cell : 0];
  };
  auto layer = [&](int cx, PF& pfc) __attribute__((always_inline)) {
    const int cur = (cx - cbeg) & 1, nxt = cur ^ 1;
    const bool last = (cx == cend - 1);   // end of this segment
    const bool glast = (cx == ncx - 1);   // end of the march
    const bool red = (cx < sa);           // redundant layer: carry only
    __syncthreads();

    // ---- prefetch: layer cx+1 into pfc (used at the end of this layer)
    const int64_t lnext = static_cast<int64_t>(cx + 1) * P * A.ps;
    issue(pfc, cx + 1);
    T(&pf_r)[NPF] = pfc.r;
    T(&pf_p)[NPF] = pfc.p;
    T(&pf_x)[NPF] = pfc.x;
    T(&pf_v)[NPV] = pfc.v;

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
      const T kcell = A.kc ? s_kc[cur][c] : A.kappa;
      const T sc = cell_on ? kcell * fast_rcp(det) : T(0);
      G00 = sc * (K00 * K00 + K01 * K01 + K02 * K02);
      G01 = sc * (K00 * K10 + K01 * K11 + K02 * K12);
      G02 = sc * (K00 * K20 + K01 * K21 + K02 * K22);
      G11 = sc * (K10 * K10 + K11 * K11 + K12 * K12);
      G12 = sc * (K10 * K20 + K11 * K21 + K12 * K22);
      G22 = sc * (K20 * K20 + K21 * K21 + K22 * K22);
    }

    // ------------------------------------------------ MFMA core
    // lane (g, xi, cs): u[cell][l][j][k = g] for all (l, j)
    const T* __restrict__ ub = su + (cy * P) * DZP + cz * P + g;
    T uu[ND][ND];
#pragma unroll
    for (int l = 0; l < ND; ++l)
#pragma unroll
      for (int j = 0; j < ND; ++j) uu[l][j] = ub[l * PLP + j * DZP];
    bdx_f64x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    auto block = [&](int t, const T (&V)[ND], T gt) {
      const bdx_f64x2 a01 = *reinterpret_cast<const bdx_f64x2*>(s_Al + (2 * t) * 128);
      const bdx_f64x2 a23 = *reinterpret_cast<const bdx_f64x2*>(s_Al + (2 * t + 1) * 128);
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a01[0], gt * V[0], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a01[1], gt * V[1], acc1, 0, 0, 0);
      acc0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a23[0], gt * V[2], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a23[1], gt * V[3], acc1, 0, 0, 0);
    };
    auto xcontract = [&](int m, T (&V)[ND]) {
      const bdx_f64x2 x01 = *reinterpret_cast<const bdx_f64x2*>(XrL + m * 16);
      const bdx_f64x2 x23 = *reinterpret_cast<const bdx_f64x2*>(XrL + m * 16 + 2);
      const T xr[ND] = {x01[0], x01[1], x23[0], x23[1]};
#pragma unroll
      for (int j = 0; j < ND; ++j) {
        T s = T(0);
#pragma unroll
        for (int l = 0; l < ND; ++l) s += xr[l] * uu[l][j];
        V[j] = s;
      }
    };
    {
      // Cells whose Jacobian is diagonal (axis-aligned boxes) have
      // G01 = G02 = G12 = 0 exactly; when that holds for every cell of the
      // wave the five mixed blocks contribute exact zeros to the MFMA
      // accumulators and are skipped (wave-uniform branch, bit-identical
      // result).
      const bool mixed = __any((G01 != T(0)) || (G02 != T(0)) || (G12 != T(0)));
      T V[ND];
      xcontract(1, V);  // K1 along x
      block(0, V, G00);
      if (mixed) {
        xcontract(2, V);  // C1
        block(4, V, G01);
        block(6, V, G02);
        xcontract(3, V);  // C1^T
        block(5, V, G01);
        block(7, V, G02);
      }
      xcontract(0, V);  // M1
      block(1, V, G11);
      block(2, V, G22);
      if (mixed) block(3, V, G12);
    }
    const bdx_f64x4 ye = acc0 + acc1;
    // lane holds y_e[cell][x = xi][y = r][z = g], r = 0..3
    if constexpr (MODE == kFusedCG) {
      if (cell_on && !red) {
#pragma unroll
        for (int r = 0; r < ND; ++r)
          pap += static_cast<double>(ub[xi * PLP + r * DZP]) * static_cast<double>(ye[r]);
      }
    }
    {
      T* __restrict__ eo = s_e + c * PC + g * RP + xi;
#pragma unroll
      for (int r = 0; r < ND; ++r) eo[r * P1] = cell_on ? ye[r] : T(0);
    }
    __syncthreads();

    // ------------------------------------------------ stage the next layer (LDS)
    // The prefetched values go to LDS before any global store of this layer
    // is issued: vmcnt retires in order, so the wait for the prefetch batch
    // never includes a store, and the stores below (gather, then the staging
    // writes) drain while the next layer computes.  The wait is explicit and
    // unconditional (vmcnt(0) only; gfx9 encoding) so the waitcnt pass sees
    // no prefetch register pending on any path after this point.
    __builtin_amdgcn_s_waitcnt(0x0F70);  // pfc landed
    if (!last) {
      T* __restrict__ un = s_u[nxt];
#pragma unroll
      for (int k = 0; k < NCP; ++k)
        if (cp_lds[k] >= 0) un[cp_lds[k]] = su[P * PLP + cp_lds[k]];
      // branch-free: every prefetch register is rewritten here by a VALU op,
      // so no later store can find one of them still pending (the waitcnt
      // pass is conservative across branches)
#pragma unroll
      for (int k = 0; k < NPF; ++k) {
        const int m = st_meta[k];
        const int gxx = (cx + 1) * P + ((m >> 4) & 15);
        T val;
        if constexpr (MODE == kFusedCG) {
          val = pf_r[k] + beta * pf_p[k];
          pf_x[k] += xalpha * pf_p[k];
        } else {
          val = pf_r[k];
        }
        pf_r[k] = val;  // p (CG) / u (action) of the node: stored below
        const bool bcn = (m & kBcYZ) || gxx == A.bcx_hi;
        if constexpr (MODE == kFusedCG) {
          const bool rown = (m & kValid) && (m & kOwnT) && (m & kRownYZ) && gxx < A.ownx;
          pap += (bcn && rown) ? static_cast<double>(val) * static_cast<double>(val) : 0.0;
        }
        const T v = ((m & kValid) && !bcn) ? val : T(0);
        BDX_DASSERT(tid + k * NT >= P * PL || ((m >> 8) >= 0 && (m >> 8) < ND * PLP));
        if (tid + k * NT < P * PL) un[m >> 8] = v;
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
      if (A.kc) s_kc[nxt][c] = cell_on ? pfc.kc : T(0);  // (the batch has landed here)
    }

    // ------------------------------------------------ gather-sum and write out
    {
      const int64_t lbase = static_cast<int64_t>(cx) * P;
      T* __restrict__ ybase[4] = {A.y + lbase * A.ps, A.yb + lbase * A.ybps,
                                  A.zb + lbase * A.zbps, A.cb + lbase * A.cbps};
#pragma unroll
      for (int k = 0; k < NOUT; ++k) {
        const int m = o_meta[k];
        if (!(m & kValid)) continue;
        const int pl = (m >> 8) & 15, rem = m >> 12;
        const int os0 = o_src[k][tid][0], os1 = o_src[k][tid][1];
        BDX_DASSERT((os0 & 0xffff) <= ZSLOT && (os0 >> 16) <= ZSLOT && (os1 & 0xffff) <= ZSLOT &&
                    (os1 >> 16) <= ZSLOT && rem < PL);
        T v = s_e[os0 & 0xffff] + s_e[os0 >> 16] + s_e[os1 & 0xffff] + s_e[os1 >> 16];
        if (pl == 0) v += s_c[cur][rem];
        if (pl == P && !last) {
          s_c[nxt][rem] = v;
          continue;
        }
        // a redundant layer only carries; a segment's end plane is completed
        // (and written) by the next segment
        if (red || (pl == P && !glast)) continue;
        const int gxx = cx * P + pl;
        const bool bc = (m & kBcYZ) || gxx == A.bcx_lo || gxx == A.bcx_hi;
        const int kind = (m >> 4) & 3;
        if (bc) {
          if (kind == 0) continue;  // Dirichlet y was written at staging
          v = T(0);
        }
        if (BDX_OOB(lbase * (kind == 0 ? A.ps : kind == 1 ? A.ybps : kind == 2 ? A.zbps : A.cbps) +
                        o_off[k], kind == 0 ? A.vsize : A.ibsize, "f4 gather store"))
          continue;
        if (kind == 0)
          st_stream(ybase[0] + o_off[k], v);
        else
          (kind == 1 ? ybase[1] : kind == 2 ? ybase[2] : ybase[3])[o_off[k]] = v;
      }
    }

    // ------------------------------------------------ staging stores
    if (!last) {
      T* __restrict__ pnl = A.pnew + lnext;
      T* __restrict__ yl = A.y + lnext;
#pragma unroll
      for (int k = 0; k < NPF; ++k) {
        const int m = st_meta[k];
        if (tid + k * NT < P * PL && (m & kValid) && (m & kOwnT)) {
          if (BDX_OOB(lnext + st_goff[k], A.vsize, "f4 staging store")) continue;
          const int gxx = (cx + 1) * P + ((m >> 4) & 15);
          if constexpr (MODE == kFusedCG) {
            st_stream(pnl + st_goff[k], pf_r[k]);
            if (xupd) st_stream(A.x + lnext + st_goff[k], pf_x[k]);
          }
          if ((m & kBcYZ) || gxx == A.bcx_hi) {
            const bool rown = (m & kRownYZ) && gxx < A.ownx;
            yl[st_goff[k]] = rown ? pf_r[k] : T(0);
          }
        }
      }
    }
  };
  // two layers per trip, alternating register sets (the rolled loop with one
  // set spills 8 dwords in the CG instance)
  PF pfa, pfb;
  for (int cx = cbeg; cx < cend; cx += 2) {
    layer(cx, pfa);
    if (cx + 1 < cend) layer(cx + 1, pfb);
  }
  if constexpr (MODE == kFusedCG) {
    const double t = block_sum(pap, s_red);
    // indexed by (tile, segment): invariant under any launch split
    if (tid == 0) A.partials[(ty * A.ntz + tz) * A.nseg + seg] = t;
  }
}

// 1D matrices of the quadrature rule (host, double): M1 = B^T W B,
// K1 = Dd^T W Dd, C1 = Dd^T W B with B = phi0 (nq x 4), Dd = dphi1 phi0.
inline int pack_tables4(int nd, int nq, const double* phi0, const double* Dd, const double* wts,
                        double* out) {
  if (nd != 4 || nq < 1 || nq > kMaxNq) return -1;
  if (!out) return kFusedTabMax;
  for (int i = 0; i < kFusedTabMax; ++i) out[i] = 0.0;
  for (int i = 0; i < 4; ++i)
    for (int l = 0; l < 4; ++l) {
      double m = 0, k = 0, c = 0;
      for (int q = 0; q < nq; ++q) {
        m += wts[q] * phi0[q * 4 + i] * phi0[q * 4 + l];
        k += wts[q] * Dd[q * 4 + i] * Dd[q * 4 + l];
        c += wts[q] * Dd[q * 4 + i] * phi0[q * 4 + l];
      }
      out[i * 4 + l] = m;
      out[16 + i * 4 + l] = k;
      out[32 + i * 4 + l] = c;
    }
  return kFusedTabMax;
}

template <int MODE>
int launch_fused4(const Fused2Args<double>& a, const FusedTables<double>& tb, hipStream_t st) {
  constexpr int TY = kF4TY, TZ = kF4TZ;
  const int nblk = a.nblk;
  if (nblk <= 0) return 0;
  lap_fused4_kernel<TY, TZ, MODE><<<nblk, TY * TZ * 16, 0, st>>>(a, tb);
  return static_cast<int>(hipGetLastError());
}
