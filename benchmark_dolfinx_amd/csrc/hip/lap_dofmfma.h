// Reference data model (cell -> dof map, stored G [cell][6][nq^3], atomic
// scatter) with the tensor contractions on the matrix pipe: FP64
// v_mfma_f64_16x16x4_f64, one cell per wave, no workgroup barriers.
//
// The reference runs each 1D contraction as a thread-per-quadrature-point loop
// over an LDS image behind a __syncthreads (src/laplacian_gpu.hpp:188-251
// forward, :307-420 transposed).  Here every contraction over a NODE index (K
// = nd <= 8, one or two k-steps) and every contraction over a QUADRATURE index
// of the transposed pass is an MFMA whose operand is the previous MFMA's
// accumulator as it stands: an accumulator register r holds rows
// (lane >> 4) + 4 r, column lane & 15, which is exactly an A (row = column of
// the previous result) or B operand whose k index is those 4 rows.  The only
// lane movement is one DPP row_ror:8 exchange per node index in each
// direction; no LDS image, no table loads inside the contraction loops.
//
// Stacked 1D table S (16 rows): rows 0-7 phi0 (interpolation to the
// quadrature points), rows 8-15 Dd = dphi1 phi0 (derivative at the points);
// columns = nodes.  Kronecker structure of the reference gradient:
//   d/dx = Dd (x) phi (x) phi,  d/dy = phi (x) Dd (x) phi,  d/dz = phi (x) phi (x) Dd.
//
// Forward (u_e -> grad u at the points):
//   Z  C1_t = sum_s A(u_e: lines (i, j) x k-step s) . B(S^T: k x 16)       TZ*KS MFMAs
//      -> rows (i, j) of tile t, columns qz' (phi rows 0-7 | Dd rows 8-15)
//   Y  C2_i = sum_c A(C1 reg of (i, chunk c)) . B(S^T)                     ND*KS MFMAs
//      -> rows qz', columns qy' (phi | Dd)
//   X  DPP exchange (lanes n, n ^ 8) so that lane (g, n) holds the three
//      combinations (phi z, phi y), (phi z, Dd y), (Dd z, phi y) of ONE point
//      (qy = n & 7, qz = g + 4 (n >> 3)); then the x contraction is
//      lane-local: d/dx = sum_i Dd[qx][i] Vx_i, d/dy, d/dz with phi.
// Point stage: F = kappa G grad u (G: 6 loads per point, coalesced over the
//   lanes), p.Ap += grad u . F (= u_e . A_e u_e).
// Transposed (F -> y_e), the forward run backwards:
//   X^T lane-local R_i = sum_qx {Dd, phi, phi}[qx][i] F, DPP exchange back
//      to the C layout (rows qz', columns qy')
//   Z^T C3_t = sum_{i in t} sum_r' A(R_i reg r') . B(S: qz' chunk x kz)    ND*4 MFMAs
//      (two node indices i per 16 columns: block-diagonal B)
//   Y^T C4_t = sum_r A(S^T chunk: j x qy') . B(C3_t reg r)                 TZ*4 MFMAs
//      -> rows j, columns (i, kz): y_e of the cell in 16-lane z-runs.
// The gather / CG stores / identity rows are the element stage of
// lap_dofmap.h in the A-operand layout of Z (lane (g, n): line 16 t + n, node
// 4 s + g); the scatter reads the dof of each C4 element from an LDS copy of
// the cell's scatter targets.
//
// Instances: T = double, nd <= 8, nq <= 8 (Q1-Q7 at qmode 0 / 1, GLL or Gauss).
#pragma once
// attribution builds only (wrong numerics): BDX_EXP_NOG=1 replaces the stored
// G by constants, so a timing shows the kernel without its G stream
#ifndef BDX_EXP_NOG
#define BDX_EXP_NOG 0
#endif

template <int ND, int NQ>
struct DofMfmaShape {
  static constexpr int JP = ND <= 4 ? 4 : 8;            // line pitch of j (and of kz in C4)
  static constexpr int KS = (ND + 3) / 4;               // k-steps over a node index
  static constexpr int IPT = 16 / JP;                   // node indices i per 16 columns
  static constexpr int TZ = (ND * JP + 15) / 16;        // line tiles of Z = column tiles of Z^T
  static constexpr bool Q8 = NQ > 4;                    // quadrature rows 4-7 / 12-15 in use
  static constexpr int WAVES = 4;
  static constexpr int NT = 64 * WAVES;
  static constexpr int NE = TZ * KS;                    // element A-fragments per lane
  static constexpr int ND3 = ND * ND * ND, NQ3 = NQ * NQ * NQ;
  static constexpr int DSC = ((ND3 + 63) / 64) * 64;    // LDS scatter targets per wave
};

// dofmap (reference data model) operator with the contractions on v_mfma_f64_16x16x4_f64.
template <int ND, int NQ, int GEOM, int MODE>
__global__ void __launch_bounds__(256, 2)
    lap_dofmfma_kernel(DofArgs<double> A) {
  using T = double;
  using S = DofMfmaShape<ND, NQ>;
  using V4 = bdx_f64x4;
  constexpr int JP = S::JP, KS = S::KS, IPT = S::IPT, TZ = S::TZ, ND3 = S::ND3, NQ3 = S::NQ3;
  __shared__ int s_dsc[S::WAVES][2][S::DSC];
  __shared__ T s_X[S::WAVES][24];
  __shared__ double s_red[16];

  // wave index as a wave-uniform value (cell ids, descriptors and the G
  // block base then live in SGPRs: no waterfall loops)
  const int tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, n = lane & 15;
  const bool hi = n >= 8;

  // ---- tables.  A.tab = [phi0 nq x nd | dphi1 nq x nq | qpts | wts | Dd nq x nd |
  // phi0^T nd x nq | Dd^T nd x nq] (the transposed copies: the nq values of one
  // node index are contiguous, so each x-stage step loads them in one scalar load)
  typedef const __attribute__((address_space(4))) T CT;
  constexpr int OFF_D = NQ * ND, OFF_QP = OFF_D + NQ * NQ, OFF_W = OFF_QP + NQ, OFF_DD = OFF_W + NQ;
  constexpr int OFF_PT = OFF_DD + NQ * ND, OFF_DT = OFF_PT + ND * NQ;
  CT* const tab0 = (CT*)A.tab;  // NOLINT: address-space cast (scalar loads)
  auto lphase = [&](T dep) -> CT* {  // per-phase reload of the uniform rows
    CT* p = tab0;
    asm volatile("" : "+s"(p) : "v"(dep));
    return p;
  };
  // S[row][col] (row: 0-7 phi, 8-15 Dd; zero outside nq x nd)
  auto Sv = [&](int row, int col) -> T {
    const int q = row & 7;
    if (q >= NQ || col >= ND) return T(0);
    return row < 8 ? A.tab[q * ND + col] : A.tab[OFF_DD + q * ND + col];
  };
  // per-lane operand constants
  T Bz[KS];  // B of Z / Y: B[k = g][n] = S[n][4 s + g]
#pragma unroll
  for (int s = 0; s < KS; ++s) Bz[s] = Sv(n, 4 * s + g);
  T Bt[4];   // B of Z^T (before the block mask): S[g + 4 r'][n % JP]
#pragma unroll
  for (int r = 0; r < 4; ++r) Bt[r] = Sv(g + 4 * r, n % JP);
  T At[4];   // A of Y^T: A[m = n = j][k = g] = S[4 r + g][j]
#pragma unroll
  for (int r = 0; r < 4; ++r) At[r] = n < ND ? Sv(4 * r + g, n) : T(0);
  const int bt_blk = n / JP;  // the i % IPT this lane's Z^T column belongs to

  T beta = T(0), xalpha = T(0);
  if constexpr (MODE == kDofCG) {
    if (A.beta_num >= 0) beta = static_cast<T>(A.scal[A.beta_num] / A.scal[A.beta_den]);
    if (A.xa_num >= 0) xalpha = static_cast<T>(A.scal[A.xa_num] / A.scal[A.xa_den]);
  }
  double pap = 0.0;

  // XCD-aware bijective block remap (as lap_dofmap_kernel)
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  const int c_beg = bid * A.cells_per_block;
  const int c_end = min(c_beg + A.cells_per_block, A.ncl);

  // range-checked buffer descriptors (out-of-range offset: load 0 / store dropped)
  constexpr unsigned kOOB = 0xfffffff0u;
  const unsigned vbytes = static_cast<unsigned>(A.nvec * sizeof(T));
  auto rsrc = [](const void* ptr, unsigned bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(ptr), 0, static_cast<int>(bytes),
                                             0x00020000);
  };
  const auto rs_u = rsrc(A.u, vbytes), rs_f = rsrc(A.flags, static_cast<unsigned>(A.nvec));
  const auto rs_po = rsrc(MODE == kDofCG ? A.pold : A.u, vbytes);
  const auto rs_pn = rsrc(MODE == kDofCG ? A.pnew : A.y, MODE == kDofCG ? vbytes : 0u);
  const auto rs_x = rsrc(MODE == kDofCG ? A.x : A.y, MODE == kDofCG ? vbytes : 0u);
  const auto rs_y = rsrc(A.y, vbytes);
  auto ldv = [](__amdgpu_buffer_rsrc_t r, unsigned off) -> T {
    return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
  };
  auto stv = [](__amdgpu_buffer_rsrc_t r, unsigned off, T v) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(bdx_u32x2, v), r, off, 0, 0);
  };

  // element A-fragment e of this lane: line 16 t + n, node 4 s + g
  auto e_loc = [&](int f) -> int {  // local dof, -1 outside the cell
    const int t = f / KS, s = f % KS;
    const int p = 16 * t + n, i = p / JP, j = p % JP, k = 4 * s + g;
    return (i < ND && j < ND && k < ND) ? (i * ND + j) * ND + k : -1;
  };

  struct Gather {
    int d[S::NE];
    unsigned f[S::NE];
    T u[S::NE], po[S::NE], x[S::NE];
  };
  auto load_dofs = [&](int cell, int (&d)[S::NE]) {
#pragma unroll
    for (int f = 0; f < S::NE; ++f) {
      const int e = e_loc(f);
      d[f] = e >= 0 ? A.cdofs[static_cast<int64_t>(cell) * ND3 + e] : -1;
    }
  };
  auto gather = [&](const int (&d)[S::NE], Gather& G) {
#pragma unroll
    for (int f = 0; f < S::NE; ++f) {
      G.d[f] = d[f];
      const bool on = d[f] != -1;
      const unsigned dd = static_cast<unsigned>(d[f] & 0x7fffffff);
      G.f[f] = __builtin_amdgcn_raw_buffer_load_b8(rs_f, on ? dd : kOOB, 0, 0);
      G.u[f] = ldv(rs_u, on ? dd * 8u : kOOB);
      G.po[f] = MODE == kDofCG ? ldv(rs_po, on ? dd * 8u : kOOB) : T(0);
      const bool xw = on & (d[f] < 0) & (MODE == kDofCG) & (A.xa_num >= 0);
      G.x[f] = MODE == kDofCG ? ldv(rs_x, xw ? dd * 8u : kOOB) : T(0);
    }
  };

  // ---- element stage of one cell (consumes its gathers): p = r + beta
  // p_old, writer stores, identity rows; returns the A fragments of Z in ue
  // and writes the scatter targets to s_dsc[wv][buf]
  auto element = [&](const Gather& G, T (&ue)[S::NE], int buf) {
#pragma unroll
    for (int f = 0; f < S::NE; ++f) {
      const int dof = G.d[f];
      const bool on = dof != -1;
      const int d = dof & 0x7fffffff;
      const bool wr = on && dof < 0;
      const unsigned fl = (on ? G.f[f] : 0u) | (wr ? 4u : 0u);
      T v = G.u[f];
      if constexpr (MODE == kDofCG) {
        v = G.u[f] + beta * G.po[f];
        stv(rs_pn, wr ? static_cast<unsigned>(d) * 8u : kOOB, v);
        stv(rs_x, (wr && A.xa_num >= 0) ? static_cast<unsigned>(d) * 8u : kOOB,
            G.x[f] + xalpha * G.po[f]);
      }
      const bool bc = fl & 1u;
      const bool idrow = (fl & 7u) == 7u;  // Dirichlet, owned, writer
      stv(rs_y, idrow ? static_cast<unsigned>(d) * 8u : kOOB, v);
      if constexpr (MODE == kDofCG) {
        if (idrow) pap += v * v;
      }
      ue[f] = (on && !bc) ? v : T(0);
      const int e = e_loc(f);
      if (e >= 0) s_dsc[wv][buf][e] = (on && !bc) ? d : -1;
    }
  };

  // software pipeline over this wave's cells (list index wfirst + WAVES it).
  // Iteration it: the gathers of cell it + 1 (issued at its start) land
  // under the forward pass and are consumed after the point stage (its
  // element stage: ue of the next cell, scatter targets in the other s_dsc
  // buffer); the dofs of cell it + 2 are loaded at its start.
  const int wfirst = c_beg + wv;
  const int nit = wfirst < c_end ? (c_end - wfirst + S::WAVES - 1) / S::WAVES : 0;
  T ue[S::NE];
  int dn[S::NE];
  int cell_cur = 0, cell_next = 0;
  if (nit > 0) {
    cell_cur = A.cells[wfirst];
    int d0[S::NE];
    load_dofs(cell_cur, d0);
    Gather g0;
    gather(d0, g0);
    element(g0, ue, 0);
    if (nit > 1) {
      cell_next = A.cells[wfirst + S::WAVES];
      load_dofs(cell_next, dn);
    }
  }

  for (int it = 0; it < nit; ++it) {
    const int li = wfirst + it * S::WAVES;  // < c_end
    const int64_t cell = cell_cur;
    const int buf = it & 1;
    const T kap = A.kc ? A.kc[cell] : A.kappa;
    if constexpr (GEOM == kGeomOTF) {
      if (lane < 24) s_X[wv][lane] = A.coords[3 * static_cast<int64_t>(A.cverts[cell * 8 + lane / 3]) + lane % 3];
    }

    // the next cell's gathers, the dofs of the one after
    const bool more = it + 1 < nit;
    Gather gn;
    if (more) {
      gather(dn, gn);
      cell_cur = cell_next;
      if (it + 2 < nit) {
        cell_next = A.cells[li + 2 * S::WAVES];
        load_dofs(cell_next, dn);
      }
    }

    // ---- Z (contract k) one line tile at a time, then Y (contract j) and X
    // (contract i, lane-local) for the node indices i of that tile: one
    // accumulator tile live at a time
    T dX[NQ], dY[NQ], dZ[NQ];
#pragma unroll
    for (int q = 0; q < NQ; ++q) dX[q] = dY[q] = dZ[q] = T(0);
#pragma unroll
    for (int t = 0; t < TZ; ++t) {
      V4 C1 = V4{0, 0, 0, 0};
#pragma unroll
      for (int s = 0; s < KS; ++s) C1 = bdx_mfma16x4(ue[t * KS + s], Bz[s], C1);
#pragma unroll
      for (int i = t * IPT; i < (t + 1) * IPT && i < ND; ++i) {
        V4 C2 = V4{0, 0, 0, 0};
#pragma unroll
        for (int c = 0; c < KS; ++c) C2 = bdx_mfma16x4(C1[(i % IPT) * KS + c], Bz[c], C2);
        // lane (g, n) <- the three combinations of its point (see the file head)
        const T a = dpp_row_ror8(C2[0]), b = dpp_row_ror8(C2[1]), c3 = dpp_row_ror8(C2[3]);
        const T vx = hi ? b : C2[0], vy = hi ? C2[1] : a, vz = hi ? c3 : C2[2];
        CT* const tb = lphase(vx);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          dX[q] += tb[OFF_DT + i * NQ + q] * vx;
          dY[q] += tb[OFF_PT + i * NQ + q] * vy;
          dZ[q] += tb[OFF_PT + i * NQ + q] * vz;
        }
        __builtin_amdgcn_sched_barrier(0);  // one node index at a time (registers)
      }
    }

    // ---- point stage: F = kappa G grad u at (qx, qy, qz), p.Ap
    const int qy = n & 7, qz = g + 4 * (n >> 3);
    const bool pt = qy < NQ && qz < NQ;
    const T kv = pt ? kap : T(0);
    if constexpr (GEOM == kGeomOTF) {
      T Xc[8][3];
#pragma unroll
      for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int d = 0; d < 3; ++d) Xc[v][d] = s_X[wv][v * 3 + d];
      CT* const t = lphase(dX[0]);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        T Gd[6];
        geometry_G<T>(Xc, t[OFF_QP + q], t[OFF_QP + (pt ? qy : 0)], t[OFF_QP + (pt ? qz : 0)],
                      t[OFF_W + q] * t[OFF_W + (pt ? qy : 0)] * t[OFF_W + (pt ? qz : 0)], Gd);
        const T gx = dX[q], gy = dY[q], gz = dZ[q];
        dX[q] = kv * (Gd[0] * gx + Gd[1] * gy + Gd[2] * gz);
        dY[q] = kv * (Gd[1] * gx + Gd[3] * gy + Gd[4] * gz);
        dZ[q] = kv * (Gd[2] * gx + Gd[4] * gy + Gd[5] * gz);
        if constexpr (MODE == kDofCG) pap += gx * dX[q] + gy * dY[q] + gz * dZ[q];
      }
    } else {
      // the cell's G block through a range-checked descriptor (no branch
      // around the loads; lanes without a point load 0), non-temporal (aux 2),
      // two point planes in flight ahead of the one being used
      const auto rs_g = rsrc(A.G + cell * 6 * NQ3, 6 * NQ3 * 8);
      const unsigned pbase = pt ? static_cast<unsigned>(qy * NQ + qz) * 8u : kOOB;
      // (the offset of step q + 2's loads is laundered through step q - 1's
      // result, so the compiler cannot hoist the whole cell's G ahead)
      auto gload = [&](int q, T (&Gd)[6], T dep) {
        unsigned off = pbase;
        asm volatile("" : "+v"(off) : "v"(dep));
#pragma unroll
        for (int k = 0; k < 6; ++k)
          Gd[k] = __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(
                                            rs_g, off, (k * NQ3 + q * NQ * NQ) * 8, 2));
      };
      T Gr[3][6];
      gload(0, Gr[0], kv);
      if (NQ > 1) gload(1, Gr[1], kv);
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (q + 2 < NQ) gload(q + 2, Gr[(q + 2) % 3], q > 0 ? dZ[q - 1] : kv);
        const T* Gd = Gr[q % 3];
#if BDX_EXP_NOG
        const T Gk[6] = {1.0, 0.1, 0.1, 1.0, 0.1, 1.0};
        Gd = Gk;
#endif
        const T gx = dX[q], gy = dY[q], gz = dZ[q];
        dX[q] = kv * (Gd[0] * gx + Gd[1] * gy + Gd[2] * gz);
        dY[q] = kv * (Gd[1] * gx + Gd[3] * gy + Gd[4] * gz);
        dZ[q] = kv * (Gd[2] * gx + Gd[4] * gy + Gd[5] * gz);
        if constexpr (MODE == kDofCG) pap += gx * dX[q] + gy * dY[q] + gz * dZ[q];
      }
    }

    // ---- the next cell's element stage (its gathers were in flight under Z /
    // Y / X and the point stage)
    if (more) element(gn, ue, buf ^ 1);

    // ---- X^T (lane-local), exchange back, Z^T into the column tile of i;
    // once a tile's node indices are done: Y^T (rows j, columns (i % IPT,
    // kz)) and the scatter-add
    dof_wave_sync();  // s_dsc[buf] of this cell visible to every lane
    T chain = dX[0];  // per-i dependency of the table pointer: node index i's rows
                      // load after i - 1 has finished (SGPR budget)
#pragma unroll
    for (int t = 0; t < TZ; ++t) {
      V4 C3 = V4{0, 0, 0, 0};
#pragma unroll
      for (int i = t * IPT; i < (t + 1) * IPT && i < ND; ++i) {
        CT* const tb = lphase(chain);
        T rx = T(0), ry = T(0), rz = T(0);
#pragma unroll
        for (int q = 0; q < NQ; ++q) {
          rx += tb[OFF_DT + i * NQ + q] * dX[q];
          ry += tb[OFF_PT + i * NQ + q] * dY[q];
          rz += tb[OFF_PT + i * NQ + q] * dZ[q];
        }
        chain = rz;
        const T prx = dpp_row_ror8(rx), pry = dpp_row_ror8(ry), prz = dpp_row_ror8(rz);
        T R[4];
        R[0] = hi ? pry : rx;
        R[1] = hi ? ry : prx;
        R[2] = hi ? T(0) : rz;
        R[3] = hi ? T(0) : prz;
        const bool blk = bt_blk == i % IPT;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          if (!S::Q8 && (r & 1)) continue;  // quadrature rows 4-7 / 12-15 empty
          C3 = bdx_mfma16x4(R[r], blk ? Bt[r] : T(0), C3);
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      V4 C4 = V4{0, 0, 0, 0};
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (!S::Q8 && (r & 1)) continue;
        C4 = bdx_mfma16x4(At[r], C3[r], C4);
      }
      const int i = t * IPT + n / JP, kz = n % JP;
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        const int j = g + 4 * r;
        if (i < ND && j < ND && kz < ND) {
          const int dsc = s_dsc[wv][buf][(i * ND + j) * ND + kz];
          if (dsc >= 0) atomicAdd(A.y + dsc, C4[r]);
        }
      }
    }
    dof_wave_sync();  // the cell after next rewrites s_dsc[buf]
  }

  // zero this block's slice of the other y buffer (native runtime ping-pong)
  if constexpr (MODE == kDofCG) {
    if (A.yz) {
      typedef T ZV __attribute__((ext_vector_type(2)));
      const int64_t nv = A.nz / 2, per = (nv + nblk - 1) / nblk;
      const int64_t v0 = static_cast<int64_t>(ob) * per, v1 = v0 + per < nv ? v0 + per : nv;
      for (int64_t v = v0 + tid; v < v1; v += S::NT)
        __builtin_nontemporal_store(ZV(0), reinterpret_cast<ZV*>(A.yz + v * 2));
      if (ob == 0)
        for (int64_t i = nv * 2 + tid; i < A.nz; i += S::NT) A.yz[i] = T(0);
    }
    const double t = block_sum(pap, s_red);
    if (tid == 0) A.partials[bid] = t;
  }
}
