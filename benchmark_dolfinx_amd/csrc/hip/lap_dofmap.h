// Unstructured-data-model operator ("dofmap"): the reference's general mesh
// representation instead of lattice index arithmetic.
//
// Inputs are the arrays a DOLFINx mesh carries (reference src/laplacian.hpp:
// 105-114 and src/laplacian_gpu.hpp:153-170, built in src/mesh.cpp:87-102):
//   cell_dofs  [ncells][ND^3]  cell -> dof map (tensor-product order i, j, k);
//                              the sign bit marks the one (cell, local dof)
//                              occurrence that writes a dof's CG vectors
//   cell_verts [ncells][8]     cell -> geometry-node map (v = 4a + 2b + c)
//   coords     [nverts][3]     geometry nodes
//   dof_flags  [ndofs]         bit 0: Dirichlet dof, bit 1: owned by this rank
//   cells      [ncl]           the cells of this launch (interior or boundary
//                              list, so the halo exchange can overlap the
//                              interior cells as in src/laplacian.hpp:281-349)
// and optionally stored G [ncells][6][nq^3] (the reference layout) and a
// per-cell coefficient.  Any hexahedral mesh, any cell order and any dof
// numbering work: nothing is derived from a lattice.
//
// Kernel design (MI355X, one wave per CPW = 64 / NQ^2 cells, no workgroup
// barriers): the reference runs one thread per quadrature point with every
// 1D contraction read from LDS behind a __syncthreads (10 per cell,
// src/laplacian_gpu.hpp:172-412).  Here a lane owns a whole 1D line of the
// cell and contracts it in registers; LDS only transposes between the line
// directions, inside the wave:
//   element    lane + 64 r:   one local dof of one of the wave's cells, in
//                             cell_dofs order (gather, CG stores, scatter):
//                             a wave-instruction reads one dofmap row and
//                             touches the dofs in z-runs, not one per lane
//   nodal      lane (i, j):   z-line of the element vector
//   mixed      lane (i, qz):  y-lines of the half-interpolated arrays
//   quadrature lane (qy, qz): x-lines of U, grad U, G grad U (G loads are
//                             contiguous across these lanes), with the y- and
//                             z-derivatives formed by lanes (qx, qz) / (qx, qy)
// The stored-G loads of a cell are issued before its first contraction, so
// they are in flight under the interpolation and gradient stages (at Q3 as
// 16-byte chunks of the cells' contiguous G blocks, redistributed to the
// quadrature lanes through LDS).
//
// CG mode fuses the reference's BLAS-1 calls (src/cg.hpp:121-167) into the
// gather: p = r + beta p_old is formed per gathered dof, the designated
// writer of each dof stores p and the lagged x += alpha p_old, the element
// dots p_e . (A_e p_e) give p.Ap, and the y scatter-add uses float atomics as
// the reference does.  With the update pass (r -= alpha y, r.r, y = 0) one
// CG iteration moves 11 vector streams instead of the generic 15.
#pragma once
#include "lap_v1.h"

enum { kDofAction = 0, kDofCG = 1 };

// Pipeline schedule (switches kept with their A/B records): kDofEarly issues
// the next cell's gathers (and the dofs of the cell after it) as soon as the
// element stage has consumed the current ones, and the next cell's stored G
// as soon as the F stage has moved the current G to LDS, so both are in
// flight for a whole iteration instead of from the end of one to the start /
// middle of the next (instances that prefetch G).  kDofGnt streams G
// non-temporally (66.6 GB per apply at Q3, read once: kept out of the caches
// that the gathers reuse).  A direct-to-LDS form of the G staging
// (global_load_lds_dwordx4) compiles to a vmcnt(0) before the next read of
// any LDS array (the waitcnt pass cannot separate s_G from s_buf), which
// would expose the G latency at once: not used.
constexpr bool kDofEarly = true;
constexpr bool kDofGnt = true;
// kDofZMerge: the Q3 instance scatters the z-lines of its two z-neighbour
// cells as one 7-dof run (see the scatter at the end of the cell loop)
constexpr bool kDofZMerge = true;
// kDofWgMerge: the one-cell-per-wave instances (NQ >= 8) and the FP64 Q3 one
// (two cells per wave) scatter the z-lines of the workgroup's cells of an
// iteration (consecutive in the launch list: z-neighbours on a lexicographic
// mesh) as one run per line, after a workgroup barrier
constexpr bool kDofWgMerge = true;
typedef unsigned bdx_u32x2 __attribute__((ext_vector_type(2)));

template <int NQ>
struct DofShape {
  static constexpr int NQ2 = NQ * NQ;
  static constexpr int CPW = NQ2 <= 64 ? 64 / NQ2 : 1;  // cells per wave
  static constexpr int LPL = (NQ2 + 63) / 64;           // lines per lane (NQ = 9: 2)
  static constexpr int NQP = NQ | 1;                    // odd z pitch: conflict-free z-lines
  static constexpr int BUF = NQ * NQ * NQP;             // one transpose buffer per cell
  static constexpr int WAVES = 4;
  static constexpr int NT = 64 * WAVES;
  // stored G of the lane's x-lines held in registers from the start of the
  // cell (in flight under the interpolation and gradient); larger rules load
  // it where it is used
  static constexpr bool GPREF = 6 * NQ * LPL <= 30;
};

template <typename T>
struct DofArgs {
  const int* cells;
  int ncl;
  int cells_per_block;
  int64_t nvec;  // entries of every vector (range of the buffer descriptors)
  const int* cdofs;
  const int* cverts;
  const T* coords;
  const unsigned char* flags;
  const T* G;
  const T* tab;  // device [phi0 (nq x nd) | dphi1 (nq x nq) | qpts | wts]
  T kappa;
  const T* kc;
  const T* u;      // action: input; CG: r
  const T* pold;   // CG
  T* pnew;         // CG
  T* x;            // CG
  T* y;
  const double* scal;
  int beta_num, beta_den, xa_num, xa_den;  // -1: beta = 0 / no x update
  double* partials;                        // CG: p.Ap per block
  // native CG runtime: the other y buffer of its ping-pong (consumed by the
  // last update pass), zeroed by this launch for the next operator; null: none
  T* yz;
  int64_t nz;
};

// wave-local LDS exchange (the lanes of one wave run in lockstep)
__device__ __forceinline__ void dof_wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}

// dofmap: line-per-lane sum factorisation on an explicit cell->dof map (any hex mesh).
template <typename T, int ND, int NQ, int GEOM, int MODE>
__global__ void __launch_bounds__(DofShape<NQ>::NT)
    lap_dofmap_kernel(DofArgs<T> A) {
  using S = DofShape<NQ>;
  constexpr int CPW = S::CPW, LPL = S::LPL, NQP = S::NQP, BUF = S::BUF, NQ2 = NQ * NQ;
  constexpr int ND3 = ND * ND * ND, NQ3 = NQ * NQ * NQ;
  constexpr bool IDENT = ND == NQ;  // qmode 0, GLL: phi0 = I (quirk Q5 guarantees it)
  constexpr bool GPREF = GEOM == kGeomStored && S::GPREF;
  // early issue: instances with prefetched stored G.  On-the-fly geometry is
  // register-bound (the early gathers push its Q5 / Q6 CG instances to 1
  // wave / SIMD); with G loaded where it is used (NQ >= 6) the in-order
  // vmcnt makes those loads wait for the early gathers too (Q6 -6 %,
  // profiles/r5_dofmap_pipeline.md)
  constexpr bool EARLY = kDofEarly && GPREF;
  // GLDS: the prefetched stored G of the wave's cells moves as 16-byte
  // chunks (each cell's G block is contiguous) and is redistributed to the
  // quadrature lanes through LDS at the F stage: 12 instead of 30 load
  // instructions per cell pair at Q3, 194 -> 140 VGPRs, +2.9 % same box
  // (scripts/r3_dofglds.sh).  Two cells per wave (NQ = 5) only: with more
  // cells per wave the 12-24 KB of staging per wave would cut the workgroups
  // per CU below what the register version reaches.
  constexpr int GE = CPW * 6 * NQ3;  // stored-G values of the wave's cells
  constexpr bool GLDS = GPREF && CPW <= 2 && (6 * NQ3 * sizeof(T)) % 16 == 0;
  constexpr int GW = 16 / sizeof(T), GCH = GLDS ? (GE / GW + 63) / 64 : 1;
  static_assert(ND * ND <= 64, "nodal z-lines: one per lane");
  __shared__ __attribute__((aligned(16))) T s_buf[S::WAVES][CPW][3][BUF];
  __shared__ T s_X[S::WAVES][CPW][24];
  __shared__ int s_ids[S::WAVES][2][64];  // per-wave ring of cell ids (two blocks)
  __shared__ double s_red[16];
  __shared__ __attribute__((aligned(16))) T s_G[GLDS ? S::WAVES : 1][GLDS ? GE : GW];

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int slot = CPW > 1 ? lane / NQ2 : 0;
  const int sl = lane - slot * NQ2;  // lane within the cell's slot (CPW > 1: < NQ2)
  const bool slot_on = slot < CPW;
  T* const Ab = s_buf[wv][slot_on ? slot : 0][0];
  T* const Bb = s_buf[wv][slot_on ? slot : 0][1];
  T* const Cb = s_buf[wv][slot_on ? slot : 0][2];

  // lane roles (see the file head); quadrature / mixed lines are numbered
  // l = sl + 64 rp, rp < LPL
  const bool r_nod = slot_on && sl < ND * ND;
  const int ni = sl / ND, nj = sl % ND;
  auto q_on = [&](int rp) { return slot_on && sl + 64 * rp < NQ2; };
  auto qa_of = [&](int rp) { return (sl + 64 * rp) / NQ; };
  auto qb_of = [&](int rp) { return (sl + 64 * rp) % NQ; };

  T beta = T(0), xalpha = T(0);
  if constexpr (MODE == kDofCG) {
    if (A.beta_num >= 0) beta = static_cast<T>(A.scal[A.beta_num] / A.scal[A.beta_den]);
    if (A.xa_num >= 0) xalpha = static_cast<T>(A.scal[A.xa_num] / A.scal[A.xa_den]);
  }
  double pap = 0.0;

  // 1D tables: wave-uniform scalar loads from the operator's device buffer.
  // Each contraction phase reads its table through a pointer laundered with
  // the phase's first input value, so the phase's rows load together (one
  // scalar-cache round trip per phase, not per row) and are not hoisted out
  // of the cell loop (all tables at once would overflow the SGPR file and
  // spill to VGPR lanes).
  typedef const __attribute__((address_space(4))) T CT;
  constexpr int OFF_D = NQ * ND, OFF_QP = OFF_D + NQ * NQ, OFF_W = OFF_QP + NQ;
  CT* const tab0 = (CT*)A.tab;  // NOLINT: address-space cast (as in lap_fused5.h)
  auto lphase = [&](T dep) -> CT* {
    CT* p = tab0;
    asm volatile("" : "+s"(p) : "v"(dep));
    return p;
  };

  // XCD-aware bijective block remap: consecutive cell chunks on one XCD (its
  // L2 then holds the dofs neighbouring cells share)
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  const int c_beg = bid * A.cells_per_block;
  const int c_end = min(c_beg + A.cells_per_block, A.ncl);

  // Range-checked buffer descriptors of the gathered / scattered vectors: an
  // offset past the range loads 0 and drops a store, so masked lanes (no
  // cell, not a writer, Dirichlet) need no branch and every load of a cell
  // issues back to back (a branch around a load makes the waitcnt pass fall
  // back to vmcnt(0), which would wait for the prefetched G as well).
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
  // per-cell coefficient: range 0 when there is none (the load returns 0)
  const auto rs_kc = rsrc(A.kc ? A.kc : A.y, A.kc ? 0x7ffffff0u : 0u);
  auto ldv = [](__amdgpu_buffer_rsrc_t r, unsigned off) -> T {
    if constexpr (sizeof(T) == 8)
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0));
    else
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
  };
  auto stv = [](__amdgpu_buffer_rsrc_t r, unsigned off, T v) {
    if constexpr (sizeof(T) == 8)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(bdx_u32x2, v), r, off, 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
  };

  // ---- software pipeline over this wave's cells (iteration j: list index
  // li = first + STEP j).  Cell ids come from a per-wave LDS ring filled one
  // block of IB iterations ahead (no global-load latency on the id), each
  // iteration issues the next cell's gathers and stored G and the dofs of the
  // cell after it, and the loop is unrolled by two with alternating dof /
  // vertex register sets, so no register holding an in-flight load is ever
  // copied (a copy would make the wave wait for it at the loop latch).
  constexpr int STEP = S::WAVES * CPW;
  constexpr int IB = 64 / CPW;               // iterations per id block
  constexpr int XPL = (24 + NQ2 - 1) / NQ2;  // vertex coordinates per lane (OTF)
  constexpr int NE = CPW * ND3, RE = (NE + 63) / 64;  // gathered elements / rounds per lane
  // merged z-line scatter of the wave's two cells (see the scatter below)
  // (FP64 only: the FP32 instance would drop from 3 to 2 waves / SIMD)
  constexpr bool ZMERGE = kDofZMerge && CPW == 2 && ND == 4 && sizeof(T) == 8;
  // workgroup-merged scatter of the waves' cells (supersedes ZMERGE)
  constexpr bool WGMERGE = kDofWgMerge && (CPW == 1 || ZMERGE) && ND3 <= 512;
  const int first = c_beg + wv * CPW + slot;
  const int last_li = c_end - 1;
  const int wbase = c_beg + wv * CPW;  // list index of (iteration 0, slot 0)
  const int id_lane = (lane / CPW) * STEP + lane % CPW;  // this lane's entry of a block
  auto id_load = [&](int blk) -> int {
    const int li = wbase + blk * IB * STEP + id_lane;
    return A.cells[li < last_li ? li : last_li];
  };
  auto id_put = [&](int blk, int v) {
    if (lane < IB * CPW) s_ids[wv][blk & 1][lane] = v;
  };
  auto cell_at = [&](int j, int s) -> int { return s_ids[wv][(j / IB) & 1][(j % IB) * CPW + s]; };
  auto cell_of = [&](int j) -> int { return cell_at(j, slot_on ? slot : 0); };
  // element role of the gather / CG stores / scatter: lane + 64 r is entry
  // e_ of cell slot s_ (local dofs in cell_dofs order, k fastest), so each
  // wave-instruction reads a cell's dofmap row and its dofs' values in
  // contiguous z-runs instead of one dof per lane
  auto e_slot = [&](int r) { return (lane + 64 * r) / ND3; };
  auto e_loc = [&](int r) { return (lane + 64 * r) % ND3; };
  auto e_on = [&](int j, int r) {  // element of a cell of this launch
    return lane + 64 * r < NE && wbase + e_slot(r) + j * STEP < c_end;
  };
  auto load_dofs = [&](int j, int (&d)[RE]) {
#pragma unroll
    for (int r = 0; r < RE; ++r) {
      const int s = lane + 64 * r < NE ? e_slot(r) : 0;
      d[r] = A.cdofs[static_cast<int64_t>(cell_at(j, s)) * ND3 + e_loc(r)];
    }
  };
  auto load_verts = [&](int c32, int (&vx)[XPL]) {
    const int64_t c = c32;
#pragma unroll
    for (int e = 0; e < XPL; ++e) {
      const int x = sl + NQ2 * e;
      vx[e] = GEOM == kGeomOTF ? A.cverts[c * 8 + (x < 24 ? x / 3 : 0)] : 0;
    }
  };
  struct Gather {
    T u[RE], po[RE], x[RE], X[XPL];
    unsigned f[RE];
    T kc;
  };
  auto gather = [&](const int (&d)[RE], const int (&vx)[XPL], int j, int c32, Gather& g) {
#pragma unroll
    for (int r = 0; r < RE; ++r) {
      const unsigned dd = static_cast<unsigned>(d[r] & 0x7fffffff);
      const bool on = e_on(j, r);
      g.f[r] = __builtin_amdgcn_raw_buffer_load_b8(rs_f, on ? dd : kOOB, 0, 0);
      g.u[r] = ldv(rs_u, on ? dd * sizeof(T) : kOOB);
      g.po[r] = MODE == kDofCG ? ldv(rs_po, on ? dd * sizeof(T) : kOOB) : T(0);
      const bool xw = on & (d[r] < 0) & (MODE == kDofCG) & (A.xa_num >= 0);
      g.x[r] = MODE == kDofCG ? ldv(rs_x, xw ? dd * sizeof(T) : kOOB) : T(0);
    }
#pragma unroll
    for (int e = 0; e < XPL; ++e) {
      const int x = sl + NQ2 * e;
      g.X[e] = GEOM == kGeomOTF ? A.coords[3 * static_cast<int64_t>(vx[e]) + (x < 24 ? x % 3 : 0)]
                                : T(0);
    }
    g.kc = ldv(rs_kc, static_cast<unsigned>(c32) * sizeof(T));
  };
  T Gr[LPL][GPREF && !GLDS ? 6 * NQ : 1];
  typedef T GV __attribute__((ext_vector_type(16 / sizeof(T))));
  GV Gv[GCH];
  auto load_G = [&](int j, int c32) {
    if constexpr (GLDS) {
#pragma unroll
      for (int m = 0; m < GCH; ++m) {
        const int e = (lane + 64 * m) * GW;  // first value of this lane's chunk
        if (e < GE) {
          const int s = e / (6 * NQ3);
          const GV* gp = reinterpret_cast<const GV*>(A.G + static_cast<int64_t>(cell_at(j, s)) * 6 * NQ3 +
                                                     (e - s * 6 * NQ3));
          Gv[m] = kDofGnt ? __builtin_nontemporal_load(gp) : *gp;
        }
      }
    } else if constexpr (GPREF) {
      const T* Gc = A.G + static_cast<int64_t>(c32) * 6 * NQ3;
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp)
#pragma unroll
        for (int qx = 0; qx < NQ; ++qx)
#pragma unroll
          for (int k = 0; k < 6; ++k)
            Gr[rp][k * NQ + qx] = Gc[k * NQ3 + qx * NQ2 + (q_on(rp) ? sl + 64 * rp : 0)];
    }
  };

  // WGMERGE: every wave of the block runs the block's iteration count (the
  // scatter has workgroup barriers); a wave past the end runs masked cells
  const bool wave_on = WGMERGE ? c_beg < c_end : wbase < c_end;
  const int nit = !wave_on ? 0 : (c_end - (WGMERGE ? c_beg : wbase) + STEP - 1) / STEP;
  int dA[RE], dB[RE], vA[XPL], vB[XPL];
  int cell_cur = 0, id_next = 0;
  Gather gc;
  if (wave_on) {
    id_put(0, id_load(0));
    dof_wave_sync();
    cell_cur = cell_of(0);
    load_dofs(0, dA);
    load_verts(cell_cur, vA);
    gather(dA, vA, 0, cell_cur, gc);
    load_G(0, cell_cur);
    load_dofs(1, dB);
    load_verts(cell_of(1), vB);
  }

  // one cell of the pipeline: (dc, vc) hold its dofs / vertices (landed),
  // (dn, vn) the next cell's (in flight); the advance overwrites (dc, vc)
  // with the dofs of the cell after next
  auto iter = [&](int j, int (&dc)[RE], int (&dn)[RE], int (&vc)[XPL], int (&vn)[XPL])
      __attribute__((always_inline)) {
    const int li = first + j * STEP;
    const bool valid = slot_on && li < c_end;
    const int64_t cell = cell_cur;
    (void)vc;
    // id ring: block b + 1 is loaded when block b starts and written to the
    // ring half a block later (before any cell_of reaches into it)
    if (j % IB == 0) id_next = id_load(j / IB + 1);
    if (j % IB == IB / 2) id_put(j / IB + 1, id_next);
    const T kap = A.kc ? gc.kc : A.kappa;

    // ---- the gathered elements (element role): p = r + beta p_old (CG), the
    // writer's p / lagged x stores, Dirichlet identity rows; the element
    // vector goes to LDS in the nodal layout, the scatter target stays here
    // (-1: Dirichlet dof, entry of no cell)
    int dsc[RE];
    T ue[RE];
#pragma unroll
    for (int r = 0; r < RE; ++r) {
      const int dof = dc[r];
      const int d = dof & 0x7fffffff;
      const bool on = e_on(j, r);
      const bool wr = on && dof < 0;
      const unsigned fl = (on ? gc.f[r] : 0u) | (wr ? 4u : 0u);
      T v = gc.u[r];
      if constexpr (MODE == kDofCG) {
        v = gc.u[r] + beta * gc.po[r];
        stv(rs_pn, wr ? static_cast<unsigned>(d) * sizeof(T) : kOOB, v);
        stv(rs_x, (wr && A.xa_num >= 0) ? static_cast<unsigned>(d) * sizeof(T) : kOOB,
            gc.x[r] + xalpha * gc.po[r]);
      }
      const bool bc = fl & 1u;
      const bool idrow = (fl & 7u) == 7u;  // Dirichlet, owned, writer
      stv(rs_y, idrow ? static_cast<unsigned>(d) * sizeof(T) : kOOB, v);
      if constexpr (MODE == kDofCG) {
        if (idrow) pap += static_cast<double>(v) * static_cast<double>(v);
      }
      ue[r] = bc ? T(0) : v;  // zero column
      dsc[r] = (on && !bc) ? d : -1;
      if (lane + 64 * r < NE) {
        const int e = e_loc(r);
        s_buf[wv][e_slot(r)][0][((e / (ND * ND)) * NQ + (e / ND) % ND) * NQP + e % ND] = ue[r];
      }
    }
    if constexpr (GEOM == kGeomOTF) {
#pragma unroll
      for (int e = 0; e < XPL; ++e) {
        const int x = sl + NQ2 * e;
        if (slot_on && x < 24) s_X[wv][slot][x] = gc.X[e];
      }
    }
    dof_wave_sync();
    // early advance: the next cell's gathers into the registers just consumed,
    // the dofs of the cell after it into dc (the scatter targets are in dsc)
    if constexpr (EARLY) {
      const int cn = cell_of(j + 1), cnn = cell_of(j + 2);
      gather(dn, vn, j + 1, cn, gc);
      load_dofs(j + 2, dc);
      load_verts(cnn, vc);
      cell_cur = cn;
    }

    // ---- interpolation to the quadrature points: z (nodal lanes), y (mixed), x (quad)
    T U[LPL][NQ];
    if constexpr (IDENT) {
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp)
#pragma unroll
        for (int qx = 0; qx < NQ; ++qx)
          U[rp][qx] = q_on(rp) ? Ab[(qx * NQ + qa_of(rp)) * NQP + qb_of(rp)] : T(0);
    } else {
      if (r_nod) {  // z-line (i, j) of the element vector, rewritten in place
        T un[ND];
#pragma unroll
        for (int k = 0; k < ND; ++k) un[k] = Ab[(ni * NQ + nj) * NQP + k];
        CT* const t = lphase(un[0]);
#pragma unroll
        for (int qz = 0; qz < NQ; ++qz) {
          T s = T(0);
#pragma unroll
          for (int k = 0; k < ND; ++k) s += t[qz * ND + k] * un[k];
          Ab[(ni * NQ + nj) * NQP + qz] = s;
        }
      }
      dof_wave_sync();
#pragma unroll
      for (int rp = 0; rp < (ND * NQ + 63) / 64; ++rp) {
        const int l = sl + 64 * rp, mi = l / NQ, mq = l % NQ;
        if (slot_on && l < ND * NQ) {  // mixed lane (i, qz)
          T in[ND];
#pragma unroll
          for (int j = 0; j < ND; ++j) in[j] = Ab[(mi * NQ + j) * NQP + mq];
          CT* const t = lphase(in[0]);
#pragma unroll
          for (int qy = 0; qy < NQ; ++qy) {
            T s = T(0);
#pragma unroll
            for (int j = 0; j < ND; ++j) s += t[qy * ND + j] * in[j];
            Bb[(mi * NQ + qy) * NQP + mq] = s;
          }
        }
      }
      dof_wave_sync();
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp) {
        T in[ND];
#pragma unroll
        for (int i = 0; i < ND; ++i)
          in[i] = q_on(rp) ? Bb[(i * NQ + qa_of(rp)) * NQP + qb_of(rp)] : T(0);
        CT* const t = lphase(in[0]);
#pragma unroll
        for (int qx = 0; qx < NQ; ++qx) {
          T s = T(0);
#pragma unroll
          for (int i = 0; i < ND; ++i) s += t[qx * ND + i] * in[i];
          U[rp][qx] = s;
        }
        if (q_on(rp)) {
#pragma unroll
          for (int qx = 0; qx < NQ; ++qx) Ab[(qx * NQ + qa_of(rp)) * NQP + qb_of(rp)] = U[rp][qx];
        }
      }
      dof_wave_sync();
    }

    // ---- reference gradient: x in registers, y / z by the transposed lane roles
#pragma unroll
    for (int rp = 0; rp < LPL; ++rp) {
      if (!q_on(rp)) continue;
      const int a = qa_of(rp), b = qb_of(rp);
      T in[NQ], o[NQ];
#pragma unroll
      for (int m = 0; m < NQ; ++m) in[m] = Ab[(a * NQ + m) * NQP + b];  // y-line (qx, qz)
      CT* const t = lphase(in[0]);  // dphi1 rows for both lines
#pragma unroll
      for (int qy = 0; qy < NQ; ++qy) {
        T s = T(0);
#pragma unroll
        for (int m = 0; m < NQ; ++m) s += t[OFF_D + qy * NQ + m] * in[m];
        o[qy] = s;
      }
#pragma unroll
      for (int qy = 0; qy < NQ; ++qy) Bb[(a * NQ + qy) * NQP + b] = o[qy];
#pragma unroll
      for (int m = 0; m < NQ; ++m) in[m] = Ab[(a * NQ + b) * NQP + m];  // z-line (qx, qy)
#pragma unroll
      for (int qz = 0; qz < NQ; ++qz) {
        T s = T(0);
#pragma unroll
        for (int m = 0; m < NQ; ++m) s += t[OFF_D + qz * NQ + m] * in[m];
        o[qz] = s;
      }
#pragma unroll
      for (int qz = 0; qz < NQ; ++qz) Cb[(a * NQ + b) * NQP + qz] = o[qz];
    }
    dof_wave_sync();

    // ---- F = kappa G grad U at the points of this lane's x-lines (qy, qz) = (a, b)
    T Fx[LPL][NQ];
    if constexpr (GEOM == kGeomOTF) {
      T Xc[8][3];
#pragma unroll
      for (int v = 0; v < 8; ++v)
#pragma unroll
        for (int d = 0; d < 3; ++d) Xc[v][d] = s_X[wv][slot_on ? slot : 0][v * 3 + d];
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp) {
        const int a = qa_of(rp), b = qb_of(rp);
        CT* const t = lphase(U[rp][0]);
#pragma unroll
        for (int qx = 0; qx < NQ; ++qx) {
          Fx[rp][qx] = T(0);
          if (!q_on(rp)) continue;
          T gx = T(0);
#pragma unroll
          for (int m = 0; m < NQ; ++m) gx += t[OFF_D + qx * NQ + m] * U[rp][m];
          const T gy = Bb[(qx * NQ + a) * NQP + b], gz = Cb[(qx * NQ + a) * NQP + b];
          T Gd[6];
          geometry_G<T>(Xc, t[OFF_QP + qx], t[OFF_QP + a], t[OFF_QP + b],
                        t[OFF_W + qx] * t[OFF_W + a] * t[OFF_W + b], Gd);
          const T kv = valid ? kap : T(0);
          Fx[rp][qx] = kv * (Gd[0] * gx + Gd[1] * gy + Gd[2] * gz);
          Bb[(qx * NQ + a) * NQP + b] = kv * (Gd[1] * gx + Gd[3] * gy + Gd[4] * gz);
          Cb[(qx * NQ + a) * NQP + b] = kv * (Gd[2] * gx + Gd[4] * gy + Gd[5] * gz);
        }
      }
    } else {
      if constexpr (GLDS) {
#pragma unroll
        for (int m = 0; m < GCH; ++m) {
          const int e = (lane + 64 * m) * GW;
          if (e < GE) *reinterpret_cast<GV*>(&s_G[wv][e]) = Gv[m];
        }
        dof_wave_sync();
        if constexpr (EARLY) load_G(j + 1, cell_of(j + 1));
      }
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp) {
        const int a = qa_of(rp), b = qb_of(rp);
        CT* const t = lphase(U[rp][0]);
#pragma unroll
        for (int qx = 0; qx < NQ; ++qx) {
          Fx[rp][qx] = T(0);
          if (!q_on(rp)) continue;
          T gx = T(0);
#pragma unroll
          for (int m = 0; m < NQ; ++m) gx += t[OFF_D + qx * NQ + m] * U[rp][m];
          const T gy = Bb[(qx * NQ + a) * NQP + b], gz = Cb[(qx * NQ + a) * NQP + b];
          T Gd[6];
#pragma unroll
          for (int k = 0; k < 6; ++k) {
            if constexpr (GLDS)
              Gd[k] = s_G[wv][(slot_on ? slot : 0) * 6 * NQ3 + k * NQ3 + qx * NQ2 + sl + 64 * rp];
            else if constexpr (GPREF)
              Gd[k] = Gr[rp][k * NQ + qx];
            else if constexpr (kDofGnt)
              Gd[k] = __builtin_nontemporal_load(&A.G[cell * 6 * NQ3 + k * NQ3 + qx * NQ2 + sl + 64 * rp]);
            else
              Gd[k] = A.G[cell * 6 * NQ3 + k * NQ3 + qx * NQ2 + sl + 64 * rp];
          }
          Fx[rp][qx] = kap * (Gd[0] * gx + Gd[1] * gy + Gd[2] * gz);
          Bb[(qx * NQ + a) * NQP + b] = kap * (Gd[1] * gx + Gd[3] * gy + Gd[4] * gz);
          Cb[(qx * NQ + a) * NQP + b] = kap * (Gd[2] * gx + Gd[4] * gy + Gd[5] * gz);
        }
      }
      if constexpr (EARLY && GPREF && !GLDS) load_G(j + 1, cell_of(j + 1));
    }
    dof_wave_sync();

    // ---- transposed gradient: y / z lines by the transposed lanes (in place:
    // every line is read whole before it is rewritten, lines are disjoint)
#pragma unroll
    for (int rp = 0; rp < LPL; ++rp) {
      if (!q_on(rp)) continue;
      const int a = qa_of(rp), b = qb_of(rp);
      T in[NQ], o[NQ];
#pragma unroll
      for (int m = 0; m < NQ; ++m) in[m] = Bb[(a * NQ + m) * NQP + b];
      CT* const t = lphase(in[0]);  // dphi1 columns for both lines
#pragma unroll
      for (int qy = 0; qy < NQ; ++qy) {
        T s = T(0);
#pragma unroll
        for (int m = 0; m < NQ; ++m) s += t[OFF_D + m * NQ + qy] * in[m];
        o[qy] = s;
      }
#pragma unroll
      for (int qy = 0; qy < NQ; ++qy) Bb[(a * NQ + qy) * NQP + b] = o[qy];
#pragma unroll
      for (int m = 0; m < NQ; ++m) in[m] = Cb[(a * NQ + b) * NQP + m];
#pragma unroll
      for (int qz = 0; qz < NQ; ++qz) {
        T s = T(0);
#pragma unroll
        for (int m = 0; m < NQ; ++m) s += t[OFF_D + m * NQ + qz] * in[m];
        o[qz] = s;
      }
#pragma unroll
      for (int qz = 0; qz < NQ; ++qz) Cb[(a * NQ + b) * NQP + qz] = o[qz];
    }
    dof_wave_sync();
    T R[LPL][NQ];
#pragma unroll
    for (int rp = 0; rp < LPL; ++rp) {
      const int a = qa_of(rp), b = qb_of(rp);
      CT* const t = lphase(Fx[rp][0]);
#pragma unroll
      for (int qx = 0; qx < NQ; ++qx) {
        T s = q_on(rp) ? Bb[(qx * NQ + a) * NQP + b] + Cb[(qx * NQ + a) * NQP + b] : T(0);
#pragma unroll
        for (int m = 0; m < NQ; ++m) s += t[OFF_D + m * NQ + qx] * Fx[rp][m];
        R[rp][qx] = s;
      }
    }

    // ---- transposed interpolation: x (quad lanes), y (mixed), z (nodal lanes)
    T ye[ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) ye[k] = T(0);
    if constexpr (IDENT) {
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp) {
        if (!q_on(rp)) continue;
#pragma unroll
        for (int qx = 0; qx < NQ; ++qx) Ab[(qx * NQ + qa_of(rp)) * NQP + qb_of(rp)] = R[rp][qx];
      }
      dof_wave_sync();
      if (r_nod) {
#pragma unroll
        for (int k = 0; k < ND; ++k) ye[k] = Ab[(ni * NQ + nj) * NQP + k];
      }
    } else {
#pragma unroll
      for (int rp = 0; rp < LPL; ++rp) {
        if (!q_on(rp)) continue;
        CT* const t = lphase(R[rp][0]);
#pragma unroll
        for (int i = 0; i < ND; ++i) {
          T s = T(0);
#pragma unroll
          for (int qx = 0; qx < NQ; ++qx) s += t[qx * ND + i] * R[rp][qx];
          Ab[(i * NQ + qa_of(rp)) * NQP + qb_of(rp)] = s;
        }
      }
      dof_wave_sync();
#pragma unroll
      for (int rp = 0; rp < (ND * NQ + 63) / 64; ++rp) {
        const int l = sl + 64 * rp, mi = l / NQ, mq = l % NQ;
        if (slot_on && l < ND * NQ) {  // mixed lane (i, qz)
          T in[NQ];
#pragma unroll
          for (int qy = 0; qy < NQ; ++qy) in[qy] = Ab[(mi * NQ + qy) * NQP + mq];
          CT* const t = lphase(in[0]);
#pragma unroll
          for (int j = 0; j < ND; ++j) {
            T s = T(0);
#pragma unroll
            for (int qy = 0; qy < NQ; ++qy) s += t[qy * ND + j] * in[qy];
            Bb[(mi * NQ + j) * NQP + mq] = s;
          }
        }
      }
      dof_wave_sync();
      if (r_nod) {
        T in[NQ];
#pragma unroll
        for (int qz = 0; qz < NQ; ++qz) in[qz] = Bb[(ni * NQ + nj) * NQP + qz];
        CT* const t = lphase(in[0]);
#pragma unroll
        for (int k = 0; k < ND; ++k) {
          T s = T(0);
#pragma unroll
          for (int qz = 0; qz < NQ; ++qz) s += t[qz * ND + k] * in[qz];
          ye[k] = s;
        }
      }
    }

    // ---- A_e p_e of every cell to LDS in local-dof order (k fastest)
    dof_wave_sync();  // every lane has read the last stage's buffer
    if (r_nod) {
#pragma unroll
      for (int k = 0; k < ND; ++k) Cb[(ni * ND + nj) * ND + k] = ye[k];
    }

    // ---- advance the pipeline: the next cell's gathers and G, the dofs of
    // the one after (issued before this cell's atomics, which need no wait)
    if constexpr (!EARLY) {
      dof_wave_sync();  // the id ring entry of j + 1 / j + 2 is visible
      const int cn = cell_of(j + 1), cnn = cell_of(j + 2);
      gather(dn, vn, j + 1, cn, gc);
      load_G(j + 1, cn);
      load_dofs(j + 2, dc);
      load_verts(cnn, vc);
      cell_cur = cn;
    }

    // ---- element role: the element dot p_e . (A_e p_e) and the scatter-add
    // of the non-Dirichlet dofs; consecutive lanes add to consecutive local
    // dofs, so on a mesh whose z-lines are numbered contiguously a
    // wave-instruction carries ND-dof runs instead of one dof per lane (float
    // atomics execute as 64-B memory-side requests: MI355X_MICROARCH.md,
    // "Global float atomics")
    if constexpr (ZMERGE && !WGMERGE) {
      // two cells per wave with 4-dof z-lines (Q3): the wave's cells are
      // consecutive in the launch list, i.e. z-neighbours on a lexicographic
      // mesh, so each z-line of cell 0 ends at the dof where cell 1's begins.
      // Where the scatter targets say so (per line, any mesh), the two lines
      // are added as ONE 7-dof run with the shared dof summed first: 16 runs
      // of 56 bytes per cell pair instead of 32 runs of 32 bytes, i.e. fewer
      // 64-byte memory-side atomic requests (and one atomic per shared dof).
      // Lines that do not meet take the spare lanes 112..127 for cell 1's
      // first dof.
      int* const tg = reinterpret_cast<int*>(s_buf[wv][0][1]);  // Bb: free since the last sync
#pragma unroll
      for (int r = 0; r < RE; ++r) {
        const T v = s_buf[wv][r][2][lane];
        if constexpr (MODE == kDofCG) {
          if (dsc[r] >= 0) pap += static_cast<double>(ue[r]) * static_cast<double>(v);
        }
        tg[64 * r + lane] = dsc[r];
      }
      dof_wave_sync();
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const int q = lane + 64 * r;
        int t;
        T v;
        if (q < 112) {
          const int l = q / 7, m = q - (q / 7) * 7;  // line, position in the 7-dof run
          if (m < 3) {
            t = tg[l * 4 + m];
            v = s_buf[wv][0][2][l * 4 + m];
          } else if (m == 3) {  // the shared dof: cell 1's part joins when the lines meet
            t = tg[l * 4 + 3];
            const bool meet = t == tg[64 + l * 4];
            v = s_buf[wv][0][2][l * 4 + 3] + (meet ? s_buf[wv][1][2][l * 4] : T(0));
          } else {
            t = tg[64 + l * 4 + m - 3];
            v = s_buf[wv][1][2][l * 4 + m - 3];
          }
        } else {
          const int l = q - 112;  // cell 1's first dof of line l when the lines do not meet
          t = tg[l * 4 + 3] == tg[64 + l * 4] ? -1 : tg[64 + l * 4];
          v = s_buf[wv][1][2][l * 4];
        }
        if (t >= 0) atomicAdd(A.y + t, v);
      }
    } else if constexpr (WGMERGE) {
      // the workgroup's cells of this iteration are consecutive in the launch
      // list (wave w, slot s: list entry c_beg + CPW w + s + STEP j), i.e. a
      // z-run of cells on a lexicographic mesh: every z-line goes out as one
      // run through them, each junction's shared dof summed first when the
      // scatter targets say the lines meet (per line and junction, so any
      // mesh stays correct; a junction that does not meet gives the next
      // cell's first dof to an extra entry).  One run of NC (ND - 1) + 1 dofs
      // per line instead of NC runs of ND: fewer 64-byte memory-side atomic
      // requests, one atomic per shared dof.
      int* const tg = reinterpret_cast<int*>(s_buf[wv][0][1]);  // Bb: free since the last sync
#pragma unroll
      for (int r = 0; r < RE; ++r) {
        if (lane + 64 * r < NE) {
          if constexpr (MODE == kDofCG) {
            if (dsc[r] >= 0)
              pap += static_cast<double>(ue[r]) *
                     static_cast<double>(s_buf[wv][e_slot(r)][2][e_loc(r)]);
          }
          tg[lane + 64 * r] = dsc[r];  // slot s's entries at s ND^3
        }
      }
      __syncthreads();
      constexpr int W4 = S::WAVES * CPW, RL = W4 * (ND - 1) + 1, NXL = W4 - 1;  // run / extras per line
      constexpr int NLN = ND * ND, NB = NLN * (RL + NXL);
      // cell c of the iteration: wave c / CPW, slot c % CPW
      auto tgt = [&](int c, int e) {
        return reinterpret_cast<const int*>(s_buf[c / CPW][0][1])[(c % CPW) * ND3 + e];
      };
      auto val = [&](int c, int e) { return s_buf[c / CPW][c % CPW][2][e]; };
#pragma unroll 1
      for (int q = tid; q < NB; q += S::NT) {
        int t;
        T v;
        if (q < NLN * RL) {
          const int l = q / RL, m = q - (q / RL) * RL;
          // position m of the run: cell w = m / (ND - 1), its dof k = m % (ND - 1),
          // except the last cell's last dof (m = RL - 1)
          const int w = m < RL - 1 ? m / (ND - 1) : W4 - 1;
          const int k = m < RL - 1 ? m - w * (ND - 1) : ND - 1;
          t = tgt(w, l * ND + k);
          v = val(w, l * ND + k);
          if (k == 0 && w > 0) {
            // a junction: this entry carries the previous cell's last dof
            // (summed with ours when they meet); ours alone goes out as an
            // extra entry otherwise
            const int tp = tgt(w - 1, l * ND + ND - 1);
            const T vp = val(w - 1, l * ND + ND - 1);
            v = tp == t ? vp + v : vp;
            t = tp;
          }
        } else {
          const int q2 = q - NLN * RL, l = q2 / NXL, w = q2 - (q2 / NXL) * NXL + 1;
          const int tn = tgt(w, l * ND);  // cell w's first dof when the junction does not meet
          t = tgt(w - 1, l * ND + ND - 1) == tn ? -1 : tn;
          v = val(w, l * ND);
        }
        if (t >= 0) atomicAdd(A.y + t, v);
      }
      __syncthreads();  // every wave's buffers are read before the next cell reuses them
    } else {
#pragma unroll
      for (int r = 0; r < RE; ++r) {
        if (lane + 64 * r < NE && dsc[r] >= 0) {
          const T v = s_buf[wv][e_slot(r)][2][e_loc(r)];
          if constexpr (MODE == kDofCG) pap += static_cast<double>(ue[r]) * static_cast<double>(v);
          atomicAdd(A.y + dsc[r], v);
        }
      }
    }
    dof_wave_sync();  // the next cell reuses the wave's buffers
  };
  for (int j = 0; j < nit; j += 2) {
    iter(j, dA, dB, vA, vB);
    if (j + 1 < nit) iter(j + 1, dB, dA, vB, vA);
  }
  // zero this block's slice of the other y buffer (after the cell loop, so
  // the stores never sit in front of a wait for the pipeline's loads)
  if constexpr (MODE == kDofCG) {
    if (A.yz) {
      constexpr int W = 16 / sizeof(T);
      typedef T ZV __attribute__((ext_vector_type(16 / sizeof(T))));
      const int64_t nv = A.nz / W, per = (nv + nblk - 1) / nblk;
      const int64_t v0 = static_cast<int64_t>(ob) * per, v1 = v0 + per < nv ? v0 + per : nv;
      for (int64_t v = v0 + tid; v < v1; v += S::NT)
        __builtin_nontemporal_store(ZV(0), reinterpret_cast<ZV*>(A.yz + v * W));
      if (ob == 0)
        for (int64_t i = nv * W + tid; i < A.nz; i += S::NT) A.yz[i] = T(0);
    }
    const double t = block_sum(pap, s_red);
    if (tid == 0) A.partials[bid] = t;
  }
}

#include "lap_dofmfma.h"

// Which operator kernel the dofmap launches take in FP64 where both exist
// (nd <= 8, nq <= 8): the MFMA one (lap_dofmfma.h) or the line-per-lane VALU
// one above.  BDX_DOFMAP_MFMA=1 / 0 forces it (A/B builds and tests); unset:
// kDofMfmaDefault(nq).  bdx_dofmap_set_mfma() overrides both (-1: back to
// the environment / default).
extern "C" int bdx_dofmap_set_mfma(int mode);
int bdx_dofmap_mfma_mode();
// Round 6, same box, bench.py --kernel dofmap --geometry stored, GDoF/s (VALU
// / MFMA): Q3 14.47 / 10.74, Q6 22.79 / 21.31 (profiles/r6_dofmap_mfma.md):
// the VALU kernel stays the default.
constexpr bool kDofMfmaDefault(int nq) { return nq < 0; }

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

// Writer designation: the first occurrence (in launch order: the cell list
// `cells`, position p = list index * ND^3 + local dof) of every dof.
static __global__ void __launch_bounds__(256)
    dofmap_first_kernel(const int* __restrict__ cells, int ncl, const int* __restrict__ cdofs,
                        int nd3, unsigned pos0, unsigned* __restrict__ first) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(ncl) * nd3) return;
  const int64_t li = t / nd3;
  const int loc = static_cast<int>(t - li * nd3);
  const int d = cdofs[static_cast<int64_t>(cells[li]) * nd3 + loc] & 0x7fffffff;
  atomicMin(first + d, pos0 + static_cast<unsigned>(t));
}
static __global__ void __launch_bounds__(256)
    dofmap_mark_kernel(const int* __restrict__ cells, int ncl, int* __restrict__ cdofs, int nd3,
                       unsigned pos0, const unsigned* __restrict__ first) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(ncl) * nd3) return;
  const int64_t li = t / nd3;
  const int loc = static_cast<int>(t - li * nd3);
  int* e = cdofs + static_cast<int64_t>(cells[li]) * nd3 + loc;
  const int d = *e & 0x7fffffff;
  *e = (first[d] == pos0 + static_cast<unsigned>(t)) ? (d | static_cast<int>(0x80000000u)) : d;
}

// Vectors per thread and pass of dofmap_cg_update_kernel (below).
constexpr int kDofUpdU = 4;

// CG update of the dofmap path: alpha = s[rn] / s[pap]; r -= alpha y over
// every local dof, r.r over the owned ones, y = 0 for the next operator
// (ZERO; the native runtime's y ping-pong leaves that to the next operator
// launch, DofArgs::yz).
// 16-byte vectors (and W flag bytes); block 0 takes the tail.  Non-temporal
// r / y loads and stores (a pure stream): update pass Q3 2.29 -> 2.00 ms, Q6
// 3.07 -> 2.74, +1.5 % / +2-4 % GDoF/s same box (profiles/r4_update_pass_ab.txt).
// Round 5: U vectors per thread per pass of the grid-stride loop, every load
// of a pass issued before any arithmetic (the tiled update pass's form,
// fused_common.hip): with one vector per thread and pass the loop kept a
// single 16-byte r / y pair in flight per thread and ran 1.56 ms on one box
// and 2.17 ms on another at Q3 (profiles/r5_dofmap_update.md).
template <typename T, int U, bool ZERO>
__global__ void __launch_bounds__(256)
    dofmap_cg_update_kernel(int64_t n, const unsigned char* __restrict__ flags, T* __restrict__ r,
                            T* __restrict__ y, const double* __restrict__ scal, int rn_slot,
                            int pap_slot, double* __restrict__ partials) {
  __shared__ double lds[16];
  const T alpha = static_cast<T>(scal[rn_slot] / scal[pap_slot]);
  constexpr int W = 16 / sizeof(T);
  typedef T V __attribute__((ext_vector_type(W)));
  typedef unsigned char F __attribute__((ext_vector_type(W)));
  double acc = 0.0;
  const int64_t nv = n / W;
  const int64_t stride = static_cast<int64_t>(gridDim.x) * (256 * U);
  for (int64_t vb = static_cast<int64_t>(blockIdx.x) * (256 * U) + threadIdx.x; vb < nv;
       vb += stride) {
    V vr[U], vy[U];
    F fl[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = vb + u * 256;
      if (v < nv) {
        vr[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(r + v * W));
        vy[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(y + v * W));
        fl[u] = *reinterpret_cast<const F*>(flags + v * W);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = vb + u * 256;
      if (v >= nv) break;
      const V rn = vr[u] - alpha * vy[u];
      __builtin_nontemporal_store(rn, reinterpret_cast<V*>(r + v * W));
      if constexpr (ZERO) __builtin_nontemporal_store(V(0), reinterpret_cast<V*>(y + v * W));
#pragma unroll
      for (int w = 0; w < W; ++w)
        if (fl[u][w] & 2u) acc += static_cast<double>(rn[w]) * static_cast<double>(rn[w]);
    }
  }
  if (blockIdx.x == 0) {
    for (int64_t i = nv * W + threadIdx.x; i < n; i += blockDim.x) {
      const T rn = r[i] - alpha * y[i];
      r[i] = rn;
      if constexpr (ZERO) y[i] = T(0);
      if (flags[i] & 2u) acc += static_cast<double>(rn) * static_cast<double>(rn);
    }
  }
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// x += (s[num] / s[den]) p over every local dof (the lagged x update's flush)
template <typename T>
__global__ void __launch_bounds__(256)
    dofmap_xflush_kernel(int64_t n, T* __restrict__ x, const T* __restrict__ p,
                         const double* __restrict__ scal, int num, int den) {
  const T a = static_cast<T>(scal[num] / scal[den]);
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * blockDim.x)
    x[i] += a * p[i];
}

constexpr int kDofMaxBlocks = 16384;  // partials per launch (<= bdx_hip_partials_size / 2)

// Blocks of a launch over ncl cells: whole waves of cells per block, at most
// kDofMaxBlocks blocks (each marches a contiguous chunk of the cell list).
template <int NQ>
inline int dofmap_blocks(int ncl, int* cells_per_block) {
  constexpr int step = DofShape<NQ>::WAVES * DofShape<NQ>::CPW;
  int64_t nb = (static_cast<int64_t>(ncl) + step - 1) / step;
  int64_t cpb = step;
  if (nb > kDofMaxBlocks) {
    cpb = ((static_cast<int64_t>(ncl) + kDofMaxBlocks - 1) / kDofMaxBlocks + step - 1) / step * step;
    nb = (ncl + cpb - 1) / cpb;
  }
  *cells_per_block = static_cast<int>(cpb);
  return static_cast<int>(nb);
}

template <typename T, int ND, int NQ>
int launch_dofmap(int geom, int mode, DofArgs<T> a, int* nblocks, hipStream_t st) {
  *nblocks = 0;
  if (a.ncl <= 0) return 0;
  const int nb = dofmap_blocks<NQ>(a.ncl, &a.cells_per_block);
  *nblocks = nb;
  constexpr int NT = DofShape<NQ>::NT;
  if constexpr (sizeof(T) == 8 && ND <= 8 && NQ <= 8) {
    const int mm = bdx_dofmap_mfma_mode();
    if (mm == 1 || (mm < 0 && kDofMfmaDefault(NQ))) {
      static_assert(DofMfmaShape<ND, NQ>::NT == NT && NT == 256, "block shape of the VALU kernel");
#define BDX_DM(G, M) lap_dofmfma_kernel<ND, NQ, G, M><<<nb, NT, 0, st>>>(a)
      if (geom == kGeomStored)
        (mode == kDofCG) ? BDX_DM(kGeomStored, kDofCG) : BDX_DM(kGeomStored, kDofAction);
      else
        (mode == kDofCG) ? BDX_DM(kGeomOTF, kDofCG) : BDX_DM(kGeomOTF, kDofAction);
#undef BDX_DM
      return static_cast<int>(hipGetLastError());
    }
  }
#define BDX_DL(G, M) lap_dofmap_kernel<T, ND, NQ, G, M><<<nb, NT, 0, st>>>(a)
  if (geom == kGeomStored)
    (mode == kDofCG) ? BDX_DL(kGeomStored, kDofCG) : BDX_DL(kGeomStored, kDofAction);
  else
    (mode == kDofCG) ? BDX_DL(kGeomOTF, kDofCG) : BDX_DL(kGeomOTF, kDofAction);
#undef BDX_DL
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

// apply: mode 0 = action (u -> y += A u), 1 = CG operator (u = r); returns the
// number of p.Ap partials written at partials (CG) in *nblocks.
#define BDX_DOFMAP_API(T, SUF)                                                                    \
  extern "C" int bdx_dofmap_apply_yz_##SUF(                                                       \
      int, int, int, int, const T*, const int*, int, int64_t, const int*, const int*, const T*,   \
      const unsigned char*, const T*, double, const T*, const T*, const T*, T*, T*, T*, T*,       \
      const double*, int, int, int, int, double*, int*, hipStream_t);                             \
  extern "C" int bdx_dofmap_cg_update_z_##SUF(int64_t, const unsigned char*, T*, T*,              \
                                              const double*, int, int, double*, int*, int,        \
                                              hipStream_t);                                       \
  extern "C" int bdx_dofmap_apply_##SUF(                                                          \
      int P, int nq, int geom, int mode, const T* tab, const int* cells, int ncl, int64_t nvec,   \
      const int* cdofs, const int* cverts, const T* coords, const unsigned char* flags,           \
      const T* G, double kappa, const T* kc, const T* u, const T* pold, T* pnew, T* x, T* y,      \
      const double* scal, int beta_num, int beta_den, int xa_num, int xa_den, double* partials,   \
      int* nblocks, hipStream_t st) {                                                             \
    return bdx_dofmap_apply_yz_##SUF(P, nq, geom, mode, tab, cells, ncl, nvec, cdofs, cverts,     \
                                     coords, flags, G, kappa, kc, u, pold, pnew, x, y, nullptr,   \
                                     scal, beta_num, beta_den, xa_num, xa_den, partials, nblocks, \
                                     st);                                                         \
  }                                                                                               \
  extern "C" int bdx_dofmap_apply_yz_##SUF(                                                       \
      int P, int nq, int geom, int mode, const T* tab, const int* cells, int ncl, int64_t nvec,   \
      const int* cdofs, const int* cverts, const T* coords, const unsigned char* flags,           \
      const T* G, double kappa, const T* kc, const T* u, const T* pold, T* pnew, T* x, T* y,      \
      T* yz, const double* scal, int beta_num, int beta_den, int xa_num, int xa_den,              \
      double* partials, int* nblocks, hipStream_t st) {                                           \
    DofArgs<T> a{cells, ncl, 0, nvec, cdofs, cverts, coords, flags, G, tab,                       \
                 static_cast<T>(kappa), kc, u, pold, pnew, x, y, scal, beta_num, beta_den,        \
                 xa_num, xa_den, partials, yz, yz ? nvec : 0};                                    \
    if (nvec * static_cast<int64_t>(sizeof(T)) >= 0xfffffff0LL)                                   \
      return static_cast<int>(hipErrorInvalidValue);                                              \
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
  }                                                                                               \
  extern "C" int bdx_dofmap_cg_update_##SUF(int64_t n, const unsigned char* flags, T* r, T* y,    \
                                            const double* scal, int rn_slot, int pap_slot,        \
                                            double* partials, int* nblocks, hipStream_t st) {     \
    return bdx_dofmap_cg_update_z_##SUF(n, flags, r, y, scal, rn_slot, pap_slot, partials,        \
                                        nblocks, 1, st);                                          \
  }                                                                                               \
  extern "C" int bdx_dofmap_cg_update_z_##SUF(int64_t n, const unsigned char* flags, T* r, T* y,  \
                                              const double* scal, int rn_slot, int pap_slot,      \
                                              double* partials, int* nblocks, int zero_y,         \
                                              hipStream_t st) {                                   \
    const int64_t want = (n / (16 / static_cast<int64_t>(sizeof(T))) + 256 * kDofUpdU - 1) /      \
                         (256 * kDofUpdU);                                                        \
    const int g = static_cast<int>(want < kDofMaxBlocks ? (want > 0 ? want : 1) : kDofMaxBlocks); \
    if (zero_y)                                                                                   \
      dofmap_cg_update_kernel<T, kDofUpdU, true>                                                  \
          <<<g, 256, 0, st>>>(n, flags, r, y, scal, rn_slot, pap_slot, partials);                 \
    else                                                                                          \
      dofmap_cg_update_kernel<T, kDofUpdU, false>                                                 \
          <<<g, 256, 0, st>>>(n, flags, r, y, scal, rn_slot, pap_slot, partials);                 \
    *nblocks = g;                                                                                 \
    return static_cast<int>(hipGetLastError());                                                   \
  }                                                                                               \
  extern "C" int bdx_dofmap_xflush_##SUF(int64_t n, T* x, const T* p, const double* scal,         \
                                         int num, int den, hipStream_t st) {                      \
    const int64_t want = (n + 1023) / 1024;                                                       \
    const int g = static_cast<int>(want < kDofMaxBlocks ? (want > 0 ? want : 1) : kDofMaxBlocks); \
    dofmap_xflush_kernel<T><<<g, 256, 0, st>>>(n, x, p, scal, num, den);                          \
    return static_cast<int>(hipGetLastError());                                                   \
  }

#define BDX_DOFMAP_CASE(T, PP)                                                                    \
  case PP * 16 + PP + 1:                                                                          \
    return launch_dofmap<T, PP + 1, PP + 1>(geom, mode, a, nblocks, st);                          \
  case PP * 16 + PP + 2:                                                                          \
    return launch_dofmap<T, PP + 1, PP + 2>(geom, mode, a, nblocks, st);
