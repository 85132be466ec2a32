// Fused-kernel helpers: tile query, table packing, the interface-partials
// finalize pass and the fused2/3 CG update.
#include <cstdlib>
#include "lap_fused3.h"

// Packed 1D tables of the fused kernel (layout: FusedShape::OFF_*), written
// to host memory `out` (which the caller uploads).  Returns the count.
template <typename T, int ND, int NQ>
int pack_tables(const double* phi0, const double* dphi1, T* out) {
  using S = FusedShape<T, ND, NQ, 1, 1>;
  if (!out) return kFusedTabMax;
  for (int i = 0; i < kFusedTabMax; ++i) out[i] = T(0);
  for (int q = 0; q < NQ; ++q)
    for (int m = 0; m < NQ; ++m) {
      out[S::OFF_DR + q * S::XP + m] = static_cast<T>(dphi1[q * NQ + m]);
      out[S::OFF_DC + m * S::XP + q] = static_cast<T>(dphi1[q * NQ + m]);
    }
  for (int q = 0; q < NQ; ++q)
    for (int i = 0; i < ND; ++i) {
      out[S::OFF_PR + q * S::NP + i] = static_cast<T>(phi0[q * ND + i]);
      out[S::OFF_PC + i * S::XP + q] = static_cast<T>(phi0[q * ND + i]);
    }
  return kFusedTabMax;
}


// kPartialsCap is the partials capacity every caller provides
// (bdx_hip_partials_size).  The flat update pass wants a non-persistent grid (a persistent 8192/16384-block
// grid-stride version measured 1.70 ms vs 1.52 at Q3); its up to 65280 block
// partials are summed in two fixed-order stages (256 slices into the last 256
// slots of the partials buffer, then one block): deterministic like the rest.
constexpr int kPartialsCap = 65536, kStage1 = 256;
constexpr int kUpdGrid = kPartialsCap - kStage1;  // update pass grid cap
constexpr int kUpdU = 2;  // vectors per thread of the tiled update pass
constexpr bool kUpdPre = true;  // cg_update_tiled_pre_kernel (interface loads issued up front)

// CG update of the fused2..5 paths: alpha = s[rn] / s[pap];
//   r -= alpha (y + interface partials);  partial r.r
// The tile-interface partials (YB/ZB/CB) are folded here on the fly instead of
// by a separate finalize pass over y (same sum as fused_finalize_kernel).
// x is not touched: its update x += alpha p is lagged into the next fused
// launch (staging reads p there anyway) and flushed by bdx_xflush at the end.
// Flat pass (a row-per-wave kernel measured slower): the owned rows j < o1 of an
// x-plane are one contiguous block of o1 * ld elements (row pitch ld, a
// multiple of 16 elements: no 16-byte vector straddles two rows), so the pass
// runs as a plain stream -- one chunk of 256 threads x 2 vectors per block,
// blocks up to the partials capacity (grid-stride beyond), both loads of a
// thread in flight before any arithmetic.  Same arithmetic per element as the
// row kernel above (fold, r update, r.r); columns k >= o2 are left as read.
template <typename T>
__global__ void __launch_bounds__(256)
    cg_update_flat_kernel(int64_t L1, int64_t ld, int64_t o0, int64_t o1, int64_t o2,
                          int64_t Lz, T* __restrict__ r, const T* __restrict__ y,
                          const T* __restrict__ yb, const T* __restrict__ zb,
                          const T* __restrict__ cb, int nty, int ntz, int sy, int sz,
                          const double* __restrict__ scal, int rn_slot, int pap_slot,
                          double* __restrict__ partials) {
  __shared__ double lds[16];
  const T alpha = static_cast<T>(scal[rn_slot] / scal[pap_slot]);
  constexpr int W = 16 / sizeof(T), U = 2, CH = 256 * U;
  typedef T V __attribute__((ext_vector_type(W)));
  const int ldv = static_cast<int>(ld / W);
  const int nvp = static_cast<int>(o1) * ldv;
  const int nch = (nvp + CH - 1) / CH;
  const int64_t nwork = o0 * nch;
  const float inv_sz = 1.0f / static_cast<float>(sz);
  const float inv_ldv = 1.0f / static_cast<float>(ldv);
  double acc = 0.0;
  for (int64_t c = blockIdx.x; c < nwork; c += gridDim.x) {
    const int64_t i = c / nch;
    const int v0 = static_cast<int>(c - i * nch) * CH + static_cast<int>(threadIdx.x) * U;
    const int64_t pbase = i * L1 * ld;
    V vy[U], vr[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (v0 + u < nvp) {
        vy[u] = ld_stream(reinterpret_cast<const V*>(y + pbase + static_cast<int64_t>(v0 + u) * W));
        vr[u] = ld_stream(reinterpret_cast<const V*>(r + pbase + static_cast<int64_t>(v0 + u) * W));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int v = v0 + u;
      if (v >= nvp) continue;
      int j = static_cast<int>(static_cast<float>(v) * inv_ldv);
      if (j * ldv > v) --j;
      if ((j + 1) * ldv <= v) ++j;
      const int k0 = (v - j * ldv) * W;
      const int tyy = j / sy;
      const int yrow = (j - tyy * sy == 0 && tyy >= 1 && tyy < nty) ? tyy - 1 : -1;
#pragma unroll
      for (int e = 0; e < W; ++e) {
        const int k = k0 + e;
        if (k >= o2) continue;
        T t = vy[u][e];
        if (yrow >= 0) t += yb[(i * (nty - 1) + yrow) * Lz + k];
        int zq = static_cast<int>(static_cast<float>(k) * inv_sz);
        if (zq * sz > k) --zq;
        if ((zq + 1) * sz <= k) ++zq;
        if (zq * sz == k && zq >= 1 && zq < ntz) {
          t += zb[(i * (ntz - 1) + zq - 1) * L1 + j];
          if (yrow >= 0) t += cb[(i * (nty - 1) + yrow) * (ntz - 1) + zq - 1];
        }
        const T rn = vr[u][e] - alpha * t;
        vr[u][e] = rn;
        acc += static_cast<double>(rn) * static_cast<double>(rn);
      }
      st_stream(reinterpret_cast<V*>(r + pbase + static_cast<int64_t>(v) * W), vr[u]);
    }
  }
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// The r update of the tiled storage (bdx_lattice.h, tsy != 0): the same
// arithmetic per node as the flat kernel above, in the layout's element order.
// Chunks of tsy * tsz elements are one tile's patch of one x-plane; a vector
// of W elements never straddles a chunk (tsy * tsz * sizeof(T) is a multiple
// of 16 bytes, checked by the host wrapper).  ROW: tsz is a multiple of W as
// well, so a vector lies in one z-row of its chunk and its position, owned
// mask and y-interface term are resolved once per vector instead of once per
// element.  Used for FP32 (4 elements per 16-byte vector): Q6 FP32 update
// 1.58 -> 1.41 ms, +3 % GDoF/s; FP64 keeps the per-element form (ROW: Q3
// update 1.555 -> 1.583 ms), same box (scripts/r3_updrow.sh).  Blocks stay in
// launch order: an XCD-aware remap (contiguous slabs per XCD) made the pass
// 8-40 % slower (Q6 FP64 update 2.54 -> 3.54 ms, scripts/r3_updxcd.sh).
// Round 4: U = 2 vectors per thread with both loads in flight, and the chunk ->
// (tile, x) split in 32-bit arithmetic (it was two 64-bit divisions per
// vector): update pass Q3 1.79 -> 1.54 ms, Q6 2.76 -> 2.59, Q6 FP32 1.58 ->
// 1.37, same box (U = 1: 1.57 at Q3, U = 4: no gain;
// profiles/r4_update_pass_ab.txt).  The pass's r / y loads and r stores are
// non-temporal (whole 16-byte vectors, full lines; unlike the operator's
// march, nothing here relies on L2 merging partial rows): update Q3 1.53 ->
// 1.46 ms, Q6 FP64 2.50 -> 2.30, +1.6-1.8 % GDoF/s same box (same file).
template <typename T, bool ROW, int U>
__global__ void __launch_bounds__(256)
    cg_update_tiled_kernel(int64_t L0, int64_t L1, int64_t Lz, int tsy, int tsz, int tntz,
                           int64_t o0, int64_t o1, int64_t o2, int64_t nvec, T* __restrict__ r,
                           const T* __restrict__ y, const T* __restrict__ yb,
                           const T* __restrict__ zb, const T* __restrict__ cb, int nty, int ntz,
                           const double* __restrict__ scal, int rn_slot, int pap_slot,
                           double* __restrict__ partials) {
  __shared__ double lds[16];
  const T alpha = static_cast<T>(scal[rn_slot] / scal[pap_slot]);
  constexpr int W = 16 / sizeof(T);
  typedef T V __attribute__((ext_vector_type(W)));
  const int64_t ch = static_cast<int64_t>(tsy) * tsz;
  const double inv_ch = 1.0 / static_cast<double>(ch);
  const float inv_l0 = 1.0f / static_cast<float>(L0), inv_tntz = 1.0f / static_cast<float>(tntz);
  const float inv_tsz = 1.0f / static_cast<float>(tsz);
  const int l0 = static_cast<int>(L0);
  double acc = 0.0;
  for (int64_t vb = static_cast<int64_t>(blockIdx.x) * (256 * U) + threadIdx.x; vb < nvec;
       vb += static_cast<int64_t>(gridDim.x) * (256 * U)) {
    // U vectors per thread, 256 apart (each load coalesced over the block), all
    // loads in flight before the index math and the arithmetic
    V vyu[U], vru[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = vb + u * 256;
      if (v < nvec) {
        vyu[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(y + v * W));
        vru[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(r + v * W));
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = vb + u * 256;
      if (v >= nvec) break;
      const int64_t e0 = v * W;
      int64_t c = static_cast<int64_t>(static_cast<double>(e0) * inv_ch);  // chunk
      if (c * ch > e0) --c;
      if ((c + 1) * ch <= e0) ++c;
      // chunk -> (tile, x): 32-bit (chunks < 2^31), float reciprocals + exact fix-ups
      const int ci = static_cast<int>(c);
      int blk = static_cast<int>(static_cast<float>(ci) * inv_l0);
      while (blk * l0 > ci) --blk;
      while ((blk + 1) * l0 <= ci) ++blk;
      const int x = ci - blk * l0;
      int tY = static_cast<int>(static_cast<float>(blk) * inv_tntz);
      while (tY * tntz > blk) --tY;
      while ((tY + 1) * tntz <= blk) ++tY;
      const int tZ = blk - tY * tntz;
      if (x >= o0) continue;
      const int ein = static_cast<int>(e0 - c * ch);
      if (BDX_OOB(e0 + W - 1, nvec * W, "tiled update")) continue;
      // (y, z) of the vector's first element
      int ly = static_cast<int>(static_cast<float>(ein) * inv_tsz);
      if (ly * tsz > ein) --ly;
      if ((ly + 1) * tsz <= ein) ++ly;
      if constexpr (ROW) {
        const int lz0 = ein - ly * tsz;
        const int64_t gy = static_cast<int64_t>(tY) * tsy + ly, gz0 = static_cast<int64_t>(tZ) * tsz + lz0;
        if (gy >= o1 || gz0 >= o2) continue;
        V t = vyu[u];
        V vr = vru[u];
        const int yrow = (ly == 0 && tY >= 1 && tY < nty) ? tY - 1 : -1;
        const int nw = o2 - gz0 < W ? static_cast<int>(o2 - gz0) : W;  // owned elements
        if (yrow >= 0) {
          const T* yr = yb + (x * (nty - 1) + yrow) * Lz + gz0;
#pragma unroll
          for (int w = 0; w < W; ++w)
            if (w < nw) t[w] += yr[w];
        }
        if (lz0 == 0 && tZ >= 1 && tZ < ntz) {
          t[0] += zb[(x * (ntz - 1) + tZ - 1) * L1 + gy];
          if (yrow >= 0) t[0] += cb[(x * (nty - 1) + yrow) * (ntz - 1) + tZ - 1];
        }
#pragma unroll
        for (int w = 0; w < W; ++w) {
          const T rn = vr[w] - alpha * t[w];
          if (w < nw) {
            vr[w] = rn;
            acc += static_cast<double>(rn) * static_cast<double>(rn);
          }
        }
        __builtin_nontemporal_store(vr, reinterpret_cast<V*>(r + e0));
      } else {
        const V vy = vyu[u];
        V vr = vru[u];
        bool any = false;
        // the other elements step along z
        int lz = ein - ly * tsz - 1;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          if (++lz == tsz) {
            lz = 0;
            ++ly;
          }
          const int64_t gy = static_cast<int64_t>(tY) * tsy + ly, gz = static_cast<int64_t>(tZ) * tsz + lz;
          if (gy >= o1 || gz >= o2) continue;
          any = true;
          const int yrow = (ly == 0 && tY >= 1 && tY < nty) ? tY - 1 : -1;
          T t = vy[w];
          if (yrow >= 0) t += yb[(x * (nty - 1) + yrow) * Lz + gz];
          if (lz == 0 && tZ >= 1 && tZ < ntz) {
            t += zb[(x * (ntz - 1) + tZ - 1) * L1 + gy];
            if (yrow >= 0) t += cb[(x * (nty - 1) + yrow) * (ntz - 1) + tZ - 1];
          }
          const T rn = vr[w] - alpha * t;
          vr[w] = rn;
          acc += static_cast<double>(rn) * static_cast<double>(rn);
        }
        if (any) __builtin_nontemporal_store(vr, reinterpret_cast<V*>(r + e0));
      }
    }
  }
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// The tiled r update with the tile-interface partials loaded together with
// the vector's y and r (round 5): in cg_update_tiled_kernel they are loaded
// inside the branches that need them, after the wave has waited for y and r,
// so every vector next to a tile interface (a third of them in FP32 at Q6)
// pays a second memory latency.  Here every load of a pass -- y, r and the
// YB / ZB / CB terms of each element -- is issued first, as range-checked
// buffer loads whose offset is out of range (the load returns 0, no memory
// access) where an element has no such term; the arithmetic follows.  Same
// sums in the same order as cg_update_tiled_kernel.
template <typename T, bool ROW, int U>
__global__ void __launch_bounds__(256)
    cg_update_tiled_pre_kernel(int64_t L0, int64_t L1, int64_t Lz, int tsy, int tsz, int tntz,
                               int64_t o0, int64_t o1, int64_t o2, int64_t nvec, T* __restrict__ r,
                               const T* __restrict__ y, const T* yb, const T* zb, const T* cb,
                               int nty, int ntz, const double* __restrict__ scal, int rn_slot,
                               int pap_slot, double* __restrict__ partials) {
  __shared__ double lds[16];
  const T alpha = static_cast<T>(scal[rn_slot] / scal[pap_slot]);
  constexpr int W = 16 / sizeof(T);
  constexpr int NI = ROW ? W + 2 : 3 * W;  // interface loads per vector
  typedef T V __attribute__((ext_vector_type(W)));
  constexpr unsigned kOOB = 0xfffffff0u;
  auto rsrc = [](const T* ptr, int64_t n) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<T*>(ptr), 0,
                                             static_cast<int>(n * static_cast<int64_t>(sizeof(T))),
                                             0x00020000);
  };
  const auto rs_yb = rsrc(yb, L0 * (nty - 1) * Lz), rs_zb = rsrc(zb, L0 * L1 * (ntz - 1)),
             rs_cb = rsrc(cb, L0 * (nty - 1) * (ntz - 1));
  auto ldb = [](__amdgpu_buffer_rsrc_t rs, unsigned off) -> T {
    if constexpr (sizeof(T) == 8)
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
    else
      return __builtin_bit_cast(T, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 0, 0));
  };
  auto bo = [](bool on, int64_t e) { return on ? static_cast<unsigned>(e * sizeof(T)) : kOOB; };
  const int64_t ch = static_cast<int64_t>(tsy) * tsz;
  const double inv_ch = 1.0 / static_cast<double>(ch);
  const float inv_l0 = 1.0f / static_cast<float>(L0), inv_tntz = 1.0f / static_cast<float>(tntz);
  const float inv_tsz = 1.0f / static_cast<float>(tsz);
  const int l0 = static_cast<int>(L0);
  double acc = 0.0;
  for (int64_t vb = static_cast<int64_t>(blockIdx.x) * (256 * U) + threadIdx.x; vb < nvec;
       vb += static_cast<int64_t>(gridDim.x) * (256 * U)) {
    V vyu[U], vru[U];
    T ia[U][NI];
    int own[U];  // bit w: element w is owned
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = vb + u * 256;
      own[u] = 0;
#pragma unroll
      for (int i = 0; i < NI; ++i) ia[u][i] = T(0);
      if (v >= nvec) continue;
      vyu[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(y + v * W));
      vru[u] = __builtin_nontemporal_load(reinterpret_cast<const V*>(r + v * W));
      const int64_t e0 = v * W;
      int64_t c = static_cast<int64_t>(static_cast<double>(e0) * inv_ch);  // chunk
      if (c * ch > e0) --c;
      if ((c + 1) * ch <= e0) ++c;
      const int ci = static_cast<int>(c);
      int blk = static_cast<int>(static_cast<float>(ci) * inv_l0);
      while (blk * l0 > ci) --blk;
      while ((blk + 1) * l0 <= ci) ++blk;
      const int x = ci - blk * l0;
      int tY = static_cast<int>(static_cast<float>(blk) * inv_tntz);
      while (tY * tntz > blk) --tY;
      while ((tY + 1) * tntz <= blk) ++tY;
      const int tZ = blk - tY * tntz;
      const int ein = static_cast<int>(e0 - c * ch);
      int ly = static_cast<int>(static_cast<float>(ein) * inv_tsz);
      if (ly * tsz > ein) --ly;
      if ((ly + 1) * tsz <= ein) ++ly;
      const bool xin = x < o0 && !BDX_OOB(e0 + W - 1, nvec * W, "tiled update");
      const bool zt = tZ >= 1 && tZ < ntz;
      if constexpr (ROW) {
        const int lz0 = ein - ly * tsz;
        const int64_t gy = static_cast<int64_t>(tY) * tsy + ly, gz0 = static_cast<int64_t>(tZ) * tsz + lz0;
        const bool row = xin && gy < o1;
        const int yrow = (ly == 0 && tY >= 1 && tY < nty) ? tY - 1 : -1;
#pragma unroll
        for (int w = 0; w < W; ++w) own[u] |= (row && gz0 + w < o2) ? 1 << w : 0;
        // the vector's YB terms: one 16-byte load when they lie in one YB row
        // (dword-aligned offsets are allowed; the terms of unowned elements
        // are loaded but not applied), else one load per owned element
        const bool yneed = row && gz0 < o2 && yrow >= 0;
        const int64_t ye = (x * (nty - 1) + yrow) * Lz + gz0;
        if (gz0 + W <= Lz) {
          const V yv = __builtin_bit_cast(V, __builtin_amdgcn_raw_buffer_load_b128(rs_yb, bo(yneed, ye), 0, 0));
#pragma unroll
          for (int w = 0; w < W; ++w) ia[u][w] = yv[w];
        } else {
#pragma unroll
          for (int w = 0; w < W; ++w) ia[u][w] = ldb(rs_yb, bo(yneed && gz0 + w < o2, ye + w));
        }
        const bool z0 = row && gz0 < o2 && lz0 == 0 && zt;
        ia[u][W] = ldb(rs_zb, bo(z0, (x * (ntz - 1) + tZ - 1) * L1 + gy));
        ia[u][W + 1] = ldb(rs_cb, bo(z0 && yrow >= 0, (x * (nty - 1) + yrow) * (ntz - 1) + tZ - 1));
      } else {
        int lz = ein - ly * tsz - 1;
#pragma unroll
        for (int w = 0; w < W; ++w) {
          if (++lz == tsz) {
            lz = 0;
            ++ly;
          }
          const int64_t gy = static_cast<int64_t>(tY) * tsy + ly, gz = static_cast<int64_t>(tZ) * tsz + lz;
          const bool on = xin && gy < o1 && gz < o2;
          own[u] |= on ? 1 << w : 0;
          const int yrow = (ly == 0 && tY >= 1 && tY < nty) ? tY - 1 : -1;
          const bool zf = on && lz == 0 && zt;
          ia[u][3 * w] = ldb(rs_yb, bo(on && yrow >= 0, (x * (nty - 1) + yrow) * Lz + gz));
          ia[u][3 * w + 1] = ldb(rs_zb, bo(zf, (x * (ntz - 1) + tZ - 1) * L1 + gy));
          ia[u][3 * w + 2] = ldb(rs_cb, bo(zf && yrow >= 0, (x * (nty - 1) + yrow) * (ntz - 1) + tZ - 1));
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t v = vb + u * 256;
      if (v >= nvec || !own[u]) continue;
      V vr = vru[u];
#pragma unroll
      for (int w = 0; w < W; ++w) {
        T t = vyu[u][w];
        if constexpr (ROW) {  // the order of cg_update_tiled_kernel: y + YB, + ZB, + CB
          t += ia[u][w];
          if (w == 0) {
            t += ia[u][W];
            t += ia[u][W + 1];
          }
        } else {
          t += ia[u][3 * w];
          t += ia[u][3 * w + 1];
          t += ia[u][3 * w + 2];
        }
        const T rn = vr[w] - alpha * t;
        if (own[u] & (1 << w)) {
          vr[w] = rn;
          acc += static_cast<double>(rn) * static_cast<double>(rn);
        }
      }
      __builtin_nontemporal_store(vr, reinterpret_cast<V*>(r + v * W));
    }
  }
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// x += (s[num] / s[den]) p over the owned rows (flush of the lagged x update).
template <typename T>
__global__ void __launch_bounds__(256)
    xflush_kernel(int64_t L1, int64_t ld, int64_t o0, int64_t o1, int64_t o2, T* __restrict__ x,
                  const T* __restrict__ p, const double* __restrict__ scal, int num, int den) {
  // den < 0: alpha stored directly in scal[num] (kScalXSave, runtime.hip)
  const T alpha = static_cast<T>(den < 0 ? scal[num] : scal[num] / scal[den]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nrows = o0 * o1;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + wid; row < nrows;
       row += static_cast<int64_t>(gridDim.x) * 4) {
    const int64_t i = row / o1, j = row - i * o1;
    const int64_t base = (i * L1 + j) * ld;
    for (int64_t k = lane; k < o2; k += 64) x[base + k] += alpha * p[base + k];
  }
}

// stage 1 of the two-stage sum: block b sums slice b of partials[0, n) into out[b]
__global__ void reduce_partials_slices(const double* __restrict__ partials, int n,
                                       double* __restrict__ out) {
  __shared__ double lds[16];
  const int per = (n + static_cast<int>(gridDim.x) - 1) / static_cast<int>(gridDim.x);
  const int lo = static_cast<int>(blockIdx.x) * per, hi = lo + per < n ? lo + per : n;
  double acc = 0.0;
  for (int i = lo + static_cast<int>(threadIdx.x); i < hi; i += blockDim.x) acc += partials[i];
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) out[blockIdx.x] = t;
}

// Fixed-order sum of the per-tile p.Ap partials into one device scalar slot.
__global__ void reduce_partials_fixed(const double* __restrict__ partials, int n,
                                      double* __restrict__ out, int slot) {
  __shared__ double lds[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) out[slot] = t;
}

static int rows_grid(int64_t nrows) {
  const int64_t want = (nrows + 3) / 4;
  return static_cast<int>(want < 2048 ? (want > 0 ? want : 1) : 2048);
}

extern "C" {

#define BDX_CGI(T, SUF)                                                              \
  int bdx_cg_update_iface_##SUF(const int64_t* latd, const int64_t* own, T* r,      \
                                const T* y, const T* yb, const T* zb, const T* cb,  \
                                int nty, int ntz, int sy, int sz, double* scal,     \
                                int rn_slot, int pap_slot, int out_slot,            \
                                double* partials, hipStream_t st) {                 \
    const BdxLattice lat = BdxLattice::from(latd);                                  \
    int g;                                                                          \
    {                                                             \
      const int64_t nvp = own[1] * (lat.ld * static_cast<int64_t>(sizeof(T)) / 16); \
      const int64_t want = own[0] * ((nvp + 511) / 512);                            \
      g = static_cast<int>(want < kUpdGrid ? (want > 0 ? want : 1) : kUpdGrid); \
      cg_update_flat_kernel<T><<<g, 256, 0, st>>>(lat.L[1], lat.ld, own[0], own[1], \
                                                  own[2], lat.L[2], r, y, yb, zb, cb, \
                                                  nty, ntz, sy, sz, scal, rn_slot,  \
                                                  pap_slot, partials);              \
    }                                                                               \
    if (g > 4 * kStage1) {                                                          \
      double* stage = partials + kPartialsCap - kStage1;                            \
      reduce_partials_slices<<<kStage1, 256, 0, st>>>(partials, g, stage);          \
      reduce_partials_fixed<<<1, 256, 0, st>>>(stage, kStage1, scal, out_slot);     \
    } else {                                                                        \
      reduce_partials_fixed<<<1, 256, 0, st>>>(partials, g, scal, out_slot);        \
    }                                                                               \
    return static_cast<int>(hipGetLastError());                                     \
  }                                                                                 \
  int bdx_xflush_##SUF(const int64_t* latd, const int64_t* own, T* x, const T* p,   \
                       const double* scal, int num, int den, hipStream_t st) {      \
    const BdxLattice lat = BdxLattice::from(latd);                                  \
    xflush_kernel<T><<<rows_grid(own[0] * own[1]), 256, 0, st>>>(                   \
        lat.L[1], lat.ld, own[0], own[1], own[2], x, p, scal, num, den);            \
    return static_cast<int>(hipGetLastError());                                     \
  }
BDX_CGI(double, f64)
BDX_CGI(float, f32)
#undef BDX_CGI

// Tiled-storage variants of the r update and the x flush (latd: the tiled
// descriptor of bdx_lattice.h).
#define BDX_CGT(T, SUF)                                                                         \
  int bdx_cg_update_tiled_##SUF(const int64_t* latd, const int64_t* own, T* r, const T* y,     \
                                const T* yb, const T* zb, const T* cb, int nty, int ntz,       \
                                double* scal, int rn_slot, int pap_slot, int out_slot,         \
                                double* partials, hipStream_t st) {                            \
    const BdxLattice L = BdxLattice::from(latd);                                               \
    if (!L.tsy || (L.tsy * L.tsz * static_cast<int64_t>(sizeof(T))) % 16)                     \
      return static_cast<int>(hipErrorInvalidValue);                                           \
    const int64_t nvec = L.size() / (16 / static_cast<int64_t>(sizeof(T)));                    \
    const int64_t want = (nvec + 256 * kUpdU - 1) / (256 * kUpdU);                             \
    const int g = static_cast<int>(want < kUpdGrid ? (want > 0 ? want : 1) : kUpdGrid); \
    /* interface partials prefetched (byte offsets of the buffers fit 31 bits); the   */      \
    /* plain kernel serves larger blocks (BDX_UPD_PLAIN=1 forces it: the test hook of */      \
    /* tests/test_gpu_runtime.py::test_tiled_update_plain_path_matches)               */      \
    const bool force_plain = std::getenv("BDX_UPD_PLAIN") != nullptr;                         \
    const bool pre = kUpdPre && !force_plain &&                                                \
                     L.L[0] * L.L[1] * (ntz > 1 ? ntz - 1 : 1) * 8 < (1LL << 31) &&            \
                     L.L[0] * (nty > 1 ? nty - 1 : 1) * L.L[2] * 8 < (1LL << 31);              \
    if (pre && sizeof(T) == 4 && L.tsz % 4 == 0)                                               \
      cg_update_tiled_pre_kernel<T, true, kUpdU><<<g, 256, 0, st>>>(                           \
          L.L[0], L.L[1], L.L[2], static_cast<int>(L.tsy), static_cast<int>(L.tsz),            \
          static_cast<int>(L.tntz), own[0], own[1], own[2], nvec, r, y, yb, zb, cb, nty, ntz,  \
          scal, rn_slot, pap_slot, partials);                                                  \
    else if (pre)                                                                              \
      cg_update_tiled_pre_kernel<T, false, kUpdU><<<g, 256, 0, st>>>(                          \
          L.L[0], L.L[1], L.L[2], static_cast<int>(L.tsy), static_cast<int>(L.tsz),            \
          static_cast<int>(L.tntz), own[0], own[1], own[2], nvec, r, y, yb, zb, cb, nty, ntz,  \
          scal, rn_slot, pap_slot, partials);                                                  \
    else if (sizeof(T) == 4 && L.tsz % 4 == 0)                                                 \
      cg_update_tiled_kernel<T, true, kUpdU><<<g, 256, 0, st>>>(                               \
          L.L[0], L.L[1], L.L[2], static_cast<int>(L.tsy), static_cast<int>(L.tsz),            \
          static_cast<int>(L.tntz), own[0], own[1], own[2], nvec, r, y, yb, zb, cb, nty, ntz,  \
          scal, rn_slot, pap_slot, partials);                                                  \
    else                                                                                       \
      cg_update_tiled_kernel<T, false, kUpdU><<<g, 256, 0, st>>>(                              \
          L.L[0], L.L[1], L.L[2], static_cast<int>(L.tsy), static_cast<int>(L.tsz),            \
          static_cast<int>(L.tntz), own[0], own[1], own[2], nvec, r, y, yb, zb, cb, nty, ntz,  \
          scal, rn_slot, pap_slot, partials);                                                  \
    if (g > 4 * kStage1) {                                                                     \
      double* stage = partials + kPartialsCap - kStage1;                                       \
      reduce_partials_slices<<<kStage1, 256, 0, st>>>(partials, g, stage);                     \
      reduce_partials_fixed<<<1, 256, 0, st>>>(stage, kStage1, scal, out_slot);                \
    } else {                                                                                   \
      reduce_partials_fixed<<<1, 256, 0, st>>>(partials, g, scal, out_slot);                   \
    }                                                                                          \
    return static_cast<int>(hipGetLastError());                                                \
  }
BDX_CGT(double, f64)
BDX_CGT(float, f32)
#undef BDX_CGT

// Tile shape (cells in y, z) used by the fused kernel for a given nq.
int bdx_fused_tile(int nq, int* ty, int* tz) {
  switch (nq) {
#define BDX_T(NQ)                 \
  case NQ:                        \
    *ty = TileFor<NQ>::TY;        \
    *tz = TileFor<NQ>::TZ;        \
    return 0;
    BDX_T(2) BDX_T(3) BDX_T(4) BDX_T(5) BDX_T(6) BDX_T(7) BDX_T(8) BDX_T(9)
#undef BDX_T
  }
  return static_cast<int>(hipErrorInvalidValue);
}

#define BDX_FIN(T, SUF)                                                          \
  int bdx_fused_finalize_##SUF(const int64_t* latd, T* y, const T* yb, const T* zb, \
                               const T* cb, int nty, int ntz, int sy, int sz,      \
                               int ghost_only, hipStream_t st) {                   \
    const BdxLattice lat = BdxLattice::from(latd);                                 \
    if (ghost_only) {                                                              \
      const int64_t Lx = lat.L[0], Ly = lat.L[1], Lz = lat.L[2];                   \
      const int64_t xB = lat.gh[0] ? Lx - 1 : Lx;                                  \
      const int64_t n = (lat.gh[0] ? (nty - 1) * Lz + Ly * (ntz - 1) : 0) +        \
                        (lat.gh[1] ? xB * (ntz - 1) : 0) + (lat.gh[2] ? xB * (nty - 1) : 0); \
      if (n <= 0) return 0;                                                        \
      int64_t g = (n + 255) / 256;                                                 \
      if (g > 4096) g = 4096;                                                      \
      fused_finalize_ghost_kernel<T><<<static_cast<unsigned>(g), 256, 0, st>>>(    \
          lat, y, yb, zb, cb, nty, ntz, sy, sz);                                   \
      return static_cast<int>(hipGetLastError());                                  \
    }                                                                              \
    const int64_t n = lat.L[0] * (nty - 1) * lat.L[2] + lat.L[0] * lat.L[1] * (ntz - 1); \
    if (n <= 0) return 0;                                                          \
    int64_t g = (n + 255) / 256;                                                   \
    if (g > 8192) g = 8192;                                                        \
    fused_finalize_kernel<T><<<static_cast<unsigned>(g), 256, 0, st>>>(            \
        lat, y, yb, zb, cb, nty, ntz, sy, sz, 0);                                  \
    return static_cast<int>(hipGetLastError());                                    \
  }

BDX_FIN(double, f64)
BDX_FIN(float, f32)

#define BDX_TABS(T, SUF)                                                           \
  int bdx_fused_tables_##SUF(int nd, int nq, const double* phi0, const double* dphi1, \
                             T* out) {                                             \
    switch (nd * 16 + nq) {                                                        \
      case 2 * 16 + 2: return pack_tables<T, 2, 2>(phi0, dphi1, out);              \
      case 2 * 16 + 3: return pack_tables<T, 2, 3>(phi0, dphi1, out);              \
      case 3 * 16 + 3: return pack_tables<T, 3, 3>(phi0, dphi1, out);              \
      case 3 * 16 + 4: return pack_tables<T, 3, 4>(phi0, dphi1, out);              \
      case 4 * 16 + 4: return pack_tables<T, 4, 4>(phi0, dphi1, out);              \
      case 4 * 16 + 5: return pack_tables<T, 4, 5>(phi0, dphi1, out);              \
      case 5 * 16 + 5: return pack_tables<T, 5, 5>(phi0, dphi1, out);              \
      case 5 * 16 + 6: return pack_tables<T, 5, 6>(phi0, dphi1, out);              \
      case 6 * 16 + 6: return pack_tables<T, 6, 6>(phi0, dphi1, out);              \
      case 6 * 16 + 7: return pack_tables<T, 6, 7>(phi0, dphi1, out);              \
      case 7 * 16 + 7: return pack_tables<T, 7, 7>(phi0, dphi1, out);              \
      case 7 * 16 + 8: return pack_tables<T, 7, 8>(phi0, dphi1, out);              \
      case 8 * 16 + 8: return pack_tables<T, 8, 8>(phi0, dphi1, out);              \
      case 8 * 16 + 9: return pack_tables<T, 8, 9>(phi0, dphi1, out);              \
    }                                                                              \
    return -1;                                                                     \
  }
BDX_TABS(double, f64)
BDX_TABS(float, f32)

#define BDX_TABS3(T, SUF)                                                          \
  int bdx_fused3_tables_##SUF(int nd, int nq, const double* phi0, const double* Dd, \
                              T* out) {                                            \
    switch (nd * 16 + nq) {                                                        \
      case 2 * 16 + 3: return pack_tables3<T, 2, 3>(phi0, Dd, out);                \
      case 3 * 16 + 4: return pack_tables3<T, 3, 4>(phi0, Dd, out);                \
      case 4 * 16 + 5: return pack_tables3<T, 4, 5>(phi0, Dd, out);                \
      case 5 * 16 + 6: return pack_tables3<T, 5, 6>(phi0, Dd, out);                \
      case 6 * 16 + 7: return pack_tables3<T, 6, 7>(phi0, Dd, out);                \
      case 7 * 16 + 8: return pack_tables3<T, 7, 8>(phi0, Dd, out);                \
      case 8 * 16 + 9: return pack_tables3<T, 8, 9>(phi0, Dd, out);                \
    }                                                                              \
    return -1;                                                                     \
  }
BDX_TABS3(double, f64)
BDX_TABS3(float, f32)

}  // extern "C"
