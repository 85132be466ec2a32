// Device BLAS-1, CG vector updates, halo pack/unpack (gfx950).
//
// Replaces the reference's Thrust calls (src/vector.hpp:151-292,
// src/cg.hpp:21-79) and pack/unpack kernels (src/vector.hpp:31-62).
// Differences by design:
//   * every reduction is device-resident: per-block partials + one
//     fixed-order final pass into a float64 scalar slot (deterministic, no
//     host round trip); the all-reduce then runs on that device scalar;
//   * the CG scalars (alpha, beta) are formed on the device from those slots;
//   * x/r updates and the r.r reduction are one fused pass;
//   * reductions and updates walk the owned sub-box of the local lattice
//     one z-row per wave (rows are 128-byte aligned by the storage pitch).
#include "bdx_common.h"

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

struct RowSpace {
  int64_t L1, ld;       // storage strides
  int64_t o0, o1, o2;   // owned extents
};

__device__ __forceinline__ int64_t row_base(const RowSpace& s, int64_t row) {
  const int64_t i = row / s.o1, j = row - i * s.o1;
  return (i * s.L1 + j) * s.ld;
}

// Fused dot-product kernel: per-block partial sums of a.b (deterministic order).
template <typename T>
__global__ void __launch_bounds__(kBlock)
    dot_rows_kernel(RowSpace s, const T* __restrict__ a, const T* __restrict__ b,
                    double* __restrict__ partials) {
  __shared__ double lds[16];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nrows = s.o0 * s.o1;
  double acc = 0.0;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wid; row < nrows;
       row += static_cast<int64_t>(gridDim.x) * kWaves) {
    const int64_t base = row_base(s, row);
    for (int64_t k = lane; k < s.o2; k += 64)
      acc += static_cast<double>(a[base + k]) * static_cast<double>(b[base + k]);
  }
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// Fixed-order sum of partials into out[slot] (single block).
__global__ void __launch_bounds__(kBlock)
    reduce_partials_kernel(const double* __restrict__ partials, int n,
                           double* __restrict__ out, int slot) {
  __shared__ double lds[16];
  double acc = 0.0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) acc += partials[i];
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) out[slot] = t;
}

// CG: alpha = s[rn] / s[pap];  x += alpha p;  r -= alpha y;  partial r.r
template <typename T>
__global__ void __launch_bounds__(kBlock)
    cg_update_kernel(RowSpace s, T* __restrict__ x, T* __restrict__ r,
                     const T* __restrict__ p, const T* __restrict__ y,
                     const double* __restrict__ scal, int rn_slot, int pap_slot,
                     double* __restrict__ partials) {
  __shared__ double lds[16];
  const T alpha = static_cast<T>(scal[rn_slot] / scal[pap_slot]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nrows = s.o0 * s.o1;
  double acc = 0.0;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wid; row < nrows;
       row += static_cast<int64_t>(gridDim.x) * kWaves) {
    const int64_t base = row_base(s, row);
    for (int64_t k = lane; k < s.o2; k += 64) {
      const int64_t i = base + k;
      x[i] = x[i] + alpha * p[i];
      const T rn = r[i] - alpha * y[i];
      r[i] = rn;
      acc += static_cast<double>(rn) * static_cast<double>(rn);
    }
  }
  const double t = block_sum(acc, lds);
  if (threadIdx.x == 0) partials[blockIdx.x] = t;
}

// p = beta p + r with beta = s[num] / s[den] (owned rows).
template <typename T>
__global__ void __launch_bounds__(kBlock)
    p_update_kernel(RowSpace s, T* __restrict__ p, const T* __restrict__ r,
                    const double* __restrict__ scal, int num, int den) {
  const T beta = static_cast<T>(scal[num] / scal[den]);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nrows = s.o0 * s.o1;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wid; row < nrows;
       row += static_cast<int64_t>(gridDim.x) * kWaves) {
    const int64_t base = row_base(s, row);
    for (int64_t k = lane; k < s.o2; k += 64) p[base + k] = beta * p[base + k] + r[base + k];
  }
}

// out = alpha x + y over owned rows (reference axpy, src/vector.hpp:228-240).
template <typename T>
__global__ void __launch_bounds__(kBlock)
    axpy_kernel(RowSpace s, T* __restrict__ out, T alpha, const T* __restrict__ x,
                const T* __restrict__ y) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int64_t nrows = s.o0 * s.o1;
  for (int64_t row = static_cast<int64_t>(blockIdx.x) * kWaves + wid; row < nrows;
       row += static_cast<int64_t>(gridDim.x) * kWaves) {
    const int64_t base = row_base(s, row);
    for (int64_t k = lane; k < s.o2; k += 64) out[base + k] = alpha * x[base + k] + y[base + k];
  }
}

// ------------------------------------------------------------- halo boxes
// Box table in device memory: per box {lo0,lo1,lo2, e0,e1,e2, offset} (int64).
constexpr int kBoxFields = 7;

// MODE 0 pack, 1 unpack (assign), 2 unpack (add).  `only` >= 0 restricts the
// pass to one box: the owned lower-face boxes overlap on edges/corners (a dof
// there receives partial sums from up to 7 neighbours), so the add-unpack runs
// box by box -- race-free and in a fixed order.
// Storage index of lattice node (i, j, k): the lattice layout or the tiled
// one of the CG runtime (bdx_lattice.h, tsy != 0).
struct VecIdx {
  int64_t L1, ld, tsy, tsz, tntz, tcol;
  __device__ __forceinline__ int64_t operator()(int64_t i, int64_t j, int64_t k) const {
    if (tsy) return ((j / tsy) * tntz + k / tsz) * tcol + (i * tsy + j % tsy) * tsz + k % tsz;
    return (i * L1 + j) * ld + k;
  }
};

// Pack / unpack of the halo boxes (see the box table above).
template <typename T, int MODE>
__global__ void __launch_bounds__(kBlock)
    box_copy_kernel(T* __restrict__ vec, VecIdx vi,
                    const int64_t* __restrict__ boxes, int nboxes, int64_t total,
                    T* __restrict__ buf, int only = -1) {
  int64_t t0 = 0, t1 = total;
  if (only >= 0) {
    t0 = boxes[only * kBoxFields + 6];
    t1 = only + 1 < nboxes ? boxes[(only + 1) * kBoxFields + 6] : total;
  }
  for (int64_t t = t0 + static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; t < t1;
       t += static_cast<int64_t>(gridDim.x) * kBlock) {
    int b = only >= 0 ? only : 0;
    while (only < 0 && b + 1 < nboxes && boxes[(b + 1) * kBoxFields + 6] <= t) ++b;
    const int64_t* bx = boxes + b * kBoxFields;
    const int64_t o = t - bx[6];
    const int64_t e1 = bx[4], e2 = bx[5];
    const int64_t k = o % e2, j = (o / e2) % e1, i = o / (e1 * e2);
    const int64_t v = vi(bx[0] + i, bx[1] + j, bx[2] + k);
    if constexpr (MODE == 0)
      buf[t] = vec[v];
    else if constexpr (MODE == 1)
      vec[v] = buf[t];
    else
      vec[v] += buf[t];
  }
}

// Lattice layout <-> tiled layout of one vector, every node of the local
// lattice (owned and ghost).  dir 0: tiled[t(i,j,k)] = lat[l(i,j,k)]; 1: back.
template <typename T>
__global__ void __launch_bounds__(kBlock)
    layout_convert_kernel(int dir, VecIdx lat, VecIdx til, int64_t L0, int64_t L1v,
                          int64_t L2, T* __restrict__ a, T* __restrict__ t) {
  const int64_t n = L0 * L1v * L2;
  for (int64_t e = static_cast<int64_t>(blockIdx.x) * kBlock + threadIdx.x; e < n;
       e += static_cast<int64_t>(gridDim.x) * kBlock) {
    // e enumerates the tiled order (tile, x, ly, lz) of valid nodes would need
    // divisions by run-time tile sizes; enumerate lattice order instead (the
    // lattice side then streams, the tiled side moves in 8..16-node runs)
    const int64_t k = e % L2, r = e / L2, j = r % L1v, i = r / L1v;
    if (BDX_OOB(til(i, j, k), til.tsy ? ((L1v - 1) / til.tsy + 1) * til.tntz * til.tcol : n,
                "layout convert"))
      continue;
    if (dir == 0)
      t[til(i, j, k)] = a[lat(i, j, k)];
    else
      a[lat(i, j, k)] = t[til(i, j, k)];
  }
}

constexpr int kFeTiles = 16;  // tiles per flush_export block along z

// End of a CG call on tiled storage: the lagged x terms folded into the tiled
// iterate and the result exported to the lattice layout in one pass
// (t += a1 p1 [+ a2 p2]; lat = t) instead of a flush pass per term plus a
// conversion pass.  a = scal[num] / scal[den], den < 0: scal[num] itself.
// One block per (x-plane, tile row, group of kFeTiles tiles along z): it
// reads the group's tiled chunks ([tile][x][ly][lz], contiguous) in 16-byte
// vectors, stages the result in LDS in lattice order and writes the group's
// z-rows contiguously, so both sides stream (the element-wise forms ran at
// 2-3.7 TB/s: 64-bit divisions per element, then 96-byte lattice runs).
// Every access is non-temporal (+0.2 % on the 20-step Q3 / Q6 runs that
// carry one flush each, profiles/r4_update_pass_ab.txt).
template <typename T>
__global__ void __launch_bounds__(kBlock)
    flush_export_kernel(int64_t L0, int64_t L1, int64_t L2, int64_t ld, int tsy, int tsz,
                        int tntz, int ngz, T* __restrict__ a, T* __restrict__ t,
                        const T* __restrict__ p1, const T* __restrict__ p2,
                        const double* __restrict__ scal, int num1, int den1, int num2, int den2,
                        int p2mask) {
  extern __shared__ __attribute__((aligned(16))) unsigned char fe_lds[];
  T* const sv = reinterpret_cast<T*>(fe_lds);  // [tsy][kFeTiles * tsz]
  const T a1 = static_cast<T>(den1 < 0 ? scal[num1] : scal[num1] / scal[den1]);
  const T a2 = p2 ? static_cast<T>(den2 < 0 ? scal[num2] : scal[num2] / scal[den2]) : T(0);
  constexpr int W = 16 / sizeof(T);
  typedef T V __attribute__((ext_vector_type(W)));
  // block -> (x, tile row ty, z group g); x fastest
  const int64_t bidx = blockIdx.x;
  const int64_t x = bidx % L0, rest = bidx / L0;
  const int g = static_cast<int>(rest % ngz), ty = static_cast<int>(rest / ngz);
  const int tz0 = g * kFeTiles;
  const int nt = tntz - tz0 < kFeTiles ? tntz - tz0 : kFeTiles;  // tiles of this group
  const int C = tsy * tsz, CV = C / W;                              // chunk, vectors per chunk
  const int pitch = kFeTiles * tsz;                                 // LDS row pitch
  const int64_t cbase = (static_cast<int64_t>(ty) * tntz + tz0) * L0 + x;  // chunk index of tile tz0
  for (int q = threadIdx.x; q < nt * CV; q += kBlock) {
    const int tl = q / CV, e = (q - tl * CV) * W;
    const int64_t off = (cbase + static_cast<int64_t>(tl) * L0) * C + e;
    V vt = __builtin_nontemporal_load(reinterpret_cast<const V*>(t + off));
    vt += a1 * __builtin_nontemporal_load(reinterpret_cast<const V*>(p1 + off));
    // p2mask: the tile colours ((ty + tz) & 1) with the second term pending
    if (p2 && ((p2mask >> ((ty + tz0 + tl) & 1)) & 1))
      vt += a2 * __builtin_nontemporal_load(reinterpret_cast<const V*>(p2 + off));
    if (!(p2mask & 4)) __builtin_nontemporal_store(vt, reinterpret_cast<V*>(t + off));
    int ly = e / tsz, lz = e - ly * tsz;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      sv[ly * pitch + tl * tsz + lz] = vt[w];
      if (++lz == tsz) {
        lz = 0;
        ++ly;
      }
    }
  }
  __syncthreads();
  const int64_t k0 = static_cast<int64_t>(tz0) * tsz;
  const int64_t kend = (k0 + nt * tsz < L2) ? k0 + nt * tsz : L2;
  const int nk = static_cast<int>(kend - k0);
  const int64_t j0 = static_cast<int64_t>(ty) * tsy;
  const int nj = static_cast<int>((j0 + tsy <= L1) ? tsy : L1 - j0);
  for (int r = threadIdx.x; r < nj * nk; r += kBlock) {
    const int ly = r / nk, kk = r - ly * nk;
    __builtin_nontemporal_store(sv[ly * pitch + kk], a + (x * L1 + j0 + ly) * ld + k0 + kk);
  }
}

template <typename T>
int box_copy_vi(int mode, T* vec, VecIdx vi, const int64_t* boxes, int nboxes, int64_t total,
                T* buf, hipStream_t st) {
  if (total <= 0) return 0;
  const int64_t g64 = (total + kBlock - 1) / kBlock;
  const int g = static_cast<int>(g64 < 4096 ? g64 : 4096);
  if (mode == 0) {
    box_copy_kernel<T, 0><<<g, kBlock, 0, st>>>(vec, vi, boxes, nboxes, total, buf);
  } else if (mode == 1) {
    box_copy_kernel<T, 1><<<g, kBlock, 0, st>>>(vec, vi, boxes, nboxes, total, buf);
  } else {  // add: boxes may overlap (edges/corners), one launch per box
    for (int b = 0; b < nboxes; ++b)
      box_copy_kernel<T, 2><<<g, kBlock, 0, st>>>(vec, vi, boxes, nboxes, total, buf, b);
  }
  return static_cast<int>(hipGetLastError());
}

int grid_for_rows(int64_t nrows) {
  const int64_t want = (nrows + kWaves - 1) / kWaves;
  return static_cast<int>(want < 2048 ? (want > 0 ? want : 1) : 2048);
}

}  // namespace

extern "C" {

int bdx_hip_partials_size() { return 65536; }  // >= kPartialsCap (fused_common.hip)

// Fixed-order reduction of n per-block partials into out[slot].
int bdx_reduce_partials(const double* partials, int n, double* out, int slot,
                        hipStream_t st) {
  reduce_partials_kernel<<<1, kBlock, 0, st>>>(partials, n, out, slot);
  return static_cast<int>(hipGetLastError());
}

#define BDX_BLAS_API(T, SUF)                                                  \
  int bdx_dot_##SUF(int64_t L1, int64_t ld, int64_t o0, int64_t o1, int64_t o2, \
                    const T* a, const T* b, double* partials, double* out,    \
                    int slot, hipStream_t st) {                               \
    RowSpace s{L1, ld, o0, o1, o2};                                           \
    const int g = grid_for_rows(o0 * o1);                                     \
    dot_rows_kernel<T><<<g, kBlock, 0, st>>>(s, a, b, partials);              \
    reduce_partials_kernel<<<1, kBlock, 0, st>>>(partials, g, out, slot);     \
    return static_cast<int>(hipGetLastError());                               \
  }                                                                           \
  int bdx_cg_update_##SUF(int64_t L1, int64_t ld, int64_t o0, int64_t o1,     \
                          int64_t o2, T* x, T* r, const T* p, const T* y,     \
                          double* scal, int rn_slot, int pap_slot,            \
                          int out_slot, double* partials, hipStream_t st) {   \
    RowSpace s{L1, ld, o0, o1, o2};                                           \
    const int g = grid_for_rows(o0 * o1);                                     \
    cg_update_kernel<T><<<g, kBlock, 0, st>>>(s, x, r, p, y, scal, rn_slot,   \
                                              pap_slot, partials);            \
    reduce_partials_kernel<<<1, kBlock, 0, st>>>(partials, g, scal, out_slot); \
    return static_cast<int>(hipGetLastError());                               \
  }                                                                           \
  int bdx_p_update_##SUF(int64_t L1, int64_t ld, int64_t o0, int64_t o1,      \
                         int64_t o2, T* p, const T* r, const double* scal,    \
                         int num, int den, hipStream_t st) {                  \
    RowSpace s{L1, ld, o0, o1, o2};                                           \
    p_update_kernel<T><<<grid_for_rows(o0 * o1), kBlock, 0, st>>>(s, p, r,    \
                                                                  scal, num,  \
                                                                  den);       \
    return static_cast<int>(hipGetLastError());                               \
  }                                                                           \
  int bdx_axpy_##SUF(int64_t L1, int64_t ld, int64_t o0, int64_t o1,          \
                     int64_t o2, T* out, double alpha, const T* x, const T* y, \
                     hipStream_t st) {                                        \
    RowSpace s{L1, ld, o0, o1, o2};                                           \
    axpy_kernel<T><<<grid_for_rows(o0 * o1), kBlock, 0, st>>>(                \
        s, out, static_cast<T>(alpha), x, y);                                 \
    return static_cast<int>(hipGetLastError());                               \
  }                                                                           \
  int bdx_box_copy_##SUF(int mode, T* vec, int64_t L1, int64_t ld,            \
                         const int64_t* boxes, int nboxes, int64_t total,     \
                         T* buf, hipStream_t st) {                            \
    const VecIdx vi{L1, ld, 0, 0, 0, 0};                                      \
    return box_copy_vi<T>(mode, vec, vi, boxes, nboxes, total, buf, st);      \
  }                                                                           \
  /* the same on a lattice descriptor (lattice or tiled storage) */           \
  int bdx_box_copy_lat_##SUF(int mode, T* vec, const int64_t* latd,           \
                             const int64_t* boxes, int nboxes, int64_t total, \
                             T* buf, hipStream_t st) {                        \
    const BdxLattice L = BdxLattice::from(latd);                              \
    const VecIdx vi{L.L[1], L.ld, L.tsy, L.tsz, L.tntz, L.tcol};              \
    return box_copy_vi<T>(mode, vec, vi, boxes, nboxes, total, buf, st);      \
  }                                                                           \
  /* lattice <-> tiled copy of a vector (dir 0: to tiled, 1: back) */         \
  int bdx_layout_convert_##SUF(int dir, const int64_t* latd_tiled, T* lat,    \
                               T* tiled, hipStream_t st) {                    \
    const BdxLattice L = BdxLattice::from(latd_tiled);                        \
    if (!L.tsy) return static_cast<int>(hipErrorInvalidValue);                \
    const VecIdx lv{L.L[1], L.ld, 0, 0, 0, 0};                                \
    const VecIdx tv{L.L[1], L.ld, L.tsy, L.tsz, L.tntz, L.tcol};              \
    const int64_t n = L.L[0] * L.L[1] * L.L[2];                               \
    const int64_t g64 = (n + kBlock - 1) / kBlock;                            \
    const int g = static_cast<int>(g64 < 65536 ? g64 : 65536);                \
    layout_convert_kernel<T><<<g, kBlock, 0, st>>>(dir, lv, tv, L.L[0], L.L[1], \
                                                   L.L[2], lat, tiled);       \
    return static_cast<int>(hipGetLastError());                               \
  }                                                                           \
  /* tiled x += a1 p1 [+ a2 p2], exported to the lattice layout (p2 may be */ \
  /* null; p2mask bits 0-1: tile colours that take it, bit 2: export only, */ \
  /* the tiled iterate keeps its lagged terms pending) */                     \
  int bdx_flush_export_##SUF(const int64_t* latd_tiled, T* lat, T* tiled,     \
                             const T* p1, const T* p2, const double* scal,    \
                             int num1, int den1, int num2, int den2,          \
                             int p2mask, hipStream_t st) {                    \
    const BdxLattice L = BdxLattice::from(latd_tiled);                        \
    if (!L.tsy || (L.tsy * L.tsz * static_cast<int64_t>(sizeof(T))) % 16)    \
      return static_cast<int>(hipErrorInvalidValue);                          \
    const int64_t nty = (L.L[1] - 1) / L.tsy + 1;                             \
    const int ngz = static_cast<int>((L.tntz + kFeTiles - 1) / kFeTiles);     \
    const int64_t nblk = L.L[0] * nty * ngz;                                  \
    const size_t lds = static_cast<size_t>(L.tsy) * kFeTiles * L.tsz * sizeof(T); \
    if (nblk <= 0) return 0;                                                  \
    if (nblk > 0x7fffffffLL || lds > 64 * 1024)                               \
      return static_cast<int>(hipErrorInvalidValue);                          \
    flush_export_kernel<T><<<static_cast<unsigned>(nblk), kBlock, lds, st>>>( \
        L.L[0], L.L[1], L.L[2], L.ld, static_cast<int>(L.tsy),                \
        static_cast<int>(L.tsz), static_cast<int>(L.tntz), ngz, lat, tiled,   \
        p1, p2, scal, num1, den1, num2, den2, p2mask);                        \
    return static_cast<int>(hipGetLastError());                               \
  }

BDX_BLAS_API(double, f64)
BDX_BLAS_API(float, f32)

}  // extern "C"
