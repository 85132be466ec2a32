// Common device-side helpers for the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

#include "bdx_lattice.h"

#define BDX_CHECK(expr)                                                     \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) return static_cast<int>(_e);                      \
  } while (0)

constexpr int kMaxNd = 8;
constexpr int kMaxNq = 9;
// packed 1D-table capacity of every fused kernel family (the largest: fused
// v1 TAB for nd=8, nq=9 at the f32 pitch); the runtime copies this many
// entries
constexpr int kFusedTabMax = 2 * 9 * 12 + 9 * 8 + 8 * 12;

enum { kGeomStored = 0, kGeomOTF = 1 };

// FP64 MFMA operand / accumulator vectors (v_mfma_f64_16x16x4f64: 4 results per lane)
typedef double bdx_f64x4 __attribute__((ext_vector_type(4)));
typedef double bdx_f64x2 __attribute__((ext_vector_type(2)));
// FP32 (v_mfma_f32_16x16x4_f32: 4 results per lane, exact f32 fma chain)
typedef float bdx_f32x4 __attribute__((ext_vector_type(4)));

// 16 x 16 x 4 MFMA in T: A / B one T per lane (lane l: A[l & 15][k = l >> 4],
// B[k = l >> 4][l & 15]); C / D 4 per lane.
template <typename T> struct BdxMfmaAcc;
template <> struct BdxMfmaAcc<double> { using type = bdx_f64x4; };
template <> struct BdxMfmaAcc<float> { using type = bdx_f32x4; };
__device__ __forceinline__ bdx_f64x4 bdx_mfma16x4(double a, double b, bdx_f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ bdx_f32x4 bdx_mfma16x4(float a, float b, bdx_f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// The result row of accumulator element r in lane group g (= lane >> 4) is
// g + 4 r for FP64 and 4 g + r for FP32 (cdna_hip_programming.md §3).  Code
// written for the FP64 map runs unchanged in FP32 when the row-carrying
// operand's row m is taken from source row bdx_mfma_row<T>(m): then element r
// of lane group g holds source row g + 4 r in both precisions.
template <typename T>
__device__ __forceinline__ constexpr int bdx_mfma_row(int m) {
  return sizeof(T) == 8 ? m : (m >> 2) + 4 * (m & 3);
}

// Value of lane (l ^ 8) within each 16-lane row (DPP row_ror:8 = swap of the
// row halves; two VALU moves per double, no LDS).
__device__ __forceinline__ double dpp_row_ror8(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x128, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x128, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}

// Lagged x update of the fused5 CG (Fused2Args::xmode, bits 4-5 of the apply
// entry points' mode word, set by runtime.hip): one term per iteration, save
// alpha_prev only, or fold two terms; the saved alpha's slot of the CG scalars.
enum { kXSingle = 0, kXSave = 1, kXPair = 2 };
constexpr int kScalXSave = 3;  // and kScalXSave + 1 (alternate iterations)

// Debug builds (BDX_DEBUG=1: `python -m benchmark_dolfinx_amd.ops.build
// --variant debug=-DBDX_DEBUG=1`, loaded with BDX_HIP_LIB) turn on
// device-side checks of the operator kernels' LDS and global index paths; a
// failing check prints the expression and aborts the process (HIP device
// assert) instead of reading or writing out of bounds.  Release builds compile
// them out.
#ifndef BDX_DEBUG
#define BDX_DEBUG 0
#endif
#if BDX_DEBUG
// report (do not trap: a trapped wave would take the queue down with it)
#define BDX_DASSERT(c) \
  ((c) ? (void)0 : (void)printf("[bdx ASSERT] %s:%d %s\n", __FILE__, __LINE__, #c))
// out-of-range global offset: print the first few offenders, skip the access
#define BDX_OOB(off, n, tag)                                                        \
  (((off) < 0 || (off) >= (n))                                                      \
       ? (printf("[bdx OOB] %s off=%lld n=%lld block=%d thread=%d\n", tag,          \
                 static_cast<long long>(off), static_cast<long long>(n),            \
                 static_cast<int>(blockIdx.x), static_cast<int>(threadIdx.x)),      \
          true)                                                                     \
       : false)
#else
#define BDX_DASSERT(c) ((void)0)
#define BDX_OOB(off, n, tag) false
#endif

// Streamed vectors (read or written once per CG iteration; every vector is
// far larger than the 256 MiB Infinity Cache) use the default cache policy:
// non-temporal loads AND stores measured 36-37 % SLOWER on all three headline configs (Q3 46.7 ->
// 29.9, Q6 44.6 -> 28.9, Q6-FP32 59.3 -> 35.1 GDoF/s, profiles/r2_nt_ab.md):
// the x-march writes 96-byte row segments, and only the default policy lets
// L2 merge neighbouring tiles' segments into whole lines before write-back.
// (Round 4: whole 16-byte-vector streams that no other tile re-reads -- the
// update passes, fused5's own-node staging loads and stores -- do gain from
// __builtin_nontemporal_*, see profiles/r4_fused5_nt_ab.txt; these helpers
// keep the default policy for the element-wise accesses.)
template <typename T>
__device__ __forceinline__ T ld_stream(const T* p) {
  return *p;
}
template <typename T>
__device__ __forceinline__ void st_stream(T* p, T v) {
  *p = v;
}

// 1D operator tables, passed by value as a kernel argument (< 1.5 KiB).
template <typename T>
struct OpTables {
  T phi0[kMaxNq * kMaxNd];    // nq x nd, interpolation to quadrature points
  T dphi1[kMaxNq * kMaxNq];   // nq x nq, derivative on quadrature nodes
  T wts[kMaxNq];              // 1D quadrature weights
  T qpts[kMaxNq];             // 1D quadrature points on [0, 1]
  int identity;               // phi0 == I (collocated: qmode 0 + GLL)
};

template <typename T>
inline OpTables<T> make_op_tables(int nd, int nq, const double* phi0,
                                  const double* dphi1, const double* wts,
                                  const double* qpts, int identity) {
  OpTables<T> t{};
  for (int q = 0; q < nq; ++q) {
    for (int i = 0; i < nd; ++i) t.phi0[q * nd + i] = static_cast<T>(phi0[q * nd + i]);
    for (int j = 0; j < nq; ++j) t.dphi1[q * nq + j] = static_cast<T>(dphi1[q * nq + j]);
    t.wts[q] = static_cast<T>(wts[q]);
    t.qpts[q] = static_cast<T>(qpts[q]);
  }
  t.identity = identity;
  return t;
}

// Trilinear geometry at reference point (s, t, u) of the cell with vertices
// X (v = 4a+2b+c): returns det J and writes G = w adj(J) adj(J)^T / det J.
template <typename T>
__device__ __forceinline__ T geometry_G(const T (*X)[3], T s, T t, T u, T w,
                                        T G[6]) {
  T J[3][3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    // d x_i / d s = sum over the 4 edges in s of (x_hi - x_lo) * bilinear(t, u)
    const T e00 = X[4][i] - X[0][i], e01 = X[5][i] - X[1][i];
    const T e10 = X[6][i] - X[2][i], e11 = X[7][i] - X[3][i];
    J[i][0] = (1 - t) * ((1 - u) * e00 + u * e01) + t * ((1 - u) * e10 + u * e11);
    const T f00 = X[2][i] - X[0][i], f01 = X[3][i] - X[1][i];
    const T f10 = X[6][i] - X[4][i], f11 = X[7][i] - X[5][i];
    J[i][1] = (1 - s) * ((1 - u) * f00 + u * f01) + s * ((1 - u) * f10 + u * f11);
    const T g00 = X[1][i] - X[0][i], g01 = X[3][i] - X[2][i];
    const T g10 = X[5][i] - X[4][i], g11 = X[7][i] - X[6][i];
    J[i][2] = (1 - s) * ((1 - t) * g00 + t * g01) + s * ((1 - t) * g10 + t * g11);
  }
  const T K00 = J[1][1] * J[2][2] - J[1][2] * J[2][1];
  const T K01 = J[0][2] * J[2][1] - J[0][1] * J[2][2];
  const T K02 = J[0][1] * J[1][2] - J[0][2] * J[1][1];
  const T K10 = J[1][2] * J[2][0] - J[1][0] * J[2][2];
  const T K11 = J[0][0] * J[2][2] - J[0][2] * J[2][0];
  const T K12 = J[0][2] * J[1][0] - J[0][0] * J[1][2];
  const T K20 = J[1][0] * J[2][1] - J[1][1] * J[2][0];
  const T K21 = J[0][1] * J[2][0] - J[0][0] * J[2][1];
  const T K22 = J[0][0] * J[1][1] - J[0][1] * J[1][0];
  const T det = J[0][0] * K00 + J[0][1] * K10 + J[0][2] * K20;
  const T sc = w / det;
  G[0] = (K00 * K00 + K01 * K01 + K02 * K02) * sc;
  G[1] = (K10 * K00 + K11 * K01 + K12 * K02) * sc;
  G[2] = (K20 * K00 + K21 * K01 + K22 * K02) * sc;
  G[3] = (K10 * K10 + K11 * K11 + K12 * K12) * sc;
  G[4] = (K20 * K10 + K21 * K11 + K22 * K12) * sc;
  G[5] = (K20 * K20 + K21 * K21 + K22 * K22) * sc;
  return det;
}

// Wave64 sum reduction via DPP-friendly shuffles.
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// Block sum (blockDim.x multiple of 64, <= 1024); result valid in thread 0.
template <typename T>
__device__ __forceinline__ T block_sum(T v, T* lds /* >= 16 */) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  T s = 0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int w = 0; w < nw; ++w) s += lds[w];
  }
  return s;
}
