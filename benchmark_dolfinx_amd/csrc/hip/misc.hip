// Geometry precompute (stored-G mode) and CSR SpMV (mat_comp path), gfx950.
//
// geometry_kernel: G[c][k][q] = w_q adj(J) adj(J)^T / det J, the reference's
// layout and maths (geometry_computation_gpu, src/geometry_gpu.hpp:26-132),
// one thread per (cell, quadrature point), vertices read straight from the
// local vertex lattice (no geometry dofmap), 64-bit offsets.
//
// spmv_kernel: y = A x for the assembled local matrix (src/csr.hpp:28-45 is
// one thread per row); here one wave per row with a shuffle reduction so a
// row's ~(2P+1)^3 entries are read coalesced.
#include "bdx_common.h"

namespace {

// Stored geometry: G at every quadrature point in the reference layout.
template <typename T, int NQ>
__global__ void __launch_bounds__(256)
    geometry_kernel(BdxLattice lat, OpTables<T> tb, const T* __restrict__ xv,
                    T* __restrict__ G, int64_t ncells) {
  constexpr int nq3 = NQ * NQ * NQ;
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= ncells * nq3) return;
  const int64_t c = t / nq3;
  const int q = static_cast<int>(t - c * nq3);
  const int64_t cz = c % lat.n[2], cy = (c / lat.n[2]) % lat.n[1],
                cx = c / (lat.n[1] * lat.n[2]);
  T X[8][3];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int cc = 0; cc < 2; ++cc) {
        const int64_t v = lat.vidx(cx + a, cy + b, cz + cc);
#pragma unroll
        for (int d = 0; d < 3; ++d) X[4 * a + 2 * b + cc][d] = xv[3 * v + d];
      }
  const int qx = q / (NQ * NQ), qy = (q / NQ) % NQ, qz = q % NQ;
  T Gd[6];
  geometry_G<T>(X, tb.qpts[qx], tb.qpts[qy], tb.qpts[qz],
                tb.wts[qx] * tb.wts[qy] * tb.wts[qz], Gd);
  T* out = G + c * 6 * nq3 + q;
#pragma unroll
  for (int k = 0; k < 6; ++k) out[k * nq3] = Gd[k];
}

template <typename T>
int launch_geometry(int nq, const BdxLattice& lat, const OpTables<T>& tb,
                    const T* xv, T* G, hipStream_t st) {
  const int64_t ncells = lat.n[0] * lat.n[1] * lat.n[2];
  const int64_t total = ncells * nq * nq * nq;
  const int64_t g = (total + 255) / 256;
  if (g == 0) return 0;
  switch (nq) {
#define BDX_G(NQ)                                                          \
  case NQ:                                                                 \
    geometry_kernel<T, NQ><<<static_cast<unsigned>(g), 256, 0, st>>>(      \
        lat, tb, xv, G, ncells);                                           \
    break;
    BDX_G(2)
    BDX_G(3)
    BDX_G(4)
    BDX_G(5)
    BDX_G(6)
    BDX_G(7)
    BDX_G(8)
    BDX_G(9)
#undef BDX_G
    default:
      return static_cast<int>(hipErrorInvalidValue);
  }
  return static_cast<int>(hipGetLastError());
}

// Wave-per-row CSR SpMV (the reference's assembled-matrix comparison
// operator) over the entry range [beg[row], end[row]) of each row; acc = 1
// adds to y.  Two launches with a column-split matrix give the reference's
// owned-column / ghost-column overlap (src/csr.hpp:203-217).
template <typename T>
__global__ void __launch_bounds__(256)
    spmv_kernel(int64_t nrows, const int64_t* __restrict__ beg, const int64_t* __restrict__ end,
                const int32_t* __restrict__ cols, const T* __restrict__ vals,
                const T* __restrict__ x, T* __restrict__ y, int acc_out) {
  const int lane = threadIdx.x & 63;
  const int64_t row = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int64_t b = beg[row], e = end[row];
  T acc = 0;
  for (int64_t p = b + lane; p < e; p += 64) acc += vals[p] * x[cols[p]];
  acc = wave_sum(acc);
  if (lane == 0) y[row] = acc_out ? y[row] + acc : acc;
}

}  // namespace

extern "C" {

#define BDX_MISC_API(T, SUF)                                                  \
  int bdx_geometry_##SUF(const int64_t* latd, int nq, const double* phi0,     \
                         const double* dphi1, const double* wts,              \
                         const double* qpts, const T* xv, T* G,               \
                         hipStream_t st) {                                    \
    const BdxLattice lat = BdxLattice::from(latd);                            \
    const OpTables<T> tb = make_op_tables<T>(static_cast<int>(lat.P) + 1, nq, \
                                             phi0, dphi1, wts, qpts, 0);      \
    return launch_geometry<T>(nq, lat, tb, xv, G, st);                        \
  }                                                                           \
  int bdx_spmv_##SUF(int64_t nrows, const int64_t* beg, const int64_t* end,    \
                     const int32_t* cols, const T* vals, const T* x, T* y,    \
                     int acc, hipStream_t st) {                               \
    if (nrows <= 0) return 0;                                                 \
    spmv_kernel<T><<<static_cast<unsigned>((nrows + 3) / 4), 256, 0, st>>>(   \
        nrows, beg, end, cols, vals, x, y, acc);                              \
    return static_cast<int>(hipGetLastError());                               \
  }

BDX_MISC_API(double, f64)
BDX_MISC_API(float, f32)

// Device banner (reference get_device_information, src/util.cpp:10-52).
// 1 when the library was built with the device bounds checks (BDX_DEBUG):
// correct numerics, but not a valid timing build.
int bdx_build_debug() { return BDX_DEBUG; }

int bdx_device_info(int dev, char* buf, int buflen) {
  hipDeviceProp_t p;
  hipError_t e = hipGetDeviceProperties(&p, dev);
  if (e != hipSuccess) return static_cast<int>(e);
  snprintf(buf, buflen,
           "Device: %s\n  gcnArch: %s\n  CUs: %d\n  Global memory: %.1f GB\n"
           "  LDS per block: %zu B\n  Warp size: %d\n  Max threads/block: %d\n"
           "  Clock: %.0f MHz\n  L2: %d B\n",
           p.name, p.gcnArchName, p.multiProcessorCount,
           static_cast<double>(p.totalGlobalMem) / 1e9, p.sharedMemPerBlock,
           p.warpSize, p.maxThreadsPerBlock, p.clockRate / 1000.0, p.l2CacheSize);
  return 0;
}

}  // extern "C"
