// Microbenchmark: what the x-march access pattern costs in HBM bandwidth.
//
// The fused operator kernels read and write their vectors as (y, z) tile
// patches of each x-plane: 12 x 12 owned nodes (96-byte row segments at the
// row pitch of the lattice) per plane, one workgroup per tile marching along
// x.  This program times the same bytes moved four ways on a 300 M-double
// vector (the Q3 headline size):
//   stream   : flat grid-stride, 16 B per lane (the roofline reference)
//   march    : lattice layout [x][y][z_pad], tile patches as the operator does
//   tiled    : tile-major layout [ty][tz][x][12][12] (a tile's plane patch is
//              1152 contiguous bytes), same march
// for write-only, read-only and read+write (2R1W: r, p read, p written).
// Occupancy is pinned to the operator's (3 workgroups of 256 per CU) with a
// dummy LDS allocation.  Build: hipcc -O3 --offload-arch=gfx950 march_bw.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

constexpr int TP = 12;        // owned nodes per tile side (4 Q3 cells)
constexpr int NT = 256;       // threads per workgroup
constexpr int LDS_PIN = 48 * 1024;  // 3 workgroups per CU, as fused4

struct Geo {
  int X, Y, Z, ld;            // lattice extents and row pitch (elements)
  int nty, ntz;               // tiles
};

// Lattice offset of (x, y, z) and tile-major offset of the same node.
__device__ __forceinline__ long lat_off(const Geo& g, int x, int y, int z) {
  return (static_cast<long>(x) * g.Y + y) * g.ld + z;
}
__device__ __forceinline__ long tile_off(const Geo& g, int ty, int tz, int x, int ly, int lz) {
  return ((static_cast<long>(ty) * g.ntz + tz) * g.X + x) * (TP * TP) + ly * TP + lz;
}

// mode: 0 write, 1 read, 2 read 2 + write 1.  TILED: tile-major layout.
template <int TILED>
__global__ void __launch_bounds__(NT) march_kernel(Geo g, int mode, double* __restrict__ a,
                                                   const double* __restrict__ b, double* sink) {
  __shared__ double pin[LDS_PIN / 8];
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  const int ty = bid / g.ntz, tz = bid % g.ntz;
  double acc = 0.0;
  // 4 planes per step, every load of a step in flight before any use (the
  // operator keeps one layer = 3 planes of loads in flight)
  constexpr int U = 4;
  const int e = threadIdx.x;
  const bool on = e < TP * TP;
  const int ly = e / TP, lz = e % TP;
  for (int x0 = 0; x0 < g.X; x0 += U) {
    long o[U];
    double va[U], vb[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int x = x0 + u < g.X ? x0 + u : g.X - 1;
      o[u] = TILED ? tile_off(g, ty, tz, x, ly, lz) : lat_off(g, x, ty * TP + ly, tz * TP + lz);
    }
    if (!on) continue;
    if (mode == 0) {
#pragma unroll
      for (int u = 0; u < U; ++u) a[o[u]] = static_cast<double>(x0 + u + e);
    } else if (mode == 1) {
#pragma unroll
      for (int u = 0; u < U; ++u) va[u] = a[o[u]];
#pragma unroll
      for (int u = 0; u < U; ++u) acc += va[u];
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        va[u] = a[o[u]];
        vb[u] = b[o[u]];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) a[o[u]] = va[u] + 0.5 * vb[u];
    }
  }
  if (acc == 12345.678) sink[0] = acc + pin[threadIdx.x];
}

// In-tile offset of node (ly, lz): row-major (COLFIRST = 0) or with the
// lz = 0 column stored first (COLFIRST = 1: a tile's first column, which the
// left neighbour reads as its 13th column, is contiguous).
template <int COLFIRST>
__device__ __forceinline__ int intile(int ly, int lz) {
  if (COLFIRST) return lz == 0 ? ly : TP + ly * (TP - 1) + (lz - 1);
  return ly * TP + lz;
}

// Read the operator's 13 x 13 patch of every x-plane (own 12 x 12 plus the
// neighbours' first row / column) from the tile-major layout.
template <int COLFIRST>
__global__ void __launch_bounds__(NT) patch_read_kernel(Geo g, const double* __restrict__ a,
                                                        double* sink) {
  __shared__ double pin[LDS_PIN / 8];
  const int nblk = gridDim.x, ob = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = ob % 8;
  const int bid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + ob / 8;
  const int ty = bid / g.ntz, tz = bid % g.ntz;
  constexpr int D = TP + 1, U = 4;
  const int e = threadIdx.x;
  const bool on = e < D * D;
  int ly = e / D, lz = e % D, tyy = ty, tzz = tz;
  if (ly == TP) { ly = 0; ++tyy; }
  if (lz == TP) { lz = 0; ++tzz; }
  const bool in = on && tyy < g.nty && tzz < g.ntz;
  const long base = (static_cast<long>(tyy) * g.ntz + tzz) * g.X * (TP * TP) + intile<COLFIRST>(ly, lz);
  double acc = 0.0;
  for (int x0 = 0; x0 < g.X; x0 += U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int x = x0 + u < g.X ? x0 + u : g.X - 1;
      v[u] = in ? a[base + static_cast<long>(x) * (TP * TP)] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += v[u];
  }
  if (acc == 12345.678) sink[0] = acc + pin[threadIdx.x];
}

// Flat grid-stride reference: 16 bytes per lane.
__global__ void __launch_bounds__(NT) stream_kernel(long n, int mode, double* __restrict__ a,
                                                    const double* __restrict__ b, double* sink) {
  typedef double V __attribute__((ext_vector_type(2)));
  V* av = reinterpret_cast<V*>(a);
  const V* bv = reinterpret_cast<const V*>(b);
  const long nv = n / 2;
  double acc = 0.0;
  for (long i = static_cast<long>(blockIdx.x) * NT + threadIdx.x; i < nv;
       i += static_cast<long>(gridDim.x) * NT) {
    if (mode == 0) {
      av[i] = V{1.0, 2.0};
    } else if (mode == 1) {
      const V v = av[i];
      acc += v[0] + v[1];
    } else {
      av[i] = av[i] + 0.5 * bv[i];
    }
  }
  if (acc == 12345.678) sink[0] = acc;
}

int main() {
  Geo g;
  g.nty = g.ntz = 56;
  g.Y = g.Z = g.nty * TP;          // 672 owned nodes per side
  g.ld = g.Z;                      // multiple of 16 elements
  g.X = 664;
  const long n = static_cast<long>(g.X) * g.Y * g.ld;  // ~3.0e8 doubles
  double *a, *b, *sink;
  CK(hipMalloc(&a, n * 8));
  CK(hipMalloc(&b, n * 8));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(a, 0, n * 8));
  CK(hipMemset(b, 0, n * 8));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const char* mname[3] = {"write 1W", "read 1R", "r+w 2R1W"};
  const double bytes[3] = {8.0 * n, 8.0 * n, 24.0 * n};
  const int tiles = g.nty * g.ntz;
  for (int mode = 0; mode < 3; ++mode) {
    for (int kind = 0; kind < 3; ++kind) {
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(t0));
        if (kind == 0)
          stream_kernel<<<4096, NT>>>(n, mode, a, b, sink);
        else if (kind == 1)
          march_kernel<0><<<tiles, NT>>>(g, mode, a, b, sink);
        else
          march_kernel<1><<<tiles, NT>>>(g, mode, a, b, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(t1));
        CK(hipEventSynchronize(t1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, t0, t1));
        if (rep > 0 && ms < best) best = ms;
      }
      const char* kname[3] = {"stream", "march (lattice layout)", "march (tile-major layout)"};
      std::printf("%-9s %-27s %8.3f ms  %6.2f TB/s\n", mname[mode], kname[kind], best,
                  bytes[mode] / (best * 1e-3) / 1e12);
    }
  }
  // the operator's read: 13 x 13 patches (169 reads per 144 owned nodes)
  for (int cf = 0; cf < 2; ++cf) {
    float best = 1e30f;
    for (int rep = 0; rep < 4; ++rep) {
      CK(hipEventRecord(t0));
      if (cf)
        patch_read_kernel<1><<<tiles, NT>>>(g, a, sink);
      else
        patch_read_kernel<0><<<tiles, NT>>>(g, a, sink);
      CK(hipGetLastError());
      CK(hipEventRecord(t1));
      CK(hipEventSynchronize(t1));
      float ms = 0.f;
      CK(hipEventElapsedTime(&ms, t0, t1));
      if (rep > 0 && ms < best) best = ms;
    }
    std::printf("patch 13x13 read, tile-major %-22s %8.3f ms  %6.2f TB/s (owned bytes)\n",
                cf ? "(first column first)" : "(row-major tile)", best, 8.0 * n / (best * 1e-3) / 1e12);
  }
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(sink));
  return 0;
}
