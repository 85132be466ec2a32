// Microbenchmark: does a deeper prefetch help the x-march's memory side?
//
// The fused5 CG kernel (lap_fused5.h) streams, per cell layer of P = 3
// x-planes and per (y, z) tile of 12 x 12 owned nodes: reads of r and p_old
// (the 13 x 13 patch: own nodes plus the neighbours' first row / column),
// writes of p_new (own nodes) and y (own nodes).  Its loads for layer cx + 1
// are issued when layer cx starts and consumed when layer cx ends, so one
// layer of loads is in flight under the compute of one layer.  This program
// replays that traffic pattern in the tile-major layout [ty][tz][x][12][12]
// with a tunable amount of dependent FP64 work per layer standing in for the
// contractions, at the operator's occupancy (4 workgroups of 256 per CU),
// with a whole number of rounds (no tail), and compares
//   depth 1: loads of layer cx + 1 in flight under layer cx (the kernel today)
//   depth 2: loads of layers cx + 1 and cx + 2 in flight (two register sets,
//            the march unrolled by two so no in-flight register is copied)
// Build: hipcc -O3 --offload-arch=gfx950 march_depth.hip -o march_depth
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int TP = 12, D = TP + 1, P = 3, NT = 256;
constexpr int NL = (P * D * D + NT - 1) / NT;  // patch loads per thread and layer (2)
constexpr int NS = (P * TP * TP + NT - 1) / NT;  // owned stores per thread and layer (2)

struct Geo {
  int X, nty, ntz;
};

__device__ __forceinline__ long toff(const Geo& g, int ty, int tz, int x, int ly, int lz) {
  return ((static_cast<long>(ty) * g.ntz + tz) * g.X + x) * (TP * TP) + ly * TP + lz;
}

// one layer of "compute": `work` dependent FMA chains of 8 (4 chains interleaved)
__device__ __forceinline__ double burn(double v, int work) {
  double a0 = v, a1 = v + 1, a2 = v + 2, a3 = v + 3;
  for (int i = 0; i < work; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a0 = a0 * 0.999 + 1e-3;
      a1 = a1 * 0.999 + 1e-3;
      a2 = a2 * 0.999 + 1e-3;
      a3 = a3 * 0.999 + 1e-3;
    }
  }
  return a0 + a1 + a2 + a3;
}

// The operator's traffic per layer with DEPTH layers of loads in flight.
template <int DEPTH>
__global__ void __launch_bounds__(NT) march_kernel(Geo g, int work, const double* __restrict__ r,
                                                   const double* __restrict__ p, double* __restrict__ pn,
                                                   double* __restrict__ y, double* sink, int pin_bytes) {
  extern __shared__ double lds[];
  const int tile = blockIdx.x;
  const int ty = tile / g.ntz, tz = tile % g.ntz;
  const int tid = threadIdx.x;
  // load descriptors: patch element e = tid + k NT of (plane, 13 x 13)
  long lo[NL];
  bool lon[NL];
#pragma unroll
  for (int k = 0; k < NL; ++k) {
    const int e = tid + k * NT;
    lon[k] = e < P * D * D;
    const int pl = lon[k] ? e / (D * D) : 0, rem = e % (D * D);
    int ly = rem / D, lz = rem % D, tyy = ty, tzz = tz;
    if (ly == TP) { ly = 0; ++tyy; }
    if (lz == TP) { lz = 0; ++tzz; }
    if (tyy >= g.nty || tzz >= g.ntz) lon[k] = false;
    lo[k] = lon[k] ? toff(g, tyy, tzz, pl, ly, lz) : 0;
  }
  long so[NS];
  bool son[NS];
#pragma unroll
  for (int k = 0; k < NS; ++k) {
    const int e = tid + k * NT;
    son[k] = e < P * TP * TP;
    const int pl = son[k] ? e / (TP * TP) : 0, rem = e % (TP * TP);
    so[k] = son[k] ? toff(g, ty, tz, pl, rem / TP, rem % TP) : 0;
  }
  const long lstep = static_cast<long>(P) * TP * TP;  // one layer along x in the tile's column
  const int nlay = g.X / P;
  double acc = 0.0;
  auto issue = [&](int cx, double (&vr)[NL], double (&vp)[NL]) {
#pragma unroll
    for (int k = 0; k < NL; ++k) {
      const long o = lo[k] + static_cast<long>(cx) * lstep;
      vr[k] = (lon[k] && cx < nlay) ? __builtin_nontemporal_load(r + o) : 0.0;
      vp[k] = (lon[k] && cx < nlay) ? __builtin_nontemporal_load(p + o) : 0.0;
    }
  };
  // layer cx: the compute (independent of the loads), then the landed values
  // of layer cx are used (staging stand-in) and the layer's stores issue
  auto consume = [&](int cx, const double (&vr)[NL], const double (&vp)[NL]) {
    const double c = burn(static_cast<double>(cx + tid), work);
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NL; ++k) s += vr[k] + 0.5 * vp[k];
    lds[tid] = s;
#pragma unroll
    for (int k = 0; k < NS; ++k) {
      const long o = so[k] + static_cast<long>(cx) * lstep;
      if (son[k]) {
        pn[o] = s + k;
        y[o] = c + k;
      }
    }
    acc += c;
  };
  if constexpr (DEPTH == 1) {
    // loads of one layer in flight under each layer's compute
    double vr[NL], vp[NL];
    issue(0, vr, vp);
    for (int cx = 0; cx < nlay; ++cx) {
      consume(cx, vr, vp);
      issue(cx + 1, vr, vp);
    }
  } else {
    // two layers in flight: two register sets, the march unrolled by two
    double ar[NL], ap[NL], br[NL], bp[NL];
    issue(0, ar, ap);
    issue(1, br, bp);
    for (int cx = 0; cx < nlay; cx += 2) {
      consume(cx, ar, ap);
      issue(cx + 2, ar, ap);
      if (cx + 1 < nlay) consume(cx + 1, br, bp);
      issue(cx + 3, br, bp);
    }
  }
  if (acc == 12345.678) sink[0] = acc + lds[tid];
  (void)pin_bytes;
}

// The same traffic with 16-byte accesses wherever a tile row allows: the 12
// own nodes of a row as 6 pairs, the neighbour's 13th column element and the
// corner as single loads; writes of own nodes as pairs.
__global__ void __launch_bounds__(NT) march_vec_kernel(Geo g, int work, const double* __restrict__ r,
                                                      const double* __restrict__ p, double* __restrict__ pn,
                                                      double* __restrict__ y, double* sink) {
  typedef double V __attribute__((ext_vector_type(2)));
  extern __shared__ double lds[];
  const int tile = blockIdx.x;
  const int ty = tile / g.ntz, tz = tile % g.ntz;
  const int tid = threadIdx.x;
  // load items per plane: 13 rows x 6 pairs (row 12 from the y neighbour) +
  // 13 singles (column 12 from the z neighbour, incl. the corner) = 91
  constexpr int NIT = 13 * 6 + 13, NLI = (P * NIT + NT - 1) / NT;
  long lo[NLI];
  int lk[NLI];  // 0 none, 1 pair, 2 single
#pragma unroll
  for (int k = 0; k < NLI; ++k) {
    const int e = tid + k * NT;
    lk[k] = 0;
    lo[k] = 0;
    if (e < P * NIT) {
      const int pl = e / NIT, it = e % NIT;
      int ly, lz, tyy = ty, tzz = tz;
      if (it < 78) { ly = it / 6; lz = 2 * (it % 6); lk[k] = 1; }
      else { ly = it - 78; lz = 0; ++tzz; lk[k] = 2; }
      if (ly == TP) { ly = 0; ++tyy; }
      if (tyy >= g.nty || tzz >= g.ntz) lk[k] = 0;
      lo[k] = lk[k] ? toff(g, tyy, tzz, pl, ly, lz) : 0;
    }
  }
  constexpr int NSI = (P * 72 + NT - 1) / NT;  // own pairs per layer
  long so[NSI];
  bool son[NSI];
#pragma unroll
  for (int k = 0; k < NSI; ++k) {
    const int e = tid + k * NT;
    son[k] = e < P * 72;
    const int pl = son[k] ? e / 72 : 0, it = e % 72;
    so[k] = son[k] ? toff(g, ty, tz, pl, it / 6, 2 * (it % 6)) : 0;
  }
  const long lstep = static_cast<long>(P) * TP * TP;
  const int nlay = g.X / P;
  double acc = 0.0;
  V vr[NLI], vp[NLI];
  auto issue = [&](int cx) {
#pragma unroll
    for (int k = 0; k < NLI; ++k) {
      const long o = lo[k] + static_cast<long>(cx) * lstep;
      vr[k] = V{0, 0};
      vp[k] = V{0, 0};
      if (cx < nlay && lk[k] == 1) {
        vr[k] = __builtin_nontemporal_load(reinterpret_cast<const V*>(r + o));
        vp[k] = __builtin_nontemporal_load(reinterpret_cast<const V*>(p + o));
      } else if (cx < nlay && lk[k] == 2) {
        vr[k][0] = __builtin_nontemporal_load(r + o);
        vp[k][0] = __builtin_nontemporal_load(p + o);
      }
    }
  };
  issue(0);
  for (int cx = 0; cx < nlay; ++cx) {
    const double c = burn(static_cast<double>(cx + tid), work);
    double sacc = 0.0;
#pragma unroll
    for (int k = 0; k < NLI; ++k) sacc += vr[k][0] + vr[k][1] + 0.5 * (vp[k][0] + vp[k][1]);
    lds[tid] = sacc;
#pragma unroll
    for (int k = 0; k < NSI; ++k) {
      const long o = so[k] + static_cast<long>(cx) * lstep;
      if (son[k]) {
        *reinterpret_cast<V*>(pn + o) = V{sacc + k, sacc};
        *reinterpret_cast<V*>(y + o) = V{c + k, c};
      }
    }
    acc += c;
    issue(cx + 1);
  }
  if (acc == 12345.678) sink[0] = acc + lds[tid];
}

int main(int argc, char** argv) {
  // 1024 tiles = one round at 4 workgroups per CU on 256 CUs; ~300 M doubles
  Geo g;
  g.nty = g.ntz = 32;
  g.X = 2034;
  const int pin = argc > 1 ? std::atoi(argv[1]) : 40 * 1024;
  const long n = static_cast<long>(g.nty) * g.ntz * g.X * TP * TP;
  double *r, *p, *pn, *y, *sink;
  CK(hipMalloc(&r, n * 8));
  CK(hipMalloc(&p, n * 8));
  CK(hipMalloc(&pn, n * 8));
  CK(hipMalloc(&y, n * 8));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(r, 0, n * 8));
  CK(hipMemset(p, 0, n * 8));
  hipEvent_t t0, t1;
  CK(hipEventCreate(&t0));
  CK(hipEventCreate(&t1));
  const double bytes = 8.0 * n * (2.0 * 169.0 / 144.0 + 2.0);  // patch reads + own writes
  std::printf("n = %ld doubles, LDS pin %d B, %d tiles\n", n, pin, g.nty * g.ntz);
  for (int work : {0, 2, 4, 8, 12, 16}) {
    for (int depth = 1; depth <= 3; ++depth) {  // 3: depth 1 with 16-byte accesses
      float best = 1e30f;
      for (int rep = 0; rep < 4; ++rep) {
        CK(hipEventRecord(t0));
        if (depth == 1)
          march_kernel<1><<<g.nty * g.ntz, NT, pin>>>(g, work, r, p, pn, y, sink, pin);
        else if (depth == 2)
          march_kernel<2><<<g.nty * g.ntz, NT, pin>>>(g, work, r, p, pn, y, sink, pin);
        else
          march_vec_kernel<<<g.nty * g.ntz, NT, pin>>>(g, work, r, p, pn, y, sink);
        CK(hipGetLastError());
        CK(hipEventRecord(t1));
        CK(hipEventSynchronize(t1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, t0, t1));
        if (rep > 0 && ms < best) best = ms;
      }
      std::printf("work %2d %s: %8.3f ms  %6.2f TB/s (patch-read + own-write bytes)\n", work,
                  depth == 1 ? "depth 1      " : depth == 2 ? "depth 2      " : "depth 1, 16 B", best,
                  bytes / (best * 1e-3) / 1e12);
    }
  }
  return 0;
}
