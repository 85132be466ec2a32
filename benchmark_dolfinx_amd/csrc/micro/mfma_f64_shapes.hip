// Microbenchmark + layout probe for the two FP64 MFMA shapes of gfx950:
//   v_mfma_f64_16x16x4_f64    (one 16x16 tile, K = 4; 4 results per lane)
//   v_mfma_f64_4x4x4_4b_f64   (four independent 4x4 tiles, K = 4; 1 result per lane)
// 1. layout: small-integer A / B per lane (exact in FP64) -> D per lane, dumped
//    as text; the host side (scripts/mfma_layout.py) infers the lane maps.
// 2. issue rate: independent accumulators, one and two waves per SIMD.
// 3. dependent latency: one accumulator chain per wave.
// Build: hipcc --offload-arch=gfx950 -O3 mfma_f64_shapes.hip -o mfma_f64_shapes
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

typedef double d4 __attribute__((ext_vector_type(4)));

// one 16x16x4 MFMA of the given per-lane A / B (layout probe)
__global__ void k_layout16(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  d4 c = {0, 0, 0, 0};
  c = __builtin_amdgcn_mfma_f64_16x16x4f64(a[l], b[l], c, 0, 0, 0);
  for (int r = 0; r < 4; ++r) d[l * 4 + r] = c[r];
}
// one 4x4x4_4b MFMA of the given per-lane A / B (layout probe)
__global__ void k_layout4(const double* a, const double* b, double* d) {
  const int l = threadIdx.x;
  double c = 0;
  c = __builtin_amdgcn_mfma_f64_4x4x4f64(a[l], b[l], c, 0, 0, 0);
  d[l] = c;
}

// 16x16x4 issue-rate loop on NACC independent accumulators
template <int NACC>
__global__ void __launch_bounds__(256) k_rate16(int it, double* out) {
  d4 c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = d4{0, 0, 0, 0};
  double a = threadIdx.x * 1e-3, b = 1.0 - a;
  for (int i = 0; i < it; ++i) {
#pragma unroll
    for (int k = 0; k < 8 / NACC; ++k)
#pragma unroll
      for (int j = 0; j < NACC; ++j) c[j] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[j], 0, 0, 0);
  }
  d4 s = c[0];
  for (int j = 1; j < NACC; ++j) s += c[j];
  if (s[0] + s[1] + s[2] + s[3] == 12345.0) out[0] = 1;
}
// 4x4x4_4b issue-rate loop on NACC independent accumulators
template <int NACC>
__global__ void __launch_bounds__(256) k_rate4(int it, double* out) {
  double c[NACC];
  for (int i = 0; i < NACC; ++i) c[i] = 0;
  double a = threadIdx.x * 1e-3, b = 1.0 - a;
  for (int i = 0; i < it; ++i) {
#pragma unroll
    for (int k = 0; k < 8 / NACC; ++k)
#pragma unroll
      for (int j = 0; j < NACC; ++j) c[j] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[j], 0, 0, 0);
  }
  double s = 0;
  for (int j = 0; j < NACC; ++j) s += c[j];
  if (s == 12345.0) out[0] = 1;
}

template <typename F>
double timeit(F f) {
  f();
  hipDeviceSynchronize();
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < 5; ++r) f();
  hipDeviceSynchronize();
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / 5;
}

int main() {
  double *a, *b, *d;
  hipMalloc(&a, 64 * 8);
  hipMalloc(&b, 64 * 8);
  hipMalloc(&d, 256 * 8);
  double ha[64], hb[64], hd[256];
  unsigned s = 12345u;
  for (int trial = 0; trial < 3; ++trial) {
    for (int l = 0; l < 64; ++l) {
      s = s * 1103515245u + 12345u;
      ha[l] = static_cast<double>((s >> 16) % 7) - 3.0;
      s = s * 1103515245u + 12345u;
      hb[l] = static_cast<double>((s >> 16) % 7) - 3.0;
    }
    hipMemcpy(a, ha, 64 * 8, hipMemcpyHostToDevice);
    hipMemcpy(b, hb, 64 * 8, hipMemcpyHostToDevice);
    k_layout16<<<1, 64>>>(a, b, d);
    hipMemcpy(hd, d, 256 * 8, hipMemcpyDeviceToHost);
    printf("L16 %d A", trial);
    for (int l = 0; l < 64; ++l) printf(" %g", ha[l]);
    printf(" B");
    for (int l = 0; l < 64; ++l) printf(" %g", hb[l]);
    printf(" D");
    for (int l = 0; l < 256; ++l) printf(" %g", hd[l]);
    printf("\n");
    k_layout4<<<1, 64>>>(a, b, d);
    hipMemcpy(hd, d, 64 * 8, hipMemcpyDeviceToHost);
    printf("L4 %d A", trial);
    for (int l = 0; l < 64; ++l) printf(" %g", ha[l]);
    printf(" B");
    for (int l = 0; l < 64; ++l) printf(" %g", hb[l]);
    printf(" D");
    for (int l = 0; l < 64; ++l) printf(" %g", hd[l]);
    printf("\n");
  }
  // rates: 256 CUs x {4, 8} waves; per wave it * 8 MFMAs
  const int it = 2000;
  for (int wpc : {4, 8}) {
    const int blocks = 256 * wpc / 4;
    const double mf = static_cast<double>(blocks) * 4 * it * 8;  // MFMAs
    double t;
    t = timeit([&] { k_rate16<1><<<blocks, 256>>>(it, d); });
    printf("16x16x4 chain(1 acc)  waves/SIMD %d: %.3f ms, %.1f cyc/MFMA/SIMD @2.4GHz, %.1f TF/s\n",
           wpc / 4, t * 1e3, t * 2.4e9 / (mf / (256 * 4)), mf * 2048 / t / 1e12);
    t = timeit([&] { k_rate16<4><<<blocks, 256>>>(it, d); });
    printf("16x16x4 4 acc         waves/SIMD %d: %.3f ms, %.1f cyc/MFMA/SIMD @2.4GHz, %.1f TF/s\n",
           wpc / 4, t * 1e3, t * 2.4e9 / (mf / (256 * 4)), mf * 2048 / t / 1e12);
    t = timeit([&] { k_rate4<1><<<blocks, 256>>>(it, d); });
    printf("4x4x4_4b chain(1 acc) waves/SIMD %d: %.3f ms, %.1f cyc/MFMA/SIMD @2.4GHz, %.1f TF/s\n",
           wpc / 4, t * 1e3, t * 2.4e9 / (mf / (256 * 4)), mf * 512 / t / 1e12);
    t = timeit([&] { k_rate4<4><<<blocks, 256>>>(it, d); });
    printf("4x4x4_4b 4 acc        waves/SIMD %d: %.3f ms, %.1f cyc/MFMA/SIMD @2.4GHz, %.1f TF/s\n",
           wpc / 4, t * 1e3, t * 2.4e9 / (mf / (256 * 4)), mf * 512 / t / 1e12);
  }
  return 0;
}
