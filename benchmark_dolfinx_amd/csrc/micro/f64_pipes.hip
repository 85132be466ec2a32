// Microbenchmark: does the FP64 MFMA pipe run concurrently with FP64 VALU
// FMAs on gfx950?  Three kernels of equal per-wave work:
//   valu: every wave runs independent v_fma_f64 chains
//   mfma: every wave runs v_mfma_f64_16x16x4_f64 on 4 independent accumulators
//   mix : waves 0-3 of a 512-thread workgroup run the VALU loop, waves 4-7 the
//         MFMA loop (so each SIMD hosts one of each).
// Build: hipcc --offload-arch=gfx950 -O3 f64_pipes.hip -o /tmp/f64_pipes
#include <hip/hip_runtime.h>
#include <cstdio>
#include <chrono>

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double valu_loop(int iters, double x) {
  double a0 = x, a1 = x + 1, a2 = x + 2, a3 = x + 3, a4 = x + 4, a5 = x + 5, a6 = x + 6, a7 = x + 7;
  const double m = 0.999999, c = 1e-7;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a0 = fma(a0, m, c); a1 = fma(a1, m, c); a2 = fma(a2, m, c); a3 = fma(a3, m, c);
      a4 = fma(a4, m, c); a5 = fma(a5, m, c); a6 = fma(a6, m, c); a7 = fma(a7, m, c);
    }
  }
  return a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

__device__ __forceinline__ double mfma_loop(int iters, double x) {
  d4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double a = x, b = 1.0 - x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c3, 0, 0, 0);
    }
  }
  d4 s = c0 + c1 + c2 + c3;
  return s[0] + s[1] + s[2] + s[3];
}

// FP64 VALU FMA throughput loop.
__global__ void __launch_bounds__(512) k_valu(int it, double* out) {
  double r = valu_loop(it, threadIdx.x * 1e-3);
  if (r == 12345.0) out[0] = r;
}
// FP64 MFMA 16x16x4 throughput loop.
__global__ void __launch_bounds__(512) k_mfma(int it, double* out) {
  double r = mfma_loop(it, threadIdx.x * 1e-3);
  if (r == 12345.0) out[0] = r;
}
// VALU waves and MFMA waves side by side (pipe sharing).
__global__ void __launch_bounds__(512) k_mix(int itv, int itm, double* out) {
  double r;
  if (threadIdx.x < 256) r = valu_loop(itv, threadIdx.x * 1e-3);
  else r = mfma_loop(itm, threadIdx.x * 1e-3);
  if (r == 12345.0) out[0] = r;
}

// ---- f32: v_fma_f32 (and packed) VALU vs v_mfma_f32_16x16x4_f32
typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float valu32_loop(int iters, float x) {
  f2 a0 = {x, x + 1}, a1 = {x + 2, x + 3}, a2 = {x + 4, x + 5}, a3 = {x + 6, x + 7};
  f2 a4 = a0 + 8.f, a5 = a1 + 8.f, a6 = a2 + 8.f, a7 = a3 + 8.f;
  const f2 m = {0.999999f, 0.999999f}, c = {1e-7f, 1e-7f};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a0 = __builtin_elementwise_fma(a0, m, c); a1 = __builtin_elementwise_fma(a1, m, c);
      a2 = __builtin_elementwise_fma(a2, m, c); a3 = __builtin_elementwise_fma(a3, m, c);
      a4 = __builtin_elementwise_fma(a4, m, c); a5 = __builtin_elementwise_fma(a5, m, c);
      a6 = __builtin_elementwise_fma(a6, m, c); a7 = __builtin_elementwise_fma(a7, m, c);
    }
  }
  f2 s = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  return s[0] + s[1];
}
__device__ __forceinline__ float mfma32_loop(int iters, float x) {
  f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  float a = x, b = 1.0f - x;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c3, 0, 0, 0);
    }
  }
  f4 s = c0 + c1 + c2 + c3;
  return s[0] + s[1] + s[2] + s[3];
}
// FP32 packed-FMA throughput loop.
__global__ void __launch_bounds__(512) k_valu32(int it, float* out) {
  float r = valu32_loop(it, threadIdx.x * 1e-3f);
  if (r == 12345.0f) out[0] = r;
}
// FP32 MFMA 16x16x4 throughput loop.
__global__ void __launch_bounds__(512) k_mfma32(int it, float* out) {
  float r = mfma32_loop(it, threadIdx.x * 1e-3f);
  if (r == 12345.0f) out[0] = r;
}
// FP32 VALU and MFMA waves side by side.
__global__ void __launch_bounds__(512) k_mix32(int itv, int itm, float* out) {
  float r;
  if (threadIdx.x < 256) r = valu32_loop(itv, threadIdx.x * 1e-3f);
  else r = mfma32_loop(itm, threadIdx.x * 1e-3f);
  if (r == 12345.0f) out[0] = r;
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
  double* out;
  hipMalloc(&out, 8);
  const int blocks = 256 * 4;
  const int itv = 2000, itm = 1000;
  // FLOPs: valu per wave-iter: 64 fma * 64 lanes * 2; mfma per wave-iter: 16 mfma * 2048
  const double fv = 2.0 * 64 * 64 * itv, fm = 16.0 * 2048 * itm;  // per wave
  double tv = timeit([&] { k_valu<<<blocks, 512>>>(itv, out); });
  double tm = timeit([&] { k_mfma<<<blocks, 512>>>(itm, out); });
  double tx = timeit([&] { k_mix<<<blocks, 512>>>(itv, itm, out); });
  const double waves = blocks * 8.0;
  printf("valu: %.3f ms  %.1f TF/s\n", tv * 1e3, waves * fv / tv / 1e12);
  printf("mfma: %.3f ms  %.1f TF/s\n", tm * 1e3, waves * fm / tm / 1e12);
  printf("mix : %.3f ms  %.1f TF/s (half waves each: valu %.1f + mfma %.1f)\n", tx * 1e3,
         waves / 2 * (fv + fm) / tx / 1e12, waves / 2 * fv / tx / 1e12, waves / 2 * fm / tx / 1e12);
  printf("(if concurrent: mix ~= max(valu, mfma)/2 of the pure times = %.3f ms; if shared: sum/2 = %.3f ms)\n",
         0.5 * (tv > tm ? tv : tm) * 1e3, 0.5 * (tv + tm) * 1e3);
  {
    float* o32 = reinterpret_cast<float*>(out);
    const int itv32 = 4000, itm32 = 2000;
    // valu per wave-iter: 64 packed fma (2 lanes each) * 64 lanes * 2 flop; mfma: 16 * 16*16*4*2
    const double fv32 = 2.0 * 2 * 64 * 64 * itv32, fm32 = 16.0 * 2048 * itm32;
    double a = timeit([&] { k_valu32<<<blocks, 512>>>(itv32, o32); });
    double b = timeit([&] { k_mfma32<<<blocks, 512>>>(itm32, o32); });
    double c = timeit([&] { k_mix32<<<blocks, 512>>>(itv32, itm32, o32); });
    printf("f32 valu (pk_fma): %.3f ms  %.1f TF/s\n", a * 1e3, waves * fv32 / a / 1e12);
    printf("f32 mfma 16x16x4: %.3f ms  %.1f TF/s\n", b * 1e3, waves * fm32 / b / 1e12);
    printf("f32 mix : %.3f ms  %.1f TF/s (concurrent ~ %.3f ms, shared ~ %.3f ms)\n", c * 1e3,
           waves / 2 * (fv32 + fm32) / c / 1e12, 0.5 * (a > b ? a : b) * 1e3, 0.5 * (a + b) * 1e3);
  }
  return 0;
}
