// Microbenchmark: when does a small kernel on a second stream get CUs while a
// large grid fills the chip?
//
// The split CG schedule (runtime.hip, CGRuntime::step) runs the interior
// tiles of the operator as one large launch on the compute stream while the
// comm stream runs forward exchange -> boundary tiles -> reverse send.  The
// round-4 probe (profiles/r4_overlap_probe.md) showed the boundary tiles of a
// Q3 operator (4 workgroups per CU, LDS-bound) finishing only in the
// interior's last round although the comm stream has the device's greatest
// priority.  This program isolates the dispatcher with stand-in kernels of
// the same residency (256 threads, 38 KB LDS: 4 workgroups per CU), each
// workgroup holding its slot for a fixed wall-clock time and recording its
// start / end / CU:
//
//   L   the interior: nL workgroups on stream A;
//   B   the chain on stream B: delay (the forward exchange), H1, H2 (the
//       boundary tile launches), delay (the reverse send).
//
// Variants: stream priorities, enqueue order, and CU masks that reserve a
// few CUs per XCD for stream B (hipExtStreamCreateWithCUMask).
// Build: hipcc -O3 --offload-arch=gfx950 dispatch_prio.hip -o dispatch_prio
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <set>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

// rec[4 b + 0..3] = start tick, end tick, smid, 0 (wall clock: 100 MHz)
__global__ void __launch_bounds__(256) hold_kernel(long long ticks, long long* rec) {
  extern __shared__ double lds[];
  if (threadIdx.x == 0) {
    const long long t0 = wall_clock64();
    lds[0] = 1.0;
    long long t = t0;
    // bounded: ends after `ticks` of the constant clock whatever else runs
    while (t - t0 < ticks) {
      __builtin_amdgcn_s_sleep(4);
      t = wall_clock64();
    }
    long long* r = rec + 4 * static_cast<long long>(blockIdx.x);
    r[0] = t0;
    r[1] = t;
    r[2] = static_cast<long long>(__smid());
    r[3] = static_cast<long long>(lds[0]);
  }
  __syncthreads();
}

struct Launch {
  int nwg;
  long long ticks;
  size_t lds;
  long long* rec;
};

static void launch(const Launch& l, hipStream_t s) {
  hipLaunchKernelGGL(hold_kernel, dim3(l.nwg), dim3(256), l.lds, s, l.ticks, l.rec);
  CK(hipGetLastError());
}

struct Span {
  long long first, median, last_start, last_end;
};
static Span span(const std::vector<long long>& rec, int n, long long t0) {
  std::vector<long long> st(n);
  long long le = 0;
  for (int i = 0; i < n; ++i) {
    st[i] = rec[4 * i] - t0;
    le = std::max(le, rec[4 * i + 1] - t0);
  }
  std::sort(st.begin(), st.end());
  return {st[0], st[n / 2], st[n - 1], le};
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int ncu = prop.multiProcessorCount;
  int prio_lo = 0, prio_hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi));
  // 250 us per workgroup (wall clock: 100 ticks per us), 9 rounds of 4
  // workgroups per CU for L
  const long long hold = 25000;
  const int nL = ncu * 4 * 9;
  const int nH = 168;  // a boundary tile row x 3 x segments
  const size_t lds = 38 * 1024;
  long long *recL, *recH1, *recH2, *recD1, *recD2;
  CK(hipMalloc(&recL, 4 * sizeof(long long) * nL));
  CK(hipMalloc(&recH1, 4 * sizeof(long long) * nH));
  CK(hipMalloc(&recH2, 4 * sizeof(long long) * nH));
  CK(hipMalloc(&recD1, 4 * sizeof(long long)));
  CK(hipMalloc(&recD2, 4 * sizeof(long long)));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(hold_kernel),
                         hipFuncAttributeMaxDynamicSharedMemorySize, 64 * 1024));

  // reserved CUs: `per_xcd` mask bits per 32-bit word chunk; bit order of the
  // mask is checked by the census below (which smids each stream's grid used)
  auto masks = [&](int nres, std::vector<uint32_t>& ma, std::vector<uint32_t>& mb,
                   int pattern) {
    const int words = (ncu + 31) / 32;
    ma.assign(words, 0xffffffffu);
    mb.assign(words, 0u);
    // pattern 0: the first nres bits; 1: every (ncu / nres)-th bit
    for (int k = 0; k < nres; ++k) {
      const int bit = pattern == 0 ? k : k * (ncu / nres);
      ma[bit / 32] &= ~(1u << (bit % 32));
      mb[bit / 32] |= 1u << (bit % 32);
    }
  };

  struct Variant {
    const char* name;
    bool b_high, b_first;
    int nres, pattern;
    bool b_only_reserved;
  };
  const Variant vars[] = {
      {"prio_hi_chain_first", true, true, 0, 0, false},
      {"prio_same_chain_first", false, true, 0, 0, false},
      {"prio_hi_interior_first", true, false, 0, 0, false},
      {"mask16_first_bits_b_all", true, true, 16, 0, false},
      {"mask16_spread_b_all", true, true, 16, 1, false},
      {"mask16_spread_b_reserved", true, true, 16, 1, true},
      {"mask8_spread_b_reserved", true, true, 8, 1, true},
  };
  for (const Variant& v : vars) {
    hipStream_t A = nullptr, B = nullptr;
    std::vector<uint32_t> ma, mb;
    if (v.nres > 0) {
      masks(v.nres, ma, mb, v.pattern);
      CK(hipExtStreamCreateWithCUMask(&A, static_cast<uint32_t>(ma.size()), ma.data()));
      if (v.b_only_reserved)
        CK(hipExtStreamCreateWithCUMask(&B, static_cast<uint32_t>(mb.size()), mb.data()));
      else
        CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, v.b_high ? prio_hi : prio_lo));
    } else {
      CK(hipStreamCreateWithPriority(&A, hipStreamNonBlocking, prio_lo));
      CK(hipStreamCreateWithPriority(&B, hipStreamNonBlocking, v.b_high ? prio_hi : prio_lo));
    }
    for (int rep = 0; rep < reps; ++rep) {
      CK(hipDeviceSynchronize());
      const Launch L{nL, hold, lds, recL}, H1{nH, hold, lds, recH1}, H2{nH, hold, lds, recH2};
      const Launch D1{1, 20000, 0, recD1}, D2{1, 20000, 0, recD2};  // 200 us "exchanges"
      auto chain = [&] {
        launch(D1, B);
        launch(H1, B);
        launch(H2, B);
        launch(D2, B);
      };
      if (v.b_first) {
        chain();
        launch(L, A);
      } else {
        launch(L, A);
        chain();
      }
      CK(hipDeviceSynchronize());
      std::vector<long long> rl(4 * nL), r1(4 * nH), r2(4 * nH), d1(4), d2(4);
      CK(hipMemcpy(rl.data(), recL, rl.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r1.data(), recH1, r1.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r2.data(), recH2, r2.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(d1.data(), recD1, 32, hipMemcpyDeviceToHost));
      CK(hipMemcpy(d2.data(), recD2, 32, hipMemcpyDeviceToHost));
      long long t0 = d1[0];
      for (int i = 0; i < nL; ++i) t0 = std::min(t0, rl[4 * i]);
      const Span sl = span(rl, nL, t0), s1 = span(r1, nH, t0), s2 = span(r2, nH, t0);
      std::set<long long> cul, cub;
      for (int i = 0; i < nL; ++i) cul.insert(rl[4 * i + 2]);
      for (int i = 0; i < nH; ++i) cub.insert(r1[4 * i + 2]);
      for (int i = 0; i < nH; ++i) cub.insert(r2[4 * i + 2]);
      int overlap = 0;
      for (long long c : cub) overlap += cul.count(c) ? 1 : 0;
      // times in microseconds (wall clock 100 MHz)
      std::printf(
          "{\"variant\": \"%s\", \"rep\": %d, \"L_first_us\": %.1f, \"L_end_us\": %.1f, "
          "\"D1_end_us\": %.1f, \"H1_first_us\": %.1f, \"H1_median_us\": %.1f, "
          "\"H1_last_start_us\": %.1f, \"H1_end_us\": %.1f, \"H2_first_us\": %.1f, "
          "\"H2_end_us\": %.1f, \"D2_end_us\": %.1f, \"L_cus\": %zu, \"B_cus\": %zu, "
          "\"B_cus_shared_with_L\": %d, \"ideal_L_us\": %.1f}\n",
          v.name, rep, sl.first / 100.0, sl.last_end / 100.0, (d1[1] - t0) / 100.0,
          s1.first / 100.0, s1.median / 100.0, s1.last_start / 100.0, s1.last_end / 100.0,
          s2.first / 100.0, s2.last_end / 100.0, (d2[1] - t0) / 100.0, cul.size(), cub.size(),
          overlap, 9 * hold / 100.0);
      std::fflush(stdout);
    }
    CK(hipStreamDestroy(A));
    CK(hipStreamDestroy(B));
  }
  // mask bit -> smid census: one workgroup per CU on a 1-bit mask stream
  {
    std::vector<uint32_t> m((ncu + 31) / 32, 0u);
    long long* rc;
    CK(hipMalloc(&rc, 4 * sizeof(long long) * 8));
    std::printf("{\"census\": [");
    for (int bit = 0; bit < 16; ++bit) {
      std::fill(m.begin(), m.end(), 0u);
      m[bit / 32] |= 1u << (bit % 32);
      hipStream_t s;
      CK(hipExtStreamCreateWithCUMask(&s, static_cast<uint32_t>(m.size()), m.data()));
      const Launch c{8, 100, 0, rc};
      launch(c, s);
      CK(hipStreamSynchronize(s));
      std::vector<long long> r(32);
      CK(hipMemcpy(r.data(), rc, 32 * 8, hipMemcpyDeviceToHost));
      std::set<long long> ids;
      for (int i = 0; i < 8; ++i) ids.insert(r[4 * i + 2]);
      std::printf("%s{\"bit\": %d, \"smids\": [", bit ? ", " : "", bit);
      int k = 0;
      for (long long id : ids) std::printf("%s%lld", k++ ? ", " : "", id);
      std::printf("]}");
      CK(hipStreamDestroy(s));
    }
    std::printf("]}\n");
    CK(hipFree(rc));
  }
  CK(hipFree(recL));
  CK(hipFree(recH1));
  CK(hipFree(recH2));
  CK(hipFree(recD1));
  CK(hipFree(recD2));
  return 0;
}
