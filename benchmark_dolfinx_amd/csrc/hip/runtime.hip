// Native CG runtime: the whole timed CG loop of the fused operator in C++.
//
// The reference drives its CG from C++ (src/cg.hpp:89-169) over GPU-aware MPI
// with host round trips per dot product and two halo scatters per iteration
// (SURVEY.md quirks Q2/Q3), overlapping the forward scatter with the
// interior-cell kernel (src/laplacian.hpp:281-349).  This runtime owns one
// rank's iteration on two HIP streams, every scalar device-resident:
//
//   compute stream                     comm stream
//   --------------                     -----------
//   fused op, all interior tiles  ||   pack r faces -> RCCL send/recv -> unpack ghosts
//                                 ||   fused op, ghost-touching tiles (last row / column)
//                                 ||   ghost-plane finalize
//                                 ||   pack y ghosts -> RCCL send/recv
//   (join) unpack-add y faces
//   reduce(p.Ap) -> all-reduce -> r update (+ r.r) -> all-reduce
//
// The tile split needs an unsplit march axis (x): the partition keeps x whole
// on the GPU platform (fem/mesh.py partition_grid), so only the last (y, z)
// tile row / column touches a ghost plane and every other tile can run while
// the halo is in flight.  The whole comm-stream chain -- both exchanges and
// the small boundary launches -- runs under the one large interior launch.  Otherwise (x split, one
// rank) the iteration runs serially on the compute stream.  Halos are
// grouped RCCL point-to-point sends/receives with the <= 7 neighbours over
// xGMI; the steady-state iterations (two parities: the p buffers and the r.r
// slots ping-pong) are captured once into hipGraphs (fork/join over the two
// streams) and replayed.
//
// Failure containment: every blocking RCCL call and host wait runs inside a
// bdx::Watchdog scope (csrc/include/bdx_watchdog.h); past the deadline
// (BDX_RCCL_TIMEOUT_S, default 300 s) or on an asynchronous communicator
// error the communicator is aborted and the call returns an error that
// Python raises.  A second transport runs R ranks as threads of one process
// on one GPU (host barriers + device copies) so the multi-rank orchestration
// is testable on a single-GPU box.
//
// Python (solvers/native.py) builds the problem, runs the CG prologue
// (r0 = b - A x0, rho0) and hands the device buffers to this runtime.
#include <rccl/rccl.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "bdx_common.h"
#include "bdx_watchdog.h"

extern "C" {
int bdx_box_copy_f64(int, double*, int64_t, int64_t, const int64_t*, int, int64_t, double*,
                     hipStream_t);
int bdx_box_copy_f32(int, float*, int64_t, int64_t, const int64_t*, int, int64_t, float*,
                     hipStream_t);
int bdx_reduce_partials(const double*, int, double*, int, hipStream_t);
int bdx_fused_finalize_f64(const int64_t*, double*, const double*, const double*,
                           const double*, int, int, int, int, int, hipStream_t);
int bdx_fused_finalize_f32(const int64_t*, float*, const float*, const float*, const float*,
                           int, int, int, int, int, hipStream_t);
int bdx_cg_update_iface_f64(const int64_t*, const int64_t*, double*, const double*,
                            const double*, const double*, const double*, int, int, int, int,
                            double*, int, int, int, double*, hipStream_t);
int bdx_cg_update_iface_f32(const int64_t*, const int64_t*, float*, const float*, const float*,
                            const float*, const float*, int, int, int, int, double*, int, int,
                            int, double*, hipStream_t);
int bdx_xflush_f64(const int64_t*, const int64_t*, double*, const double*, const double*, int,
                   int, hipStream_t);
int bdx_xflush_f32(const int64_t*, const int64_t*, float*, const float*, const double*, int,
                   int, hipStream_t);
int bdx_box_copy_lat_f64(int, double*, const int64_t*, const int64_t*, int, int64_t, double*,
                         hipStream_t);
int bdx_box_copy_lat_f32(int, float*, const int64_t*, const int64_t*, int, int64_t, float*,
                         hipStream_t);
int bdx_layout_convert_f64(int, const int64_t*, double*, double*, hipStream_t);
int bdx_layout_convert_f32(int, const int64_t*, float*, float*, hipStream_t);
int bdx_flush_export_f64(const int64_t*, double*, double*, const double*, const double*,
                         const double*, int, int, int, int, int, hipStream_t);
int bdx_flush_export_f32(const int64_t*, float*, float*, const float*, const float*,
                         const double*, int, int, int, int, int, hipStream_t);
int bdx_cg_update_tiled_f64(const int64_t*, const int64_t*, double*, const double*, const double*,
                            const double*, const double*, int, int, double*, int, int, int,
                            double*, hipStream_t);
int bdx_cg_update_tiled_f32(const int64_t*, const int64_t*, float*, const float*, const float*,
                            const float*, const float*, int, int, double*, int, int, int, double*,
                            hipStream_t);
}

// The fused2, fused3 and fused5 operator entry points (lap_fused{2,3,5}_<suf>_p<P>.hip);
// weak so that experiment builds holding a subset of the operator TUs still
// load (a missing instance resolves to null and bdx_rt_create refuses it).
#define BDX_DECL_APPLY(V, T, SUF, PP)                                                        \
  extern "C" __attribute__((weak)) int bdx_fused##V##_apply_##SUF##_p##PP(                  \
      int, int, const int64_t*, int, const double*, const double*, const T*, const T*, T*, \
      T*, T*, T*, T*, T*, const T*, const T*, const T*, double, const double*, double*, int, \
      int, int, int, int, int, const int*, hipStream_t);
#define BDX_DECL_ALL(V)                                                                    \
  BDX_DECL_APPLY(V, double, f64, 1) BDX_DECL_APPLY(V, double, f64, 2)                      \
  BDX_DECL_APPLY(V, double, f64, 3) BDX_DECL_APPLY(V, double, f64, 4)                      \
  BDX_DECL_APPLY(V, double, f64, 5) BDX_DECL_APPLY(V, double, f64, 6)                      \
  BDX_DECL_APPLY(V, double, f64, 7) BDX_DECL_APPLY(V, float, f32, 1)                       \
  BDX_DECL_APPLY(V, float, f32, 2) BDX_DECL_APPLY(V, float, f32, 3)                        \
  BDX_DECL_APPLY(V, float, f32, 4) BDX_DECL_APPLY(V, float, f32, 5)                        \
  BDX_DECL_APPLY(V, float, f32, 6) BDX_DECL_APPLY(V, float, f32, 7)
BDX_DECL_ALL(2)
BDX_DECL_ALL(3)
#define BDX_DECL_F5(T, SUF) \
  BDX_DECL_APPLY(5, T, SUF, 3) BDX_DECL_APPLY(5, T, SUF, 4) BDX_DECL_APPLY(5, T, SUF, 5) \
  BDX_DECL_APPLY(5, T, SUF, 6) BDX_DECL_APPLY(5, T, SUF, 7)
BDX_DECL_F5(double, f64)
BDX_DECL_F5(float, f32)

// The dofmap data model's entry points (lap_dofmap.h, lap_dofmap_f{32,64}.hip).
#define BDX_DECL_DOF(T, SUF)                                                                  \
  extern "C" int bdx_dofmap_apply_##SUF(                                                      \
      int, int, int, int, const T*, const int*, int, int64_t, const int*, const int*, const T*, \
      const unsigned char*, const T*, double, const T*, const T*, const T*, T*, T*, T*,        \
      const double*, int, int, int, int, double*, int*, hipStream_t);                          \
  extern "C" int bdx_dofmap_cg_update_##SUF(int64_t, const unsigned char*, T*, T*,              \
                                            const double*, int, int, double*, int*, hipStream_t); \
  extern "C" int bdx_dofmap_apply_yz_##SUF(                                                   \
      int, int, int, int, const T*, const int*, int, int64_t, const int*, const int*, const T*, \
      const unsigned char*, const T*, double, const T*, const T*, const T*, T*, T*, T*, T*,    \
      const double*, int, int, int, int, double*, int*, hipStream_t);                          \
  extern "C" int bdx_dofmap_cg_update_z_##SUF(int64_t, const unsigned char*, T*, T*,            \
                                              const double*, int, int, double*, int*, int,      \
                                              hipStream_t);                                     \
  extern "C" int bdx_dofmap_xflush_##SUF(int64_t, T*, const T*, const double*, int, int,        \
                                         hipStream_t);
BDX_DECL_DOF(double, f64)
BDX_DECL_DOF(float, f32)
// p.Ap partials of a dofmap launch (lap_dofmap_f64.hip)
extern "C" int bdx_dofmap_nblocks(int nq, int ncl);
// capacity of the partials buffers (blas.hip)
extern "C" int bdx_hip_partials_size();

namespace {

template <typename T>
using ApplyFn = int (*)(int, int, const int64_t*, int, const double*, const double*, const T*,
                        const T*, T*, T*, T*, T*, T*, T*, const T*, const T*, const T*, double,
                        const double*, double*, int, int, int, int, int, int, const int*,
                        hipStream_t);

template <typename T>
ApplyFn<T> apply_fn(int version, int P);
template <>
ApplyFn<double> apply_fn<double>(int version, int P) {
#define BDX_CASE(V, PP) \
  if (version == V && P == PP) return bdx_fused##V##_apply_f64_p##PP;
  BDX_CASE(2, 1) BDX_CASE(2, 2) BDX_CASE(2, 3) BDX_CASE(2, 4) BDX_CASE(2, 5) BDX_CASE(2, 6)
  BDX_CASE(2, 7) BDX_CASE(3, 1) BDX_CASE(3, 2) BDX_CASE(3, 3) BDX_CASE(3, 4) BDX_CASE(3, 5)
  BDX_CASE(3, 6) BDX_CASE(3, 7) BDX_CASE(5, 3) BDX_CASE(5, 4) BDX_CASE(5, 5) BDX_CASE(5, 6)
  BDX_CASE(5, 7)
#undef BDX_CASE
  return nullptr;
}
template <>
ApplyFn<float> apply_fn<float>(int version, int P) {
#define BDX_CASE(V, PP) \
  if (version == V && P == PP) return bdx_fused##V##_apply_f32_p##PP;
  BDX_CASE(2, 1) BDX_CASE(2, 2) BDX_CASE(2, 3) BDX_CASE(2, 4) BDX_CASE(2, 5) BDX_CASE(2, 6)
  BDX_CASE(2, 7) BDX_CASE(3, 1) BDX_CASE(3, 2) BDX_CASE(3, 3) BDX_CASE(3, 4) BDX_CASE(3, 5)
  BDX_CASE(3, 6) BDX_CASE(3, 7) BDX_CASE(5, 3) BDX_CASE(5, 4) BDX_CASE(5, 5) BDX_CASE(5, 6)
  BDX_CASE(5, 7)
#undef BDX_CASE
  return nullptr;
}

// Error codes returned to Python (besides hipError_t values).
constexpr int kErrAborted = -20;   // the watchdog aborted the communicator
constexpr int kErrNotConnected = -21;

// ------------------------------------------------------------------ transports
struct Transport {
  virtual ~Transport() = default;
  // Grouped point-to-point exchange: rank p receives rcnt[p] elements from
  // each peer (into rbuf + roff[p]) and sends scnt[p] elements to it.
  virtual int exchange(const void* sbuf, const std::vector<int64_t>& scnt,
                       const std::vector<int64_t>& soff, void* rbuf,
                       const std::vector<int64_t>& rcnt, const std::vector<int64_t>& roff,
                       int esize, hipStream_t st) = 0;
  virtual int allreduce_sum(double* dev, int n, hipStream_t st) = 0;
  virtual bool capturable() const = 0;
  virtual int ranks() const = 0;
  // Host wait for `ev` (the end of queued work that may contain
  // communication), bounded by the transport's deadline.
  virtual int wait(hipEvent_t ev) { return static_cast<int>(hipEventSynchronize(ev)); }
  virtual bool aborted() const { return false; }
  // Deadline watchdog whose Busy scopes must cover every host call that can
  // block behind a stuck peer (RCCL only; null otherwise).
  virtual bdx::Watchdog* watchdog() { return nullptr; }
};

double rccl_timeout_s() {
  const char* e = std::getenv("BDX_RCCL_TIMEOUT_S");
  return e ? std::atof(e) : 300.0;
}

struct RcclTransport final : Transport {
  std::atomic<ncclComm_t> comm{nullptr};
  int nranks = 1;
  std::atomic<bool> was_aborted{false};
  std::unique_ptr<bdx::Watchdog> wd;

  RcclTransport() {
    wd = std::make_unique<bdx::Watchdog>(
        rccl_timeout_s(),
        [this] {
          ncclComm_t c = comm.load();
          if (!c || was_aborted.load()) return false;
          ncclResult_t e = ncclSuccess;
          if (ncclCommGetAsyncError(c, &e) != ncclSuccess) return true;
          return e != ncclSuccess && e != ncclInProgress;
        },
        [this] {
          ncclComm_t c = comm.load();
          if (!c) {
            // still inside ncclCommInitRank: nothing to abort, fail fast
            std::fprintf(stderr,
                         "[bdx] RCCL communicator init exceeded %.0f s; a peer never joined. "
                         "Exiting.\n",
                         wd->timeout_s());
            std::fflush(stderr);
            std::_Exit(124);
          }
          std::fprintf(stderr, "[bdx] RCCL %s; aborting the communicator\n",
                       wd->reason() == 1 ? "call exceeded the deadline" : "asynchronous error");
          std::fflush(stderr);
          was_aborted.store(true);
          ncclCommAbort(c);
        });
  }
  ~RcclTransport() override {
    if (wd) wd->stop();
    ncclComm_t c = comm.load();
    if (c && !was_aborted.load()) ncclCommDestroy(c);
  }
  int connect(const ncclUniqueId& id, int n, int rank) {
    nranks = n;
    wd->start();
    bdx::Watchdog::Busy b(wd.get());
    ncclComm_t c = nullptr;
    if (ncclCommInitRank(&c, n, id, rank) != ncclSuccess) return -1;
    comm.store(c);
    return 0;
  }
  bool aborted() const override { return was_aborted.load(); }
  bdx::Watchdog* watchdog() override { return wd.get(); }
  int exchange(const void* sbuf, const std::vector<int64_t>& scnt,
               const std::vector<int64_t>& soff, void* rbuf, const std::vector<int64_t>& rcnt,
               const std::vector<int64_t>& roff, int esize, hipStream_t st) override {
    ncclComm_t c = comm.load();
    if (!c) return kErrNotConnected;
    if (was_aborted.load()) return kErrAborted;
    bdx::Watchdog::Busy b(wd.get());
    const ncclDataType_t dt = esize == 8 ? ncclFloat64 : ncclFloat32;
    if (ncclGroupStart() != ncclSuccess) return -1;
    for (int p = 0; p < nranks; ++p) {
      if (scnt[p] > 0 &&
          ncclSend(static_cast<const char*>(sbuf) + soff[p] * esize, scnt[p], dt, p, c, st) !=
              ncclSuccess)
        return -2;
      if (rcnt[p] > 0 &&
          ncclRecv(static_cast<char*>(rbuf) + roff[p] * esize, rcnt[p], dt, p, c, st) !=
              ncclSuccess)
        return -3;
    }
    const ncclResult_t e = ncclGroupEnd();
    if (was_aborted.load()) return kErrAborted;
    return e == ncclSuccess ? 0 : -4;
  }
  int allreduce_sum(double* dev, int n, hipStream_t st) override {
    ncclComm_t c = comm.load();
    if (!c) return kErrNotConnected;
    if (was_aborted.load()) return kErrAborted;
    bdx::Watchdog::Busy b(wd.get());
    const ncclResult_t e = ncclAllReduce(dev, dev, n, ncclFloat64, ncclSum, c, st);
    if (was_aborted.load()) return kErrAborted;
    return e == ncclSuccess ? 0 : -5;
  }
  int wait(hipEvent_t ev) override {
    bdx::Watchdog::Busy b(wd.get());
    for (;;) {
      const hipError_t e = hipEventQuery(ev);
      if (e == hipSuccess) return 0;
      if (e != hipErrorNotReady) return static_cast<int>(e);
      if (was_aborted.load()) return kErrAborted;
      std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
  }
  bool capturable() const override { return true; }
  int ranks() const override {
    ncclComm_t c = comm.load();
    int n = 0;
    if (!c || ncclCommCount(c, &n) != ncclSuccess) return -1;
    return n;
  }
};

// Emulated link (one rank of an N-rank run alone on this device: bench /
// scripts/emulate_rank.py).  Every exchange is a device copy of the send
// buffer into the receive buffer by a few workgroups (RCCL's p2p kernels
// occupy a few CUs the same way) that hold their CUs until the modelled link
// time has passed: max over peers of the bytes to or from that peer /
// link_gbps (one xGMI link per peer) + lat_us.  An all-reduce is a single
// workgroup held for allreduce_us.  The copies carry the rank's own face
// data, not a peer's: the emulation is for timing the schedule, not for
// results.  Bounded: each workgroup waits on the 100 MHz constant clock from
// its own start, nothing else.
__global__ void __launch_bounds__(256)
    bdx_link_emu_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t n16,
                        int64_t ticks) {
  const long long t0 = wall_clock64();
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16;
       i += static_cast<int64_t>(gridDim.x) * 256)
    dst[i] = src[i];
  if (threadIdx.x == 0) {
    while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  }
  __syncthreads();
}

struct LinkEmuTransport final : Transport {
  int nranks = 1;
  double link_gbps = 50.0, lat_us = 10.0, allreduce_us = 20.0;
  int nwg = 8;
  static double env(const char* k, double d) {
    const char* e = std::getenv(k);
    return e ? std::atof(e) : d;
  }
  LinkEmuTransport() {
    link_gbps = env("BDX_EMU_LINK_GBPS", 50.0);
    lat_us = env("BDX_EMU_LINK_LAT_US", 10.0);
    allreduce_us = env("BDX_EMU_ALLREDUCE_US", 20.0);
    nwg = static_cast<int>(env("BDX_EMU_LINK_WG", 8));
    if (nwg < 1) nwg = 1;
  }
  // modelled link time of one exchange, microseconds
  double exchange_us(const std::vector<int64_t>& scnt, const std::vector<int64_t>& rcnt,
                     int esize) const {
    int64_t worst = 0;
    for (size_t p = 0; p < scnt.size() && p < rcnt.size(); ++p)
      worst = std::max(worst, std::max(scnt[p], rcnt[p]) * esize);
    if (worst == 0) return 0.0;
    return worst / (link_gbps * 1e3) + lat_us;  // bytes / (1e3 link_gbps) = us
  }
  int exchange(const void* sbuf, const std::vector<int64_t>& scnt,
               const std::vector<int64_t>& soff, void* rbuf, const std::vector<int64_t>& rcnt,
               const std::vector<int64_t>& roff, int esize, hipStream_t st) override {
    (void)soff;
    (void)roff;
    int64_t ns = 0, nr = 0;
    for (int64_t c : scnt) ns += c;
    for (int64_t c : rcnt) nr += c;
    const double us = exchange_us(scnt, rcnt, esize);
    if (us <= 0.0) return 0;
    const int64_t n16 = std::min(ns, nr) * esize / 16;
    hipLaunchKernelGGL(bdx_link_emu_kernel, dim3(nwg), dim3(256), 0, st,
                       static_cast<const uint4*>(sbuf), static_cast<uint4*>(rbuf), n16,
                       static_cast<int64_t>(us * 100.0));
    return static_cast<int>(hipGetLastError());
  }
  int allreduce_sum(double*, int, hipStream_t st) override {
    hipLaunchKernelGGL(bdx_link_emu_kernel, dim3(1), dim3(256), 0, st, nullptr, nullptr,
                       int64_t{0}, static_cast<int64_t>(allreduce_us * 100.0));
    return static_cast<int>(hipGetLastError());
  }
  bool capturable() const override { return true; }
  int ranks() const override { return nranks; }
};

// Single rank: no communication at all.
struct NoTransport final : Transport {
  int exchange(const void*, const std::vector<int64_t>&, const std::vector<int64_t>&, void*,
               const std::vector<int64_t>&, const std::vector<int64_t>&, int,
               hipStream_t) override {
    return 0;
  }
  int allreduce_sum(double*, int, hipStream_t) override { return 0; }
  bool capturable() const override { return true; }
  int ranks() const override { return 1; }
};

// R ranks = R threads of one process on one device (tests): host barriers,
// device-to-device copies from the peers' posted buffers, fixed-order sums.
struct ThreadGroupState {
  std::mutex m;
  std::condition_variable cv;
  int size = 0, arrived = 0;
  long generation = 0;
  std::vector<const void*> sbuf;
  std::vector<const std::vector<int64_t>*> soff;
  std::vector<hipEvent_t> packed, copied;
  std::vector<double*> red;
  void barrier() {
    std::unique_lock<std::mutex> lk(m);
    const long gen = generation;
    if (++arrived == size) {
      arrived = 0;
      ++generation;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return generation != gen; });
    }
  }
};
std::mutex g_groups_m;
std::map<int64_t, std::shared_ptr<ThreadGroupState>> g_groups;

// The exchange is stream-ordered, as RCCL's: the host only swaps buffer
// pointers and event handles at two barriers and never waits for the device,
// so the compute stream's interior tiles really run while the copies do.
//   1. record `packed` on the caller's stream (after the pack kernel);
//   2. barrier: every rank's send buffer / offsets / `packed` are published;
//   3. per peer: wait for its `packed`, copy its slice into the receive buffer;
//      record `copied`;
//   4. barrier: every `copied` is published; wait for the `copied` of each
//      peer that reads this rank's send buffer, so a later write to it (the
//      next pack, stream-ordered after this) cannot overtake their copies.
// Event reuse is safe: a rank re-records `packed` only after barrier 2 of
// the previous exchange (every peer's wait on it was issued before that
// barrier) and `copied` only after barrier 1 of the next exchange (every
// peer issues its wait on it before arriving there).
struct ThreadTransport final : Transport {
  std::shared_ptr<ThreadGroupState> g;
  int rank = 0;
  hipEvent_t ev_packed = nullptr, ev_copied = nullptr;
  ~ThreadTransport() override {
    if (ev_packed) hipEventDestroy(ev_packed);
    if (ev_copied) hipEventDestroy(ev_copied);
  }
  int exchange(const void* sbuf, const std::vector<int64_t>& scnt,
               const std::vector<int64_t>& soff, void* rbuf, const std::vector<int64_t>& rcnt,
               const std::vector<int64_t>& roff, int esize, hipStream_t st) override {
    if (!ev_packed) {
      BDX_CHECK(hipEventCreateWithFlags(&ev_packed, hipEventDisableTiming));
      BDX_CHECK(hipEventCreateWithFlags(&ev_copied, hipEventDisableTiming));
    }
    BDX_CHECK(hipEventRecord(ev_packed, st));
    g->sbuf[rank] = sbuf;
    g->soff[rank] = &soff;
    g->packed[rank] = ev_packed;
    g->barrier();
    for (int p = 0; p < g->size; ++p) {
      if (rcnt[p] <= 0) continue;
      const char* src = static_cast<const char*>(g->sbuf[p]) + (*g->soff[p])[rank] * esize;
      BDX_CHECK(hipStreamWaitEvent(st, g->packed[p], 0));
      BDX_CHECK(hipMemcpyAsync(static_cast<char*>(rbuf) + roff[p] * esize, src, rcnt[p] * esize,
                               hipMemcpyDeviceToDevice, st));
    }
    BDX_CHECK(hipEventRecord(ev_copied, st));
    g->copied[rank] = ev_copied;
    g->barrier();
    for (int p = 0; p < g->size; ++p)
      if (scnt[p] > 0) BDX_CHECK(hipStreamWaitEvent(st, g->copied[p], 0));
    return 0;
  }
  int allreduce_sum(double* dev, int n, hipStream_t st) override {
    BDX_CHECK(hipStreamSynchronize(st));
    g->red[rank] = dev;
    g->barrier();
    std::vector<double> acc(n, 0.0), v(n);
    for (int p = 0; p < g->size; ++p) {  // fixed rank order: deterministic
      BDX_CHECK(hipMemcpy(v.data(), g->red[p], n * sizeof(double), hipMemcpyDeviceToHost));
      for (int i = 0; i < n; ++i) acc[i] += v[i];
    }
    g->barrier();
    BDX_CHECK(hipMemcpy(dev, acc.data(), n * sizeof(double), hipMemcpyHostToDevice));
    g->barrier();
    return 0;
  }
  bool capturable() const override { return false; }
  int ranks() const override { return g->size; }
};

// ------------------------------------------------------------------ the CG loop
constexpr int kRR0 = 0, kRR1 = 1, kPAP = 2;

// Phase marks of one iteration (bdx_rt_profile).  In the serial schedule the
// marks that belong to the split schedule coincide with their neighbours.
enum Mark {
  kMStart = 0,   // compute stream: iteration start
  kMFwdBeg,      // comm stream: forward exchange start
  kMFwdEnd,      // comm stream: ghost planes of r unpacked
  kMOpA,         // compute: interior tiles / cells done (serial: the whole operator)
  kMBnd,         // comm: ghost-touching tiles / cells (+ ghost finalize) done
  kMRevBeg,      // comm: reverse exchange start
  kMRevEnd,      // comm: reverse send done (serial: + unpack-add)
  kMJoin,        // compute: comm stream joined, received sums added
  kMPap,         // compute: reduce + all-reduce(p.Ap) done
  kMUpd,         // compute: r update (+ r.r) done
  kMEnd,         // compute: all-reduce(r.r) done
  kNMarks
};

// What the fused-structured and the dofmap CG runtimes share: the transport,
// the two streams, the plane halo, the batched / watchdog-bounded iteration
// loop with its graph capture, the phase profiler and the pre-flight.  A
// derived runtime supplies one iteration (`step`) and the final x flush.
struct LoopBase {
  std::unique_ptr<Transport> tr;
  int nranks = 1, rank = 0;
  int esize = 8;  // vector element bytes
  // comm stream priority (hipDeviceGetStreamPriorityRange: least, greatest;
  // the priority cs was created with)
  int prio_least = 0, prio_greatest = 0, prio_cs = 0;
  double* pf_scal = nullptr;  // pre-flight all-reduce slot
  // own non-blocking streams (graph capture is not allowed on the legacy
  // default stream torch may be using); ordered against the caller's stream
  // `ext` with events at the start and end of every iterate()
  hipStream_t st = nullptr, cs = nullptr, ext = nullptr;
  // Split schedule, interior launch: on st (si == nullptr), or on its own
  // stream si whose CU mask leaves `reserve` CUs to the comm stream's chain
  // (BDX_SPLIT=mask; make_interior_stream).  cu_mask_cs: cs was created with
  // the complementary mask (BDX_SPLIT=maskr: the chain on the reserved CUs
  // only).
  hipStream_t si = nullptr;
  hipEvent_t ev_int = nullptr;
  int reserve = 0;
  std::vector<uint32_t> mask_si, mask_cs;
  hipEvent_t ev_in = nullptr, ev_out = nullptr, ev_fork = nullptr, ev_rev = nullptr;
  // halo: owned lower faces <-> ghost planes (parallel/halo.py layout), on
  // the storage layout `wlatd` describes
  bool halo = false, split = false;
  const int64_t* wlatd = nullptr;
  void *hbuf_a = nullptr, *hbuf_b = nullptr;
  const int64_t *face_boxes = nullptr, *ghost_boxes = nullptr;
  int nface_boxes = 0, nghost_boxes = 0;
  int64_t face_total = 0, ghost_total = 0;
  std::vector<int64_t> face_cnt, face_off, ghost_cnt, ghost_off;
  // phase profiling (eager iterations only)
  bool prof = false;
  hipEvent_t pev[kNMarks] = {};
  // state
  long it = 0;
  // Lagged x update: `pend` terms alpha_j p_j are not yet in x (0, 1 or 2).
  // One-term kernels fold alpha_prev p_old into x at every iteration (pend
  // stays 1).  fused5 pairs them (xpair): an iteration
  // with one term pending only saves alpha_prev (kXSave), the next folds
  // both, reading p_prev2 from the p buffer it is about to overwrite (kXPair)
  // -- x is read and written every other iteration, for one extra p read:
  // 5.5 instead of 6 operator streams per iteration, but unevenly spread.
  int pend = 0;
  bool xpair = false;
  // Staggered pairing (xpair on tiled storage, BDX_XSTAGGER): the odd tiles
  // ((ty + tz) odd) run the save / pair cycle one iteration out of phase
  // with their own pending count pend1, so every iteration carries half of
  // the x stream instead of all of it every other iteration.  The saved
  // alpha alternates between two scalar slots (kScalXSave + iteration parity).
  bool stagger = false;
  int pend1 = 0;
  int cur_m1 = kXSingle;  // the odd tiles' mode of the iteration being launched
  bool use_graph = true, graph_ok[4] = {false, false, false, false};
  hipGraphExec_t graph[4] = {nullptr, nullptr, nullptr, nullptr};
  hipEvent_t ev_batch[2] = {nullptr, nullptr};  // in-flight bound (iterate_on_stream)
  std::vector<hipEvent_t> tev;                  // per-step timing events

  virtual ~LoopBase() {
    drop_graphs();
    for (auto& e : pev)
      if (e) hipEventDestroy(e);
    for (hipEvent_t e : tev) hipEventDestroy(e);
    for (hipEvent_t e : {ev_in, ev_out, ev_fork, ev_rev, ev_batch[0], ev_batch[1]})
      if (e) hipEventDestroy(e);
    if (si) hipStreamDestroy(si);
    if (ev_int) hipEventDestroy(ev_int);
    if (st) hipStreamDestroy(st);
    if (cs) hipStreamDestroy(cs);
    if (pf_scal) hipFree(pf_scal);
  }
  // One CG iteration with explicit parity / flags (stream-ordered, no sync).
  // xm: kXSingle (pend 0: no x term; else alpha_prev p_old), kXSave, kXPair.
  virtual int step(long k, bool first, bool xlag, int xm) = 0;
  // x += the pending lagged terms (end of iterate() / profile())
  virtual int flush() = 0;
  // bring the prologue's state into the loop's own storage (tiled layouts)
  virtual int import_state() { return 0; }
  // the vector the forward halo carries (the pre-flight exchanges it)
  virtual void* halo_vector() = 0;
  virtual bool tiled() const { return false; }

  void mark(int id, hipStream_t s) {
    if (prof) (void)hipEventRecord(pev[id], s);
  }

  // The interior launch's stream of the split schedule (BDX_SPLIT):
  //   prio  (default) the compute stream st; the comm stream has the
  //         device's greatest priority;
  //   mask  its own stream si whose CU mask excludes BDX_SPLIT_RESERVE CUs
  //         (default 16), so the comm stream's chain -- RCCL kernels,
  //         boundary tiles, ghost fold -- always finds free CUs instead of
  //         queueing behind the interior grid's workgroups;
  //   maskr as mask, and the comm stream is confined to the reserved CUs.
  // The reserved CUs are mask bits 0 .. reserve-1, which the hardware deals
  // round-robin over the XCDs (csrc/micro/dispatch_prio.hip census).
  // hipExtStreamCreateWithCUMask takes no flags or priority: si (mask, maskr)
  // and the re-created cs (maskr) are BLOCKING streams at the DEFAULT
  // priority, unlike the non-blocking greatest-priority cs of init_common.
  // So in maskr the comm chain loses its priority, and both streams
  // synchronise with the legacy null stream: any work the caller submits to
  // the null stream while iterate() runs serialises with them.  The mask /
  // maskr A/Bs (profiles/r5_split_schedule.md) ran with nothing on the null
  // stream; comm_priority() reports the priority cs really has.
  int make_interior_stream() {
    const char* e = std::getenv("BDX_SPLIT");
    const std::string mode = e ? e : "prio";
    if (mode == "prio" || mode.empty()) return 0;
    if (mode != "mask" && mode != "maskr") return static_cast<int>(hipErrorInvalidValue);
    int dev = 0, ncu = 0;
    BDX_CHECK(hipGetDevice(&dev));
    BDX_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    const char* r = std::getenv("BDX_SPLIT_RESERVE");
    reserve = r ? std::atoi(r) : 16;
    if (reserve < 1 || reserve >= ncu) return static_cast<int>(hipErrorInvalidValue);
    const int words = (ncu + 31) / 32;
    mask_si.assign(words, 0u);
    mask_cs.assign(words, 0u);
    for (int b = 0; b < ncu; ++b) (b < reserve ? mask_cs : mask_si)[b / 32] |= 1u << (b % 32);
    BDX_CHECK(hipExtStreamCreateWithCUMask(&si, static_cast<uint32_t>(words), mask_si.data()));
    BDX_CHECK(hipEventCreateWithFlags(&ev_int, hipEventDisableTiming));
    if (mode == "maskr") {
      BDX_CHECK(hipStreamDestroy(cs));
      cs = nullptr;
      BDX_CHECK(hipExtStreamCreateWithCUMask(&cs, static_cast<uint32_t>(words), mask_cs.data()));
      BDX_CHECK(hipStreamGetPriority(cs, &prio_cs));
    }
    return 0;
  }
  // interior launch `f(stream)` of the split schedule on si or st; st
  // continues after it (the caller then joins the comm stream)
  template <typename F>
  int interior(F&& f) {
    if (!si) return f(st);
    BDX_CHECK(hipStreamWaitEvent(si, ev_fork, 0));
    if (int rc = f(si)) return rc;
    BDX_CHECK(hipEventRecord(ev_int, si));
    BDX_CHECK(hipStreamWaitEvent(st, ev_int, 0));
    return 0;
  }

  // Streams, events, halo tables and the transport (every runtime kind).
  // ptrs: hbuf_a, hbuf_b, face_boxes, ghost_boxes.
  int init_common(hipStream_t ext_stream, void* const* hptrs, const int64_t* halo_sizes,
                  const int64_t* fcnt, const int64_t* gcnt, int transport, int n, int r,
                  int64_t group_id) {
    nranks = n;
    rank = r;
    ext = ext_stream;
    // The comm stream runs at the greatest priority the device offers: its
    // chain (RCCL send/recv kernels, the boundary work, the reverse send) is
    // dispatched ahead of the interior launch's queued workgroups as soon as
    // resident ones retire, instead of after the whole interior grid.
    if (hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest) != hipSuccess) {
      (void)hipGetLastError();
      prio_least = prio_greatest = 0;
    }
    BDX_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    BDX_CHECK(hipStreamCreateWithPriority(&cs, hipStreamNonBlocking, prio_greatest));
    BDX_CHECK(hipStreamGetPriority(cs, &prio_cs));
    for (hipEvent_t* e : {&ev_in, &ev_out, &ev_fork, &ev_rev, &ev_batch[0], &ev_batch[1]})
      BDX_CHECK(hipEventCreateWithFlags(e, hipEventDisableTiming));
    hbuf_a = hptrs[0];
    hbuf_b = hptrs[1];
    face_boxes = static_cast<const int64_t*>(hptrs[2]);
    ghost_boxes = static_cast<const int64_t*>(hptrs[3]);
    nface_boxes = static_cast<int>(halo_sizes[0]);
    face_total = halo_sizes[1];
    nghost_boxes = static_cast<int>(halo_sizes[2]);
    ghost_total = halo_sizes[3];
    face_cnt.assign(fcnt, fcnt + n);
    ghost_cnt.assign(gcnt, gcnt + n);
    face_off.assign(n, 0);
    ghost_off.assign(n, 0);
    for (int p = 1; p < n; ++p) {
      face_off[p] = face_off[p - 1] + face_cnt[p - 1];
      ghost_off[p] = ghost_off[p - 1] + ghost_cnt[p - 1];
    }
    halo = n > 1 && (face_total + ghost_total) > 0;
    if (transport == 1 && n > 1) {  // RCCL: connected by bdx_rt_connect
      auto t = std::make_unique<RcclTransport>();
      t->nranks = n;
      tr = std::move(t);
    } else if (transport == 2 && n > 1) {  // in-process threads
      auto t = std::make_unique<ThreadTransport>();
      {
        std::lock_guard<std::mutex> lk(g_groups_m);
        auto& g = g_groups[group_id];
        if (!g) {
          g = std::make_shared<ThreadGroupState>();
          g->size = n;
          g->sbuf.assign(n, nullptr);
          g->soff.assign(n, nullptr);
          g->packed.assign(n, nullptr);
          g->copied.assign(n, nullptr);
          g->red.assign(n, nullptr);
        }
        t->g = g;
      }
      t->rank = r;
      tr = std::move(t);
    } else if (transport == 3 && n > 1) {  // emulated links (one rank alone)
      auto t = std::make_unique<LinkEmuTransport>();
      t->nranks = n;
      tr = std::move(t);
    } else {  // single rank: no communication
      tr = std::make_unique<NoTransport>();
      halo = false;
    }
    return 0;
  }

  int box_copy(int mode, void* vec, const int64_t* boxes, int nb, int64_t total, void* buf,
               hipStream_t s) {
    if (esize == 8)
      return bdx_box_copy_lat_f64(mode, static_cast<double*>(vec), wlatd, boxes, nb, total,
                                  static_cast<double*>(buf), s);
    return bdx_box_copy_lat_f32(mode, static_cast<float*>(vec), wlatd, boxes, nb, total,
                                static_cast<float*>(buf), s);
  }
  // forward: owned lower faces of v -> peers' ghost planes (pack, exchange, unpack)
  int halo_forward(void* v, hipStream_t s) {
    int rc = box_copy(0, v, face_boxes, nface_boxes, face_total, hbuf_a, s);
    if (rc || (rc = tr->exchange(hbuf_a, face_cnt, face_off, hbuf_b, ghost_cnt, ghost_off,
                                 esize, s)))
      return rc;
    return box_copy(1, v, ghost_boxes, nghost_boxes, ghost_total, hbuf_b, s);
  }
  // reverse, first half: ghost-plane partial sums of v -> peers (pack, exchange)
  int halo_reverse_send(void* v, hipStream_t s) {
    const int rc = box_copy(0, v, ghost_boxes, nghost_boxes, ghost_total, hbuf_a, s);
    if (rc) return rc;
    return tr->exchange(hbuf_a, ghost_cnt, ghost_off, hbuf_b, face_cnt, face_off, esize, s);
  }
  // reverse, second half: add the received sums into the owned lower faces
  int halo_reverse_add(void* v, hipStream_t s) {
    return box_copy(2, v, face_boxes, nface_boxes, face_total, hbuf_b, s);
  }

  // x mode of the next iteration (kXSingle with pend == 0: no x update)
  int next_xmode() const {
    if (pend == 0 || !xpair) return kXSingle;
    return pend == 1 ? kXSave : kXPair;
  }
  // the odd tiles' mode for an even-tile mode m0 (staggered pairing)
  int next_xmode1(int m0) const {
    if (!stagger) return m0;
    if (m0 == kXSave) return pend1 == 2 ? kXPair : kXSingle;
    if (m0 == kXPair) return kXSave;
    return kXSingle;
  }
  static int advanced(int p, int xm) { return (p == 0 || xm == kXPair) ? 1 : (xm == kXSave ? 2 : 1); }
  void advance_pend(int xm, int xm1) {
    pend = advanced(pend, xm);
    pend1 = stagger ? advanced(pend1, xm1) : pend;
  }
  // the periodic regime, in which one graph per (parity, even-tile mode) holds
  static bool periodic(int m0, int m1) {
    return (m0 == kXSave && m1 == kXPair) || (m0 == kXPair && m1 == kXSave);
  }

  // Capture the steady-state iteration of a parity and x mode (it > 0,
  // lagged x update pending); graph index = parity + 2 * (xm == kXPair).
  bool capture(int parity, int xm) {
    hipGraph_t g = nullptr;
    if (hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    const int rc = step(parity, false, true, xm);
    const hipError_t e = hipStreamEndCapture(st, &g);
    if (rc || e != hipSuccess || !g) {
      if (g) hipGraphDestroy(g);
      (void)hipGetLastError();
      return false;
    }
    const int gi = parity + 2 * (xm == kXPair);
    const bool ok = hipGraphInstantiate(&graph[gi], g, nullptr, nullptr, 0) == hipSuccess;
    hipGraphDestroy(g);
    if (!ok) (void)hipGetLastError();
    return ok;
  }

  void drop_graphs() {
    for (int i = 0; i < 4; ++i) {
      if (graph[i]) hipGraphExecDestroy(graph[i]);
      graph[i] = nullptr;
      graph_ok[i] = false;
    }
  }

  // n iterations; step_ms (may be null): n per-step device times from
  // timing events recorded between the iterations (no extra work, no sync)
  int iterate(long n, float* step_ms = nullptr) {
    if (tr->aborted()) return kErrAborted;
    BDX_CHECK(hipEventRecord(ev_in, ext));
    BDX_CHECK(hipStreamWaitEvent(st, ev_in, 0));
    int rc = iterate_on_stream(n, step_ms);
    BDX_CHECK(hipEventRecord(ev_out, st));
    BDX_CHECK(hipStreamWaitEvent(ext, ev_out, 0));
    if (!rc && step_ms) {
      if ((rc = tr->wait(ev_out))) return rc;
      for (long i = 0; i < n; ++i) {
        BDX_CHECK(hipEventElapsedTime(&step_ms[i], tev[i], tev[i + 1]));
      }
    }
    return rc;
  }

  // Iterations are enqueued in batches of kBatch under a watchdog Busy
  // scope, and before each batch the host waits (bounded by the deadline)
  // for the batch before the previous one: at most 2 kBatch iterations are
  // in flight, so an enqueue can never block for long behind a stuck peer
  // outside a deadline-covered scope, and a long run never trips it.
  static constexpr long kBatch = 32;
  int iterate_on_stream(long n, float* step_ms) {
    if (int rc = import_state()) return rc;
    if (step_ms) {
      while (static_cast<long>(tev.size()) < n + 1) {
        hipEvent_t e = nullptr;
        BDX_CHECK(hipEventCreate(&e));
        tev.push_back(e);
      }
      BDX_CHECK(hipEventRecord(tev[0], st));
    }
    for (long i0 = 0; i0 < n; i0 += kBatch) {
      if (i0 >= 2 * kBatch) {
        if (int rc = tr->wait(ev_batch[(i0 / kBatch) % 2])) return rc;
      }
      bdx::Watchdog::Busy busy(tr->watchdog());
      for (long i = i0; i < n && i < i0 + kBatch; ++i) {
        const bool first = (it == 0);
        const int par = static_cast<int>(it % 2);
        const int xm = next_xmode();
        cur_m1 = next_xmode1(xm);
        const int gi = par + 2 * (xm == kXPair);
        const bool steady = !first && pend > 0 && !prof && (!stagger || periodic(xm, cur_m1));
        if (steady && use_graph && tr->capturable() && !graph_ok[gi]) {
          graph_ok[gi] = capture(par, xm);
          if (!graph_ok[gi]) use_graph = false;  // fall back to eager launches
        }
        if (steady && use_graph && graph_ok[gi]) {
          BDX_CHECK(hipGraphLaunch(graph[gi], st));
        } else {
          const int rc = step(it, first, pend > 0, xm);
          if (rc) return rc;
        }
        advance_pend(xm, cur_m1);
        ++it;
        if (step_ms) BDX_CHECK(hipEventRecord(tev[i + 1], st));
      }
      BDX_CHECK(hipEventRecord(ev_batch[(i0 / kBatch) % 2], st));
    }
    bdx::Watchdog::Busy busy(tr->watchdog());
    return flush();
  }

  // n eager iterations with timing events between the phases; out[i] = mean
  // ms of interval i (see bdx_rt_profile for the list).
  static constexpr int kNPhases = 13;
  int profile(long n, double* out, int nout) {
    if (nout < kNPhases) return static_cast<int>(hipErrorInvalidValue);
    for (int i = 0; i < kNMarks; ++i)
      if (!pev[i]) BDX_CHECK(hipEventCreate(&pev[i]));
    for (int i = 0; i < nout; ++i) out[i] = 0.0;
    BDX_CHECK(hipEventRecord(ev_in, ext));
    BDX_CHECK(hipStreamWaitEvent(st, ev_in, 0));
    // prof is cleared on every exit path (an early error return must not
    // leave later iterate() calls eager and recording phase events)
    struct ProfGuard {
      bool& f;
      ~ProfGuard() { f = false; }
    } guard{prof};
    prof = true;
    bdx::Watchdog::Busy busy(tr->watchdog());
    int rc = import_state();
    for (long i = 0; i < n && !rc; ++i) {
      const bool first = (it == 0);
      const int xm = next_xmode();
      cur_m1 = next_xmode1(xm);
      rc = step(it, first, pend > 0, xm);
      if (rc) break;
      advance_pend(xm, cur_m1);
      ++it;
      if ((rc = static_cast<int>(hipEventRecord(ev_out, st)))) break;
      if ((rc = tr->wait(ev_out))) break;
      auto dt = [&](int a, int b) {
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, pev[a], pev[b]);
        return static_cast<double>(ms);
      };
      out[0] += dt(kMFwdBeg, kMFwdEnd);
      out[1] += dt(kMStart, kMOpA);
      // split: forward-halo end -> boundary work; serial: the boundary work
      // only (kMFwdEnd precedes the whole operator there)
      out[2] += split ? dt(kMFwdEnd, kMBnd) : dt(kMOpA, kMBnd);
      out[3] += dt(kMRevBeg, kMRevEnd);
      out[4] += dt(kMOpA, kMJoin);
      out[5] += dt(kMJoin, kMPap);
      out[6] += dt(kMPap, kMUpd);
      out[7] += dt(kMUpd, kMEnd);
      out[8] += dt(kMStart, kMEnd);
      // timeline offsets from the iteration start: the comm-stream chain is
      // hidden when it completes before the interior work does
      out[9] += dt(kMStart, kMFwdEnd);
      out[10] += dt(kMStart, kMBnd);
      out[11] += dt(kMStart, kMRevEnd);
      out[12] += dt(kMStart, kMOpA);
    }
    prof = false;
    if (!rc) rc = flush();
    BDX_CHECK(hipEventRecord(ev_out, st));
    BDX_CHECK(hipStreamWaitEvent(ext, ev_out, 0));
    for (int i = 0; i < kNPhases && n > 0; ++i) out[i] /= static_cast<double>(n);
    return rc;
  }

  // Pre-flight of the transport before any timed work (bench.py at N > 1):
  // one forward halo exchange of the loop's halo vector and a device
  // all-reduce of (rank + 1), under a deadline of timeout_s instead of the
  // run's.  out[0] = host ms of both, out[1] = the all-reduce result
  // (n (n + 1) / 2 when every rank took part).  A peer that never joins
  // aborts the communicator: the error comes back here instead of a hang
  // inside the warmup.
  int preflight(double timeout_s, double* out) {
    if (!pf_scal) BDX_CHECK(hipMalloc(&pf_scal, sizeof(double)));
    const double v = rank + 1.0;
    bdx::Watchdog* wd = tr->watchdog();
    const double old = wd ? wd->timeout_s() : 0.0;
    if (wd && timeout_s > 0) wd->set_timeout(timeout_s);
    struct Restore {
      bdx::Watchdog* w;
      double t;
      ~Restore() {
        if (w) w->set_timeout(t);
      }
    } restore{wd, old};
    BDX_CHECK(hipEventRecord(ev_in, ext));
    BDX_CHECK(hipStreamWaitEvent(st, ev_in, 0));
    const int64_t t0 = bdx::Watchdog::now_ns();
    int rc = 0;
    {
      bdx::Watchdog::Busy busy(wd);
      BDX_CHECK(hipMemcpyAsync(pf_scal, &v, sizeof(double), hipMemcpyHostToDevice, st));
      if (halo) rc = halo_forward(halo_vector(), st);
      if (!rc && nranks > 1) rc = tr->allreduce_sum(pf_scal, 1, st);
      if (!rc) rc = static_cast<int>(hipEventRecord(ev_out, st));
    }
    if (!rc) rc = tr->wait(ev_out);
    if (rc) return rc;
    out[0] = (bdx::Watchdog::now_ns() - t0) * 1e-6;
    BDX_CHECK(hipMemcpy(&out[1], pf_scal, sizeof(double), hipMemcpyDeviceToHost));
    BDX_CHECK(hipStreamWaitEvent(ext, ev_out, 0));
    return 0;
  }
};

// ---------------------------------------------------- fused structured operator
struct RtConfig {
  int64_t latd[21];
  int64_t latdT[21];  // tiled-storage descriptor (tsy = 0: lattice layout)
  int64_t own[3];
  int version, affine, P, nq, nblocks, nty, ntz, sy, sz, nseg;
  double kappa;
  std::vector<double> wts, qpts;
};

template <typename T>
struct CGRuntime final : LoopBase {
  RtConfig cfg;
  ApplyFn<T> apply = nullptr;
  std::vector<T> tabs_host;
  const T* tabs = nullptr;  // host copy (fused2/3: kernarg tables) or device buffer (fused5)
  T *x, *r, *pa, *pb, *y, *yb, *zb, *cb;
  // Tiled storage (cfg.latdT[17] != 0): the iteration runs on tiled copies
  // xt, rt, pat, pbt, yt (allocated zeroed by the caller: the padding stays
  // zero); r and x are imported after each prologue and x is exported after
  // every iterate() / profile().  wx .. wy: the buffers the loop works on.
  bool is_tiled = false, need_import = false;
  T *xt = nullptr, *rt_ = nullptr, *pat = nullptr, *pbt = nullptr, *yt = nullptr;
  T *wx, *wr, *wpa, *wpb, *wy;
  const T* xv;
  const T* kc = nullptr;
  double *scal, *partials, *upart;
  // overlapped schedule: tile rectangles {ty0, ty1, tz0, tz1}
  int rect_a[4], rect_r1[4], rect_r2[4];  // interior, last tile row, last tile column

  bool tiled() const override { return is_tiled; }
  void* halo_vector() override { return wr; }

  int convert(int dir, T* lat, T* til, hipStream_t s) {
    if constexpr (sizeof(T) == 8)
      return bdx_layout_convert_f64(dir, cfg.latdT, lat, til, s);
    else
      return bdx_layout_convert_f32(dir, cfg.latdT, lat, til, s);
  }
  // tiled: bring the prologue's r and x into the tiled copies, p_old = 0
  int import_state() override {
    if (!is_tiled || !need_import) return 0;
    need_import = false;
    int rc;
    if ((rc = convert(0, r, rt_, st)) || (rc = convert(0, x, xt, st))) return rc;
    const BdxLattice L = BdxLattice::from(cfg.latdT);
    return static_cast<int>(hipMemsetAsync(pat, 0, L.size() * sizeof(T), st));
  }
  int finalize_ghost(hipStream_t s) {
    if constexpr (sizeof(T) == 8)
      return bdx_fused_finalize_f64(wlatd, wy, yb, zb, cb, cfg.nty, cfg.ntz, cfg.sy, cfg.sz, 1,
                                    s);
    else
      return bdx_fused_finalize_f32(wlatd, wy, yb, zb, cb, cfg.nty, cfg.ntz, cfg.sy, cfg.sz, 1,
                                    s);
  }

  // The fused operator of iteration k on the tile rectangle `rect` (null:
  // every tile) on stream s.
  int launch_op(long k, bool first, bool xlag, int xm, const int* rect, hipStream_t s) {
    const int cur = (k % 2 == 0) ? kRR0 : kRR1, nxt = cur == kRR0 ? kRR1 : kRR0;
    T* pold = (k % 2 == 0) ? wpa : wpb;
    T* pnew = (k % 2 == 0) ? wpb : wpa;
    // mode word: CG | x mode (bits 4-5) | odd-tile x mode + 1 (6-7, 0: not
    // staggered) | segments (8-15) | saved-alpha slot parity to write (16)
    // and to read (17)
    const int m1 = stagger ? cur_m1 + 1 : 0;
    const int word = 1 | (xm << 4) | (m1 << 6) | (cfg.nseg << 8) | static_cast<int>((k & 1) << 16) |
                     static_cast<int>(((k + 1) & 1) << 17);
    return apply(word, cfg.affine, wlatd, cfg.nq, cfg.wts.data(),
                 cfg.qpts.data(), wr, pold, pnew, wx, wy, yb, zb, cb, xv, kc, tabs, cfg.kappa,
                 scal, partials, first ? -1 : cur, first ? -1 : nxt, xlag ? nxt : -1,
                 xlag ? kPAP : -1, cfg.nty, cfg.ntz, rect, s);
  }

  int step(long k, bool first, bool xlag, int xm) override {
    const int cur = (k % 2 == 0) ? kRR0 : kRR1, nxt = cur == kRR0 ? kRR1 : kRR0;
    T* const r = wr;
    T* const y = wy;
    auto op = [&](const int* rect, hipStream_t s) {
      return launch_op(k, first, xlag, xm, rect, s);
    };
    int rc;
    mark(kMStart, st);
    if (split) {
      // Two streams (reference src/laplacian.hpp:281-349, redesigned):
      //   cs: forward exchange -> boundary tiles (the last tile row and
      //       column, which read the ghost planes) -> ghost-plane fold ->
      //       reverse send;
      //   st: every interior tile, concurrently -- the exchanges and the
      //       small boundary launches all ride under the interior launch, so
      //       none of them is on the critical path as long as the interior
      //       work outlasts them;
      //   st: wait for cs, add the received sums into the owned faces.
      // Write sets are disjoint: a tile writes only its own nodes and its own
      // interface partials, and the ghost-plane fold reads only partials of
      // boundary tiles (fused_finalize_ghost_kernel).
      BDX_CHECK(hipEventRecord(ev_fork, st));
      BDX_CHECK(hipStreamWaitEvent(cs, ev_fork, 0));
      mark(kMFwdBeg, cs);
      if ((rc = halo_forward(r, cs))) return rc;
      mark(kMFwdEnd, cs);
      if ((rc = op(rect_r1, cs)) || (rc = op(rect_r2, cs)) || (rc = finalize_ghost(cs)))
        return rc;
      mark(kMBnd, cs);
      mark(kMRevBeg, cs);
      if ((rc = halo_reverse_send(y, cs))) return rc;
      BDX_CHECK(hipEventRecord(ev_rev, cs));
      mark(kMRevEnd, cs);
      if ((rc = interior([&](hipStream_t s) {
             const int r2 = op(rect_a, s);
             mark(kMOpA, s);
             return r2;
           })))
        return rc;
      BDX_CHECK(hipStreamWaitEvent(st, ev_rev, 0));
      if ((rc = halo_reverse_add(y, st))) return rc;
      mark(kMJoin, st);
    } else {
      mark(kMFwdBeg, st);
      if (halo && (rc = halo_forward(r, st))) return rc;
      mark(kMFwdEnd, st);
      if ((rc = op(nullptr, st))) return rc;
      mark(kMOpA, st);
      if (halo && (rc = finalize_ghost(st))) return rc;
      mark(kMBnd, st);
      mark(kMRevBeg, st);
      if (halo && ((rc = halo_reverse_send(y, st)) || (rc = halo_reverse_add(y, st)))) return rc;
      mark(kMRevEnd, st);
      mark(kMJoin, st);
    }
    if ((rc = bdx_reduce_partials(partials, cfg.nblocks, scal, kPAP, st))) return rc;
    if (nranks > 1 && (rc = tr->allreduce_sum(scal + kPAP, 1, st))) return rc;
    mark(kMPap, st);
    if (is_tiled) {
      if constexpr (sizeof(T) == 8)
        rc = bdx_cg_update_tiled_f64(wlatd, cfg.own, r, y, yb, zb, cb, cfg.nty, cfg.ntz, scal, cur,
                                     kPAP, nxt, upart, st);
      else
        rc = bdx_cg_update_tiled_f32(wlatd, cfg.own, r, y, yb, zb, cb, cfg.nty, cfg.ntz, scal, cur,
                                     kPAP, nxt, upart, st);
    } else if constexpr (sizeof(T) == 8) {
      rc = bdx_cg_update_iface_f64(cfg.latd, cfg.own, r, y, yb, zb, cb, cfg.nty, cfg.ntz, cfg.sy,
                                   cfg.sz, scal, cur, kPAP, nxt, upart, st);
    } else {
      rc = bdx_cg_update_iface_f32(cfg.latd, cfg.own, r, y, yb, zb, cb, cfg.nty, cfg.ntz, cfg.sy,
                                   cfg.sz, scal, cur, kPAP, nxt, upart, st);
    }
    if (rc) return rc;
    mark(kMUpd, st);
    if (nranks > 1 && (rc = tr->allreduce_sum(scal + nxt, 1, st))) return rc;
    mark(kMEnd, st);
    return 0;
  }

  // x += alpha_last p_last (and, with two terms pending, the saved
  // alpha_prev p_prev, which is the last iteration's p_old)
  int flush() override {
    if (pend == 0 && pend1 == 0) return 0;
    const int last = ((it - 1) % 2 == 0) ? kRR0 : kRR1;
    T* plast = ((it - 1) % 2 == 0) ? wpb : wpa;  // p_new of the last iteration
    T* pprev = ((it - 1) % 2 == 0) ? wpa : wpb;  // its p_old
    // two terms pending: alpha_prev was saved by the last iteration
    const int slot = kScalXSave + static_cast<int>((it - 1) & 1);
    const bool two = pend == 2, two1 = stagger ? pend1 == 2 : two;
    if (is_tiled) {
      // export x + the pending terms in one pass; the tiled iterate keeps
      // them pending (the next call continues the lagged chain), which saves
      // the write-back of the tiled x (one of five streams of the pass)
      const T* p2 = (two || two1) ? pprev : nullptr;
      const int mask = (two ? 1 : 0) | (two1 ? 2 : 0) | 4;  // tile colours with two terms
      if constexpr (sizeof(T) == 8)
        return bdx_flush_export_f64(cfg.latdT, x, wx, plast, p2, scal, last, kPAP, slot, -1, mask,
                                    st);
      else
        return bdx_flush_export_f32(cfg.latdT, x, wx, plast, p2, scal, last, kPAP, slot, -1, mask,
                                    st);
    }
    pend = pend1 = 0;
    auto one = [&](T* p, int num, int den) {
      if constexpr (sizeof(T) == 8)
        return bdx_xflush_f64(cfg.latd, cfg.own, x, p, scal, num, den, st);
      else
        return bdx_xflush_f32(cfg.latd, cfg.own, x, p, scal, num, den, st);
    };
    int rc = one(plast, last, kPAP);
    if (!rc && two) rc = one(pprev, slot, -1);
    return rc;
  }

  // Overlap probe (one rank only): does a comm-stream chain get CUs while the
  // interior launch fills the chip?  The chain of the split schedule of a
  // rank with y and z ghost planes (the N = 8 1 x 2 x 4 split) is replayed
  // on cs with a 1-rank RCCL communicator: grouped self send/recv of n
  // doubles (buf[0, n) -> buf[n, 2n)), the last tile row and column, the
  // reverse send/recv; concurrently st runs the interior tile rectangle.
  // out (ms, medians over reps): 0 chain alone, 1 interior alone, 2 chain
  // done and 3 interior done measured from the common fork, 4 one exchange
  // alone.  The CG state is clobbered: the caller restarts CG afterwards.
  int overlap_probe(int64_t n, double* buf, int reps, double* out) {
    if (nranks != 1 || cfg.nty < 2 || cfg.ntz < 2 || n <= 0 || reps <= 0)
      return static_cast<int>(hipErrorInvalidValue);
    ncclUniqueId id;
    if (ncclGetUniqueId(&id) != ncclSuccess) return -10;
    RcclTransport t;
    if (t.connect(id, 1, 0)) return -11;
    const std::vector<int64_t> cnt{n}, off0{0}, offn{n};
    auto xchg = [&](hipStream_t s) {
      return t.exchange(buf, cnt, off0, buf, cnt, offn, sizeof(double), s);
    };
    const int iy = cfg.nty - 1, iz = cfg.ntz - 1;
    const int ra[4] = {0, iy, 0, iz}, r1[4] = {iy, cfg.nty, 0, cfg.ntz}, r2[4] = {0, iy, iz, cfg.ntz};
    // ev (optional): recorded when the forward exchange is done
    auto chain = [&](hipStream_t s, hipEvent_t ev = nullptr) {
      int rc = xchg(s);
      if (!rc && ev) rc = static_cast<int>(hipEventRecord(ev, s));
      if (!rc) rc = launch_op(0, true, false, kXSingle, r1, s);
      if (!rc) rc = launch_op(0, true, false, kXSingle, r2, s);
      if (!rc) rc = xchg(s);
      return rc;
    };
    hipEvent_t e[5] = {};
    struct Free {  // before the creation loop: a failed create leaks nothing
      hipEvent_t* e;
      ~Free() {
        for (int i = 0; i < 5; ++i)
          if (e[i]) hipEventDestroy(e[i]);
      }
    } fr{e};
    for (auto& x : e) BDX_CHECK(hipEventCreate(&x));
    auto ms = [&](int a, int b) {
      float v = 0.f;
      (void)hipEventElapsedTime(&v, e[a], e[b]);
      return static_cast<double>(v);
    };
    BDX_CHECK(hipDeviceSynchronize());
    int rc = chain(cs);  // warm-up: RCCL connection setup, first launches
    if (!rc) rc = launch_op(0, true, false, kXSingle, ra, st);
    if (rc) return rc;
    BDX_CHECK(hipDeviceSynchronize());
    std::vector<double> v[6];
    bdx::Watchdog::Busy busy(t.watchdog());
    for (int it = 0; it < reps; ++it) {
      // alone: the chain, the interior, one exchange (each drained before the next)
      BDX_CHECK(hipEventRecord(e[0], cs));
      if ((rc = chain(cs))) return rc;
      BDX_CHECK(hipEventRecord(e[1], cs));
      BDX_CHECK(hipDeviceSynchronize());
      BDX_CHECK(hipEventRecord(e[2], st));
      if ((rc = launch_op(0, true, false, kXSingle, ra, st))) return rc;
      BDX_CHECK(hipEventRecord(e[3], st));
      BDX_CHECK(hipDeviceSynchronize());
      v[0].push_back(ms(0, 1));
      v[1].push_back(ms(2, 3));
      BDX_CHECK(hipEventRecord(e[0], cs));
      if ((rc = xchg(cs))) return rc;
      BDX_CHECK(hipEventRecord(e[1], cs));
      BDX_CHECK(hipDeviceSynchronize());
      v[4].push_back(ms(0, 1));
      // together, enqueued in the runtime's order: fork, cs chain, st interior
      BDX_CHECK(hipEventRecord(e[0], st));
      BDX_CHECK(hipStreamWaitEvent(cs, e[0], 0));
      if ((rc = chain(cs, e[4]))) return rc;
      BDX_CHECK(hipEventRecord(e[1], cs));
      if ((rc = launch_op(0, true, false, kXSingle, ra, st))) return rc;
      BDX_CHECK(hipEventRecord(e[2], st));
      BDX_CHECK(hipDeviceSynchronize());
      v[2].push_back(ms(0, 1));
      v[3].push_back(ms(0, 2));
      v[5].push_back(ms(0, 4));
    }
    for (int i = 0; i < 6; ++i) {
      std::sort(v[i].begin(), v[i].end());
      out[i] = v[i][v[i].size() / 2];
    }
    return 0;
  }
};

// -------------------------------------------------------------- dofmap operator
// The reference's data model (explicit cell -> dof map, stored or on-the-fly G,
// atomic scatter; csrc/hip/lap_dofmap.h) on the same loop: the interior cells
// run on the compute stream while the comm stream does the forward exchange,
// the boundary cells (those touching a ghost dof) and the reverse send of the
// ghost partial sums -- the reference's scatter_fwd_begin / lcells /
// scatter_fwd_end / bcells schedule (src/laplacian.hpp:281-349), without its
// host syncs and with the boundary cells off the critical path.
struct DofConfig {
  int64_t latd[21];
  int P, nq, geom, n_inner, n_outer, nb_inner, nb_outer;
  int64_t nvec;
  double kappa;
};

template <typename T>
struct DofCGRuntime final : LoopBase {
  DofConfig cfg;
  const T* tab = nullptr;
  const int *inner = nullptr, *outer = nullptr, *cdofs = nullptr, *cverts = nullptr;
  const T *coords = nullptr, *G = nullptr, *kc = nullptr;
  const unsigned char* flags = nullptr;
  T *x, *r, *pa, *pb, *y;
  double *scal, *partials, *upart;
  // y ping-pong: iteration k's operator adds into yk(k) and zeroes yk(k + 1)
  // (consumed by the update pass of iteration k - 1), so the update pass
  // streams r, y and r back and no longer writes y = 0 (one vector stream
  // less per iteration; the zero stores ride in the operator's tail).  y2 is
  // the runtime's own second buffer; y (the caller's) is yk of even k.
  // Invariant: after iterate() the caller's y holds A p of the last even
  // iteration (NOT zero) and y2 may be dirty.  Only reset() (called by
  // DofmapLaplacianGPU.cg_start, which zeroes the caller's y first) makes
  // the loop valid again: iteration 0 then adds into a zero y and zeroes y2
  // before iteration 1 adds into it.  No caller may read y after iterate()
  // or hand the solve to the Python driver mid-way without cg_start
  // (tests/test_gpu_dofmap.py::test_dofmap_native_second_solve_*).
  T* y2 = nullptr;
  T* yk(long k) const { return (k % 2 == 0) ? y : y2; }

  ~DofCGRuntime() override {
    if (y2) (void)hipFree(y2);
  }

  void* halo_vector() override { return r; }

  // zero: this launch also zeroes yk(k + 1)
  int run(const int* cells, int ncl, double* part, long k, bool first, bool xlag, bool zero,
          hipStream_t s) {
    if (ncl <= 0) return 0;
    const int cur = (k % 2 == 0) ? kRR0 : kRR1, nxt = cur == kRR0 ? kRR1 : kRR0;
    T* pold = (k % 2 == 0) ? pa : pb;
    T* pnew = (k % 2 == 0) ? pb : pa;
    T* const yz = zero ? yk(k + 1) : nullptr;
    int nb = 0;
    int rc;
    if constexpr (sizeof(T) == 8)
      rc = bdx_dofmap_apply_yz_f64(cfg.P, cfg.nq, cfg.geom, 1, tab, cells, ncl, cfg.nvec, cdofs,
                                   cverts, coords, flags, G, cfg.kappa, kc, r, pold, pnew, x,
                                   yk(k), yz, scal, first ? -1 : cur, first ? -1 : nxt,
                                   xlag ? nxt : -1, xlag ? kPAP : -1, part, &nb, s);
    else
      rc = bdx_dofmap_apply_yz_f32(cfg.P, cfg.nq, cfg.geom, 1, tab, cells, ncl, cfg.nvec, cdofs,
                                   cverts, coords, flags, G, cfg.kappa, kc, r, pold, pnew, x,
                                   yk(k), yz, scal, first ? -1 : cur, first ? -1 : nxt,
                                   xlag ? nxt : -1, xlag ? kPAP : -1, part, &nb, s);
    return rc;
  }

  int step(long k, bool first, bool xlag, int /*xm*/) override {
    const int cur = (k % 2 == 0) ? kRR0 : kRR1, nxt = cur == kRR0 ? kRR1 : kRR0;
    double* const part_b = partials + cfg.nb_inner;
    T* const yc = yk(k);
    // the interior launch zeroes yk(k + 1); the boundary one when there is none
    const bool z_in = cfg.n_inner > 0, z_out = !z_in;
    int rc;
    mark(kMStart, st);
    if (cfg.n_inner <= 0 && cfg.n_outer <= 0)  // a rank without cells: no launch zeroes it
      BDX_CHECK(hipMemsetAsync(yk(k + 1), 0, static_cast<size_t>(cfg.nvec) * sizeof(T), st));
    if (split) {
      // cs: forward exchange -> boundary cells -> reverse send of the ghost
      // partials; st: the interior cells (they touch no ghost dof), then the
      // received sums are added into the owned faces.  Both kernels add into
      // y with float atomics and write p / x only at their designated dofs
      // (lap_dofmap.h writer marks), so they may run concurrently.
      BDX_CHECK(hipEventRecord(ev_fork, st));
      BDX_CHECK(hipStreamWaitEvent(cs, ev_fork, 0));
      mark(kMFwdBeg, cs);
      if ((rc = halo_forward(r, cs))) return rc;
      mark(kMFwdEnd, cs);
      if ((rc = run(outer, cfg.n_outer, part_b, k, first, xlag, z_out, cs))) return rc;
      mark(kMBnd, cs);
      mark(kMRevBeg, cs);
      if ((rc = halo_reverse_send(yc, cs))) return rc;
      BDX_CHECK(hipEventRecord(ev_rev, cs));
      mark(kMRevEnd, cs);
      if ((rc = interior([&](hipStream_t s) {
             const int r2 = run(inner, cfg.n_inner, partials, k, first, xlag, z_in, s);
             mark(kMOpA, s);
             return r2;
           })))
        return rc;
      BDX_CHECK(hipStreamWaitEvent(st, ev_rev, 0));
      if ((rc = halo_reverse_add(yc, st))) return rc;
      mark(kMJoin, st);
    } else {
      mark(kMFwdBeg, st);
      if (halo && (rc = halo_forward(r, st))) return rc;
      mark(kMFwdEnd, st);
      if ((rc = run(inner, cfg.n_inner, partials, k, first, xlag, z_in, st))) return rc;
      mark(kMOpA, st);
      if ((rc = run(outer, cfg.n_outer, part_b, k, first, xlag, z_out, st))) return rc;
      mark(kMBnd, st);
      mark(kMRevBeg, st);
      if (halo && ((rc = halo_reverse_send(yc, st)) || (rc = halo_reverse_add(yc, st)))) return rc;
      mark(kMRevEnd, st);
      mark(kMJoin, st);
    }
    if ((rc = bdx_reduce_partials(partials, cfg.nb_inner + cfg.nb_outer, scal, kPAP, st)))
      return rc;
    if (nranks > 1 && (rc = tr->allreduce_sum(scal + kPAP, 1, st))) return rc;
    mark(kMPap, st);
    int nu = 0;
    if constexpr (sizeof(T) == 8)
      rc = bdx_dofmap_cg_update_z_f64(cfg.nvec, flags, r, yc, scal, cur, kPAP, upart, &nu, 0, st);
    else
      rc = bdx_dofmap_cg_update_z_f32(cfg.nvec, flags, r, yc, scal, cur, kPAP, upart, &nu, 0, st);
    if (rc || (rc = bdx_reduce_partials(upart, nu, scal, nxt, st))) return rc;
    mark(kMUpd, st);
    if (nranks > 1 && (rc = tr->allreduce_sum(scal + nxt, 1, st))) return rc;
    mark(kMEnd, st);
    return 0;
  }

  int flush() override {
    if (pend == 0) return 0;
    pend = 0;
    const int last = ((it - 1) % 2 == 0) ? kRR0 : kRR1;
    T* plast = ((it - 1) % 2 == 0) ? pb : pa;  // p_new of the last iteration
    if constexpr (sizeof(T) == 8)
      return bdx_dofmap_xflush_f64(cfg.nvec, x, plast, scal, last, kPAP, st);
    else
      return bdx_dofmap_xflush_f32(cfg.nvec, x, plast, scal, last, kPAP, st);
  }
};

// iparams of the fused kind: version, affine, P, nq, nblocks, nty, ntz, sy,
// sz, use_graph, overlap, nseg (nblocks = nty * ntz * nseg p.Ap partials)
template <typename T>
LoopBase* create(const int64_t* latd, const int64_t* own, const int* iparams, double kappa,
                 const double* wts, const double* qpts, const void* tabs, void* const* ptrs,
                 const int64_t* halo_sizes, const int64_t* face_cnt, const int64_t* ghost_cnt,
                 int transport, int nranks, int rank, int64_t group_id, hipStream_t st,
                 const int64_t* latd_tiled, void* const* tptrs) {
  auto rt = std::make_unique<CGRuntime<T>>();
  rt->esize = sizeof(T);
  RtConfig& c = rt->cfg;
  std::memcpy(c.latd, latd, sizeof(c.latd));
  std::memset(c.latdT, 0, sizeof(c.latdT));
  if (latd_tiled && latd_tiled[17] && tptrs) std::memcpy(c.latdT, latd_tiled, sizeof(c.latdT));
  std::memcpy(c.own, own, sizeof(c.own));
  c.version = iparams[0];
  c.affine = iparams[1];
  c.P = iparams[2];
  c.nq = iparams[3];
  c.nblocks = iparams[4];
  c.nty = iparams[5];
  c.ntz = iparams[6];
  c.sy = iparams[7];
  c.sz = iparams[8];
  rt->use_graph = iparams[9] != 0;
  const bool overlap = iparams[10] != 0;
  c.nseg = iparams[11] > 0 ? iparams[11] : 1;
  c.kappa = kappa;
  c.wts.assign(wts, wts + c.nq);
  c.qpts.assign(qpts, qpts + c.nq);
  rt->apply = apply_fn<T>(c.version, c.P);
  // paired lagged x update (fused5 only; BDX_XPAIR=0 folds one term per
  // iteration).  Paired on every tile at once, every other iteration carries
  // x, x and p_prev2 and the FP64 operator does not hide that burst (one
  // term per iteration was 2-4 % faster at Q6 FP64); staggered over the two
  // tile colours (tiled storage, below) the x stream is spread evenly and
  // the paired form is the fastest at Q3, Q6 and Q6 FP32
  // (profiles/r5_xpair_ab.md).
  {
    const char* e = std::getenv("BDX_XPAIR");
    rt->xpair = c.version == 5 && !(e && e[0] == '0');
  }
  if (!rt->apply || !tabs) return nullptr;
  if (c.version == 5) {
    rt->tabs = static_cast<const T*>(tabs);  // the operator's device table buffer
  } else {
    const T* tb = static_cast<const T*>(tabs);
    rt->tabs_host.assign(tb, tb + kFusedTabMax);
    rt->tabs = rt->tabs_host.data();
  }
  int i = 0;
  rt->x = static_cast<T*>(ptrs[i++]);
  rt->r = static_cast<T*>(ptrs[i++]);
  rt->pa = static_cast<T*>(ptrs[i++]);
  rt->pb = static_cast<T*>(ptrs[i++]);
  rt->y = static_cast<T*>(ptrs[i++]);
  rt->yb = static_cast<T*>(ptrs[i++]);
  rt->zb = static_cast<T*>(ptrs[i++]);
  rt->cb = static_cast<T*>(ptrs[i++]);
  rt->xv = static_cast<const T*>(ptrs[i++]);
  rt->scal = static_cast<double*>(ptrs[i++]);
  rt->partials = static_cast<double*>(ptrs[i++]);
  rt->upart = static_cast<double*>(ptrs[i++]);
  void* const* hptrs = ptrs + i;  // hbuf_a, hbuf_b, face_boxes, ghost_boxes
  i += 4;
  rt->kc = static_cast<const T*>(ptrs[i++]);
  rt->is_tiled = c.latdT[17] != 0;
  if (rt->is_tiled) {
    // only the x-march kernels whose tile is the storage tile address it
    if ((c.version != 3 && c.version != 5) || c.latdT[17] != c.sy || c.latdT[18] != c.sz)
      return nullptr;
    rt->xt = static_cast<T*>(tptrs[0]);
    rt->rt_ = static_cast<T*>(tptrs[1]);
    rt->pat = static_cast<T*>(tptrs[2]);
    rt->pbt = static_cast<T*>(tptrs[3]);
    rt->yt = static_cast<T*>(tptrs[4]);
    if (!rt->xt || !rt->rt_ || !rt->pat || !rt->pbt || !rt->yt) return nullptr;
  }
  // staggered pairing needs the flush's per-tile colours (tiled storage);
  // BDX_XSTAGGER=0 pairs every tile on the same iterations
  {
    const char* e = std::getenv("BDX_XSTAGGER");
    rt->stagger = rt->xpair && rt->is_tiled && !(e && e[0] == '0');
  }
  rt->wx = rt->is_tiled ? rt->xt : rt->x;
  rt->wr = rt->is_tiled ? rt->rt_ : rt->r;
  rt->wpa = rt->is_tiled ? rt->pat : rt->pa;
  rt->wpb = rt->is_tiled ? rt->pbt : rt->pb;
  rt->wy = rt->is_tiled ? rt->yt : rt->y;
  rt->wlatd = rt->is_tiled ? c.latdT : c.latd;
  if (rt->init_common(st, hptrs, halo_sizes, face_cnt, ghost_cnt, transport, nranks, rank,
                      group_id))
    return nullptr;
  // overlapped schedule: x whole, so only the last tile row (y ghost plane)
  // and the last tile column (z ghost plane) touch ghosts
  const BdxLattice L = BdxLattice::from(c.latd);
  const int g1 = static_cast<int>(L.gh[1]), g2 = static_cast<int>(L.gh[2]);
  if (overlap && rt->halo && L.gh[0] == 0 && (g1 || g2)) {
    const int iy = c.nty - g1, iz = c.ntz - g2;  // interior tile extents
    const int ra[4] = {0, iy, 0, iz};
    const int r1[4] = {iy, c.nty, 0, c.ntz}, r2[4] = {0, iy, iz, c.ntz};
    std::memcpy(rt->rect_a, ra, sizeof(ra));
    std::memcpy(rt->rect_r1, r1, sizeof(r1));
    std::memcpy(rt->rect_r2, r2, sizeof(r2));
    rt->split = true;
    if (rt->make_interior_stream()) return nullptr;
  }
  return rt.release();
}

// iparams of the dofmap kind: P, nq, geom, n_inner, n_outer, use_graph,
// overlap; ptrs: x, r, p_a, p_b, y, scal, partials, upart, hbuf_a, hbuf_b,
// face_boxes, ghost_boxes, tab, inner, outer, cdofs, cverts, coords, flags, G,
// kc (G / kc may be null)
template <typename T>
LoopBase* create_dofmap(const int64_t* latd, const int* iparams, int64_t nvec, double kappa,
                        void* const* ptrs, const int64_t* halo_sizes, const int64_t* face_cnt,
                        const int64_t* ghost_cnt, int transport, int nranks, int rank,
                        int64_t group_id, hipStream_t st) {
  auto rt = std::make_unique<DofCGRuntime<T>>();
  rt->esize = sizeof(T);
  DofConfig& c = rt->cfg;
  std::memcpy(c.latd, latd, sizeof(c.latd));
  c.P = iparams[0];
  c.nq = iparams[1];
  c.geom = iparams[2];
  c.n_inner = iparams[3];
  c.n_outer = iparams[4];
  rt->use_graph = iparams[5] != 0;
  const bool overlap = iparams[6] != 0;
  c.nvec = nvec;
  c.kappa = kappa;
  c.nb_inner = bdx_dofmap_nblocks(c.nq, c.n_inner);
  c.nb_outer = bdx_dofmap_nblocks(c.nq, c.n_outer);
  if (c.nb_inner < 0 || c.nb_outer < 0 || c.nb_inner + c.nb_outer > bdx_hip_partials_size())
    return nullptr;
  int i = 0;
  rt->x = static_cast<T*>(ptrs[i++]);
  rt->r = static_cast<T*>(ptrs[i++]);
  rt->pa = static_cast<T*>(ptrs[i++]);
  rt->pb = static_cast<T*>(ptrs[i++]);
  rt->y = static_cast<T*>(ptrs[i++]);
  rt->scal = static_cast<double*>(ptrs[i++]);
  rt->partials = static_cast<double*>(ptrs[i++]);
  rt->upart = static_cast<double*>(ptrs[i++]);
  void* const* hptrs = ptrs + i;
  i += 4;
  rt->tab = static_cast<const T*>(ptrs[i++]);
  rt->inner = static_cast<const int*>(ptrs[i++]);
  rt->outer = static_cast<const int*>(ptrs[i++]);
  rt->cdofs = static_cast<const int*>(ptrs[i++]);
  rt->cverts = static_cast<const int*>(ptrs[i++]);
  rt->coords = static_cast<const T*>(ptrs[i++]);
  rt->flags = static_cast<const unsigned char*>(ptrs[i++]);
  rt->G = static_cast<const T*>(ptrs[i++]);
  rt->kc = static_cast<const T*>(ptrs[i++]);
  if (!rt->tab || !rt->cdofs || !rt->flags || (c.geom == kGeomStored && !rt->G)) return nullptr;
  if (hipMalloc(&rt->y2, static_cast<size_t>(nvec) * sizeof(T)) != hipSuccess ||
      hipMemset(rt->y2, 0, static_cast<size_t>(nvec) * sizeof(T)) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  rt->wlatd = c.latd;
  if (rt->init_common(st, hptrs, halo_sizes, face_cnt, ghost_cnt, transport, nranks, rank,
                      group_id))
    return nullptr;
  rt->split = overlap && rt->halo && c.n_outer > 0;
  if (rt->split && rt->make_interior_stream()) return nullptr;
  return rt.release();
}

template <typename F>
auto with_rt(void* h, F&& f) {
  return f(static_cast<LoopBase*>(h));
}

}  // namespace

extern "C" {

int bdx_rt_nccl_unique_id(void* out128) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -1;
  std::memcpy(out128, &id, sizeof(id));
  return static_cast<int>(sizeof(id));
}

// Hardware self-test of the RCCL transport on one GPU (a 1-rank communicator):
// the grouped send/recv of RcclTransport::exchange to itself (buf[0, n) ->
// buf[n, 2n)), the device-scalar all-reduce of buf[2n, 2n+2), then the same
// pair captured into a hipGraph and replayed (into buf[2n+2, 3n+2)).  The
// multi-rank loop issues the identical calls over xGMI.  Returns 0 on success.
int bdx_rt_rccl_selftest(double* buf, int n, hipStream_t st) {
  ncclUniqueId id;
  if (ncclGetUniqueId(&id) != ncclSuccess) return -10;
  RcclTransport t;
  if (t.connect(id, 1, 0)) return -11;
  if (t.ranks() != 1) return -19;
  const std::vector<int64_t> cnt{n}, off0{0}, offn{n}, offg{2 * static_cast<int64_t>(n) + 2};
  int rc = t.exchange(buf, cnt, off0, buf, cnt, offn, sizeof(double), st);
  if (!rc) rc = t.allreduce_sum(buf + 2 * n, 2, st);
  if (!rc && hipStreamSynchronize(st) != hipSuccess) rc = -12;
  if (rc) return rc;
  // capture on an own non-blocking stream, as the runtime does (the caller's
  // stream may be the legacy default stream, which cannot be captured)
  hipStream_t cs = nullptr;
  if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return -13;
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  if (hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal) != hipSuccess) {
    hipStreamDestroy(cs);
    return -14;
  }
  rc = t.exchange(buf, cnt, off0, buf, cnt, offg, sizeof(double), cs);
  if (!rc) rc = t.allreduce_sum(buf + 2 * n, 2, cs);
  if (hipStreamEndCapture(cs, &g) != hipSuccess || !g) rc = rc ? rc : -15;
  if (!rc && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) rc = -16;
  if (!rc && hipGraphLaunch(ge, cs) != hipSuccess) rc = -17;
  hipEvent_t ev = nullptr;
  if (!rc && hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) rc = -18;
  if (!rc && hipEventRecord(ev, cs) != hipSuccess) rc = -18;
  if (!rc) rc = t.wait(ev);  // the watchdog-bounded host wait of the runtime
  if (ev) hipEventDestroy(ev);
  if (ge) hipGraphExecDestroy(ge);
  if (g) hipGraphDestroy(g);
  hipStreamDestroy(cs);
  return rc;
}

// latd_tiled / tptrs (may be null): the tiled-storage descriptor and the
// runtime's tiled x, r, p_a, p_b, y buffers (zero-initialised by the caller).
void* bdx_rt_create(int is_f64, const int64_t* latd, const int64_t* own, const int* iparams,
                    double kappa, const double* wts, const double* qpts, const void* tabs,
                    void* const* ptrs, const int64_t* halo_sizes, const int64_t* face_cnt,
                    const int64_t* ghost_cnt, int transport, int nranks, int rank,
                    int64_t group_id, hipStream_t st, const int64_t* latd_tiled,
                    void* const* tptrs) {
  if (is_f64)
    return create<double>(latd, own, iparams, kappa, wts, qpts, tabs, ptrs, halo_sizes,
                          face_cnt, ghost_cnt, transport, nranks, rank, group_id, st, latd_tiled,
                          tptrs);
  return create<float>(latd, own, iparams, kappa, wts, qpts, tabs, ptrs, halo_sizes, face_cnt,
                       ghost_cnt, transport, nranks, rank, group_id, st, latd_tiled, tptrs);
}

// The dofmap data model's CG loop (see create_dofmap for the arguments).
void* bdx_rt_create_dofmap(int is_f64, const int64_t* latd, const int* iparams, int64_t nvec,
                           double kappa, void* const* ptrs, const int64_t* halo_sizes,
                           const int64_t* face_cnt, const int64_t* ghost_cnt, int transport,
                           int nranks, int rank, int64_t group_id, hipStream_t st) {
  if (is_f64)
    return create_dofmap<double>(latd, iparams, nvec, kappa, ptrs, halo_sizes, face_cnt,
                                 ghost_cnt, transport, nranks, rank, group_id, st);
  return create_dofmap<float>(latd, iparams, nvec, kappa, ptrs, halo_sizes, face_cnt, ghost_cnt,
                              transport, nranks, rank, group_id, st);
}

// Comm stream priority: out[0] least, out[1] greatest (device range),
// out[2] the priority the comm stream runs at.
int bdx_rt_comm_priority(void* h, int* out) {
  return with_rt(h, [&](LoopBase* rt) {
    out[0] = rt->prio_least;
    out[1] = rt->prio_greatest;
    out[2] = rt->prio_cs;
    return 0;
  });
}

// Transport pre-flight (see LoopBase::preflight); out[2].
int bdx_rt_preflight(void* h, double timeout_s, double* out) {
  return with_rt(h, [&](LoopBase* rt) { return rt->preflight(timeout_s, out); });
}

// Comm/compute overlap probe on one GPU (see CGRuntime::overlap_probe;
// fused operators only); buf: 2 n doubles; out[6].
int bdx_rt_overlap_probe(void* h, int64_t n, double* buf, int reps, double* out) {
  return with_rt(h, [&](LoopBase* rt) -> int {
    if (auto* f = dynamic_cast<CGRuntime<double>*>(rt)) return f->overlap_probe(n, buf, reps, out);
    if (auto* f = dynamic_cast<CGRuntime<float>*>(rt)) return f->overlap_probe(n, buf, reps, out);
    return static_cast<int>(hipErrorInvalidValue);
  });
}

// 1 if the loop runs on the tiled storage layout.
int bdx_rt_tiled(void* h) {
  return with_rt(h, [](LoopBase* rt) { return rt->tiled() ? 1 : 0; });
}

// Open the runtime's RCCL communicator (collective over the ranks; every
// rank calls it only after all ranks created their runtime).  Bounded by the
// watchdog deadline.  0 on success (or when the transport is not RCCL).
int bdx_rt_connect(void* h, const void* uid, int rank) {
  return with_rt(h, [&](LoopBase* rt) -> int {
    auto* t = dynamic_cast<RcclTransport*>(rt->tr.get());
    if (!t) return 0;
    ncclUniqueId id;
    std::memcpy(&id, uid, sizeof(id));
    return t->connect(id, t->nranks, rank);
  });
}

// Ranks of the transport (ncclCommCount for RCCL; -1 if not connected).
int bdx_rt_comm_count(void* h) {
  return with_rt(h, [](LoopBase* rt) { return rt->tr->ranks(); });
}

// 1 if the overlapped (split, two-stream) schedule is active.
int bdx_rt_overlap(void* h) {
  return with_rt(h, [](LoopBase* rt) { return rt->split ? 1 : 0; });
}

// Reset the CG state after a new prologue (p_a zeroed by the caller).
int bdx_rt_reset(void* h) {
  return with_rt(h, [](LoopBase* rt) {
    rt->it = 0;
    rt->pend = rt->pend1 = 0;
    if (auto* f = dynamic_cast<CGRuntime<double>*>(rt)) f->need_import = f->is_tiled;
    if (auto* f = dynamic_cast<CGRuntime<float>*>(rt)) f->need_import = f->is_tiled;
    return 0;
  });
}

// Bind a new iterate buffer x (DeviceCG.start with another x): the captured
// graphs hold the old pointer, so they are dropped and re-captured.
int bdx_rt_bind_x(void* h, void* x) {
  return with_rt(h, [&](LoopBase* rt) -> int {
    auto rebind = [&](auto* f) -> int {
      using T = std::remove_pointer_t<decltype(f->x)>;
      if (f->x == static_cast<T*>(x)) return 0;
      const hipError_t e = hipStreamSynchronize(f->st);
      f->drop_graphs();
      f->x = static_cast<T*>(x);
      if constexpr (std::is_same_v<std::remove_pointer_t<decltype(f)>, CGRuntime<T>>) {
        if (!f->is_tiled) f->wx = f->x;
      }
      return static_cast<int>(e);
    };
    if (auto* f = dynamic_cast<CGRuntime<double>*>(rt)) return rebind(f);
    if (auto* f = dynamic_cast<CGRuntime<float>*>(rt)) return rebind(f);
    if (auto* f = dynamic_cast<DofCGRuntime<double>*>(rt)) return rebind(f);
    if (auto* f = dynamic_cast<DofCGRuntime<float>*>(rt)) return rebind(f);
    return static_cast<int>(hipErrorInvalidValue);
  });
}

int bdx_rt_iterate(void* h, long n) {
  return with_rt(h, [&](LoopBase* rt) { return rt->iterate(n); });
}

// iterate() plus the device time of each of the n steps (timing events
// between the steps, read after a bounded host wait): step_ms[n]
int bdx_rt_iterate_timed(void* h, long n, float* step_ms) {
  return with_rt(h, [&](LoopBase* rt) { return rt->iterate(n, step_ms); });
}

// Host wait for everything iterate() queued, bounded by the RCCL deadline
// (a hung peer aborts the communicator instead of blocking forever).
int bdx_rt_wait(void* h) {
  return with_rt(h, [](LoopBase* rt) { return rt->tr->wait(rt->ev_out); });
}

// n eager CG iterations with hipEvent phase timers; out (13 doubles, mean ms):
//   0 forward halo (comm stream: pack, exchange, unpack)
//   1 operator, interior tiles / cells (serial schedule: the first launch)
//   2 boundary work: split: ghost-touching tiles / cells (+ ghost fold)
//     after the forward halo; serial: what follows the first launch
//   3 reverse halo (pack, exchange; serial: + unpack-add)
//   4 interior done -> comm stream joined, received sums added
//   5 reduce + all-reduce(p.Ap)
//   6 r update + r.r
//   7 all-reduce(r.r)
//   8 whole iteration
//   9..12 end of the forward halo / boundary work / reverse halo / interior
//         work, measured from the iteration start (overlap evidence)
int bdx_rt_profile(void* h, long n, double* out, int nout) {
  return with_rt(h, [&](LoopBase* rt) { return rt->profile(n, out, nout); });
}

// it (iterations done) and whether steady-state graphs are in use.
int bdx_rt_state(void* h, long* it, int* graphs) {
  return with_rt(h, [&](LoopBase* rt) {
    *it = rt->it;
    *graphs = rt->use_graph &&
              (rt->graph_ok[0] || rt->graph_ok[1] || rt->graph_ok[2] || rt->graph_ok[3]);
    return 0;
  });
}

void bdx_rt_destroy(void* h) { delete static_cast<LoopBase*>(h); }

void bdx_rt_release_group(int64_t group_id) {
  std::lock_guard<std::mutex> lk(g_groups_m);
  g_groups.erase(group_id);
}

}  // extern "C"
