// Deadline watchdog for blocking communication calls (host C++, no HIP).
//
// The reference has no failure containment: a lost MPI peer hangs the job
// until the scheduler kills it.  The native CG runtime issues
// RCCL calls that block the host (connection setup inside ncclGroupEnd) or
// the device (a peer that never posts its matching send), so every such
// call, and every host wait on work that contains one, runs inside a
// `Watchdog::Busy` scope.  A monitor thread fires when a scope has been open
// longer than the deadline, or when `poll_error` reports an asynchronous
// communicator error; `on_fire` then aborts the communicator
// (ncclCommAbort), which makes the blocked call return, and the runtime turns
// the abort into an error code that Python raises as a non-zero exit.
//
// The policy (`check`) is a pure function of the clock value so it is unit
// tested on the CPU (bdx_watchdog_selftest in bdx_host.cpp).
#pragma once

#include <atomic>
#include <chrono>
#include <cstdint>
#include <functional>
#include <thread>

namespace bdx {

class Watchdog {
 public:
  using Clock = std::chrono::steady_clock;

  Watchdog(double timeout_s, std::function<bool()> poll_error, std::function<void()> on_fire)
      : timeout_ns_(static_cast<int64_t>(timeout_s * 1e9)),
        poll_error_(std::move(poll_error)),
        on_fire_(std::move(on_fire)) {}
  Watchdog(const Watchdog&) = delete;
  Watchdog& operator=(const Watchdog&) = delete;
  ~Watchdog() { stop(); }

  static int64_t now_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(Clock::now().time_since_epoch())
        .count();
  }

  // RAII scope around a call that may block on a peer.
  class Busy {
   public:
    explicit Busy(Watchdog* w) : w_(w) {
      if (w_) w_->enter(now_ns());
    }
    ~Busy() {
      if (w_) w_->leave();
    }
    Busy(const Busy&) = delete;
    Busy& operator=(const Busy&) = delete;

   private:
    Watchdog* w_;
  };

  void enter(int64_t t) {
    if (depth_.fetch_add(1) == 0) busy_since_.store(t);
  }
  void leave() {
    if (depth_.fetch_sub(1) == 1) busy_since_.store(0);
  }

  // One monitor decision at clock value `t`: fire (once) if a busy scope
  // has exceeded the deadline or the communicator reports an error.
  bool check(int64_t t) {
    if (fired_.load()) return true;
    const int64_t b = busy_since_.load(), lim = timeout_ns_.load();
    const bool late = b != 0 && lim > 0 && t - b > lim;
    const bool err = poll_error_ && poll_error_();
    if (!(late || err)) return false;
    bool expected = false;
    if (fired_.compare_exchange_strong(expected, true)) {
      reason_.store(late ? 1 : 2);
      if (on_fire_) on_fire_();
    }
    return true;
  }

  void start(double period_s = 0.05) {
    if (thread_.joinable()) return;
    stop_.store(false);
    const auto period = std::chrono::duration<double>(period_s);
    thread_ = std::thread([this, period] {
      while (!stop_.load()) {
        if (check(now_ns())) return;
        std::this_thread::sleep_for(period);
      }
    });
  }
  void stop() {
    stop_.store(true);
    if (thread_.joinable()) thread_.join();
  }

  bool fired() const { return fired_.load(); }
  int reason() const { return reason_.load(); }  // 0 none, 1 deadline, 2 async error
  double timeout_s() const { return timeout_ns_.load() * 1e-9; }
  // A shorter (or longer) deadline (the bench pre-flight bounds its first
  // exchange far below the run deadline).  check() reads the deadline on
  // every poll, so it applies at once to every open Busy scope, including
  // one already open on another thread -- not only to scopes opened later.
  void set_timeout(double timeout_s) { timeout_ns_.store(static_cast<int64_t>(timeout_s * 1e9)); }

 private:
  std::atomic<int64_t> timeout_ns_;
  std::function<bool()> poll_error_;
  std::function<void()> on_fire_;
  std::atomic<int64_t> busy_since_{0};
  std::atomic<int> depth_{0};
  std::atomic<bool> fired_{false};
  std::atomic<int> reason_{0};
  std::atomic<bool> stop_{false};
  std::thread thread_;
};

}  // namespace bdx
