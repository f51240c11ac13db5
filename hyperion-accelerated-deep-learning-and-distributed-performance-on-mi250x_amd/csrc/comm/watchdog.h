// Collective watchdog: deadline + async-error supervision for in-flight collectives.
//
// Reference behaviour being replaced: every reference collective ran under a process-group
// timeout (`02_development/distributed_utils.py:106-111`, 5 min; `test_nccl.py:26-29`, 30 s) that
// ProcessGroupNCCL's watchdog thread enforces; the reference's launcher then DISABLED the kill
// (`run_language_fsdp.sh:10`, TORCH_NCCL_ASYNC_ERROR_HANDLING=0).  Hyperion's native RCCL
// communicator bypasses ProcessGroupNCCL, so it carries its own supervisor:
//
//  * every collective registers a completion probe (in production: hipEventQuery on the event
//    recorded after the RCCL call on the comm stream) with a deadline = issue time + timeout;
//  * ONE thread per communicator polls the probes oldest-first (collectives on one stream retire
//    in order, so only the head can be the laggard) plus the communicator's async-error probe
//    (ncclCommGetAsyncError);
//  * on the first expired deadline or async error it records WHY, then runs the failure action
//    (ncclCommAbort: RCCL kernels spinning on a dead peer exit, so a host blocked in a stream
//    synchronize returns) exactly once; every later collective / wait() raises that message;
//  * optional process exit (HYPERION_COMM_ON_TIMEOUT=exit) for launchers that restart workers.
//
// The class knows nothing about HIP or RCCL (probes are std::functions), so the same logic is
// unit-tested on the CPU with simulated work handles (`WatchdogSim` in rccl_comm.cpp,
// tests/test_comm_watchdog_cpu.py).
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>

namespace hypcomm {

class Watchdog {
 public:
  using Clock = std::chrono::steady_clock;
  // probe result: kDone (retire), kPending (check the deadline), kFailed (error now)
  enum Status { kDone = 0, kPending = 1, kFailed = 2 };
  using Probe = std::function<int()>;

  // thread_init runs first on the watchdog thread (e.g. switch it to relaxed graph-capture mode)
  Watchdog(double timeout_s, double poll_ms, std::function<std::string()> async_error,
           std::function<void(const std::string&)> on_fail, std::function<void()> thread_init = nullptr)
      : timeout_(std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(timeout_s))),
        poll_(std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double, std::milli>(poll_ms))),
        async_error_(std::move(async_error)),
        on_fail_(std::move(on_fail)) {
    thread_ = std::thread([this, init = std::move(thread_init)] {
      if (init) init();
      loop();
    });
  }
  ~Watchdog() { stop(); }
  Watchdog(const Watchdog&) = delete;
  Watchdog& operator=(const Watchdog&) = delete;

  // register an in-flight operation; `what` names it in the failure message
  void watch(Probe probe, std::string what) {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(Entry{std::move(probe), Clock::now() + timeout_, std::move(what), Clock::now()});
    cv_.notify_all();
  }

  // "" while healthy, else the first failure's message (sticky)
  std::string error() const {
    std::lock_guard<std::mutex> g(mu_);
    return error_;
  }
  bool failed() const { return failed_.load(std::memory_order_acquire); }
  size_t pending() const {
    std::lock_guard<std::mutex> g(mu_);
    return q_.size();
  }
  double timeout_s() const { return std::chrono::duration<double>(timeout_).count(); }

  // block (host) until every registered operation retired or the watchdog failed; false on failure
  bool drain() {
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return q_.empty() || failed_.load() || stop_; });
    return !failed_.load();
  }

  void stop() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (stop_) return;
      stop_ = true;
      cv_.notify_all();
    }
    if (thread_.joinable()) thread_.join();
  }

  // mark failed from outside (e.g. an init deadline) with the same once-only action
  void fail(const std::string& why) { fail_locked_out(why); }

 private:
  struct Entry {
    Probe probe;
    Clock::time_point deadline;
    std::string what;
    Clock::time_point issued;
  };

  void fail_locked_out(const std::string& why) {
    bool first = false;
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!failed_.load()) {
        error_ = why;
        failed_.store(true, std::memory_order_release);
        first = true;
      }
      q_.clear();
      cv_.notify_all();
    }
    if (first && on_fail_) on_fail_(why);
  }

  void loop() {
    for (;;) {
      std::string why;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait_for(lk, poll_, [this] { return stop_; });
        if (stop_) return;
        if (failed_.load()) continue;
        // retire completed operations oldest-first; the first pending one decides the deadline
        while (!q_.empty()) {
          Entry& e = q_.front();
          const int s = e.probe();
          if (s == kDone) {
            q_.pop_front();
            continue;
          }
          if (s == kFailed) {
            why = "collective '" + e.what + "' failed on the device";
          } else if (Clock::now() > e.deadline) {
            const double waited = std::chrono::duration<double>(Clock::now() - e.issued).count();
            why = "collective '" + e.what + "' did not complete within the " + std::to_string(timeout_s()) +
                  " s timeout (waited " + std::to_string(waited) + " s; a peer rank is dead, stalled or " +
                  "issued a different collective)";
          }
          break;
        }
        if (q_.empty()) cv_.notify_all();  // drain() waiters
      }
      if (why.empty() && async_error_) {
        const std::string a = async_error_();
        if (!a.empty()) why = "communicator async error: " + a;
      }
      if (!why.empty()) fail_locked_out(why);
    }
  }

  const Clock::duration timeout_, poll_;
  std::function<std::string()> async_error_;
  std::function<void(const std::string&)> on_fail_;
  mutable std::mutex mu_;
  std::condition_variable cv_;
  std::deque<Entry> q_;
  std::string error_;
  std::atomic<bool> failed_{false};
  bool stop_ = false;
  std::thread thread_;
};

}  // namespace hypcomm
