// host_pool.h -- one persistent pool of host worker threads for the host-side
// loops of the engine (sweep plans, graph loads) and of odl::LinkState
// (snapshots, ingest, route builds).
//
// Those loops ran on threads created per call: at F100k a sweep plan makes
// ~15 such calls and a thread's creation + join costs tens of microseconds on
// the box's host, for loops whose work is a few hundred microseconds. The
// pool's workers sleep on a condition variable between jobs. One job at a
// time: a caller that finds the pool busy (another host thread's job, or a
// loop nested in a job) gets false and runs its loop some other way.
#ifndef OPENR_HOST_POOL_H
#define OPENR_HOST_POOL_H

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <system_error>
#include <thread>
#include <vector>

#include <unistd.h>

namespace host_pool {

class Pool {
 public:
  using Fn = std::function<void(uint32_t, uint32_t)>;

  static Pool& get() {
    static Pool p;
    return p;
  }

  // fn(lo, hi) over [0, n) in chunks of `grain` on up to `threads` threads
  // (the caller included); false (nothing run) when the pool is busy or has
  // no workers. The first exception a chunk throws is rethrown here after
  // the job drained.
  bool run(uint32_t n, uint32_t grain, uint32_t threads, const Fn& fn) {
    // (a forked child has the pool's state but none of its threads)
    if (in_worker() || workers_.empty() || threads <= 1 || getpid() != pid_) return false;
    std::unique_lock<std::mutex> job(job_mu_, std::try_to_lock);
    if (!job.owns_lock()) return false;
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      n_ = n;
      grain_ = std::max(1u, grain);
      next_.store(0);
      failed_.store(false);
      err_ = nullptr;
      want_ = std::min<uint32_t>((uint32_t)workers_.size(), threads - 1);
      active_ = want_;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> l(mu_);
    done_cv_.wait(l, [&] { return active_ == 0; });
    fn_ = nullptr;
    if (err_) {
      std::exception_ptr e = err_;
      err_ = nullptr;
      std::rethrow_exception(e);
    }
    return true;
  }

  ~Pool() {
    if (getpid() != pid_) {  // a forked child: the threads are not its own
      new std::vector<std::thread>(std::move(workers_));  // (never destroyed)
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  Pool() : pid_(getpid()) {
    uint32_t hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
    if (const char* e = std::getenv("OPENR_HOST_THREADS")) hw = (uint32_t)std::max(1, std::atoi(e));
    for (uint32_t i = 0; i + 1 < hw; ++i) {
      try {
        workers_.emplace_back([this, i] { loop(i); });
      } catch (const std::system_error&) {
        break;
      }
    }
  }

  static bool& in_worker() {
    static thread_local bool w = false;
    return w;
  }

  void work() {
    for (;;) {
      if (failed_.load(std::memory_order_relaxed)) return;
      const uint32_t lo = next_.fetch_add(grain_);
      if (lo >= n_) return;
      try {
        (*fn_)(lo, std::min(n_, lo + grain_));
      } catch (...) {
        std::lock_guard<std::mutex> g(mu_);
        if (!failed_.exchange(true)) err_ = std::current_exception();
        return;
      }
    }
  }

  void loop(uint32_t idx) {
    in_worker() = true;
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> l(mu_);
        cv_.wait(l, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        if (idx >= want_) continue;  // not wanted for this job
      }
      work();
      {
        std::lock_guard<std::mutex> g(mu_);
        if (--active_ == 0) done_cv_.notify_all();
      }
    }
  }

  std::mutex job_mu_, mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<std::thread> workers_;
  const Fn* fn_ = nullptr;
  uint32_t n_ = 0, grain_ = 1, want_ = 0, active_ = 0;
  std::atomic<uint32_t> next_{0};
  std::atomic<bool> failed_{false};
  std::exception_ptr err_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  const pid_t pid_;
};

}  // namespace host_pool

#endif
