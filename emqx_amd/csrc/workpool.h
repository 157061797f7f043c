// A small pool of worker threads for the host bookkeeping of the subscriber tables
// (fanout.cpp: threaded plain ops, commit patch lists): run(fn, t) runs fn on the caller and on
// t - 1 workers and returns when all are done.  One run at a time (a lock of its own).
//
// Runs come in bursts (remove, add, the commit's passes).  Workers can spin on the run
// generation for a while after each run (and the caller on the completion count) before they
// block, so that a run following within the window starts without a wake-up
// (EMQX_POOL_SPIN_US; default 0, never spin: measured, the S churn line did not gain — a run's
// time is its ops' cache misses — and the T storm at 4096 callers lost half its rate to the
// spinning workers, 12.7 -> 6.7 M ops/s, profiles/r4_q39_bench_T.json).  Everything the spin
// reads is an atomic; the blocking path keeps the usual lock-then-notify order, so no wake-up
// is lost.
#pragma once

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstddef>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace emqx {

class WorkPool {
 public:
  static WorkPool& get() {
    static WorkPool* p = [] {
      auto* w = new WorkPool();  // never destroyed: workers may outlive static teardown
      if (const char* e = std::getenv("EMQX_POOL_SPIN_US")) w->set_spin_us(static_cast<uint32_t>(std::atoi(e)));
      return w;
    }();
    return *p;
  }
  // spin budget of a waiting thread before it blocks (tests set it to 0 or large)
  void set_spin_us(uint32_t us) { spin_us_.store(us, std::memory_order_relaxed); }

  void run(const std::function<void()>& fn, unsigned t) {
    std::lock_guard<std::mutex> one(run_mu_);
    t = t < 1 ? 1u : t;
    {
      std::lock_guard<std::mutex> lk(mu_);
      while (workers_.size() < t - 1) {
        try {
          workers_.emplace_back([this, id = workers_.size()] { loop(id); });
        } catch (...) {
          break;
        }
      }
      job_ = &fn;
      want_ = std::min<size_t>(t - 1, workers_.size());
      left_.store(static_cast<int>(want_), std::memory_order_relaxed);
      gen_.fetch_add(1, std::memory_order_release);  // publishes job_ / want_ to spinning workers
    }
    cv_.notify_all();
    std::exception_ptr mine;
    try {
      fn();
    } catch (...) {
      mine = std::current_exception();
    }
    if (!spin_until([&] { return left_.load(std::memory_order_acquire) == 0; })) {
      std::unique_lock<std::mutex> lk(mu_);
      done_.wait(lk, [&] { return left_.load(std::memory_order_acquire) == 0; });
    }
    std::exception_ptr theirs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      theirs = err_;
      err_ = nullptr;
    }
    if (mine) std::rethrow_exception(mine);
    if (theirs) std::rethrow_exception(theirs);
  }

 private:
  template <class Pred>
  bool spin_until(Pred p) const {
    const uint32_t us = spin_us_.load(std::memory_order_relaxed);
    if (us == 0) return p();
    const auto end = std::chrono::steady_clock::now() + std::chrono::microseconds(us);
    for (uint32_t i = 0;; ++i) {
      if (p()) return true;
      if ((i & 63) == 63 && std::chrono::steady_clock::now() >= end) return false;
#if defined(__x86_64__) || defined(__i386__)
      __builtin_ia32_pause();
#endif
    }
  }

  void loop(size_t id) {
    uint64_t seen = 0;
    for (;;) {
      if (!spin_until([&] { return gen_.load(std::memory_order_acquire) != seen; })) {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_.load(std::memory_order_acquire) != seen; });
      }
      const std::function<void()>* job;
      size_t want;
      {
        // job_ / want_ are read under mu_: run() writes them under it, before the generation
        std::lock_guard<std::mutex> lk(mu_);
        seen = gen_.load(std::memory_order_acquire);
        job = job_;
        want = want_;
      }
      if (id >= want) continue;
      try {
        (*job)();
      } catch (...) {
        std::lock_guard<std::mutex> lk(mu_);
        if (!err_) err_ = std::current_exception();
      }
      if (left_.fetch_sub(1, std::memory_order_acq_rel) == 1) {
        std::lock_guard<std::mutex> lk(mu_);  // the caller may be about to block on done_
        done_.notify_one();
      }
    }
  }

  std::mutex run_mu_, mu_;
  std::condition_variable cv_, done_;
  std::vector<std::thread> workers_;
  const std::function<void()>* job_ = nullptr;
  std::exception_ptr err_;  // first exception of a worker's job in the current run (under mu_)
  size_t want_ = 0;
  std::atomic<int> left_{0};
  std::atomic<uint64_t> gen_{0};
  std::atomic<uint32_t> spin_us_{0};
};

}  // namespace emqx
