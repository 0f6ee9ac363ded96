// A persistent host thread pool shared by the lowering (lower.cpp) and the
// staging of the host-to-host pipeline (runtime.cpp): threads are created
// once, so a batch call pays no thread start-up.
#pragma once
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <fstream>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

namespace dp {

// Host threads for staging: the CPU share of this process (cgroup cpu.max
// quota when one is set, else the hardware threads), capped.
inline int host_threads() {
  const char* e = std::getenv("DEPPY_HOST_THREADS");
  int64_t n = e && *e ? std::atoll(e) : 0;
  if (n > 0) return (int)std::min<int64_t>(n, 256);
  unsigned hw = std::thread::hardware_concurrency();
  n = hw ? hw : 1;
  std::ifstream f("/sys/fs/cgroup/cpu.max");
  std::string quota, period;
  if (f >> quota >> period && quota != "max") {
    const double q = std::atof(quota.c_str()), p = std::atof(period.c_str());
    if (q > 0 && p > 0) n = std::min<int64_t>(n, std::max<int64_t>(1, (int64_t)(q / p)));
  }
  return (int)std::min<int64_t>(n, 32);
}

// A persistent pool: run(n, fn) calls fn(i, t) for every i < n on the
// workers and the calling thread (dynamic, in blocks; t < size() names the
// thread, 0 = the caller), and returns when all are done.
class Pool {
 public:
  using Fn = std::function<void(int64_t, int)>;
  explicit Pool(int n) {
    for (int t = 1; t < n; ++t) th_.emplace_back([this, t] { loop(t); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      ++gen_;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int size() const { return (int)th_.size() + 1; }
  void run(int64_t n, const Fn& fn, int64_t block = 16) {
    if (n <= 0) return;
    if (th_.empty() || n <= block) {
      for (int64_t i = 0; i < n; ++i) fn(i, 0);
      return;
    }
    std::lock_guard<std::mutex> one(run_mu_);  // one run at a time (callers on several threads)
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &fn;
      n_ = n;
      block_ = block;
      next_.store(0);
      busy_ = (int)th_.size();
      ++gen_;
    }
    cv_.notify_all();
    work(0);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return busy_ == 0; });
    fn_ = nullptr;
  }
  // the same with fn(i)
  void run(int64_t n, const std::function<void(int64_t)>& fn, int64_t block = 16) {
    run(n, Fn([&fn](int64_t i, int) { fn(i); }), block);
  }

 private:
  void work(int t) {
    for (;;) {
      const int64_t lo = next_.fetch_add(block_);
      if (lo >= n_) break;
      const int64_t hi = std::min(n_, lo + block_);
      for (int64_t i = lo; i < hi; ++i) (*fn_)(i, t);
    }
  }
  void loop(int t) {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        if (stop_) return;
      }
      work(t);
      std::lock_guard<std::mutex> lk(mu_);
      if (--busy_ == 0) done_cv_.notify_one();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_, run_mu_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  bool stop_ = false;
  const Fn* fn_ = nullptr;
  int64_t n_ = 0, block_ = 1;
  std::atomic<int64_t> next_{0};
  int busy_ = 0;
};

// The process-wide pool (host_threads() threads, created on first use).
inline Pool& host_pool() {
  static Pool pool(host_threads());
  return pool;
}

}  // namespace dp
