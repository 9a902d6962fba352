// Fork-join pool of host threads kept for a context's lifetime (the host-side scans of the
// tx-signature path: key-use counts, each chunk's byte extents). Spawning and joining 16
// std::threads cost 0.35-0.5 ms per round on the GPU box's host (two rounds 0.8-1.0 ms:
// tools/microbench/count_pass.cpp), about two thirds of a 1.3-ms count pass that gates both the
// key tables and chunk 0's copy.
//
// run(n, fn) calls fn(t) for every t in [0, n), parts claimed dynamically by the caller and the
// workers, and returns once every part is done and every woken worker is idle again (so the next
// run can reuse the job slot). fn must not throw. Runs from different threads take turns (a
// caller's fn must not call run on the same pool).
#pragma once
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace cg {

class HostPool {
 public:
  explicit HostPool(unsigned workers) {
    th_.reserve(workers);
    for (unsigned w = 0; w < workers; ++w) th_.emplace_back([this] { loop(); });
  }
  ~HostPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    go_.notify_all();
    for (auto& t : th_) t.join();
  }
  HostPool(const HostPool&) = delete;
  HostPool& operator=(const HostPool&) = delete;

  unsigned threads() const { return (unsigned)th_.size() + 1; }

  void run(uint64_t n, const std::function<void(uint64_t)>& fn) {
    if (n == 0) return;
    if (n == 1 || th_.empty()) {
      for (uint64_t t = 0; t < n; ++t) fn(t);
      return;
    }
    std::lock_guard<std::mutex> turn(run_m_);
    {
      std::lock_guard<std::mutex> g(m_);
      job_ = &fn;
      n_ = n;
      next_.store(0, std::memory_order_relaxed);
      busy_ = (unsigned)th_.size();
      ++gen_;
    }
    go_.notify_all();
    work(fn, n);
    std::unique_lock<std::mutex> g(m_);
    done_.wait(g, [this] { return busy_ == 0; });
    job_ = nullptr;
  }

 private:
  void work(const std::function<void(uint64_t)>& fn, uint64_t n) {
    for (uint64_t t = next_.fetch_add(1, std::memory_order_relaxed); t < n;
         t = next_.fetch_add(1, std::memory_order_relaxed))
      fn(t);
  }
  void loop() {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(m_);
    for (;;) {
      go_.wait(g, [&] { return stop_ || gen_ != seen; });
      if (stop_) return;
      seen = gen_;
      const std::function<void(uint64_t)>* fn = job_;
      const uint64_t n = n_;
      g.unlock();
      work(*fn, n);
      g.lock();
      if (--busy_ == 0) done_.notify_one();
    }
  }

  std::vector<std::thread> th_;
  std::mutex m_, run_m_;
  std::condition_variable go_, done_;
  const std::function<void(uint64_t)>* job_ = nullptr;
  uint64_t n_ = 0, gen_ = 0;
  unsigned busy_ = 0;
  bool stop_ = false;
  std::atomic<uint64_t> next_{0};
};

}  // namespace cg
