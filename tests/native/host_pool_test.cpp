// CPU checks of corda_amd/csrc/host_pool.h (the tx-signature path's host thread pool), driven by
// tests/test_host_pool.py: every part of every run executes exactly once and before run returns,
// across run sizes from 0 to many times the thread count, with one or several threads calling run
// on the same pool.
#include <atomic>
#include <cstdint>
#include <thread>
#include <vector>

#include "../../corda_amd/csrc/host_pool.h"

extern "C" {

// workers: pool size minus the caller; runs per caller; callers: threads sharing the pool.
// Returns the number of parts that ran a wrong number of times or after their run returned.
uint64_t hp_check(uint32_t workers, uint32_t runs, uint32_t callers) {
  cg::HostPool pool(workers);
  std::atomic<uint64_t> bad{0};
  auto caller = [&](uint32_t id) {
    for (uint32_t r = 0; r < runs; ++r) {
      const uint64_t n = (r * 7u + id * 3u) % 53u + (r % 11u == 0 ? 500u : 0u);  // includes 0 and 1
      std::vector<std::atomic<uint32_t>> hits(n);
      for (auto& h : hits) h.store(0);
      std::atomic<bool> returned{false};
      pool.run(n, [&](uint64_t t) {
        if (returned.load()) bad.fetch_add(1);
        hits[t].fetch_add(1);
      });
      returned.store(true);
      for (uint64_t t = 0; t < n; ++t)
        if (hits[t].load() != 1) bad.fetch_add(1);
    }
  };
  std::vector<std::thread> th;
  for (uint32_t c = 1; c < callers; ++c) th.emplace_back(caller, c);
  caller(0);
  for (auto& t : th) t.join();
  return bad.load();
}

// The pool's thread count as reported (workers + the caller).
uint32_t hp_threads(uint32_t workers) {
  cg::HostPool pool(workers);
  return pool.threads();
}
}
