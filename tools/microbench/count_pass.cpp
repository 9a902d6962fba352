// Host microbenchmark of the tx-signature key-use sample pass (cordagpu.cpp sample_counts, hot-call
// form: 1 block of 8 records in 32 blocks) over a synthetic 12.5M-record table: the current form
// (threads spawned per pass, demand loads) against software prefetch and the persistent pool.
// g++ -O2 -std=c++17 -pthread tools/microbench/count_pass.cpp -o /tmp/count_pass && /tmp/count_pass [threads]
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "../../corda_amd/csrc/host_pool.h"

struct Rec {
  uint64_t sig_off;
  uint32_t tx_idx, key_idx;
  uint16_t sig_len, tmpl;
  uint32_t reserved;
};

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static inline uint64_t group_start(uint64_t g, uint64_t S, uint64_t B) {
  return (g * S + (((uint32_t)g * 0x9E3779B1u) >> 24) % S) * B;
}

int main(int argc, char** argv) {
  const uint64_t nt = argc > 1 ? strtoull(argv[1], nullptr, 10) : 16;
  const uint64_t n = 12500000, n_keys = 6144, S = 32, B = 8;
  std::vector<Rec> sigs(n);
  std::mt19937_64 rng(1);
  for (uint64_t i = 0; i < n; ++i) sigs[i] = Rec{i * 64, (uint32_t)(i / 5), (uint32_t)(rng() % n_keys), 64, 0, 0};
  const uint64_t ng = (n + S * B - 1) / (S * B);
  std::vector<uint32_t> ref(n_keys, 0);
  for (uint64_t g = 0; g < ng; ++g)
    for (uint64_t i = group_start(g, S, B); i < group_start(g, S, B) + B && i < n; ++i) ++ref[sigs[i].key_idx];

  // (a) the current form: per-pass std::thread spawn, per-thread count arrays, demand loads
  auto pass_a = [&](std::vector<uint32_t>& counts) {
    std::vector<std::vector<uint32_t>> pc(nt, std::vector<uint32_t>(n_keys, 0u));
    auto scan = [&](uint64_t t) {
      uint32_t* cnt = pc[t].data();
      for (uint64_t g = ng * t / nt; g < ng * (t + 1) / nt; ++g) {
        const uint64_t i0 = group_start(g, S, B);
        for (uint64_t i = i0; i < i0 + B && i < n; ++i) ++cnt[sigs[i].key_idx];
      }
    };
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < nt; ++t) th.emplace_back(scan, t);
    for (auto& t : th) t.join();
    th.clear();
    for (uint64_t t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (uint64_t k = n_keys * t / nt; k < n_keys * (t + 1) / nt; ++k)
          for (uint64_t u = 0; u < nt; ++u) counts[k] += pc[u][k];
      });
    for (auto& t : th) t.join();
  };

  // (b) prefetch D groups ahead, same threading
  auto pass_b = [&](std::vector<uint32_t>& counts, uint64_t D) {
    std::vector<std::vector<uint32_t>> pc(nt, std::vector<uint32_t>(n_keys, 0u));
    auto scan = [&](uint64_t t) {
      uint32_t* cnt = pc[t].data();
      const uint64_t g0 = ng * t / nt, g1 = ng * (t + 1) / nt;
      for (uint64_t g = g0; g < g0 + D && g < g1; ++g) __builtin_prefetch(&sigs[group_start(g, S, B)]);
      for (uint64_t g = g0; g < g1; ++g) {
        if (g + D < g1) {
          const Rec* p = &sigs[group_start(g + D, S, B)];
          __builtin_prefetch(p);
          __builtin_prefetch((const char*)p + 64);
          __builtin_prefetch((const char*)p + 128);
        }
        const uint64_t i0 = group_start(g, S, B);
        for (uint64_t i = i0; i < i0 + B && i < n; ++i) ++cnt[sigs[i].key_idx];
      }
    };
    std::vector<std::thread> th;
    for (uint64_t t = 0; t < nt; ++t) th.emplace_back(scan, t);
    for (auto& t : th) t.join();
    th.clear();
    for (uint64_t t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (uint64_t k = n_keys * t / nt; k < n_keys * (t + 1) / nt; ++k)
          for (uint64_t u = 0; u < nt; ++u) counts[k] += pc[u][k];
      });
    for (auto& t : th) t.join();
  };

  // (c) thread spawn alone (two rounds of nt threads doing nothing)
  auto pass_c = [&] {
    for (int r = 0; r < 2; ++r) {
      std::vector<std::thread> th;
      for (uint64_t t = 0; t < nt; ++t) th.emplace_back([] {});
      for (auto& t : th) t.join();
    }
  };

  // (d) the persistent pool (host_pool.h), demand loads (the form cordagpu.cpp runs)
  cg::HostPool pool((unsigned)nt - 1);
  auto pass_d = [&](std::vector<uint32_t>& counts) {
    std::vector<std::vector<uint32_t>> pc(nt, std::vector<uint32_t>(n_keys, 0u));
    pool.run(nt, [&](uint64_t t) {
      uint32_t* cnt = pc[t].data();
      for (uint64_t g = ng * t / nt; g < ng * (t + 1) / nt; ++g) {
        const uint64_t i0 = group_start(g, S, B);
        for (uint64_t i = i0; i < i0 + B && i < n; ++i) ++cnt[sigs[i].key_idx];
      }
    });
    pool.run(nt, [&](uint64_t t) {
      for (uint64_t k = n_keys * t / nt; k < n_keys * (t + 1) / nt; ++k)
        for (uint64_t u = 0; u < nt; ++u) counts[k] += pc[u][k];
    });
  };

  for (int rep = 0; rep < 3; ++rep) {
    std::vector<uint32_t> ca(n_keys, 0), cb(n_keys, 0), cd(n_keys, 0);
    // evict: touch a large buffer between passes so the table is not cache-resident (as in the bench,
    // where a pass follows the previous call's copies)
    static std::vector<uint8_t> junk(512u << 20, 1);
    uint64_t sink = 0;
    for (size_t i = 0; i < junk.size(); i += 64) sink += junk[i]++;
    double t = now_ms();
    pass_a(ca);
    const double ta = now_ms() - t;
    for (size_t i = 0; i < junk.size(); i += 64) sink += junk[i]++;
    t = now_ms();
    pass_b(cb, 16);
    const double tb = now_ms() - t;
    for (size_t i = 0; i < junk.size(); i += 64) sink += junk[i]++;
    t = now_ms();
    pass_b(cd, 48);
    const double td = now_ms() - t;
    t = now_ms();
    pass_c();
    const double tc = now_ms() - t;
    std::vector<uint32_t> ce(n_keys, 0);
    for (size_t i = 0; i < junk.size(); i += 64) sink += junk[i]++;
    t = now_ms();
    pass_d(ce);
    const double te = now_ms() - t;
    printf("threads %llu: current %.3f ms, prefetch16 %.3f ms, prefetch48 %.3f ms, spawn-only %.3f ms, pool %.3f ms, equal %d %d %d (%llu)\n",
           (unsigned long long)nt, ta, tb, td, tc, te, ca == ref, cb == ref && cd == ref, ce == ref,
           (unsigned long long)(sink & 1));
  }
  return 0;
}
