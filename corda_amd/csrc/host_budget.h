// The host-side thread budget of a context: how many host threads one context's
// scans (host_pool.h: the key-use count pass, each chunk's byte extents) may use, decided before
// any GPU call and HIP-free (tests/native/host_budget_test.cpp runs it on the CPU).
//
// A node runs one process per GPU (bench.py under torchrun) or one process driving every GPU
// (cg_pool, a JVM node): either way the CPUs are shared. Round 4 gave every context 16 threads, so
// 8 ranks on a 16-CPU quota ran 128 scan threads. Now:
//   cg_config.host_threads > 0            that many (the caller knows its share: bench.py passes the
//                                          quota divided by LOCAL_WORLD_SIZE, a JVM node its config)
//   else CG_HOST_THREADS=<n> in the env   that many (operations override)
//   else                                   the process's CPU quota / the contexts open in it
// always clamped to [1, kHostThreadsMax].
#pragma once
#include <sched.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

namespace cg {

constexpr unsigned kHostThreadsMax = 64;

// CPUs this process may use: the cgroup v2 quota (cpu.max "Q P"), else cgroup v1
// (cfs_quota_us / cfs_period_us), bounded by the affinity mask; at least 1.
inline unsigned cpu_quota_from(const char* cpu_max, const char* cfs_quota, const char* cfs_period, unsigned affinity) {
  unsigned n = affinity ? affinity : 1;
  long long q = -1, p = 0;
  if (cpu_max && cpu_max[0]) {
    char qs[32] = {0};
    if (sscanf(cpu_max, "%31s %lld", qs, &p) == 2 && strcmp(qs, "max") != 0) q = atoll(qs);
  } else if (cfs_quota && cfs_period) {
    q = atoll(cfs_quota);
    p = atoll(cfs_period);
  }
  if (q > 0 && p > 0) {
    const long long c = q / p;  // whole CPUs (a fractional quota rounds down, at least 1)
    const unsigned cq = (unsigned)(c < 1 ? 1 : c);
    if (cq < n) n = cq;
  }
  return n ? n : 1;
}

inline unsigned cpu_quota() {
  auto slurp = [](const char* path, char* buf, size_t cap) -> const char* {
    FILE* f = fopen(path, "r");
    if (!f) return nullptr;
    const size_t r = fread(buf, 1, cap - 1, f);
    fclose(f);
    buf[r] = 0;
    return buf;
  };
  char a[64], b[64], c[64];
  const char* v2 = slurp("/sys/fs/cgroup/cpu.max", a, sizeof a);
  const char* q1 = v2 ? nullptr : slurp("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", b, sizeof b);
  const char* p1 = v2 ? nullptr : slurp("/sys/fs/cgroup/cpu/cpu.cfs_period_us", c, sizeof c);
  cpu_set_t set;
  unsigned aff = 0;
  if (sched_getaffinity(0, sizeof set, &set) == 0) aff = (unsigned)CPU_COUNT(&set);
  return cpu_quota_from(v2, q1, p1, aff);
}

// requested: cg_config.host_threads; env: CG_HOST_THREADS (0 = unset); contexts: open in this process
inline unsigned host_threads_for(unsigned requested, unsigned env, unsigned quota, unsigned contexts) {
  unsigned n = requested ? requested : env ? env : (quota ? quota : 1) / (contexts ? contexts : 1);
  if (n < 1) n = 1;
  if (n > kHostThreadsMax) n = kHostThreadsMax;
  return n;
}

inline unsigned host_threads_env() {
  const char* v = getenv("CG_HOST_THREADS");
  return v ? (unsigned)strtoul(v, nullptr, 10) : 0u;
}

// Whether a caller should register its host buffers (cg_host_register) rather than hand over pageable
// memory, by how many contexts share the node's host (round 6, VERDICT r5 item 3;
// profiles/r06/host8/summary.json): alone a rank copies fastest from pageable memory (the runtime's
// staging paces the DMA; registered -10% on one MI355X), but with 7 other ranks staging their bytes
// through the same host memory the pageable rank lost 17% and a registered one 4% (registered +5%
// over pageable at the 8-rank proxy). 4 or more contexts per node: register (4 interpolated).
constexpr unsigned kHostRegisterMinContexts = 4;
inline bool host_register_advised(unsigned contexts_per_node) { return contexts_per_node >= kHostRegisterMinContexts; }

}  // namespace cg
