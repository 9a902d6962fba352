// CPU driver of corda_amd/csrc/host_budget.h (tests/test_host_budget.py): the cgroup quota parser
// and the per-context thread budget, exported through a C ABI so the test can table its cases.
#include "../../corda_amd/csrc/host_budget.h"

extern "C" {
// cpu_max: cgroup v2 "cpu.max" text or null; cfs_quota / cfs_period: cgroup v1 texts or null
unsigned hb_quota_from(const char* cpu_max, const char* cfs_quota, const char* cfs_period, unsigned affinity) {
  return cg::cpu_quota_from(cpu_max, cfs_quota, cfs_period, affinity);
}
unsigned hb_threads_for(unsigned requested, unsigned env, unsigned quota, unsigned contexts) {
  return cg::host_threads_for(requested, env, quota, contexts);
}
unsigned hb_quota() { return cg::cpu_quota(); }
unsigned hb_max() { return cg::kHostThreadsMax; }
}
