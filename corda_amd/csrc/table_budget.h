// Which constant fixed-base tables a context gets (include/cordagpu.h
// cg_config.table_bytes_max). HIP-free: tests/test_table_budget.py drives it through the C ABI's
// cg_table_choice on the CPU.
//
// The Ed25519 B and the two curves' G tables are built once per device per process at one of three
// radixes, each a separate build of the radix-dependent kernels (Makefile VARIANTS):
//   radix 2^26: 10 rows, ~91 GB    (42 additions per Ed25519 / ECDSA wide-ladder item)
//   radix 2^24: 11 rows, ~25 GB    (43)
//   radix 2^22: 12 rows, ~6.9 GB   (44)
// One process per GPU holds the largest comfortably. The reference runs "any number of verifiers"
// against a node (docs/source/out-of-process-verification.rst:7-8; VerifierTests.kt:54-70 starts 4),
// so several processes may share a device: the third 91-GB set no longer fits in 288 GB. Rule:
//   table_bytes_max > 0   the largest set whose bytes <= table_bytes_max (none: CG_ERR_ARG)
//   table_bytes_max == 0  automatic: a set this process already holds on the device is reused;
//                         otherwise the largest set that leaves kTableHeadroom of the device's free
//                         memory for the calls' workspaces, else the smallest; and when the allocation
//                         itself fails (another process took the memory first) the next smaller set.
#pragma once
#include <cstdint>
#include <cstdlib>

namespace cgb {

// device memory left beside the tables for the calls' workspaces (a BASELINE configs[4] shard call
// holds ~15 GB: the arena window, two 2.5M-item workspaces and ~6 000 hot keys' wide tables)
constexpr uint64_t kTableHeadroom = 16ull << 30;

struct TableSet {
  uint32_t bits;   // fixed-base radix 2^bits
  uint64_t bytes;  // HBM of the B + G tables at that radix
};

// sets[0 .. n) in descending size. held: index of a set this process already holds on the device, or
// -1. Returns the index to build (or reuse), -1 when an explicit budget is below every set.
inline int pick_tables(const TableSet* sets, int n, uint64_t budget, uint64_t device_free, int held) {
  if (n <= 0) return -1;
  if (budget) {
    if (held >= 0 && sets[held].bytes <= budget) return held;
    for (int i = 0; i < n; ++i)
      if (sets[i].bytes <= budget) return i;
    return -1;
  }
  if (held >= 0) return held;
  for (int i = 0; i < n; ++i)
    if (sets[i].bytes + kTableHeadroom <= device_free) return i;
  return n - 1;
}

// CG_TABLE_BYTES_MAX=<bytes>[K|M|G] (operations / A/B runs) when cg_config.table_bytes_max is 0;
// 0 when unset or unreadable.
inline uint64_t table_bytes_env(const char* v) {
  if (!v || !v[0]) return 0;
  char* end = nullptr;
  const unsigned long long x = strtoull(v, &end, 10);
  if (end == v) return 0;
  const char s = *end;
  const int sh = s == 'K' || s == 'k' ? 10 : s == 'M' || s == 'm' ? 20 : s == 'G' || s == 'g' ? 30 : 0;
  if (sh && x > (~0ull >> sh)) return ~0ull;
  return (uint64_t)x << sh;
}

}  // namespace cgb
