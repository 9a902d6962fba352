// CPU harness for the multi-device shard plan and failure handling (corda_amd/csrc/pool.h):
// the library's own cg::pool_run, with each "device" a slot that verifies its shard through the
// C oracle (test infrastructure) and fails on demand. Built and driven by tests/test_pool.py.
#include <atomic>
#include <mutex>
#include <vector>

#include "../../corda_amd/csrc/pool.h"
#include "../../oracle/c/oracle.h"

extern "C" {

// fail_always: bit s -> slot s fails every call; fail_once: bit s -> slot s fails its first call
// only (a transient fault: the slot is still marked unhealthy, as the library does);
// fail_arg: bit s -> slot s returns CG_ERR_NOMEM (a capacity error: not a device fault);
// probe_ok: bit s -> an unhealthy slot s answers the re-probe at the start of the call.
// calls_out[s]: calls made on slot s. report_out: shards, reruns, failed_slots, not_run.
int pt_pool_verify(const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items, const uint8_t* arena,
                   uint64_t arena_len, uint32_t mode, uint8_t* status, uint32_t n_slots, uint8_t* healthy_io,
                   uint32_t fail_always, uint32_t fail_once, uint32_t fail_arg, uint32_t probe_ok,
                   uint32_t* calls_out, uint64_t* report_out) {
  std::vector<uint8_t> healthy(healthy_io, healthy_io + n_slots);
  std::vector<std::atomic<uint32_t>> calls(n_slots);
  for (auto& c : calls) c = 0;
  cg::PoolReport rep;
  const int rc = cg::pool_run(
      healthy, n_items, status,
      [&](uint32_t slot, uint64_t first, uint64_t count) -> int {
        const uint32_t n = calls[slot]++;
        if ((fail_always >> slot) & 1u) return CG_ERR_DEVICE;
        if ((fail_arg >> slot) & 1u) return CG_ERR_NOMEM;
        if (((fail_once >> slot) & 1u) && n == 0) {
          status[first] = 0;  // a partial write before the fault: pool_run must reset it
          return CG_ERR_DEVICE;
        }
        return or_verify_batch(keys, n_keys, items + first, count, arena, arena_len, mode, status + first, 1) == 0
                   ? CG_OK
                   : CG_ERR_DEVICE;
      },
      [&](uint32_t slot) { return ((probe_ok >> slot) & 1u) != 0; }, &rep);
  for (uint32_t s = 0; s < n_slots; ++s) {
    healthy_io[s] = healthy[s];
    calls_out[s] = calls[s];
  }
  report_out[0] = rep.shards;
  report_out[1] = rep.reruns;
  report_out[2] = rep.failed_slots;
  report_out[3] = rep.not_run;
  return rc;
}
}
