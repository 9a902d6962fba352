// The batch plan: item indices sorted by (scheme class, key) with a device radix sort.
//
// Each scheme's kernels then walk one dense range of `perm` (no lane idles on another scheme's
// item), and inside a range the items of one key are adjacent, so the 64 lanes of a wave
// gather from the same key's rows (k_ed_ladder went from 36% to 52% of its wave cycles waiting
// on table gathers once the B rows left LDS; key order keeps the -A rows hot in L2). The sort
// is stable (LSD radix): input order is kept within a key. No per-item atomics, so a hot key
// (a notary's) costs nothing extra.
//   k_plan_keys    composite key (class | table mode | key_idx) and the identity permutation; the
//                  mode bits (keyws.h) keep row-0, full- and wide-table items in separate waves
//   rocprim::radix_sort_pairs over key_bits + 4 bits
//   k_plan_ranges  class boundaries by binary search in the sorted keys
#include <hip/hip_runtime.h>

#include <rocprim/device/device_radix_sort.hpp>

#include "keyws.h"

namespace cg {

// Onesweep at every size above one block: rocprim's default switches to block sort + merge
// passes up to 2^20 items, which took ~300 us for 2^20 items over 14 key bits (ten merge
// passes) against ~2 onesweep passes of 8 bits.
typedef rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config, rocprim::default_config, 0>
    PlanSortConfig;

static uint32_t key_bits(uint32_t n_keys) {
  uint32_t b = 1;
  while (b < 27 && (1u << b) < n_keys) ++b;  // 2 class bits + 2 mode bits + the long bit + 27 key bits
  return b;
}

// kb = key bits + 3: below the class, the key's table mode (0 row 0, 1 full, 2 wide tables,
// keyws.h), so a wave's lanes run one ladder variant; below the mode the long bit (clear data of
// more than ITEM_LONG_MIN bytes: its items hash in waves of their own at the end of the mode's
// range instead of stalling a wave of 64 short ones; SURVEY.md §5 "long-context"); then the key
// index. Keys beyond 2^27 share sort positions (the index is masked): locality only, never a
// verdict.
__global__ void __launch_bounds__(256) k_plan_keys(const cg_item* __restrict__ items, uint64_t n_items,
                                                   const cg_key* __restrict__ keys, uint32_t n_keys, uint32_t kb,
                                                   const uint32_t* __restrict__ uses,
                                                   const uint32_t* __restrict__ wide_idx,
                                                   uint32_t* __restrict__ skey, uint32_t* __restrict__ sval) {
  front_prio();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const uint32_t k = items[i].key_idx;
  uint32_t c = PLAN_CLASSES;  // no verify kernel takes it (k_misc_status sets its status)
  if (k < n_keys) {
    const uint8_t s = keys[k].scheme;
    c = s == CG_EDDSA_ED25519_SHA512 ? PLAN_ED
      : s == CG_ECDSA_SECP256R1_SHA256 ? PLAN_R1
      : s == CG_ECDSA_SECP256K1_SHA256 ? PLAN_K1
                                       : PLAN_CLASSES;
  }
  uint32_t mode = 0;
  if (c < PLAN_CLASSES)
    mode = wide_idx[k] != KEY_NOT_WIDE         ? PLAN_MODE_WIDE
         : uses[k] >= ED_DIRECT_MAX_USES      ? PLAN_MODE_FULL
         : uses[k] >= KEY_QUARTER_MIN_USES    ? PLAN_MODE_QUART
                                              : PLAN_MODE_ROW0;
  const uint32_t lng = items[i].msg_len > ITEM_LONG_MIN ? 1u : 0u;
  skey[i] = (c << kb) |
            (c < PLAN_CLASSES ? (mode << (kb - 2)) | (lng << (kb - 3)) | (k & ((1u << (kb - 3)) - 1u)) : 0u);
  sval[i] = (uint32_t)i;
}

__global__ void k_plan_ranges(const uint32_t* __restrict__ skey, uint64_t n_items, uint32_t kb,
                              uint32_t* __restrict__ ranges) {
  front_prio();
  // lanes 0..3: class starts ranges[c] (ranges[3] = end of the verified classes); lanes 4..6:
  // ranges[PLAN_FULL + c] = first full-table item of class c; lanes 7..9: ranges[PLAN_WIDE + c] =
  // first wide-table item; lanes 10..12: ranges[PLAN_QUART + c] = first quarter-table item (the mode
  // bits, keyws.h: row 0, quarter, full, wide)
  const uint32_t t = threadIdx.x;
  if (t >= PLAN_QUART + PLAN_CLASSES) return;
  uint32_t c, target;
  if (t <= PLAN_CLASSES) {
    c = t;
    target = c << kb;
  } else if (t < PLAN_WIDE) {
    c = t - PLAN_FULL;
    target = (c << kb) | (PLAN_MODE_FULL << (kb - 2));
  } else if (t < PLAN_QUART) {
    c = t - PLAN_WIDE;
    target = (c << kb) | (PLAN_MODE_WIDE << (kb - 2));
  } else {
    c = t - PLAN_QUART;
    target = (c << kb) | (PLAN_MODE_QUART << (kb - 2));
  }
  uint64_t lo = 0, hi = n_items;  // first position with key >= target
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (skey[mid] < target) lo = mid + 1;
    else hi = mid;
  }
  ranges[t] = (uint32_t)lo;
}

size_t plan_sort_temp_bytes(uint64_t n_items) {
  size_t bytes = 0;
  rocprim::radix_sort_pairs<PlanSortConfig>((void*)nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                            (const uint32_t*)nullptr, (uint32_t*)nullptr, (size_t)(n_items ? n_items : 1), 0u,
                            32u);
  return bytes;
}

hipError_t launch_plan(const cg_item* d_items, uint64_t n_items, const cg_key* d_keys, uint32_t n_keys,
                       const uint32_t* d_uses, const uint32_t* d_wide_idx, const ItemWs& iw, hipStream_t stream) {
  const uint32_t kb = key_bits(n_keys) + 3;  // + the table-mode bits + the long bit
  const uint32_t B = 256;
  hipLaunchKernelGGL(k_plan_keys, dim3((unsigned)((n_items + B - 1) / B)), dim3(B), 0, stream, d_items, n_items,
                     d_keys, n_keys, kb, d_uses, d_wide_idx, iw.skey_in, iw.sval_in);
  size_t bytes = iw.sort_temp_bytes;
  hipError_t e = rocprim::radix_sort_pairs<PlanSortConfig>(iw.sort_temp, bytes, (const uint32_t*)iw.skey_in, iw.skey_out,
                                           (const uint32_t*)iw.sval_in, iw.perm, (size_t)n_items, 0u, kb + 2,
                                           stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_plan_ranges, dim3(1), dim3(64), 0, stream, (const uint32_t*)iw.skey_out, n_items, kb,
                     iw.ranges);
  return hipGetLastError();
}

}  // namespace cg
