// The batch plan: item indices grouped by (scheme class, table mode, long bit, key).
//
// Round 5 also built a counting plan (-DCG_PLAN_COUNTING=1) in place of the radix sort. A bucket is a
// (key, long bit) pair; the buckets are ranked by (class, mode, long) group, a key's rank inside its
// group being an atomic ticket (any order of keys serves: locality is per key). Per chunk: zero the
// counts, count every item into its bucket (the atomic's return value is the item's place in its
// bucket), scan the counts in rank order, scatter: five to seven small launches instead of the
// onesweep sort's ~15. Measured slower (plan 1.7-1.9 -> 2.5-2.7 ms per headline step, 2 x 2 runs,
// profiles/r05/plan): the 2.5M device-scope atomics with return per chunk go to ~400 counter lines
// shared by every XCD, where the onesweep passes count digits in LDS. Kept for A/B, off.
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

// ---------------------------------------------------------------- counting plan
#define PL_GROUPS 24  // 3 classes x 4 modes x (short, long); group 24 = the misc bucket (no verify class)
__device__ __forceinline__ uint32_t pl_class_of(const cg_key* keys, uint32_t n_keys, uint32_t k) {
  if (k >= n_keys) return PLAN_CLASSES;
  const uint8_t s = keys[k].scheme;
  return s == CG_EDDSA_ED25519_SHA512 ? PLAN_ED
       : s == CG_ECDSA_SECP256R1_SHA256 ? PLAN_R1
       : s == CG_ECDSA_SECP256K1_SHA256 ? PLAN_K1
                                        : PLAN_CLASSES;
}
__device__ __forceinline__ uint32_t pl_mode_of(uint32_t k, const uint32_t* uses, const uint32_t* wide_idx) {
  return wide_idx[k] != KEY_NOT_WIDE       ? PLAN_MODE_WIDE
       : uses[k] >= ED_DIRECT_MAX_USES    ? PLAN_MODE_FULL
       : uses[k] >= KEY_QUARTER_MIN_USES  ? PLAN_MODE_QUART
                                          : PLAN_MODE_ROW0;
}

__global__ void __launch_bounds__(256) k_plan_zero(uint32_t* __restrict__ cnt, uint64_t nb, uint32_t* __restrict__ grp) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < 64) grp[i] = 0;
  if (i < nb) cnt[i] = 0;
}

// per key: its ticket in the (class, mode, short) and (class, mode, long) groups
__global__ void __launch_bounds__(256) k_plan_tickets(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                      const uint32_t* __restrict__ uses,
                                                      const uint32_t* __restrict__ wide_idx,
                                                      uint32_t* __restrict__ grp, uint32_t* __restrict__ tick) {
  front_prio();
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= n_keys) return;
  const uint32_t c = pl_class_of(keys, n_keys, k);
  if (c >= PLAN_CLASSES) return;
  const uint32_t g = c * 8 + pl_mode_of(k, uses, wide_idx) * 2;
  tick[k] = atomicAdd(&grp[g], 1u);
  tick[n_keys + k] = atomicAdd(&grp[g + 1], 1u);
}

// grp[32 + g] = the rank of group g's first bucket (exclusive scan of the group sizes; the misc
// bucket, group 24, last)
__global__ void k_plan_group_base(uint32_t* __restrict__ grp) {
  if (threadIdx.x != 0) return;
  uint32_t acc = 0;
  for (int g = 0; g < PL_GROUPS; ++g) {
    grp[32 + g] = acc;
    acc += grp[g];
  }
  grp[32 + PL_GROUPS] = acc;
}

// per item: its bucket's rank, and its place in the bucket
__global__ void __launch_bounds__(256) k_plan_count(const cg_item* __restrict__ items, uint64_t n_items,
                                                    const cg_key* __restrict__ keys, uint32_t n_keys,
                                                    const uint32_t* __restrict__ uses,
                                                    const uint32_t* __restrict__ wide_idx,
                                                    const uint32_t* __restrict__ grp,
                                                    const uint32_t* __restrict__ tick, uint32_t* __restrict__ cnt,
                                                    uint32_t* __restrict__ rank, uint32_t* __restrict__ place) {
  front_prio();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const uint32_t k = items[i].key_idx;
  const uint32_t c = pl_class_of(keys, n_keys, k);
  uint32_t r;
  if (c >= PLAN_CLASSES) {
    r = grp[32 + PL_GROUPS];
  } else {
    const uint32_t lng = items[i].msg_len > ITEM_LONG_MIN ? 1u : 0u;
    const uint32_t g = c * 8 + pl_mode_of(k, uses, wide_idx) * 2 + lng;
    r = grp[32 + g] + tick[lng * n_keys + k];
  }
  rank[i] = r;
  place[i] = atomicAdd(&cnt[r], 1u);
}

// exclusive scan of nb counts: per 16k-bucket tile in one block (1024 threads x 16), then the tile
// partials (one block), then their offsets added
__device__ __forceinline__ uint32_t pl_block_exscan(uint32_t v, uint32_t* sh, uint32_t& total) {
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o, 64);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63) sh[wv] = x;
  __syncthreads();
  if (threadIdx.x < 64) {
    uint32_t w = threadIdx.x < (blockDim.x >> 6) ? sh[threadIdx.x] : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)w, o, 64);
      if (threadIdx.x >= (uint32_t)o) w += y;
    }
    sh[64 + threadIdx.x] = w;  // inclusive over waves
  }
  __syncthreads();
  total = sh[64 + (blockDim.x >> 6) - 1];
  const uint32_t before = wv ? sh[64 + wv - 1] : 0u;
  return before + x - v;
}

__global__ void __launch_bounds__(1024) k_plan_scan_tiles(const uint32_t* __restrict__ cnt, uint64_t nb,
                                                          uint32_t* __restrict__ pos, uint32_t* __restrict__ tile) {
  __shared__ uint32_t sh[128];
  const uint64_t t0 = (uint64_t)blockIdx.x * PL_TILE + (uint64_t)threadIdx.x * 16u;
  uint32_t v[16], sum = 0;
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    v[j] = t0 + j < nb ? cnt[t0 + j] : 0u;
    sum += v[j];
  }
  uint32_t total;
  uint32_t run = pl_block_exscan(sum, sh, total);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    if (t0 + j < nb) pos[t0 + j] = run;
    run += v[j];
  }
  if (threadIdx.x == 0) tile[blockIdx.x] = total;
}

__global__ void __launch_bounds__(1024) k_plan_scan_top(uint32_t* __restrict__ tile, uint32_t n_tiles) {
  __shared__ uint32_t sh[128];
  const uint32_t v = threadIdx.x < n_tiles ? tile[threadIdx.x] : 0u;
  uint32_t total;
  const uint32_t ex = pl_block_exscan(v, sh, total);
  if (threadIdx.x < n_tiles) tile[threadIdx.x] = ex;
}

__global__ void __launch_bounds__(256) k_plan_scan_add(uint32_t* __restrict__ pos, uint64_t nb,
                                                       const uint32_t* __restrict__ tile) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < nb && i >= PL_TILE) pos[i] += tile[i / PL_TILE];
}

__global__ void __launch_bounds__(256) k_plan_scatter(uint64_t n_items, const uint32_t* __restrict__ rank,
                                                      const uint32_t* __restrict__ place,
                                                      const uint32_t* __restrict__ pos, uint32_t* __restrict__ perm) {
  front_prio();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  perm[pos[rank[i]] + place[i]] = (uint32_t)i;
}

// ranges[c] = first item of class c (c = PLAN_CLASSES: the misc items), ranges[PLAN_QUART / FULL /
// WIDE + c] = first item of that mode: the start of the (class, mode, short) group's first bucket
__global__ void k_plan_ranges_cnt(const uint32_t* __restrict__ grp, const uint32_t* __restrict__ pos,
                                  uint32_t* __restrict__ ranges) {
  const uint32_t t = threadIdx.x;
  if (t >= PLAN_QUART + PLAN_CLASSES) return;
  uint32_t g;
  if (t <= PLAN_CLASSES) g = t * 8;  // t = PLAN_CLASSES: group 24, the misc bucket
  else if (t < PLAN_WIDE) g = (t - PLAN_FULL) * 8 + PLAN_MODE_FULL * 2;
  else if (t < PLAN_QUART) g = (t - PLAN_WIDE) * 8 + PLAN_MODE_WIDE * 2;
  else g = (t - PLAN_QUART) * 8 + PLAN_MODE_QUART * 2;
  ranges[t] = pos[grp[32 + g]];
}

#ifndef CG_PLAN_COUNTING
#define CG_PLAN_COUNTING 0
#endif

hipError_t launch_plan(const cg_item* d_items, uint64_t n_items, const cg_key* d_keys, uint32_t n_keys,
                       const KeyWs& w, const ItemWs& iw, hipStream_t stream) {
  const uint32_t B = 256;
  const uint64_t nb = pl_buckets(n_keys), tiles = pl_tiles(n_keys);
  if (CG_PLAN_COUNTING && tiles <= 1024) {
    const uint64_t zl = nb > 64 ? nb : 64;
    hipLaunchKernelGGL(k_plan_zero, dim3((unsigned)((zl + B - 1) / B)), dim3(B), 0, stream, w.pl_cnt, nb, w.pl_grp);
    if (n_keys)
      hipLaunchKernelGGL(k_plan_tickets, dim3((n_keys + B - 1) / B), dim3(B), 0, stream, d_keys, n_keys,
                         (const uint32_t*)w.uses, (const uint32_t*)w.wide_idx, w.pl_grp, w.pl_tick);
    hipLaunchKernelGGL(k_plan_group_base, dim3(1), dim3(64), 0, stream, w.pl_grp);
    hipLaunchKernelGGL(k_plan_count, dim3((unsigned)((n_items + B - 1) / B)), dim3(B), 0, stream, d_items, n_items,
                       d_keys, n_keys, (const uint32_t*)w.uses, (const uint32_t*)w.wide_idx,
                       (const uint32_t*)w.pl_grp, (const uint32_t*)w.pl_tick, w.pl_cnt, iw.sval_in, iw.skey_in);
    hipLaunchKernelGGL(k_plan_scan_tiles, dim3((unsigned)tiles), dim3(1024), 0, stream, (const uint32_t*)w.pl_cnt, nb,
                       w.pl_pos, w.pl_tile);
    if (tiles > 1) {
      hipLaunchKernelGGL(k_plan_scan_top, dim3(1), dim3(1024), 0, stream, w.pl_tile, (uint32_t)tiles);
      hipLaunchKernelGGL(k_plan_scan_add, dim3((unsigned)((nb + B - 1) / B)), dim3(B), 0, stream, w.pl_pos, nb,
                         (const uint32_t*)w.pl_tile);
    }
    hipLaunchKernelGGL(k_plan_scatter, dim3((unsigned)((n_items + B - 1) / B)), dim3(B), 0, stream, n_items,
                       (const uint32_t*)iw.sval_in, (const uint32_t*)iw.skey_in, (const uint32_t*)w.pl_pos, iw.perm);
    hipLaunchKernelGGL(k_plan_ranges_cnt, dim3(1), dim3(64), 0, stream, (const uint32_t*)w.pl_grp,
                       (const uint32_t*)w.pl_pos, iw.ranges);
    return hipGetLastError();
  }
  // the radix-sort plan (CG_PLAN_COUNTING=0, or more than 8M keys)
  const uint32_t kb = key_bits(n_keys) + 3;  // + the table-mode bits + the long bit
  hipLaunchKernelGGL(k_plan_keys, dim3((unsigned)((n_items + B - 1) / B)), dim3(B), 0, stream, d_items, n_items,
                     d_keys, n_keys, kb, (const uint32_t*)w.uses, (const uint32_t*)w.wide_idx, iw.skey_in, iw.sval_in);
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
