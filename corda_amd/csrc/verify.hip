// Batch signature verification for gfx950: dispatch over the per-scheme kernels.
//
// Pipeline per batch (all on the caller's stream, no host round trip):
//   key prep      verify_ed.hip k_ed_keyprep_rows/_tab, verify_ec.hip k_ec_keyprep_rows/_tab
//   items         k_misc_status (unsupported scheme / bad key index); the plan (plan_sort.hip:
//                 items sorted by (scheme, key), one dense range per scheme); then the Ed25519 stages (k_ed_verify, k_ed_finish) and per
//                 curve the ECDSA stages (k_ec_prep, k_ec_inv, k_ec_ladder) over their ranges.
//                 Each stage writes the final status byte of its items.
// Replaces, per item, the JCA call at core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559
// behind Crypto.doVerify (Crypto.kt:474-484).
#include "keyws.h"

namespace cg {

__global__ void k_misc_status(const cg_item* __restrict__ items, uint64_t n_items, const cg_key* __restrict__ keys,
                              uint32_t n_keys, uint8_t* __restrict__ status) {
  front_prio();
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const uint32_t ki = items[i].key_idx;
  if (ki >= n_keys) {
    status[i] = CG_NOT_RUN;
    return;
  }
  const uint8_t s = keys[ki].scheme;
  if (s != CG_EDDSA_ED25519_SHA512 && s != CG_ECDSA_SECP256R1_SHA256 && s != CG_ECDSA_SECP256K1_SHA256)
    status[i] = CG_UNSUPPORTED;
  else if (s == CG_EDDSA_ED25519_SHA512)
    status[i] = CG_NOT_RUN;  // until a verdict lands (k_ed_hash writes only its early verdicts: verify_ed.hip)
}

// Per-key use counts, sampled: one item in KEY_USES_SAMPLE adds KEY_USES_SAMPLE (no-return
// atomics, a quarter of the traffic of counting all), every item marks its key as used (plain
// stores: the exact "has items" bit row 0 depends on). Out-of-range key indices are
// k_misc_status's (CG_NOT_RUN) and count nowhere.
__global__ void __launch_bounds__(256) k_key_init(uint32_t n_keys, uint32_t all, uint32_t* __restrict__ uses,
                                                  uint8_t* __restrict__ seen, uint32_t* __restrict__ full_count,
                                                  uint32_t* __restrict__ wide_idx, uint32_t* __restrict__ wide_count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < PLAN_CLASSES) full_count[i] = full_count[ROW0_COUNT_AT + i] = full_count[QUART_COUNT_AT + i] = 0;
  if (i == 0) full_count[SKIP_MISMATCH_AT] = 0;
  if (i < PLAN_CLASSES + 2) wide_count[i] = 0;
  if (i >= n_keys) return;
  uses[i] = all ? KEY_USES_ALL : 0u;
  seen[i] = all ? 1 : 0;
  wide_idx[i] = KEY_NOT_WIDE;
}

__global__ void __launch_bounds__(256) k_key_uses(const cg_item* __restrict__ items, uint64_t n_items,
                                                  uint32_t n_keys, uint32_t* __restrict__ uses,
                                                  uint8_t* __restrict__ seen) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  const uint32_t k = items[i].key_idx;
  if (k >= n_keys) return;
  seen[k] = 1;
  // sample by a multiplicative hash of the index, not i % 4: a batch whose items cycle through
  // the keys with a stride (item j -> key j % n) would otherwise alias whole keys out
  if (((uint32_t)i * 0x9E3779B1u) >> 30 == 0) atomicAdd(&uses[k], KEY_USES_SAMPLE);
}

// The same, from a cg_txsig table (cg_verify_tx_signatures_device: the key tables are sized before
// any verify item exists, so the per-chunk item builds and splices can follow them).
template <class Sig>
__global__ void __launch_bounds__(256) k_key_uses_txsig(const Sig* __restrict__ sigs, uint64_t n,
                                                        uint32_t n_keys, uint32_t* __restrict__ uses,
                                                        uint8_t* __restrict__ seen) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint32_t k = sigs[i].key_idx;
  if (k >= n_keys) return;
  seen[k] = 1;
  if (((uint32_t)i * 0x9E3779B1u) >> 30 == 0) atomicAdd(&uses[k], KEY_USES_SAMPLE);
}

// Exact counts made by the host (cg_verify_tx_signatures counts while it scans the signature
// table for the copy extents, so no signature table has to be resident before the key tables).
__global__ void __launch_bounds__(256) k_key_counts(const uint32_t* __restrict__ counts, uint32_t n_keys,
                                                    uint32_t* __restrict__ uses, uint8_t* __restrict__ seen) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_keys) return;
  uses[i] = counts[i];
  seen[i] = counts[i] != 0;
}

// Append the lanes with c == k to list k (one atomic per wave and class).
__device__ __forceinline__ void list_append(int c, uint32_t i, uint32_t n_keys, uint32_t* __restrict__ list,
                                            uint32_t* __restrict__ count) {
  const uint32_t lane = threadIdx.x & 63u;
#pragma unroll
  for (int k = 0; k < PLAN_CLASSES; ++k) {
    const uint64_t m = __ballot(c == k);
    if (m == 0) continue;
    const int leader = __ffsll((long long)m) - 1;
    uint32_t base = 0;
    if ((int)lane == leader) base = atomicAdd(&count[k], (uint32_t)__popcll(m));
    base = __shfl(base, leader, 64);
    if (c == k) list[(size_t)k * n_keys + base + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = i;
  }
}

// Table mode per key: wide tables for keys with >= min_ed / min_ec items while the family's
// wide pool has slots (one atomic per wide key: they are few), else full tables from
// ED_DIRECT_MAX_USES items, quarter tables from KEY_QUARTER_MIN_USES, else row 0; the keys of each
// mode compacted per scheme class (row0 lists every used key without wide tables). One wave a block.
__global__ void __launch_bounds__(64) k_key_classify(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                     uint32_t* __restrict__ uses, const uint8_t* __restrict__ seen,
                                                     uint32_t* __restrict__ full, uint32_t* __restrict__ full_count,
                                                     uint32_t* __restrict__ wide_idx, uint32_t* __restrict__ wide,
                                                     uint32_t* __restrict__ wide_count, uint32_t* __restrict__ row0,
                                                     uint32_t* __restrict__ quart, uint32_t cap_ed, uint32_t cap_ec,
                                                     uint32_t min_ed, uint32_t min_ec, uint32_t skip_mask) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  int c = -1, cw = -1, c0 = -1, cq = -1;  // full list, wide list, row-0 list, quarter list
  uint32_t u = 0;
  if (i < n_keys) {  // the estimate, made exact where it matters: a used key counts >= 1
    u = uses[i];
    if (!seen[i]) u = 0;
    else if (u == 0) u = 1;
    uses[i] = u;
  }
  if (i < n_keys && u >= ED_DIRECT_MAX_USES) {
    const uint8_t s = keys[i].scheme;
    c = s == CG_EDDSA_ED25519_SHA512 ? PLAN_ED
      : s == CG_ECDSA_SECP256R1_SHA256 ? PLAN_R1
      : s == CG_ECDSA_SECP256K1_SHA256 ? PLAN_K1
                                       : -1;
    // KEY_USES_ALL (cg_prepare_keys_device: uses unknown) never gets wide tables
    const int pool = c == PLAN_ED ? 0 : 1;
    if (c >= 0 && u >= (pool == 0 ? min_ed : min_ec) && u != KEY_USES_ALL) {
      const uint32_t cap = pool == 0 ? cap_ed : cap_ec;
      if (cap) {
        const uint32_t slot = atomicAdd(&wide_count[PLAN_CLASSES + pool], 1u);
        if (slot < cap) {
          wide_idx[i] = slot;
          cw = c;
          c = -1;
        }
      }
    }
  }
  if (i < n_keys && u >= 1 && cw < 0) {  // every used key without wide tables gets its row 0
    const uint8_t s = keys[i].scheme;
    c0 = s == CG_EDDSA_ED25519_SHA512 ? PLAN_ED
       : s == CG_ECDSA_SECP256R1_SHA256 ? PLAN_R1
       : s == CG_ECDSA_SECP256K1_SHA256 ? PLAN_K1
                                        : -1;
    if (u >= KEY_QUARTER_MIN_USES && u < ED_DIRECT_MAX_USES) cq = c0;  // and its quarter rows 1..3
  }
  if (skip_mask && (c >= 0 || c0 >= 0)) {  // a mode whose builds / ladders the host skipped
    const int cls = c >= 0 ? c : c0;
    const uint32_t f = cls == PLAN_R1 ? 0u : cls == PLAN_K1 ? 1u : 2u;
    if ((skip_mask >> f) & 1u) atomicOr(&full_count[SKIP_MISMATCH_AT], 1u << f);
  }
  list_append(c, i, n_keys, full, full_count);
  list_append(cw, i, n_keys, wide, wide_count);
  list_append(c0, i, n_keys, row0, full_count + ROW0_COUNT_AT);
  list_append(cq, i, n_keys, quart, full_count + QUART_COUNT_AT);
}

// The items of family f's row-0 / quarter / full modes -> CG_NOT_RUN when k_key_classify flagged f
// (SKIP_MISMATCH_AT): their ladders or tables were skipped on the host's word. A uniform early exit
// otherwise (one load of the flag per wave).
__global__ void __launch_bounds__(256) k_mode_guard(const uint32_t* __restrict__ ranges,
                                                    const uint32_t* __restrict__ perm,
                                                    const uint32_t* __restrict__ full_count, uint32_t skip_mask,
                                                    uint8_t* __restrict__ status) {
  const uint32_t bad = full_count[SKIP_MISMATCH_AT] & skip_mask;
  if (!bad) return;
  for (int f = 0; f < 3; ++f) {
    if (!((bad >> f) & 1u)) continue;
    const int cls = f == 0 ? PLAN_R1 : f == 1 ? PLAN_K1 : PLAN_ED;
    const uint32_t beg = ranges[cls], end = ranges[PLAN_WIDE + cls];
    for (uint32_t p = beg + blockIdx.x * blockDim.x + threadIdx.x; p < end; p += gridDim.x * blockDim.x)
      status[perm[p]] = CG_NOT_RUN;
  }
}

hipError_t upload_constants() {
  hipError_t e = ed_upload_constants();
  if (e != hipSuccess) return e;
  return ec_upload_constants();
}

size_t keyprep_bytes(uint32_t n_keys) { return key_ws_bytes(n_keys); }
size_t wide_bytes(uint32_t n_keys, uint64_t n_items, uint32_t max_slots) {
  return wide_pool_bytes(wide_cap(n_keys, n_items, max_slots));
}
size_t wide_slot_bytes() { return wide_pool_bytes(1); }
static_assert(kKeyWideMax == KEY_WIDE_MAX, "engine.h mirrors keyws.h");
WidePool make_wide_pool(void* base, uint32_t n_keys, uint64_t n_items, uint32_t max_slots) {
  return wide_pool(base, wide_cap(n_keys, n_items, max_slots));
}
size_t item_ws_bytes(uint64_t n_items) { return item_ws_total(n_items); }
size_t btab_bytes() { return const_tab_bytes(); }
size_t btab_scratch_bytes() { return const_scratch_bytes(); }

hipError_t init_btab(void* d_btab, void* d_scratch, hipStream_t stream) {
  hipError_t e = ed_init_const(d_btab, d_scratch, stream);
  if (e != hipSuccess) return e;
  return ec_init_const(d_btab, d_scratch, stream);
}

// The deferred table builds, forked from `stream` at this point: Ed25519 first (its ladder runs
// first), the two curves after it (their ladders run after the Ed25519 ladder and finish); per
// family the wide tables, then the full / row-0 ones.
static hipError_t launch_pending_tabs(const Fork* fork, hipStream_t stream) {
  PendingTabs& p = fork->pending;
  if (!p.on) return hipSuccess;
  p.on = false;
  const KeyWs w = key_ws(p.keyprep, p.n_keys, &p.wide);
  hipError_t e = hipEventRecord(fork->planned, stream);
  if (e == hipSuccess) e = hipStreamWaitEvent(fork->side[2], fork->planned, 0);
  if (e != hipSuccess) return e;
  // every family's row builds after ALL the row-base chains: a chain is one lane per key (a few
  // dozen waves, latency-bound), and beside another family's row builds it ran 4x slower (r1: 5.6
  // instead of 1.3 ms, then its rows after it: profiles/r03/env_copyq timeline). CG_CHAINS_FIRST=0:
  // each family's builds right after its own chains (A/B). Round 4: with the chains' raised issue
  // priority (keyws.h chain_prio) the builds no longer slow them, and each family's builds start
  // as soon as its own chains end: CG_CHAINS_FIRST=1 restores the wait for all (3 x 3 runs each:
  // chunk 0's front done 0.5-0.8 ms earlier, ~+2% whole-node, profiles/r04/phase1)
  static const bool chains_first = [] {
    const char* v = getenv("CG_CHAINS_FIRST");
    return v && v[0] == '1';
  }();
  for (int k = 0; k < 3 && e == hipSuccess && chains_first; ++k)
    for (int q = 0; q < 3 && e == hipSuccess; ++q)
      if (q != k && fork->chains[q]) e = hipStreamWaitEvent(fork->side[k], fork->chains[q], 0);
  if (e != hipSuccess) return e;
  ed_launch_keyprep_tabs(p.keys, p.n_keys, w, fork->side[2], false, true);
  e = hipEventRecord(fork->ed_tabs, fork->side[2]);
  // then the full / row-0 tables (usually few keys: launched ahead of the wide builds, their
  // near-empty grids queued behind the challenge hashes, which hold every SIMD, and stalled the
  // wide builds behind them by ~1.8 ms per call: profiles/r02/sha_v2/timeline_step.txt)
  if (p.need_full[2]) ed_launch_keyprep_tabs(p.keys, p.n_keys, w, fork->side[2], true, false);
  if (e == hipSuccess) e = hipEventRecord(fork->ready[2], fork->side[2]);
  // the curves' wide builds right after their own row-base chains, beside the Ed25519 builds, so
  // that they are done before the first chunk's fronts (after the Ed25519 builds, they ran 5.8 ->
  // 9.9 ms into the step and slowed the first chunk's challenge hashes 2.4x: profiles/r03/v8
  // timeline); CG_TABS_CONCURRENT=0 (A/B): after the Ed25519 builds
  static const bool concurrent = [] {
    const char* v = getenv("CG_TABS_CONCURRENT");
    return !(v && v[0] == '0');
  }();
  for (int k = 0; k < 2 && e == hipSuccess; ++k) {
    e = hipStreamWaitEvent(fork->side[k], fork->planned, 0);
    if (e == hipSuccess && !concurrent) e = hipStreamWaitEvent(fork->side[k], fork->ed_tabs, 0);
    if (e != hipSuccess) break;
    ec_launch_keyprep_tabs(k == 0 ? CG_CURVE_R1 : CG_CURVE_K1, p.keys, p.n_keys, w, fork->side[k], false, true);
    if (p.need_full[k])
      ec_launch_keyprep_tabs(k == 0 ? CG_CURVE_R1 : CG_CURVE_K1, p.keys, p.n_keys, w, fork->side[k], true, false);
    e = hipEventRecord(fork->ready[k], fork->side[k]);
  }
  return e;
}

hipError_t launch_key_tables(const Fork* fork, hipStream_t stream) {
  return fork ? launch_pending_tabs(fork, stream) : hipSuccess;
}

// k_key_classify's outcome from the host counts: does any key of family f (0 r1, 1 k1, 2 Ed25519)
// end in row-0 or full-table mode? Mirrors the kernel (a counted key has u >= 1; wide when u >=
// max(ED_DIRECT_MAX_USES, the pool's minimum) and the pool's slots hold every such key).
static void families_needing_full(const KeyUses& src, uint32_t n_keys, const KeyWs& w, bool need[3]) {
  uint32_t hot[2] = {0, 0};  // keys asking for a wide slot, per pool (0 Ed25519, 1 ECDSA)
  bool low[3] = {false, false, false};
  for (uint32_t i = 0; i < n_keys; ++i) {
    const uint32_t u = src.host_counts[i];
    if (u == 0) continue;
    const uint8_t s = src.host_keys[i].scheme;
    const int f = s == CG_ECDSA_SECP256R1_SHA256 ? 0 : s == CG_ECDSA_SECP256K1_SHA256 ? 1 : s == CG_EDDSA_ED25519_SHA512 ? 2 : -1;
    if (f < 0) continue;
    const int pool = f == 2 ? 0 : 1;
    const uint32_t cap = pool == 0 ? w.cap_ed : w.cap_ec;
    if (u >= ED_DIRECT_MAX_USES && u >= (pool == 0 ? w.min_ed : w.min_ec) && u != KEY_USES_ALL && cap) ++hot[pool];
    else low[f] = true;
  }
  const bool over[2] = {hot[0] > w.cap_ed, hot[1] > w.cap_ec};
  for (int f = 0; f < 3; ++f) need[f] = low[f] || over[f == 2 ? 0 : 1];
}

hipError_t launch_keyprep(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                          void* d_keyprep, hipStream_t stream, const Fork* fork, const cg_item* d_items,
                          uint64_t n_items, const WidePool* wide, const KeyUses* src) {
  if (fork) {  // a call with no keys must not inherit the previous call's skip (k_mode_guard reads it)
    fork->pending.skip_mask = 0;
    for (int f = 0; f < 3; ++f) fork->pending.need_full[f] = true;
  }
  if (n_keys == 0) return hipSuccess;
  const bool counted = d_items || src;  // tables sized by the call's key uses
  if (!d_items && src) n_items = src->n;
  const KeyWs w = key_ws(d_keyprep, n_keys, counted ? wide : nullptr);
  // use counts first (main stream; the side streams fork after them)
  const uint32_t kl = n_keys > PLAN_CLASSES + 2 ? n_keys : PLAN_CLASSES + 2;
  hipLaunchKernelGGL(k_key_init, dim3((kl + 255) / 256), dim3(256), 0, stream, n_keys, counted ? 0u : 1u, w.uses,
                     w.seen, w.full_count, w.wide_idx, w.wide_count);
  if (d_items && n_items)
    hipLaunchKernelGGL(k_key_uses, dim3((unsigned)((n_items + 255) / 256)), dim3(256), 0, stream, d_items, n_items,
                       n_keys, w.uses, w.seen);
  else if (src && src->counts)
    hipLaunchKernelGGL(k_key_counts, dim3((n_keys + 255) / 256), dim3(256), 0, stream, src->counts, n_keys, w.uses,
                       w.seen);
  else if (src && src->sigs && src->n)
    hipLaunchKernelGGL(k_key_uses_txsig<cg_txsig>, dim3((unsigned)((src->n + 255) / 256)), dim3(256), 0, stream,
                       src->sigs, src->n, n_keys, w.uses, w.seen);
  else if (src && src->sigs12 && src->n)
    hipLaunchKernelGGL(k_key_uses_txsig<cg_txsig_packed>, dim3((unsigned)((src->n + 255) / 256)), dim3(256), 0,
                       stream, src->sigs12, src->n, n_keys, w.uses, w.seen);
  static const bool serial = [] {  // CG_SERIAL_KEYPREP=1: key prep on the caller's stream (A/B runs)
    const char* v = getenv("CG_SERIAL_KEYPREP");
    return v && v[0] == '1';
  }();
  static const bool skip_full = [] {  // CG_SKIP_EMPTY_TABS=0: always launch the row-0 / full builds (A/B)
    const char* v = getenv("CG_SKIP_EMPTY_TABS");
    return !(v && v[0] == '0');
  }();
  // every mode's builds and ladders unless this call's host counts prove a family has no row-0 /
  // quarter / full key; the classification checks that proof on the device (k_mode_guard)
  uint32_t skip_mask = 0;
  if (fork) {
    for (int f = 0; f < 3; ++f) fork->pending.need_full[f] = true;
    if (skip_full && !serial && !d_items && src && src->counts && src->host_counts && src->host_keys)
      families_needing_full(*src, n_keys, w, fork->pending.need_full);
    // CG_TEST_SKIP_FAMILIES=<mask> (tests only): skip those families' row-0 / quarter / full work as
    // if the host counts had proved it unneeded, so that the device check can be seen to catch it
    static const uint32_t test_skip = [] {
      const char* v = getenv("CG_TEST_SKIP_FAMILIES");
      return v ? (uint32_t)strtoul(v, nullptr, 0) & 7u : 0u;
    }();
    for (int f = 0; f < 3; ++f) {
      // serial key prep builds every table, so a test skip there would only mark good items NOT_RUN
      if (!serial && ((test_skip >> f) & 1u)) fork->pending.need_full[f] = false;
      if (!fork->pending.need_full[f]) skip_mask |= 1u << f;
    }
    fork->pending.skip_mask = skip_mask;
  }
  hipLaunchKernelGGL(k_key_classify, dim3((n_keys + 63) / 64), dim3(64), 0, stream, d_keys, n_keys, w.uses,
                     (const uint8_t*)w.seen, w.full, w.full_count, w.wide_idx, w.wide, w.wide_count, w.row0,
                     w.quart, w.cap_ed, w.cap_ec, w.min_ed, w.min_ec, skip_mask);
  if (!fork || serial) {
    if (fork) {  // the item stages still wait for these events
      fork->pending.on = false;
    }
    ed_launch_key_abyte(d_keys, n_keys, d_arena, arena_len, w, stream);
    for (int curve : {CG_CURVE_R1, CG_CURVE_K1}) {
      ec_launch_keyprep_chains(curve, d_keys, n_keys, d_arena, arena_len, w, stream, nullptr);
      ec_launch_keyprep_tabs(curve, d_keys, n_keys, w, stream, true, true);
    }
    ed_launch_keyprep_chains(d_keys, n_keys, d_arena, arena_len, w, stream);
    ed_launch_keyprep_tabs(d_keys, n_keys, w, stream, true, true);
    if (fork) {
      hipError_t e = hipSuccess;
      for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipEventRecord(fork->ec_decoded[k], stream);
      for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventRecord(fork->ready[k], stream);
      if (e != hipSuccess) return e;
    }
    return hipGetLastError();
  }
  hipError_t e = hipEventRecord(fork->start, stream);
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipStreamWaitEvent(fork->side[k], fork->start, 0);
  if (e != hipSuccess) return e;
  // now: decodes and row-base chains (few waves, latency-bound)
  ec_launch_keyprep_chains(CG_CURVE_R1, d_keys, n_keys, d_arena, arena_len, w, fork->side[0], fork->ec_decoded[0]);
  ec_launch_keyprep_chains(CG_CURVE_K1, d_keys, n_keys, d_arena, arena_len, w, fork->side[1], fork->ec_decoded[1]);
  ed_launch_keyprep_chains(d_keys, n_keys, d_arena, arena_len, w, fork->side[2]);
  for (int k = 0; k < 3 && e == hipSuccess; ++k)
    if (fork->chains[k]) e = hipEventRecord(fork->chains[k], fork->side[k]);
  if (e != hipSuccess) return e;
  // the tables (the wide ones hold every SIMD for milliseconds), wide first, then full / row 0:
  // after the first chunk's plan sort when items follow (its decoupled look-back stalls behind
  // them), else now
  fork->pending.on = true;
  fork->pending.keys = d_keys;
  fork->pending.n_keys = n_keys;
  fork->pending.keyprep = d_keyprep;
  fork->pending.wide = counted && wide ? *wide : WidePool{};
  if (!counted) e = launch_pending_tabs(fork, stream);
  if (e != hipSuccess) return e;
  // the only key work on the main stream: Abyte for k_ed_hash (no decode)
  ed_launch_key_abyte(d_keys, n_keys, d_arena, arena_len, w, stream);
  return hipGetLastError();
}

hipError_t launch_items_plan(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                             uint8_t* d_status, const void* d_keyprep, void* d_item_ws, hipStream_t stream,
                             const Fork* fork, const WidePool* wide) {
  if (n_items == 0) return hipSuccess;
  const uint32_t B = 256;
  const uint64_t grid = (n_items + B - 1) / B;
  const KeyWs w = key_ws((void*)d_keyprep, n_keys, wide);
  const ItemWs iw = item_ws(d_item_ws, n_items);
  hipLaunchKernelGGL(k_misc_status, dim3((unsigned)grid), dim3(B), 0, stream, d_items, n_items, d_keys, n_keys,
                     d_status);
  // plan: items sorted by (scheme class, key) (plan_sort.hip)
  hipError_t e = hipSuccess;
  CG_TIME(fork, CG_STAGE_PLAN, stream,
          e = launch_plan(d_items, n_items, d_keys, n_keys, w, iw,
                          stream));
  return e;
}

hipError_t launch_items_front(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                              const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                              const void* d_keyprep, void* d_item_ws, hipStream_t stream, const uint8_t* d_msgs,
                              uint64_t msgs_len, const Fork* fork, const WidePool* wide, bool planned) {
  if (n_items == 0) return hipSuccess;
  const KeyWs w = key_ws((void*)d_keyprep, n_keys, wide);
  const ItemWs iw = item_ws(d_item_ws, n_items);
  hipError_t e = hipSuccess;
  if (!planned)
    e = launch_items_plan(d_keys, n_keys, d_items, n_items, d_status, d_keyprep, d_item_ws, stream, fork, wide);
  if (e == hipSuccess && fork) e = launch_pending_tabs(fork, stream);  // the first front starts the table builds
  if (e == hipSuccess && fork && fork->mid_front) e = (*fork->mid_front)();  // (the hook clears itself)
  if (e != hipSuccess) return e;
  // fronts: Ed25519 challenges (need only Abyte), ECDSA prep + s^-1 per curve (need the decoded key).
  // CG_EC_FRONT_SIDE: each curve's front on its side stream beside the challenge hashes (its
  // s^-1 batches leave ~1 wave per SIMD: latency-bound alone), joined before that curve's ladders.
  // The side stream waits for everything enqueued on `stream` so far: this chunk's plan, and the
  // ladders of the chunk two back, which read the item workspace this front writes.
  // Round 4 default (with CG_ED_FINISH_SIDE): 282 / 287 / 282 -> 299 / 298 / 302 M sigs/s over three
  // interleaved runs (profiles/r04/side); =0 keeps them on `stream`.
  static const bool ec_side = [] {
    const char* v = getenv("CG_EC_FRONT_SIDE");
    return !(v && v[0] == '0');
  }();
  if (fork && ec_side && fork->ec_front_go) {
    e = hipEventRecord(fork->ec_front_go, stream);
    for (int k = 0; k < 2 && e == hipSuccess; ++k) {
      const int curve = k == 0 ? CG_CURVE_R1 : CG_CURVE_K1;
      e = hipStreamWaitEvent(fork->side[k], fork->ec_front_go, 0);
      if (e != hipSuccess) break;
      CG_TIME(fork, k == 0 ? CG_STAGE_R1_FRONT : CG_STAGE_K1_FRONT, fork->side[k],
              ec_launch_front(curve, d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw,
                              fork->side[k]));
      e = hipEventRecord(fork->ec_front_done[k], fork->side[k]);
    }
    if (e != hipSuccess) return e;
    fork->pending.ec_front_side = true;
    CG_TIME(fork, CG_STAGE_ED_HASH, stream,
            ed_launch_front(d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw, stream));
    return hipGetLastError();
  }
  if (fork) fork->pending.ec_front_side = false;
  CG_TIME(fork, CG_STAGE_ED_HASH, stream,
          ed_launch_front(d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw, stream));
  if (fork) hipStreamWaitEvent(stream, fork->ec_decoded[0], 0);
  CG_TIME(fork, CG_STAGE_R1_FRONT, stream,
          ec_launch_front(CG_CURVE_R1, d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw,
                          stream));
  if (fork) hipStreamWaitEvent(stream, fork->ec_decoded[1], 0);
  CG_TIME(fork, CG_STAGE_K1_FRONT, stream,
          ec_launch_front(CG_CURVE_K1, d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw,
                          stream));
  return hipGetLastError();
}

hipError_t launch_items_back(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                             const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_status, const void* d_keyprep,
                             void* d_item_ws, const void* d_btab, hipStream_t stream, const Fork* fork,
                             const WidePool* wide) {
  if (n_items == 0) return hipSuccess;
  (void)d_keys;
  const KeyWs w = key_ws((void*)d_keyprep, n_keys, wide);
  const ItemWs iw = item_ws(d_item_ws, n_items);
  hipError_t e = hipSuccess;
  // row-0 ladders: on the side streams (after their tables) when forked, else first on `stream`.
  // The full-table ladders stay on `stream`: on a side stream (round 3, for a handful of items per
  // chunk) a persistent full-GPU grid there held every slot while the main stream's next fronts
  // waited (Zipf keys: 125 -> 56 M sigs/s, profiles/r03/v12 vs v9); the stray full-table launch it
  // was meant to hide is gone with the biased count estimate.
  if (fork) {
    e = hipEventRecord(fork->front, stream);
    for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipStreamWaitEvent(fork->side[k], fork->front, 0);
    if (e != hipSuccess) return e;
  }
  // (a family whose host counts prove it has no row-0 / quarter key launches none: launch_keyprep)
  const bool* nf = fork ? fork->pending.need_full : nullptr;
  if (!nf || nf[2])
    CG_TIME(fork, CG_STAGE_ED_LADDER_ROW0, fork ? fork->side[2] : stream,
            ed_launch_ladder(false, d_items, n_items, d_status, w, iw, d_btab, fork ? fork->side[2] : stream));
  if (!nf || nf[0])
    CG_TIME(fork, CG_STAGE_R1_LADDER_ROW0, fork ? fork->side[0] : stream,
            ec_launch_ladder(CG_CURVE_R1, false, d_items, n_items, d_status, w, iw, d_btab, fork ? fork->side[0] : stream));
  if (!nf || nf[1])
    CG_TIME(fork, CG_STAGE_K1_LADDER_ROW0, fork ? fork->side[1] : stream,
            ec_launch_ladder(CG_CURVE_K1, false, d_items, n_items, d_status, w, iw, d_btab, fork ? fork->side[1] : stream));
  if (fork) {
    for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventRecord(fork->row0[k], fork->side[k]);
    if (e != hipSuccess) return e;
  }
  // full-table ladders on `stream`, each after its tables; Ed25519 finish after both ladders
  // wide-table ladders right after their class's full-table one (same tables-ready event)
  if (fork) hipStreamWaitEvent(stream, fork->ready[2], 0);
  CG_TIME(fork, CG_STAGE_ED_LADDER, stream, ed_launch_ladder(true, d_items, n_items, d_status, w, iw, d_btab, stream));
  if (w.cap_ed)
    CG_TIME(fork, CG_STAGE_ED_LADDER_WIDE, stream, ed_launch_ladder_wide(d_items, n_items, d_status, w, iw, d_btab, stream));
  // CG_ED_FINISH_SIDE: the finish (16 items per lane share an inversion: ~1.6 waves per SIMD,
  // latency-bound) runs on side stream 2 after the row-0 ladders there, beside the ECDSA ladders on
  // this stream; the stream joins on it at the end of the back
  static const bool fin_side = [] {  // default on (CG_EC_FRONT_SIDE's note); =0: on `stream`
    const char* v = getenv("CG_ED_FINISH_SIDE");
    return !(v && v[0] == '0');
  }();
  if (fork && fin_side) {
    e = hipEventRecord(fork->front, stream);  // the Ed25519 ladders on this stream are enqueued
    if (e == hipSuccess) e = hipStreamWaitEvent(fork->side[2], fork->front, 0);
    if (e != hipSuccess) return e;
    CG_TIME(fork, CG_STAGE_ED_FINISH, fork->side[2],
            ed_launch_finish(d_items, n_items, d_arena, arena_len, d_status, iw, fork->side[2]));
    e = hipEventRecord(fork->row0[2], fork->side[2]);
    if (e != hipSuccess) return e;
  } else {
    if (fork) hipStreamWaitEvent(stream, fork->row0[2], 0);
    CG_TIME(fork, CG_STAGE_ED_FINISH, stream, ed_launch_finish(d_items, n_items, d_arena, arena_len, d_status, iw, stream));
  }
  // CG_EC_LADDER_SIDE (A/B, bit 0 secp256r1, bit 1 secp256k1): the curve's full-table and wide
  // ladders on its side stream (after its front and its row-0 ladders there) instead of after the
  // Ed25519 ladders on this stream, so the issue-bound ladders fill each other's tails
  static const uint32_t ec_side = [] {
    const char* v = getenv("CG_EC_LADDER_SIDE");
    return v ? (uint32_t)strtoul(v, nullptr, 10) & 3u : 0u;
  }();
  // CG_EC_WIDE_MERGED=1 (A/B): the two curves' wide ladders as one launch after both full-table
  // ladders (k_ec_ladder_wide2), timed as the r1 wide stage
  static const bool ec_merged = [] {
    const char* v = getenv("CG_EC_WIDE_MERGED");
    return v && v[0] == '1';
  }();
  const bool merged = ec_merged && !ec_side && w.cap_ec;
  for (int k = 0; k < 2; ++k) {
    const int curve = k == 0 ? CG_CURVE_R1 : CG_CURVE_K1;
    const bool side = fork && (ec_side >> k & 1u);
    const hipStream_t s = side ? fork->side[k] : stream;
    if (fork) hipStreamWaitEvent(s, fork->ready[k], 0);
    if (fork && fork->pending.ec_front_side) hipStreamWaitEvent(s, fork->ec_front_done[k], 0);
    CG_TIME(fork, k == 0 ? CG_STAGE_R1_LADDER : CG_STAGE_K1_LADDER, s,
            ec_launch_ladder(curve, true, d_items, n_items, d_status, w, iw, d_btab, s));
    if (w.cap_ec && !merged)
      CG_TIME(fork, k == 0 ? CG_STAGE_R1_LADDER_WIDE : CG_STAGE_K1_LADDER_WIDE, s,
              ec_launch_ladder_wide(curve, d_items, n_items, d_status, w, iw, d_btab, s));
    if (side) {  // the join below waits for this stream's last ladder
      e = hipEventRecord(fork->row0[k], s);
      if (e != hipSuccess) return e;
    }
  }
  if (merged)
    CG_TIME(fork, CG_STAGE_R1_LADDER_WIDE, stream,
            ec_launch_ladder_wide_merged(d_items, n_items, d_status, w, iw, d_btab, stream));
  if (fork) {
    if (fork->mark) hipEventRecord(fork->mark, stream);
    hipStreamWaitEvent(stream, fork->row0[0], 0);
    hipStreamWaitEvent(stream, fork->row0[1], 0);
    if (fin_side) hipStreamWaitEvent(stream, fork->row0[2], 0);
    if (fork->pending.skip_mask)  // after every ladder and the finish of this chunk
      hipLaunchKernelGGL(k_mode_guard, dim3(64), dim3(256), 0, stream, (const uint32_t*)iw.ranges,
                         (const uint32_t*)iw.perm, (const uint32_t*)w.full_count, fork->pending.skip_mask, d_status);
  }
  return hipGetLastError();
}

hipError_t launch_items(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                        const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                        const void* d_keyprep, void* d_item_ws, const void* d_btab, hipStream_t stream,
                        const uint8_t* d_msgs, uint64_t msgs_len, const Fork* fork, const WidePool* wide) {
  hipError_t e = launch_items_front(d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode, d_status, d_keyprep,
                                    d_item_ws, stream, d_msgs, msgs_len, fork, wide, false);
  if (e != hipSuccess) return e;
  return launch_items_back(d_keys, n_keys, d_items, n_items, d_arena, arena_len, d_status, d_keyprep, d_item_ws,
                           d_btab, stream, fork, wide);
}

hipError_t launch_verify(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                         const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                         void* d_keyprep, void* d_item_ws, const void* d_btab, hipStream_t stream,
                         const uint8_t* d_msgs, uint64_t msgs_len, const Fork* fork, const WidePool* wide) {
  if (n_items == 0) return hipSuccess;
  hipError_t e = launch_keyprep(d_keys, n_keys, d_arena, arena_len, d_keyprep, stream, fork, d_items, n_items, wide);
  if (e != hipSuccess) return e;
  return launch_items(d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode, d_status, d_keyprep, d_item_ws,
                      d_btab, stream, d_msgs, msgs_len, fork, wide);
}

// This build's entry points for the C ABI layer (engine.h EngineVariant; one per fixed-base radix).
static_assert(ED_WIDE_BW == EC_WIDE_GW, "one fixed-base radix per build (Makefile VARIANTS)");
const EngineVariant& variant() {
  static const EngineVariant v = {(uint32_t)ED_WIDE_BW, upload_constants, keyprep_bytes, wide_bytes, wide_slot_bytes,
                                  make_wide_pool, btab_bytes, btab_scratch_bytes, init_btab, item_ws_bytes,
                                  launch_keyprep, launch_key_tables, launch_items, launch_items_plan,
                                  launch_items_front, launch_items_back};
  return v;
}

}  // namespace cg
