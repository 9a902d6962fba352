// C ABI of the MI355X batch signature-verification engine (include/cordagpu.h).
//
// Thin host layer: argument checks, per-context device workspace, H2D/D2H for the
// host-buffer entry points, and kernel launches through engine.h. No CPU fallback: every
// verdict is computed by the HIP kernels; if the device is unusable the call fails with
// CG_ERR_DEVICE and the status bytes stay CG_NOT_RUN.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/cordagpu.h"
#include "engine.h"
#include "host_budget.h"
#include "host_pool.h"
#include "pool.h"
#include "table_budget.h"

// the other builds of the radix-dependent kernels (Makefile VARIANTS; engine.h EngineVariant)
namespace cg24 {
const cgt::EngineVariant& variant();
}
namespace cg22 {
const cgt::EngineVariant& variant();
}

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, const char* detail = "") {
  char buf[512];
  snprintf(buf, sizeof buf, fmt, detail);
  g_err = buf;
  return code;
}

int hip_fail(hipError_t e, const char* where) {
  char buf[512];
  snprintf(buf, sizeof buf, "%s: %s", where, hipGetErrorString(e));
  g_err = buf;
  return e == hipErrorOutOfMemory ? CG_ERR_NOMEM : CG_ERR_DEVICE;
}

#define HIP_TRY(expr, where)               \
  do {                                     \
    hipError_t _e = (expr);                \
    if (_e != hipSuccess) return hip_fail(_e, where); \
  } while (0)

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  hipError_t ensure(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    size_t want = bytes + bytes / 4 + 256;
    hipError_t e = hipMalloc(&p, want);
    if (e == hipSuccess) cap = want;
    return e;
  }
  // exactly `bytes` (no growth margin): for the multi-GB wide-table pools
  hipError_t ensure_exact(size_t bytes) {
    if (bytes <= cap) return hipSuccess;
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes);
    if (e == hipSuccess) cap = bytes;
    return e;
  }
  void release() {
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
  }
};

}  // namespace

struct cg_ctx {
  int device = 0;
  uint64_t chunk = CG_DEFAULT_CHUNK_ITEMS;  // items per verify chunk (cg_config.chunk_items)
  bool chunk_set = false;                   // the caller chose it (else the host tx-signature path pipelines finer)
  bool fault = false;                       // cg_pool_inject_fault drill: every call fails
  hipStream_t stream = nullptr;
  cg::Fork fork = {{nullptr, nullptr, nullptr}, nullptr, {nullptr, nullptr}, {nullptr, nullptr, nullptr}, nullptr,
                   {nullptr, nullptr, nullptr}, nullptr};
  std::mutex mu;
  DevBuf keyprep, itemws, keys, items, arena, status, aux0, aux1, aux2;
  // the constant fixed-base tables (B, both curves' G; 91 GB at radix 2^26, 25 GB at 2^24, 6.9 GB at
  // 2^22), shared by every context of this process on the device (acquire_tables / release_tables),
  // and the build of the radix-dependent kernels that reads them (table_budget.h picks it at cg_open)
  void* btab = nullptr;
  const cgt::EngineVariant* eng = nullptr;
  uint64_t tab_bytes = 0;
  DevBuf wide;  // wide-table pools (keyws.h), sized by the largest call's item count
  // wide slots this context may allocate: lowered when the device's free memory cannot hold the
  // pool a call asks for (another process or context on the device), so the call runs
  // with fewer hot keys on wide tables (full tables for the rest: slower, same verdicts) instead of
  // failing with CG_ERR_NOMEM
  uint32_t wide_max = cg::kKeyWideMax;
  // transaction pipeline: verify items, spliced messages, templates; host-entry staging
  DevBuf txitems, msgs, tmpls, h_txs, h_comps, h_sigs, h_ids, h_txst;
  DevBuf sig12ws;  // the 12-byte signature table's per-block stream offsets (launch_tx_sig12_range)
  // tear-offs: leaf-hash workspace
  DevBuf ftxws;
  // host-buffer verify: a copy stream and one event per pipeline chunk (H2D of chunk k+1 overlaps
  // the verify of chunk k); timing events for cg_stats
  hipStream_t copy = nullptr;
  // the tx-signature host path's second copy stream (chunk 0's bytes while the key-use counts are
  // sampled) and a pinned buffer for those counts (a pinned copy does not queue behind a pageable one)
  hipStream_t copy2 = nullptr;
  // the exact key-use count (many keys): per host thread a byte counter per key (a wrap to 0 logs
  // the key in ovf: +256), kept across calls so a call does not page-fault 16 fresh arrays in
  std::vector<std::vector<uint8_t>> cnt8;
  std::vector<std::vector<uint32_t>> ovf;
  // host threads for the host paths' scans (host_pool.h), started on the first large call and sized
  // by the budget (host_budget.h: cg_config.host_threads, CG_HOST_THREADS, or the CPU quota divided
  // by the contexts open in the process), re-sized when the budget changes
  std::unique_ptr<cg::HostPool> hpool;
  uint32_t host_req = 0;   // cg_config.host_threads
  uint32_t quota = 1;      // the process's CPUs at cg_open
  bool counted = false;    // included in g_live_ctx
  uint32_t* pin_counts = nullptr;
  size_t pin_counts_cap = 0;
  std::vector<hipEvent_t> seg;
  hipEvent_t tev[4] = {};
  std::vector<hipEvent_t> segt;  // CG_HOST_TRACE: timing events behind each chunk's copy
  std::vector<hipEvent_t> segtab;  // CG_SPLIT_COPY: chunk k's signature-table slice landed
  hipEvent_t backt[2] = {nullptr, nullptr};  // CG_HOST_TRACE: chunk 0's back enqueued / tables ready
  std::vector<hipEvent_t> fbt;  // CG_HOST_TRACE: per chunk, the main stream reaching its front / its back's end
  std::vector<double> fbh;      // host ms at which chunk k's front kernels were enqueued
  bool htrace = false;
  // the end of the last call's device work, whatever stream it ran on: the next call waits for it
  // before touching the shared workspace (async calls on different streams)
  hipEvent_t done = nullptr;
  bool done_rec = false;
  hipEvent_t bridge = nullptr;  // a caller stream's point of entry (stream_of)
  hipEvent_t fs[2] = {nullptr, nullptr};  // the device forms' front stream (launch_chunked)
  hipStream_t caller = nullptr; // the caller's stream the current device call is bridged from
  cg::StageTimer timer;  // used when opened with CG_FLAG_STAGE_TIMING
};

namespace {

// contexts open in this process (the default host budget divides the CPU quota among them)
std::atomic<unsigned> g_live_ctx{0};

// The builds of the radix-dependent kernels, largest tables first (table_budget.h).
const cgt::EngineVariant* const kVariants[] = {&cg::variant(), &cg24::variant(), &cg22::variant()};
constexpr int kNumVariants = 3;

std::vector<cgb::TableSet> table_sets() {
  std::vector<cgb::TableSet> v;
  for (const cgt::EngineVariant* e : kVariants) v.push_back({e->fixed_base_bits, (uint64_t)e->btab_bytes()});
  return v;
}

// The constant fixed-base tables, one copy per device per process: read-only after the build, so
// every context on the device (a cg_pool's slots, a test's second context) shares it instead of
// holding its own (keyws.h const_tab_bytes: Ed25519 B and both curves' G at the variant's radix).
struct SharedTables {
  int device;
  int variant;
  void* p;
  unsigned refs;
};
std::mutex g_tab_mu;
std::vector<SharedTables> g_tabs;

// Picks the tables for a context on `device` under `budget` (0: automatic) and builds or shares them:
// *out = the tables, *variant = the kernel build that reads them. Automatic: when the device cannot
// allocate the set the free memory suggested (another process took it meanwhile), the next smaller.
hipError_t acquire_tables(int device, hipStream_t s, uint64_t budget, void** out, int* variant) {
  std::lock_guard<std::mutex> g(g_tab_mu);
  const std::vector<cgb::TableSet> sets = table_sets();
  int held = -1;
  for (const SharedTables& t : g_tabs)
    if (t.device == device && (held < 0 || t.variant < held)) held = t.variant;
  size_t free_b = 0, total_b = 0;
  if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) free_b = 0;
  const int pick = cgb::pick_tables(sets.data(), kNumVariants, budget, free_b, held);
  if (pick < 0) return hipErrorInvalidValue;
  for (SharedTables& t : g_tabs)
    if (t.device == device && t.variant == pick) {
      ++t.refs;
      *out = t.p;
      *variant = pick;
      return hipSuccess;
    }
  hipError_t e = hipErrorOutOfMemory;
  for (int v = pick; v < kNumVariants; ++v) {
    if (budget && sets[v].bytes > budget) continue;
    void* p = nullptr;
    e = hipMalloc(&p, sets[v].bytes);
    if (e == hipSuccess) {  // built once over a temporary scratch, freed afterwards
      DevBuf scratch;
      e = scratch.ensure(kVariants[v]->btab_scratch_bytes());
      if (e == hipSuccess) e = kVariants[v]->upload_constants();
      if (e == hipSuccess) e = kVariants[v]->init_btab(p, scratch.p, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      scratch.release();
      if (e == hipSuccess) {
        g_tabs.push_back({device, v, p, 1u});
        *out = p;
        *variant = v;
        return hipSuccess;
      }
      hipFree(p);
    }
    (void)hipGetLastError();
    if (e != hipErrorOutOfMemory || budget) break;  // only the automatic choice steps down
  }
  return e;
}

void release_tables(int device, void* p) {
  std::lock_guard<std::mutex> g(g_tab_mu);
  for (size_t i = 0; i < g_tabs.size(); ++i)
    if (g_tabs[i].device == device && g_tabs[i].p == p) {
      if (--g_tabs[i].refs == 0) {
        hipSetDevice(device);
        hipFree(p);
        g_tabs.erase(g_tabs.begin() + (ptrdiff_t)i);
      }
      return;
    }
}

// The host threads a call of n items may use: 1 below 2^16 items, else the budget; the pool is
// (re)made to match, so nt parts run on nt threads.
unsigned host_threads_of(cg_ctx* c, uint64_t n) {
  if (n < (1u << 16)) return 1;
  const unsigned nt = cg::host_threads_for(c->host_req, cg::host_threads_env(), c->quota, g_live_ctx.load());
  if (nt <= 1) c->hpool.reset();  // a budget of one runs inline (host_par), not on an older, larger pool
  else if (!c->hpool || c->hpool->threads() != nt) c->hpool.reset(new cg::HostPool(nt - 1));
  return nt;
}

// fn(t) for t in [0, m) on the context's pool (or inline)
void host_par(cg_ctx* c, uint64_t m, const std::function<void(uint64_t)>& fn) {
  if (m > 1 && c->hpool) {
    c->hpool->run(m, fn);
  } else {
    for (uint64_t t = 0; t < m; ++t) fn(t);
  }
}

hipError_t order_in(cg_ctx* c, hipStream_t s) { return c->done_rec ? hipStreamWaitEvent(s, c->done, 0) : hipSuccess; }
hipError_t order_out(cg_ctx* c, hipStream_t s) {
  hipError_t e = hipEventRecord(c->done, s);
  if (e == hipSuccess) c->done_rec = true;
  if (e == hipSuccess && c->caller) e = hipStreamWaitEvent(c->caller, c->done, 0);  // the bridge back
  c->caller = nullptr;
  return e;
}
// The stream a device call runs on. A caller's stream is bridged to the context's own stream: HIP
// multiplexes streams onto GPU_MAX_HW_QUEUES (4) hardware queues in creation order, and a stream
// created elsewhere (torch's, the JVM's) can share an in-order queue with one of the side streams,
// whose milliseconds-long chains and table builds then run ahead of the call's main-stream kernels
// (round 6: the device-resident headline on torch's stream sat ~3.5 ms per step behind side stream
// 0's wide chain and rows, profiles/r06/bridge). The context's stream, created first, has a queue of
// its own; it waits for everything the caller enqueued before the call, and order_out makes the
// caller's stream wait for the call's end, so the call stays ordered on the caller's stream.
// CG_STREAM_BRIDGE=0: run on the caller's stream itself (A/B).
hipStream_t stream_of(cg_ctx* c, void* hip_stream) {
  static const bool bridge = [] {
    const char* v = getenv("CG_STREAM_BRIDGE");
    return !(v && v[0] == '0');
  }();
  c->caller = nullptr;
  if (!hip_stream || (hipStream_t)hip_stream == c->stream) return c->stream;
  if (!bridge || !c->bridge || hipEventRecord(c->bridge, (hipStream_t)hip_stream) != hipSuccess ||
      hipStreamWaitEvent(c->stream, c->bridge, 0) != hipSuccess)
    return (hipStream_t)hip_stream;
  c->caller = (hipStream_t)hip_stream;
  return c->stream;
}

// Equal chunks of at most c->chunk items.
uint64_t chunk_of(const cg_ctx* c, uint64_t n) {
  if (n <= c->chunk) return n ? n : 1;
  const uint64_t k = (n + c->chunk - 1) / c->chunk;
  return (n + k - 1) / k;
}

// Key and item workspace for n_keys keys and chunks of ws_items items, plus the wide-table pools
// for a call of call_items items (0: none). Growing them waits for the device (cg_reserve ahead
// of time avoids that).
// A call of more than one chunk gets two item workspaces (launch_chunked runs chunk k + 1's front
// before chunk k's back).
size_t item_half_bytes(const cg_ctx* c, uint64_t ws_items) { return (c->eng->item_ws_bytes(ws_items) + 255) & ~(size_t)255; }
hipError_t ensure_ws(cg_ctx* c, uint32_t n_keys, uint64_t ws_items, uint64_t call_items = 0) {
  // the wide pool is sized for the full slot cap (KEY_WIDE_MAX) whenever the device can hold it: a
  // cap lowered by an earlier call that met low free memory (another process on the device) is
  // raised again here once the memory is back, instead of staying low for the
  // context's life
  const uint32_t kmax = cg::kKeyWideMax;
  size_t wide = c->eng->wide_bytes(n_keys, call_items, kmax);
  const size_t items = item_half_bytes(c, ws_items) * (call_items > ws_items ? 2 : 1);
  if (c->keyprep.cap >= c->eng->keyprep_bytes(n_keys) && c->itemws.cap >= items && c->wide.cap >= wide) {
    c->wide_max = kmax;
    return hipSuccess;
  }
  uint32_t cap = kmax;
  if (wide > c->wide.cap) {  // cap the wide pool by the device's free memory (keeping 1 GiB spare)
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess) {
      const size_t need_other = (c->keyprep.cap >= c->eng->keyprep_bytes(n_keys) ? 0 : c->eng->keyprep_bytes(n_keys)) +
                                (c->itemws.cap >= items ? 0 : items);
      const size_t avail = free_b + c->wide.cap;  // the current pool is freed before the new one
      const size_t spare = (size_t)1 << 30;
      if (wide + need_other + spare > avail) {
        const size_t room = avail > need_other + spare ? avail - need_other - spare : 0;
        cap = (uint32_t)std::min<size_t>(room / c->eng->wide_slot_bytes(), kmax);
        wide = c->eng->wide_bytes(n_keys, call_items, cap);
      }
    }
  }
  c->wide_max = cap;
  if (c->keyprep.cap >= c->eng->keyprep_bytes(n_keys) && c->itemws.cap >= items && c->wide.cap >= wide)
    return hipSuccess;  // still short of memory: the pool the context has is the largest that fits
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = c->keyprep.ensure(c->eng->keyprep_bytes(n_keys));
  if (e == hipSuccess) e = c->itemws.ensure(items);
  if (e == hipSuccess) e = c->wide.ensure_exact(wide);
  return e;
}

// The wide pools a call may use: what ensure_ws reserved for it (none if the buffer is short).
cg::WidePool wide_for(cg_ctx* c, uint32_t n_keys, uint64_t n_items) {
  static const bool off = [] {  // CG_NO_WIDE_TABLES=1: never build wide tables (A/B runs)
    const char* v = getenv("CG_NO_WIDE_TABLES");
    return v && v[0] == '1';
  }();
  if (off || c->wide.cap < c->eng->wide_bytes(n_keys, n_items, c->wide_max)) return cg::WidePool{};
  cg::WidePool p = c->eng->make_wide_pool(c->wide.p, n_keys, n_items, c->wide_max);
  static const uint32_t min_ed = [] {  // CG_WIDE_MIN_USES_ED / _EC: override the thresholds (A/B runs)
    const char* v = getenv("CG_WIDE_MIN_USES_ED");
    return v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
  }();
  static const uint32_t min_ec = [] {
    const char* v = getenv("CG_WIDE_MIN_USES_EC");
    return v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
  }();
  if (min_ed) p.min_ed = min_ed;
  if (min_ec) p.min_ec = min_ec;
  return p;
}

// Key tables once for the whole call (sized by every item's key use), then the items in chunks.
hipError_t launch_chunked(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                          const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status, hipStream_t s,
                          const uint8_t* d_msgs = nullptr, uint64_t msgs_len = 0,
                          const std::function<hipError_t(uint64_t, uint64_t, uint64_t)>* prepare = nullptr,
                          const cg::KeyUses* uses = nullptr, const std::vector<uint64_t>* bounds = nullptr,
                          bool prepare_blocks = false) {
  // prepare (the tx-signature entry points): called with (k, first item, items) just before chunk
  // k's front is enqueued; it makes chunk k's verify items (and, host form, its bytes) and orders
  // `s` after them. The key tables are then sized from `uses` and start building at once, before
  // any chunk is prepared (so they overlap the host copies).
  if (n_items == 0) return hipSuccess;
  const cg::WidePool wp = wide_for(c, n_keys, n_items);
  hipError_t e = c->eng->launch_keyprep(d_keys, n_keys, d_arena, arena_len, c->keyprep.p, s, &c->fork,
                                    uses ? nullptr : d_items, n_items, &wp, uses);
  // chunk k = items [at(k), at(k) + cnt(k)): the caller's bounds (bounds[0] = 0, bounds[nch] = n),
  // else equal chunks of chunk_of(c, n) items; `per` (the largest chunk) sizes the item workspaces
  uint64_t per = chunk_of(c, n_items);
  uint64_t nch = (n_items + per - 1) / per;
  if (bounds) {
    nch = bounds->size() - 1;
    per = 0;
    for (uint64_t k = 0; k < nch; ++k) per = std::max(per, (*bounds)[k + 1] - (*bounds)[k]);
  }
  auto at = [&](uint64_t k) { return bounds ? (*bounds)[k] : k * per; };
  auto cnt = [&](uint64_t k) {
    return bounds ? (*bounds)[k + 1] - (*bounds)[k] : (per < n_items - k * per ? per : n_items - k * per);
  };
  // chunk k's item workspace: half k % 2 when the buffer holds two (ensure_ws), else the one
  const bool two = nch > 1 && c->itemws.cap >= 2 * item_half_bytes(c, per);
  auto ws = [&](uint64_t k) { return (void*)((uint8_t*)c->itemws.p + (two ? (k & 1) * item_half_bytes(c, per) : 0)); };
  auto plan = [&](uint64_t k) {
    return c->eng->launch_items_plan(d_keys, n_keys, d_items + at(k), cnt(k), d_status + at(k), c->keyprep.p, ws(k), s,
                                 &c->fork, &wp);
  };
  const bool pre_plan = two && !prepare;
  // CG_DEV_PRE_PLAN=1 (A/B, the device tx-signature forms): both first chunks' items and plans before
  // the table builds, as pre_plan does for the batch forms, so that chunk 1's front is only its
  // hashes. Measured slower (388.3 vs 392.1 M sigs/s over 3 pairs, profiles/r06/preplan): chunk 0's
  // Ed25519 ladder then starts earlier but shares the chip with chunk 1's ECDSA fronts (12.5 vs
  // 11.9 ms of ladder per step); the chip is already full in phase 1.
  static const bool dev_pre_plan = [] {
    const char* v = getenv("CG_DEV_PRE_PLAN");
    return v && v[0] == '1';
  }();
  const bool pre_prep = two && prepare && !prepare_blocks && dev_pre_plan;
  double prep_ms = 0;  // CG_HOST_TRACE: the host's time in chunk k's prepare hook
  auto front = [&](uint64_t k) {
    if (prepare && !(pre_prep && k < 2)) {
      const auto p0 = std::chrono::steady_clock::now();
      const hipError_t w = (*prepare)(k, at(k), cnt(k));
      prep_ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - p0).count();
      if (w != hipSuccess) return w;
    }
    return c->eng->launch_items_front(d_keys, n_keys, d_items + at(k), cnt(k), d_arena, arena_len, mode, d_status + at(k),
                                  c->keyprep.p, ws(k), s, d_msgs, msgs_len, &c->fork, &wp, (pre_plan || pre_prep) && k < 2);
  };
  // chunk k + 1's front (plan, hashes, ECDSA prep) before chunk k's back (ladders): the first
  // chunk's wait for the key tables is spent on the next chunk's fronts. Without a prepare hook the
  // first two plans sort before the table builds start (their look-back stalls behind the builds);
  // with one, the builds start first: they overlap the preparation of the first chunk.
  if (e == hipSuccess && pre_plan) e = plan(0);
  if (e == hipSuccess && pre_plan) e = plan(1);
  for (uint64_t k = 0; k < 2 && pre_prep && e == hipSuccess; ++k) {
    e = (*prepare)(k, at(k), cnt(k));
    if (e == hipSuccess) e = plan(k);
  }
  // The host forms start the table builds now, so that they overlap the first chunk's copies. The
  // device forms have no copy to hide: their builds start after the first chunk's plan
  // (launch_items_front), whose onesweep look-back otherwise stalls behind the builds (round 6,
  // device-resident headline: the first plan's last pass 0.2 -> 2.7 ms in some steps,
  // profiles/r06/bridge timeline). CG_DEV_TABS_FIRST=1: start them now in the device forms too (A/B).
  static const bool dev_tabs_first = [] {
    const char* v = getenv("CG_DEV_TABS_FIRST");
    return v && v[0] == '1';
  }();
  if (e == hipSuccess && prepare && (prepare_blocks || dev_tabs_first)) e = c->eng->launch_key_tables(&c->fork, s);
  // CG_FRONT_AFTER_TABLES=1 (A/B): the first chunk's front waits for every key table, instead of
  // sharing the chip with the builds (both run at about half speed together:
  // profiles/r03/env_chains timelines)
  static const bool after_tables = [] {
    const char* v = getenv("CG_FRONT_AFTER_TABLES");
    return v && v[0] == '1';
  }();
  if (e == hipSuccess && prepare && after_tables)
    for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipStreamWaitEvent(s, c->fork.ready[k], 0);
  auto back = [&](uint64_t k) {
    if (k == 0 && c->htrace && c->backt[0]) {  // chunk 0's front done; every table family built
      hipEventRecord(c->backt[0], s);
      hipStream_t t = c->copy2;  // idle by now: the marker waits there, nothing else does
      for (int q = 0; q < 3; ++q) hipStreamWaitEvent(t, c->fork.ready[q], 0);
      hipEventRecord(c->backt[1], t);
    }
    c->fork.mark = c->htrace && 3 * k + 2 < c->fbt.size() ? c->fbt[3 * k + 2] : nullptr;  // before the joins
    const hipError_t r = c->eng->launch_items_back(d_keys, n_keys, d_items + at(k), cnt(k), d_arena, arena_len,
                                               d_status + at(k), c->keyprep.p, ws(k), c->btab, s, &c->fork, &wp);
    c->fork.mark = nullptr;
    if (c->htrace && 3 * k + 1 < c->fbt.size()) hipEventRecord(c->fbt[3 * k + 1], s);  // back k ends
    return r;
  };
  if (prepare_blocks) {
    // host copies in the prepare hook block the enqueuing thread: chunk k's back goes in before
    // chunk k + 1's copy, so the device runs chunk k's ladders during it (with chunk k + 1's front
    // first, chunk k's ladders waited for chunk k + 1's copy: profiles/r03/v5 timeline)
    // (a front stream of its own, chunk k + 1's front beside chunk k's back, measured neutral twice:
    // +1% in round 4, 315.4 -> 314.1 M sigs/s with the host pool, profiles/r04/fstr; removed in round 5)
    for (uint64_t k = 0; k < nch && e == hipSuccess; ++k) {
      const auto h0 = std::chrono::steady_clock::now();
      e = front(k);
      const auto h1 = std::chrono::steady_clock::now();
      if (e == hipSuccess) e = back(k);
      if (c->htrace)  // CG_HOST_TRACE: the host's time to enqueue chunk k (its front includes the copies)
        fprintf(stderr, "[cg host] chunk %llu enqueue: front %.3f ms (prepare %.3f, with the copies), back %.3f ms\n",
                (unsigned long long)k, std::chrono::duration<double, std::milli>(h1 - h0).count(), prep_ms,
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - h1).count());
    }
    return e;
  }
  // CG_DEV_FRONT_STREAM=1 (A/B, a two-chunk device tx-signature call): chunk 1's items and plan on the
  // caller's stream right after chunk 0's front, its hashes and ECDSA fronts on a stream of their own
  // (copy2: a hardware queue of its own, idle in the device forms), so that chunk 0's ladders start
  // as soon as the key tables are built instead of after chunk 1's hashes; chunk 1's ladders wait for
  // that front stream. Measured +0.9% (391.2 -> 394.6 M sigs/s, 3 of 3 pairs, profiles/r06/fstream), but
  // chunk 0's Ed25519 ladder then shares the chip with chunk 1's hashes (12.1 -> 13.3-13.9 ms of ladder
  // per step), so its launch time no longer measures the kernel: off by default
  static const bool dev_front_stream = [] {
    const char* v = getenv("CG_DEV_FRONT_STREAM");
    return v && v[0] == '1';
  }();
  if (e == hipSuccess && dev_front_stream && two && nch == 2 && prepare && !prepare_blocks && !pre_prep && c->copy2 &&
      c->fs[0] && c->fs[1]) {
    hipStream_t fs = c->copy2;
    e = front(0);
    if (e == hipSuccess) e = (*prepare)(1, at(1), cnt(1));
    if (e == hipSuccess) e = plan(1);
    if (e == hipSuccess) e = hipEventRecord(c->fs[0], s);
    if (e == hipSuccess) e = hipStreamWaitEvent(fs, c->fs[0], 0);
    if (e == hipSuccess)
      e = c->eng->launch_items_front(d_keys, n_keys, d_items + at(1), cnt(1), d_arena, arena_len, mode,
                                     d_status + at(1), c->keyprep.p, ws(1), fs, d_msgs, msgs_len, &c->fork, &wp, true);
    if (e == hipSuccess) e = hipEventRecord(c->fs[1], fs);
    if (e == hipSuccess) e = back(0);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, c->fs[1], 0);
    if (e == hipSuccess) e = back(1);
    return e;
  }
  if (e == hipSuccess) e = front(0);
  for (uint64_t k = 0; k < nch && e == hipSuccess; ++k) {
    if (!two && k > 0) e = front(k);
    if (two && k + 1 < nch && e == hipSuccess) e = front(k + 1);
    if (e == hipSuccess) e = back(k);
  }
  return e;
}

// ---- host-buffer verify: which arena bytes each pipeline chunk needs
struct Extent {
  uint64_t lo = UINT64_MAX, hi = 0;
  void add(uint64_t off, uint64_t len, uint64_t arena_len) {
    if (off > arena_len) return;  // outside the arena: the kernels never read it (CG_NOT_RUN)
    const uint64_t e = len > arena_len - off ? arena_len : off + len;
    if (off < lo) lo = off;
    if (e > hi) hi = e;
  }
  void merge(const Extent& o) {
    if (o.lo < lo) lo = o.lo;
    if (o.hi > hi) hi = o.hi;
  }
  bool empty() const { return lo >= hi; }
};

struct HostPlan {
  std::vector<uint64_t> first;  // chunk k = items [first[k], first[k+1])
  std::vector<Extent> ext;      // arena bytes chunk k reads
  Extent keys, win;             // key bytes; everything the call reads
};

void plan_host(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items,
               uint64_t arena_len, uint64_t per, HostPlan& P) {
  for (uint32_t k = 0; k < n_keys; ++k) P.keys.add(keys[k].off, keys[k].len, arena_len);
  const uint64_t nch = (n_items + per - 1) / per;
  P.first.resize(nch + 1);
  for (uint64_t k = 0; k <= nch; ++k) P.first[k] = n_items * k / nch;
  P.ext.assign(nch, Extent());
  // the chunks' scans on the context's host pool (the budget's threads): 32 B read per item
  auto scan = [&](uint64_t k) {
    Extent x;  // thread-local until the end (neighbouring chunks' slots share cache lines)
    for (uint64_t i = P.first[k]; i < P.first[k + 1]; ++i) {
      x.add(items[i].sig_off, items[i].sig_len, arena_len);
      x.add(items[i].msg_off, items[i].msg_len, arena_len);
    }
    P.ext[k] = x;
  };
  host_threads_of(c, n_items);
  host_par(c, nch, scan);
  P.win = P.keys;
  for (const Extent& e : P.ext) P.win.merge(e);
  if (P.win.empty()) P.win.lo = P.win.hi = 0;
  P.win.lo &= ~(uint64_t)15;  // the device window starts 16-aligned (kernels load aligned words)
}

// Copies the parts of [e.lo, e.hi) not yet resident (`have`: sorted disjoint intervals).
hipError_t copy_missing(std::vector<std::pair<uint64_t, uint64_t>>& have, const Extent& e, const uint8_t* arena,
                        uint8_t* dwin, uint64_t win_lo, hipStream_t s) {
  if (e.empty()) return hipSuccess;
  uint64_t cur = e.lo;
  std::vector<std::pair<uint64_t, uint64_t>> gaps;
  for (const auto& h : have) {
    if (h.second <= cur) continue;
    if (h.first >= e.hi) break;
    if (h.first > cur) gaps.push_back({cur, h.first});
    cur = h.second > cur ? h.second : cur;
    if (cur >= e.hi) break;
  }
  if (cur < e.hi) gaps.push_back({cur, e.hi});
  for (const auto& g : gaps) {
    hipError_t r = hipMemcpyAsync(dwin + (g.first - win_lo), arena + g.first, g.second - g.first,
                                  hipMemcpyHostToDevice, s);
    if (r != hipSuccess) return r;
  }
  have.push_back({e.lo, e.hi});
  std::sort(have.begin(), have.end());
  std::vector<std::pair<uint64_t, uint64_t>> m;
  for (const auto& h : have) {
    if (!m.empty() && h.first <= m.back().second) m.back().second = std::max(m.back().second, h.second);
    else m.push_back(h);
  }
  have.swap(m);
  return hipSuccess;
}

// cg_verify_batch with the ctx lock held. On failure the status bytes are CG_NOT_RUN.
int verify_host_locked(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items,
                       const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out, cg_stats* stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (c->fault) return fail(CG_ERR_DEVICE, "cg_verify_batch: device fault (injected by cg_pool_inject_fault)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  const uint64_t pipe = c->chunk < CG_PIPELINE_CHUNK_ITEMS ? c->chunk : CG_PIPELINE_CHUNK_ITEMS;
  HostPlan P;
  plan_host(c, keys, n_keys, items, n_items, arena_len, pipe, P);
  const uint64_t nch = P.ext.size();
  const uint64_t per_max = (n_items + nch - 1) / nch;
  HIP_TRY(c->keys.ensure(sizeof(cg_key) * (n_keys ? n_keys : 1)), "hipMalloc(keys)");
  HIP_TRY(c->items.ensure(sizeof(cg_item) * n_items), "hipMalloc(items)");
  HIP_TRY(c->arena.ensure((P.win.hi - P.win.lo) + 16), "hipMalloc(arena window)");
  HIP_TRY(c->status.ensure(n_items), "hipMalloc(status)");
  HIP_TRY(ensure_ws(c, n_keys, per_max, n_items), "hipMalloc(workspace)");
  while (c->seg.size() < nch) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    c->seg.push_back(e);
  }
  hipStream_t s = c->stream;
  uint8_t* dwin = (uint8_t*)c->arena.p;
  // the kernels index the arena by absolute offsets: hand them the window's base shifted back
  const uint8_t* dbase = dwin - P.win.lo;
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(hipEventRecord(c->tev[0], s), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(c->copy, c->tev[0], 0), "hipStreamWaitEvent");
  std::vector<std::pair<uint64_t, uint64_t>> have;
  if (n_keys)
    HIP_TRY(hipMemcpyAsync(c->keys.p, keys, sizeof(cg_key) * n_keys, hipMemcpyHostToDevice, c->copy), "H2D keys");
  HIP_TRY(copy_missing(have, P.keys, arena, dwin, P.win.lo, c->copy), "H2D key bytes");
  HIP_TRY(hipMemcpyAsync(c->items.p, items, sizeof(cg_item) * n_items, hipMemcpyHostToDevice, c->copy), "H2D items");
  // key tables sized by every item's key, built while chunk 0's arena bytes copy
  HIP_TRY(hipEventRecord(c->seg[0], c->copy), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(s, c->seg[0], 0), "hipStreamWaitEvent");
  const cg_key* dk = (const cg_key*)c->keys.p;
  const cg_item* di = (const cg_item*)c->items.p;
  uint8_t* ds = (uint8_t*)c->status.p;
  const cg::WidePool wp = wide_for(c, n_keys, n_items);
  HIP_TRY(c->eng->launch_keyprep(dk, n_keys, dbase, arena_len, c->keyprep.p, s, &c->fork, di, n_items, &wp, nullptr),
          "launch_keyprep");
  for (uint64_t k = 0; k < nch; ++k) {
    HIP_TRY(copy_missing(have, P.ext[k], arena, dwin, P.win.lo, c->copy), "H2D arena");
    HIP_TRY(hipEventRecord(c->seg[k], c->copy), "hipEventRecord");
    HIP_TRY(hipStreamWaitEvent(s, c->seg[k], 0), "hipStreamWaitEvent");
    if (k == 0) HIP_TRY(hipEventRecord(c->tev[1], s), "hipEventRecord");
    const uint64_t f = P.first[k], cnt = P.first[k + 1] - f;
    HIP_TRY(c->eng->launch_items(dk, n_keys, di + f, cnt, dbase, arena_len, mode, ds + f, c->keyprep.p, c->itemws.p,
                             c->btab, s, nullptr, 0, &c->fork, &wp), "launch_items");
  }
  HIP_TRY(hipEventRecord(c->tev[2], s), "hipEventRecord");
  HIP_TRY(hipMemcpyAsync(status_out, ds, n_items, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipEventRecord(c->tev[3], s), "hipEventRecord");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (stats) {
    float a = 0, b = 0, d = 0;
    hipEventElapsedTime(&a, c->tev[0], c->tev[1]);
    hipEventElapsedTime(&b, c->tev[1], c->tev[2]);
    hipEventElapsedTime(&d, c->tev[2], c->tev[3]);
    stats->n_items = n_items;
    stats->n_keys = n_keys;
    stats->ms_h2d = a;
    stats->ms_key_prep = 0;
    stats->ms_verify = b;
    stats->ms_d2h = d;
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return CG_OK;
}

}  // namespace

extern "C" {

int cg_abi_version(void) { return CG_ABI_VERSION; }

const char* cg_build_info(void) {
  return "corda_amd libcordagpu: HIP kernels for gfx950 (Ed25519 i2p-0.2.0 semantics, ECDSA BC-1.57 semantics, "
         "SHA-256/512, Merkle tx ids)";
}

int cg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* cg_last_error(void) { return g_err.c_str(); }

// ---- host memory registration (include/cordagpu.h: zero-copy ingestion)
namespace {
struct HostRange {
  uint64_t lo, hi;
};
std::mutex g_reg_mu;
std::vector<HostRange> g_reg;  // registered ranges, disjoint
}  // namespace

int cg_host_register(const void* p, uint64_t len) {
  if (!p || !len) return fail(CG_ERR_ARG, "cg_host_register: NULL pointer or empty range");
  const uint64_t lo = (uint64_t)(uintptr_t)p, hi = lo + len;
  if (hi < lo) return fail(CG_ERR_ARG, "cg_host_register: range wraps the address space");
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (const HostRange& r : g_reg)
    if (lo < r.hi && r.lo < hi) return fail(CG_ERR_ARG, "cg_host_register: range overlaps a registered one");
  // portable: every device's DMA engines may read the pages (a cg_pool's slots, one process per node)
  HIP_TRY(hipHostRegister(const_cast<void*>(p), (size_t)len, hipHostRegisterPortable), "hipHostRegister");
  g_reg.push_back({lo, hi});
  return CG_OK;
}

int cg_host_unregister(const void* p) {
  const uint64_t lo = (uint64_t)(uintptr_t)p;
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (size_t i = 0; i < g_reg.size(); ++i) {
    if (g_reg[i].lo != lo) continue;
    g_reg.erase(g_reg.begin() + (ptrdiff_t)i);
    HIP_TRY(hipHostUnregister(const_cast<void*>(p)), "hipHostUnregister");
    return CG_OK;
  }
  return fail(CG_ERR_ARG, "cg_host_unregister: pointer was not registered");
}

int cg_host_register_advised(uint32_t contexts_per_node) { return cg::host_register_advised(contexts_per_node) ? 1 : 0; }

int cg_host_registered(const void* p, uint64_t len) {
  const uint64_t lo = (uint64_t)(uintptr_t)p, hi = lo + len;
  std::lock_guard<std::mutex> g(g_reg_mu);
  for (const HostRange& r : g_reg)
    if (lo >= r.lo && hi <= r.hi && hi >= lo) return 1;
  return 0;
}

static_assert(sizeof(cg_config) == 56, "cg_config is 56 bytes in ABI v2");
static_assert(sizeof(cg_item) == 32 && sizeof(cg_key) == 16 && sizeof(cg_txsig) == 24 && sizeof(cg_txsig_packed) == 12,
              "ABI struct sizes");

int cg_open(cg_ctx** out, const cg_config* cfg) {
  if (!out) return fail(CG_ERR_ARG, "cg_open: out is NULL");
  *out = nullptr;
  if (cfg && (cfg->reserved0 || cfg->reserved1))
    return fail(CG_ERR_ARG, "cg_open: cg_config.reserved must be 0 (ABI v2: 56-byte cg_config)");
  const uint64_t tab_budget = cfg && cfg->table_bytes_max ? cfg->table_bytes_max
                                                          : cgb::table_bytes_env(getenv("CG_TABLE_BYTES_MAX"));
  if (tab_budget && tab_budget < table_sets().back().bytes) {
    char m[160];
    snprintf(m, sizeof m, "cg_open: table_bytes_max %llu is below the smallest fixed-base tables (%llu bytes, radix 2^%u)",
             (unsigned long long)tab_budget, (unsigned long long)table_sets().back().bytes, table_sets().back().bits);
    return fail(CG_ERR_ARG, "%s", m);
  }
  if (cfg && (cfg->flags & ~CG_FLAG_STAGE_TIMING)) return fail(CG_ERR_ARG, "cg_open: unknown cg_config.flags bits");
  int dev = cfg ? cfg->device : 0;
  int n = 0;
  HIP_TRY(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (dev < 0 || dev >= n) return fail(CG_ERR_ARG, "cg_open: device ordinal out of range");
  HIP_TRY(hipSetDevice(dev), "hipSetDevice");
  hipDeviceProp_t prop;
  HIP_TRY(hipGetDeviceProperties(&prop, dev), "hipGetDeviceProperties");
  if (strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    return fail(CG_ERR_DEVICE, "cg_open: kernels are built for gfx950, device is %s", prop.gcnArchName);
  cg_ctx* c = new cg_ctx();
  c->device = dev;
  c->host_req = cfg ? cfg->host_threads : 0u;
  c->quota = cg::cpu_quota();
  if (cfg && cfg->chunk_items) {
    c->chunk = cfg->chunk_items;
    c->chunk_set = true;
  }
  if (cfg && (cfg->flags & CG_FLAG_STAGE_TIMING)) c->fork.timer = &c->timer;
  // CG_STREAM_PRIORITY=1 (A/B): the context's stream at the device's highest priority, so its
  // blocks (the plan sort's decoupled look-back above all) dispatch ahead of the side streams'
  // table builds
  static const bool prio = [] {
    const char* v = getenv("CG_STREAM_PRIORITY");
    return v && v[0] == '1';
  }();
  int lo_pri = 0, hi_pri = 0;
  hipError_t e = hipSuccess;
  if (prio && hipDeviceGetStreamPriorityRange(&lo_pri, &hi_pri) == hipSuccess)
    e = hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, hi_pri);
  else
    e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete c;
    return hip_fail(e, "hipStreamCreate");
  }
  // Side streams: plain, created right after the context's stream. HIP multiplexes plain streams
  // onto GPU_MAX_HW_QUEUES (4) hardware queues in creation order, so the context's stream (the one a
  // caller gets with hip_stream = NULL) and the three side streams sit on four distinct queues;
  // a caller stream created elsewhere may share one with a side stream, whose latency-bound table
  // chain (milliseconds) then runs ahead of that caller's hashes (profiles/r02/wide_v2).
  // CG_MASKED_SIDE_STREAMS=1: side streams with an all-CU mask, which HIP backs with queues of
  // their own; measured slower (their chains and tables take CU share from the plan sort and the
  // hashes: gpurun_out/ab_mask), kept for A/B runs.
  {
    hipDeviceProp_t prop;
    const char* mk = getenv("CG_MASKED_SIDE_STREAMS");
    const bool masked = mk && mk[0] == '1' && hipGetDeviceProperties(&prop, c->device) == hipSuccess &&
                        prop.multiProcessorCount > 0;
    std::vector<uint32_t> mask(masked ? (prop.multiProcessorCount + 31) / 32 : 0, 0u);
    for (int cu = 0; masked && cu < prop.multiProcessorCount; ++cu) mask[cu / 32] |= 1u << (cu % 32);
    for (int k = 0; k < 3 && e == hipSuccess; ++k) {
      e = masked ? hipExtStreamCreateWithCUMask(&c->fork.side[k], (uint32_t)mask.size(), mask.data())
                 : hipStreamCreateWithFlags(&c->fork.side[k], hipStreamNonBlocking);
    }
  }
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.start, hipEventDisableTiming);
  for (int k = 0; k < 2 && e == hipSuccess; ++k)
    e = hipEventCreateWithFlags(&c->fork.ec_decoded[k], hipEventDisableTiming);
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->fork.ready[k], hipEventDisableTiming);
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->fork.row0[k], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.front, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.planned, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.ed_tabs, hipEventDisableTiming);
  for (int k = 0; k < 3 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->fork.chains[k], hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->fork.ec_front_go, hipEventDisableTiming);
  for (int k = 0; k < 2 && e == hipSuccess; ++k)
    e = hipEventCreateWithFlags(&c->fork.ec_front_done[k], hipEventDisableTiming);
  // The copy streams on hardware queues of their own (an all-CU mask makes HIP back a stream with a
  // dedicated queue): multiplexed onto the four default queues, the copy stream shared one with a
  // side stream, and the first chunk's bytes landed only after that stream's table builds (the
  // chunk's fronts started right after k_ed_keyprep_tab in every timeline; with
  // GPU_MAX_HW_QUEUES=8 they started 3 ms earlier: profiles/r03/env_hwq). CG_COPY_QUEUE_SHARED=1:
  // plain streams (A/B).
  {
    hipDeviceProp_t prop;
    const char* sh = getenv("CG_COPY_QUEUE_SHARED");
    const bool own = !(sh && sh[0] == '1') && hipGetDeviceProperties(&prop, c->device) == hipSuccess &&
                     prop.multiProcessorCount > 0;
    std::vector<uint32_t> mask(own ? (prop.multiProcessorCount + 31) / 32 : 0, 0u);
    for (int cu = 0; own && cu < prop.multiProcessorCount; ++cu) mask[cu / 32] |= 1u << (cu % 32);
    for (hipStream_t* cs : {&c->copy, &c->copy2})
      if (e == hipSuccess)
        e = own ? hipExtStreamCreateWithCUMask(cs, (uint32_t)mask.size(), mask.data())
                : hipStreamCreateWithFlags(cs, hipStreamNonBlocking);
  }
  for (int k = 0; k < 4 && e == hipSuccess; ++k) e = hipEventCreate(&c->tev[k]);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done, hipEventDisableTiming);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->bridge, hipEventDisableTiming);
  for (int k = 0; k < 2 && e == hipSuccess; ++k) e = hipEventCreateWithFlags(&c->fs[k], hipEventDisableTiming);
  int var = 0;
  if (e == hipSuccess) e = acquire_tables(c->device, c->stream, tab_budget, &c->btab, &var);
  if (e == hipSuccess) {
    c->eng = kVariants[var];
    c->tab_bytes = c->eng->btab_bytes();
    e = c->eng->upload_constants();  // per device: a table set built for another device uploaded there
  }
  if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  if (e != hipSuccess) {
    const int rc = hip_fail(e, "side streams / upload_constants / fixed-base tables");
    cg_close(c);
    return rc;
  }
  c->counted = true;
  ++g_live_ctx;
  *out = c;
  return CG_OK;
}

void cg_close(cg_ctx* c) {
  if (!c) return;
  if (c->counted) --g_live_ctx;
  hipSetDevice(c->device);
  if (c->stream) hipStreamSynchronize(c->stream);
  c->keyprep.release();
  c->itemws.release();
  c->wide.release();
  if (c->btab) release_tables(c->device, c->btab);
  c->btab = nullptr;
  c->keys.release();
  c->items.release();
  c->arena.release();
  c->status.release();
  c->aux0.release();
  c->aux1.release();
  c->aux2.release();
  for (DevBuf* b : {&c->txitems, &c->msgs, &c->tmpls, &c->h_txs, &c->h_comps, &c->h_sigs, &c->h_ids, &c->h_txst,
                    &c->ftxws, &c->sig12ws})
    b->release();
  for (int k = 0; k < 3; ++k) {
    if (c->fork.side[k]) {
      hipStreamSynchronize(c->fork.side[k]);
      hipStreamDestroy(c->fork.side[k]);
    }
    if (c->fork.ready[k]) hipEventDestroy(c->fork.ready[k]);
    if (c->fork.row0[k]) hipEventDestroy(c->fork.row0[k]);
  }
  if (c->fork.start) hipEventDestroy(c->fork.start);
  if (c->fork.front) hipEventDestroy(c->fork.front);
  if (c->fork.planned) hipEventDestroy(c->fork.planned);
  if (c->fork.ed_tabs) hipEventDestroy(c->fork.ed_tabs);
  for (int k = 0; k < 3; ++k)
    if (c->fork.chains[k]) hipEventDestroy(c->fork.chains[k]);
  if (c->fork.ec_front_go) hipEventDestroy(c->fork.ec_front_go);
  for (int k = 0; k < 2; ++k)
    if (c->fork.ec_front_done[k]) hipEventDestroy(c->fork.ec_front_done[k]);
  for (hipStream_t* cs : {&c->copy, &c->copy2})
    if (*cs) {
      hipStreamSynchronize(*cs);
      hipStreamDestroy(*cs);
    }
  for (hipEvent_t e : c->segt) hipEventDestroy(e);
  for (hipEvent_t e : c->segtab) hipEventDestroy(e);
  for (hipEvent_t e : c->fbt) hipEventDestroy(e);
  for (hipEvent_t e : c->backt)
    if (e) hipEventDestroy(e);
  if (c->pin_counts) hipHostFree(c->pin_counts);
  for (hipEvent_t e : c->seg) hipEventDestroy(e);
  for (int k = 0; k < 4; ++k)
    if (c->tev[k]) hipEventDestroy(c->tev[k]);
  if (c->done) hipEventDestroy(c->done);
  if (c->bridge) hipEventDestroy(c->bridge);
  for (hipEvent_t ev : c->fs)
    if (ev) hipEventDestroy(ev);
  for (auto* v : {&c->timer.recs, &c->timer.spare})
    for (auto& r : *v) {
      hipEventDestroy(r.a);
      hipEventDestroy(r.b);
    }
  for (int k = 0; k < 2; ++k)
    if (c->fork.ec_decoded[k]) hipEventDestroy(c->fork.ec_decoded[k]);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

uint64_t cg_table_bytes(uint32_t fixed_base_bits) {
  for (const cgb::TableSet& t : table_sets())
    if (t.bits == fixed_base_bits) return t.bytes;
  return 0;
}

uint32_t cg_table_choice(uint64_t table_bytes_max, uint64_t device_free) {
  const std::vector<cgb::TableSet> sets = table_sets();
  const int k = cgb::pick_tables(sets.data(), (int)sets.size(), table_bytes_max, device_free, -1);
  return k < 0 ? 0u : sets[k].bits;
}

int cg_context_info(const cg_ctx* c, cg_info* out) {
  if (!c || !out) return fail(CG_ERR_ARG, "cg_context_info: NULL argument");
  memset(out, 0, sizeof *out);
  out->device = c->device;
  out->fixed_base_bits = c->eng ? c->eng->fixed_base_bits : 0u;
  out->table_bytes = c->tab_bytes;
  out->host_threads = cg::host_threads_for(c->host_req, cg::host_threads_env(), c->quota, g_live_ctx.load());
  out->chunk_items = c->chunk;
  return CG_OK;
}

int cg_stage_times(cg_ctx* c, double* ms_out, uint32_t* launches_out, uint32_t n) {
  if (!c || (n && (!ms_out || !launches_out))) return fail(CG_ERR_ARG, "cg_stage_times: NULL argument");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  const uint32_t m = n < CG_STAGES ? n : CG_STAGES;
  for (uint32_t k = 0; k < m; ++k) {
    ms_out[k] = 0;
    launches_out[k] = 0;
  }
  int rc = CG_OK;
  for (auto& r : c->timer.recs) {
    float ms = 0;
    if (hipEventSynchronize(r.b) != hipSuccess || hipEventElapsedTime(&ms, r.a, r.b) != hipSuccess) rc = CG_ERR_DEVICE;
    if ((uint32_t)r.stage < m) {
      ms_out[r.stage] += ms;
      launches_out[r.stage] += 1;
    }
    c->timer.spare.push_back(r);
  }
  c->timer.recs.clear();
  return rc == CG_OK ? (int)m : fail(rc, "cg_stage_times: event wait failed");
}

int cg_reserve(cg_ctx* c, uint32_t max_keys, uint64_t max_items) {
  if (!c) return fail(CG_ERR_ARG, "cg_reserve: ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  HIP_TRY(ensure_ws(c, max_keys, chunk_of(c, max_items), max_items), "hipMalloc(workspace)");
  return CG_OK;
}

int cg_verify_batch_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items,
                           uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len, uint32_t mode,
                           uint8_t* d_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_batch_device: ctx is NULL");
  if (n_items && (!d_items || !d_status)) return fail(CG_ERR_ARG, "cg_verify_batch_device: NULL buffer");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_batch_device: bad mode");
  std::lock_guard<std::mutex> g(c->mu);
  if (c->fault) return fail(CG_ERR_DEVICE, "cg_verify_batch_device: device fault (injected)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  HIP_TRY(ensure_ws(c, n_keys, chunk_of(c, n_items), n_items), "hipMalloc(workspace)");
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(launch_chunked(c, d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode, d_status, s), "launch_verify");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_prepare_keys_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena,
                           uint64_t arena_len, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_prepare_keys_device: ctx is NULL");
  if (n_keys && !d_keys) return fail(CG_ERR_ARG, "cg_prepare_keys_device: keys is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->keyprep.cap < c->eng->keyprep_bytes(n_keys)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->keyprep.ensure(c->eng->keyprep_bytes(n_keys)), "hipMalloc(keyprep)");
  }
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(c->eng->launch_keyprep(d_keys, n_keys, d_arena, arena_len, c->keyprep.p, s, &c->fork, nullptr, 0, nullptr,
                                 nullptr),
          "launch_keyprep");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_verify_items_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items,
                           uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len, uint32_t mode,
                           uint8_t* d_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_items_device: ctx is NULL");
  if (n_items && (!d_items || !d_status)) return fail(CG_ERR_ARG, "cg_verify_items_device: NULL buffer");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_items_device: bad mode");
  std::lock_guard<std::mutex> g(c->mu);
  if (c->keyprep.cap < c->eng->keyprep_bytes(n_keys))
    return fail(CG_ERR_ARG, "cg_verify_items_device: keys were not prepared (call cg_prepare_keys_device)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  HIP_TRY(ensure_ws(c, n_keys, chunk_of(c, n_items)), "hipMalloc(item workspace)");
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  const uint64_t per = chunk_of(c, n_items);
  for (uint64_t f = 0; f < n_items; f += per) {
    const uint64_t cnt = per < n_items - f ? per : n_items - f;
    HIP_TRY(c->eng->launch_items(d_keys, n_keys, d_items + f, cnt, d_arena, arena_len, mode, d_status + f, c->keyprep.p,
                             c->itemws.p, c->btab, s, nullptr, 0, &c->fork, nullptr),
            "launch_items");
  }
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_verify_batch(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items,
                    const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out,
                    cg_stats* stats) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_batch: ctx is NULL");
  if (n_items && (!items || !status_out)) return fail(CG_ERR_ARG, "cg_verify_batch: NULL buffer");
  if (n_keys && !keys) return fail(CG_ERR_ARG, "cg_verify_batch: keys is NULL");
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_verify_batch: arena is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_batch: bad mode");
  if (n_items) memset(status_out, CG_NOT_RUN, n_items);
  if (n_items == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  const int rc = verify_host_locked(c, keys, n_keys, items, n_items, arena, arena_len, mode, status_out, stats);
  if (rc != CG_OK) memset(status_out, CG_NOT_RUN, n_items);
  return rc;
}

int cg_sha256_batch_device(cg_ctx* c, const cg_span* d_spans, uint64_t n, const uint8_t* d_arena,
                           uint64_t arena_len, uint8_t* d_digests, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_sha256_batch_device: ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(cg::launch_sha256(d_spans, n, d_arena, arena_len, d_digests, s), "launch_sha256");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

static int hash_batch(cg_ctx* c, const cg_span* spans, uint64_t n, const uint8_t* arena, uint64_t arena_len,
                      uint8_t* out, int which) {
  if (!c) return fail(CG_ERR_ARG, "hash batch: ctx is NULL");
  if (n && (!spans || !out)) return fail(CG_ERR_ARG, "hash batch: NULL buffer");
  if (n == 0) return CG_OK;
  const size_t dlen = which == 256 ? 32 : 64;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(c->items.ensure(sizeof(cg_span) * n), "hipMalloc(spans)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->aux0.ensure(dlen * n), "hipMalloc(digests)");
  HIP_TRY(hipMemcpyAsync(c->items.p, spans, sizeof(cg_span) * n, hipMemcpyHostToDevice, s), "H2D spans");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  if (which == 256)
    HIP_TRY(cg::launch_sha256((const cg_span*)c->items.p, n, (const uint8_t*)c->arena.p, arena_len,
                              (uint8_t*)c->aux0.p, s), "launch_sha256");
  else
    HIP_TRY(cg::launch_sha512((const cg_span*)c->items.p, n, (const uint8_t*)c->arena.p, arena_len,
                              (uint8_t*)c->aux0.p, s), "launch_sha512");
  HIP_TRY(hipMemcpyAsync(out, c->aux0.p, dlen * n, hipMemcpyDeviceToHost, s), "D2H digests");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

int cg_sha256_batch(cg_ctx* c, const cg_span* spans, uint64_t n, const uint8_t* arena, uint64_t arena_len,
                    uint8_t* out) {
  return hash_batch(c, spans, n, arena, arena_len, out, 256);
}
int cg_sha512_batch(cg_ctx* c, const cg_span* spans, uint64_t n, const uint8_t* arena, uint64_t arena_len,
                    uint8_t* out) {
  return hash_batch(c, spans, n, arena, arena_len, out, 512);
}

int cg_tx_ids_device(cg_ctx* c, const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps, uint64_t n_comps,
                     const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_ids, uint8_t* d_status,
                     void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_tx_ids_device: ctx is NULL");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->aux2.cap < cg::tx_ws_bytes(n_comps)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->aux2.ensure(cg::tx_ws_bytes(n_comps)), "hipMalloc(leaf ws)");
  }
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(cg::launch_tx_ids(d_txs, n_tx, d_comps, n_comps, d_arena, arena_len, d_ids, d_status,
                            (uint8_t*)c->aux2.p, s), "launch_tx_ids");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_tx_ids(cg_ctx* c, const cg_tx* txs, uint64_t n_tx, const cg_component* comps, uint64_t n_comps,
              const uint8_t* arena, uint64_t arena_len, uint8_t* ids_out, uint8_t* status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_tx_ids: ctx is NULL");
  if (n_tx && (!txs || !ids_out || !status_out)) return fail(CG_ERR_ARG, "cg_tx_ids: NULL buffer");
  if (n_tx == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(c->keys.ensure(sizeof(cg_tx) * n_tx), "hipMalloc(txs)");
  HIP_TRY(c->items.ensure(sizeof(cg_component) * (n_comps ? n_comps : 1)), "hipMalloc(comps)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->aux0.ensure(32 * n_tx), "hipMalloc(ids)");
  HIP_TRY(c->status.ensure(n_tx), "hipMalloc(status)");
  HIP_TRY(c->aux2.ensure(cg::tx_ws_bytes(n_comps)), "hipMalloc(leaf ws)");
  HIP_TRY(hipMemcpyAsync(c->keys.p, txs, sizeof(cg_tx) * n_tx, hipMemcpyHostToDevice, s), "H2D txs");
  if (n_comps)
    HIP_TRY(hipMemcpyAsync(c->items.p, comps, sizeof(cg_component) * n_comps, hipMemcpyHostToDevice, s), "H2D comps");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  HIP_TRY(cg::launch_tx_ids((const cg_tx*)c->keys.p, n_tx, (const cg_component*)c->items.p, n_comps,
                            (const uint8_t*)c->arena.p, arena_len, (uint8_t*)c->aux0.p, (uint8_t*)c->status.p,
                            (uint8_t*)c->aux2.p, s), "launch_tx_ids");
  HIP_TRY(hipMemcpyAsync(ids_out, c->aux0.p, 32 * n_tx, hipMemcpyDeviceToHost, s), "D2H ids");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n_tx, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

int cg_merkle_roots(cg_ctx* c, const uint8_t* leaves, const uint64_t* first, const uint32_t* count, uint64_t n,
                    uint8_t* roots_out, uint8_t* status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_merkle_roots: ctx is NULL");
  if (n && (!first || !count || !roots_out || !status_out)) return fail(CG_ERR_ARG, "cg_merkle_roots: NULL buffer");
  if (n == 0) return CG_OK;
  uint64_t total = 0, ws = 0;
  std::vector<uint64_t> wsoff(n);
  for (uint64_t j = 0; j < n; ++j) {
    if (first[j] + count[j] > total) total = first[j] + count[j];
    wsoff[j] = ws;
    ws += count[j];
  }
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(c->arena.ensure(32 * (total ? total : 1)), "hipMalloc(leaves)");
  HIP_TRY(c->keys.ensure(8 * n), "hipMalloc(first)");
  HIP_TRY(c->items.ensure(4 * n), "hipMalloc(count)");
  HIP_TRY(c->aux0.ensure(32 * n), "hipMalloc(roots)");
  HIP_TRY(c->status.ensure(n), "hipMalloc(status)");
  HIP_TRY(c->aux1.ensure(32 * (ws ? ws : 1)), "hipMalloc(ws)");
  HIP_TRY(c->aux2.ensure(8 * n), "hipMalloc(wsoff)");
  if (total) HIP_TRY(hipMemcpyAsync(c->arena.p, leaves, 32 * total, hipMemcpyHostToDevice, s), "H2D leaves");
  HIP_TRY(hipMemcpyAsync(c->keys.p, first, 8 * n, hipMemcpyHostToDevice, s), "H2D first");
  HIP_TRY(hipMemcpyAsync(c->items.p, count, 4 * n, hipMemcpyHostToDevice, s), "H2D count");
  HIP_TRY(hipMemcpyAsync(c->aux2.p, wsoff.data(), 8 * n, hipMemcpyHostToDevice, s), "H2D wsoff");
  HIP_TRY(cg::launch_merkle_roots((const uint8_t*)c->arena.p, (const uint64_t*)c->keys.p, (const uint32_t*)c->items.p,
                                  n, (uint8_t*)c->aux0.p, (uint8_t*)c->status.p, (uint8_t*)c->aux1.p,
                                  (const uint64_t*)c->aux2.p, s),
          "launch_merkle_roots");
  HIP_TRY(hipMemcpyAsync(roots_out, c->aux0.p, 32 * n, hipMemcpyDeviceToHost, s), "D2H roots");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

// cg_verify_transactions_device with the ctx lock held
static int verify_transactions_locked(cg_ctx* c, const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps,
                                      uint64_t n_comps, const cg_key* d_keys, uint32_t n_keys, const cg_txsig* d_sigs,
                                      uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                      const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_ids,
                                      uint8_t* d_tx_status, uint8_t* d_sig_status, hipStream_t s) {
  uint64_t maxlen = 0;
  for (uint32_t k = 0; k < n_tmpls; ++k) {
    const uint64_t l = (uint64_t)tmpls[k].prefix_len + 32u + tmpls[k].suffix_len;
    if (l > maxlen) maxlen = l;
  }
  uint64_t slot = (maxlen + 15) & ~(uint64_t)15;
  if (slot == 0) slot = 16;
  const uint64_t msgs_len = cg::tx_msgs_head(n_tmpls, slot);
  const size_t need_leaf = cg::tx_ws_bytes(n_comps), need_items = sizeof(cg_item) * (n_sigs ? n_sigs : 1),
               need_msgs = msgs_len ? msgs_len : 16, need_tmpl = sizeof(cg_signable_tmpl) * (n_tmpls ? n_tmpls : 1);
  if (c->aux2.cap < need_leaf || c->txitems.cap < need_items || c->msgs.cap < need_msgs ||
      c->tmpls.cap < need_tmpl) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->aux2.ensure(need_leaf), "hipMalloc(leaf ws)");
    HIP_TRY(c->txitems.ensure(need_items), "hipMalloc(tx items)");
    HIP_TRY(c->msgs.ensure(need_msgs), "hipMalloc(spliced messages)");
    HIP_TRY(c->tmpls.ensure(need_tmpl), "hipMalloc(templates)");
  }
  HIP_TRY(ensure_ws(c, n_keys, chunk_of(c, n_sigs), n_sigs), "hipMalloc(workspace)");
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  if (n_tmpls)
    HIP_TRY(hipMemcpyAsync(c->tmpls.p, tmpls, sizeof(cg_signable_tmpl) * n_tmpls, hipMemcpyHostToDevice, s),
            "H2D templates");
  HIP_TRY(cg::launch_tx_ids(d_txs, n_tx, d_comps, n_comps, d_arena, arena_len, d_ids, d_tx_status,
                            (uint8_t*)c->aux2.p, s), "launch_tx_ids");
  if (n_sigs) {
    HIP_TRY(cg::launch_tx_sig_items(d_sigs, n_sigs, (const cg_signable_tmpl*)c->tmpls.p, n_tmpls, d_tx_status, n_tx,
                                    d_ids, d_arena, arena_len, slot, (cg_item*)c->txitems.p, (uint8_t*)c->msgs.p, s),
            "launch_tx_sig_items");
    HIP_TRY(launch_chunked(c, d_keys, n_keys, (const cg_item*)c->txitems.p, n_sigs, d_arena, arena_len, mode,
                           d_sig_status, s, (const uint8_t*)c->msgs.p, msgs_len),
            "launch_verify");
  }
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_verify_transactions_device(cg_ctx* c, const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps,
                                  uint64_t n_comps, const cg_key* d_keys, uint32_t n_keys, const cg_txsig* d_sigs,
                                  uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                  const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_ids,
                                  uint8_t* d_tx_status, uint8_t* d_sig_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_transactions_device: ctx is NULL");
  if (n_tx && (!d_txs || !d_ids || !d_tx_status)) return fail(CG_ERR_ARG, "cg_verify_transactions_device: NULL tx buffer");
  if (n_sigs && (!d_sigs || !d_sig_status)) return fail(CG_ERR_ARG, "cg_verify_transactions_device: NULL sig buffer");
  if (n_tmpls && !tmpls) return fail(CG_ERR_ARG, "cg_verify_transactions_device: templates is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_transactions_device: bad mode");
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = stream_of(c, hip_stream);
  return verify_transactions_locked(c, d_txs, n_tx, d_comps, n_comps, d_keys, n_keys, d_sigs, n_sigs, tmpls, n_tmpls,
                                    d_arena, arena_len, mode, d_ids, d_tx_status, d_sig_status, s);
}

static int verify_transactions_host_locked(cg_ctx* c, const cg_tx* txs, uint64_t n_tx, const cg_component* comps,
                                           uint64_t n_comps, const cg_key* keys, uint32_t n_keys, const cg_txsig* sigs,
                                           uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                           const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* ids_out,
                                           uint8_t* tx_status_out, uint8_t* sig_status_out);

int cg_verify_transactions(cg_ctx* c, const cg_tx* txs, uint64_t n_tx, const cg_component* comps, uint64_t n_comps,
                           const cg_key* keys, uint32_t n_keys, const cg_txsig* sigs, uint64_t n_sigs,
                           const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* arena,
                           uint64_t arena_len, uint32_t mode, uint8_t* ids_out, uint8_t* tx_status_out,
                           uint8_t* sig_status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_transactions: ctx is NULL");
  if (n_tx && (!txs || !ids_out || !tx_status_out)) return fail(CG_ERR_ARG, "cg_verify_transactions: NULL tx buffer");
  if (n_sigs && (!sigs || !sig_status_out)) return fail(CG_ERR_ARG, "cg_verify_transactions: NULL sig buffer");
  if (n_comps && !comps) return fail(CG_ERR_ARG, "cg_verify_transactions: comps is NULL");
  if (n_keys && !keys) return fail(CG_ERR_ARG, "cg_verify_transactions: keys is NULL");
  if (n_tmpls && !tmpls) return fail(CG_ERR_ARG, "cg_verify_transactions: templates is NULL");
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_verify_transactions: arena is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_verify_transactions: bad mode");
  for (uint64_t i = 0; i < n_sigs; ++i) sig_status_out[i] = CG_NOT_RUN;
  if (n_tx == 0 && n_sigs == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  return verify_transactions_host_locked(c, txs, n_tx, comps, n_comps, keys, n_keys, sigs, n_sigs, tmpls, n_tmpls,
                                         arena, arena_len, mode, ids_out, tx_status_out, sig_status_out);
}

// cg_verify_transactions with the arguments checked and the ctx lock held (also a cg_pool slot's call)
static int verify_transactions_host_locked(cg_ctx* c, const cg_tx* txs, uint64_t n_tx, const cg_component* comps,
                                           uint64_t n_comps, const cg_key* keys, uint32_t n_keys, const cg_txsig* sigs,
                                           uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                           const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* ids_out,
                                           uint8_t* tx_status_out, uint8_t* sig_status_out) {
  if (c->fault) return fail(CG_ERR_DEVICE, "cg_verify_transactions: device fault (injected by cg_pool_inject_fault)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(c->h_txs.ensure(sizeof(cg_tx) * (n_tx ? n_tx : 1)), "hipMalloc(txs)");
  HIP_TRY(c->h_comps.ensure(sizeof(cg_component) * (n_comps ? n_comps : 1)), "hipMalloc(comps)");
  HIP_TRY(c->keys.ensure(sizeof(cg_key) * (n_keys ? n_keys : 1)), "hipMalloc(keys)");
  HIP_TRY(c->h_sigs.ensure(sizeof(cg_txsig) * (n_sigs ? n_sigs : 1)), "hipMalloc(sigs)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->h_ids.ensure(32 * (n_tx ? n_tx : 1)), "hipMalloc(ids)");
  HIP_TRY(c->h_txst.ensure(n_tx ? n_tx : 1), "hipMalloc(tx status)");
  HIP_TRY(c->status.ensure(n_sigs ? n_sigs : 1), "hipMalloc(sig status)");
  if (n_tx) HIP_TRY(hipMemcpyAsync(c->h_txs.p, txs, sizeof(cg_tx) * n_tx, hipMemcpyHostToDevice, s), "H2D txs");
  if (n_comps)
    HIP_TRY(hipMemcpyAsync(c->h_comps.p, comps, sizeof(cg_component) * n_comps, hipMemcpyHostToDevice, s),
            "H2D comps");
  if (n_keys) HIP_TRY(hipMemcpyAsync(c->keys.p, keys, sizeof(cg_key) * n_keys, hipMemcpyHostToDevice, s), "H2D keys");
  if (n_sigs)
    HIP_TRY(hipMemcpyAsync(c->h_sigs.p, sigs, sizeof(cg_txsig) * n_sigs, hipMemcpyHostToDevice, s), "H2D sigs");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  int rc = verify_transactions_locked(c, (const cg_tx*)c->h_txs.p, n_tx, (const cg_component*)c->h_comps.p, n_comps,
                                      (const cg_key*)c->keys.p, n_keys, (const cg_txsig*)c->h_sigs.p, n_sigs, tmpls,
                                      n_tmpls, (const uint8_t*)c->arena.p, arena_len, mode, (uint8_t*)c->h_ids.p,
                                      (uint8_t*)c->h_txst.p, (uint8_t*)c->status.p, s);
  if (rc != CG_OK) return rc;
  if (n_tx) {
    HIP_TRY(hipMemcpyAsync(ids_out, c->h_ids.p, 32 * n_tx, hipMemcpyDeviceToHost, s), "D2H ids");
    HIP_TRY(hipMemcpyAsync(tx_status_out, c->h_txst.p, n_tx, hipMemcpyDeviceToHost, s), "D2H tx status");
  }
  if (n_sigs) HIP_TRY(hipMemcpyAsync(sig_status_out, c->status.p, n_sigs, hipMemcpyDeviceToHost, s), "D2H sig status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

// ---------------------------------------------------------------- signatures over known tx ids
// the host tx-signature forms split a large call into at least this many chunks besides the smaller
// first one (CG_TXSIG_FIRST_DIV): round 6 A/B on the configs[4] shard, 1/6 + 4 / 1/6 + 3 / 1/6 + 2
// chunks = 345.4 / 351.3 / 334.7 M sigs/s over 3 rounds (profiles/r06/h2hchunks)
#define CG_TXSIG_MIN_CHUNKS 3u
#define CG_TXSIG_COUNT_SAMPLE 32u  // hot-key calls: 1 in 32 (blocks of 8 records): plan 3.0 -> 1.4-1.8 ms, 235 -> 237 / 247 M (profiles/r03/env_fd12)
#define CG_TXSIG_SAMPLE_BLOCK 8u
// The spliced-message slot of a template set: the longest prefix || id || suffix, 16-aligned.
static uint64_t tmpl_slot(const cg_signable_tmpl* tmpls, uint32_t n_tmpls) {
  uint64_t maxlen = 0;
  for (uint32_t k = 0; k < n_tmpls; ++k) {
    const uint64_t l = (uint64_t)tmpls[k].prefix_len + 32u + tmpls[k].suffix_len;
    if (l > maxlen) maxlen = l;
  }
  const uint64_t slot = (maxlen + 15) & ~(uint64_t)15;
  return slot ? slot : 16;
}

// Verify items, spliced messages and the template table of n_sigs signatures (waits for the device
// when a buffer grows).
static hipError_t ensure_txsig_ws(cg_ctx* c, uint64_t n_sigs, uint32_t n_tmpls, uint64_t slot) {
  const size_t need_items = sizeof(cg_item) * (n_sigs ? n_sigs : 1),
               need_msgs = cg::tx_msgs_head(n_tmpls, slot),
               need_tmpl = sizeof(cg_signable_tmpl) * (n_tmpls ? n_tmpls : 1);
  if (c->txitems.cap >= need_items && c->msgs.cap >= need_msgs && c->tmpls.cap >= need_tmpl) return hipSuccess;
  hipError_t e = hipDeviceSynchronize();
  if (e == hipSuccess) e = c->txitems.ensure(need_items);
  if (e == hipSuccess) e = c->msgs.ensure(need_msgs);
  if (e == hipSuccess) e = c->tmpls.ensure(need_tmpl);
  return e;
}

// Templates to the device (midstates + images), then the chunked verify: key tables sized from
// `uses` (sampled from the signature table on the device, or the host's exact counts), each chunk's
// verify items and spliced SignableData made just before its front (after `ready`, which the host
// form uses to land the chunk's signature table slice and bytes).
// The 12-byte table (cg_txsig_packed): d_sigs is null and `p12` says where the signatures sit: the
// stream at arena offset sig_region, chunk k's first signature at stream offset (*chunk_base)[k] (host
// form: the host sums the lengths as it scans each chunk) or every block's offset precomputed in
// d_bases (device form).
struct Packed12 {
  const cg_txsig_packed* d_sigs = nullptr;
  uint64_t sig_region = 0, sig_bytes_len = 0;
  const std::vector<uint64_t>* chunk_base = nullptr;
  const uint64_t* d_bases = nullptr;
};
static hipError_t launch_txsig(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_ids, uint64_t n_ids,
                               const cg_txsig* d_sigs, uint64_t n_sigs, const cg_signable_tmpl* tmpls,
                               uint32_t n_tmpls, const uint8_t* d_arena, uint64_t arena_len, uint32_t mode,
                               uint8_t* d_status, hipStream_t s, uint64_t slot, const cg::KeyUses& uses,
                               const std::function<hipError_t(uint64_t, uint64_t, uint64_t)>* ready,
                               const std::vector<uint64_t>* bounds = nullptr, const Packed12* p12 = nullptr) {
  if (n_sigs == 0) return hipSuccess;
  hipError_t e = hipSuccess;
  const cg_signable_tmpl* dt = (const cg_signable_tmpl*)c->tmpls.p;
  if (n_tmpls) e = hipMemcpyAsync(c->tmpls.p, tmpls, sizeof(cg_signable_tmpl) * n_tmpls, hipMemcpyHostToDevice, s);
  if (e == hipSuccess)
    e = cg::launch_tx_sig_templates(dt, n_tmpls, d_arena, arena_len, slot, d_ids, n_ids, (uint8_t*)c->msgs.p, s);
  const std::function<hipError_t(uint64_t, uint64_t, uint64_t)> prepare = [&](uint64_t k, uint64_t first,
                                                                               uint64_t cnt) {
    hipError_t r = ready ? (*ready)(k, first, cnt) : hipSuccess;
    if (r == hipSuccess && p12)
      r = cg::launch_tx_sig12_range(p12->d_sigs, first, cnt, p12->sig_region, p12->sig_bytes_len,
                                    p12->chunk_base ? (*p12->chunk_base)[k] : 0, p12->d_bases, dt, n_tmpls, n_ids,
                                    arena_len, (cg_item*)c->txitems.p, c->sig12ws.p, s);
    else if (r == hipSuccess)
      r = cg::launch_tx_sig_range(d_sigs, first, cnt, dt, n_tmpls, nullptr, n_ids, d_ids, arena_len, slot,
                                  (cg_item*)c->txitems.p, (uint8_t*)c->msgs.p, s);
    return r;
  };
  if (e == hipSuccess)
    e = launch_chunked(c, d_keys, n_keys, (const cg_item*)c->txitems.p, n_sigs, d_arena, arena_len, mode, d_status, s,
                       (const uint8_t*)c->msgs.p, cg::tx_msgs_head(n_tmpls, slot), &prepare, &uses,
                       bounds, ready != nullptr);
  return e;
}

// cg_verify_tx_signatures with the ctx lock held. Host side, in order: the key table and key bytes,
// the template bytes, the ids and the signature table (everything the key tables and the plans
// need), then the signature bytes chunk by chunk, each copy issued just before its chunk's front
// so that the key-table builds and the previous chunk's kernels run during it.
// The 12-byte form (cg_verify_tx_signatures_packed): sigs is null, sigs12 the table, the signatures
// dense in sig_bytes. On the device they follow the caller's arena at sig_region (16-aligned), so the
// kernels address every byte by an absolute arena offset as in the 24-byte form; a key or template
// that lies outside [0, arena_len) is moved out of the extended arena too (never reads a signature).
static int verify_txsig_host_locked(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const uint8_t* ids,
                                    uint64_t n_ids, const cg_txsig* sigs, uint64_t n_sigs,
                                    const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* arena,
                                    uint64_t arena_len, uint32_t mode, uint8_t* status_out, cg_stats* stats,
                                    const cg_txsig_packed* sigs12 = nullptr, const uint8_t* sig_bytes = nullptr,
                                    uint64_t sig_bytes_len = 0) {
  const auto t0 = std::chrono::steady_clock::now();
  const bool packed = sigs12 != nullptr;
  const size_t rec_bytes = packed ? sizeof(cg_txsig_packed) : sizeof(cg_txsig);
  const uint64_t caller_len = arena_len;
  const uint64_t sig_region = packed ? ((arena_len + 15) & ~(uint64_t)15) : 0;
  if (packed) arena_len = sig_region + sig_bytes_len;  // what the kernels see
  std::vector<cg_key> keys_fix;
  std::vector<cg_signable_tmpl> tmpls_fix;
  if (packed) {  // out-of-arena keys / templates stay out of range in the extended arena
    auto out = [&](uint64_t off, uint64_t len) { return off > caller_len || len > caller_len - off; };
    for (uint32_t k = 0; k < n_keys; ++k)
      if (out(keys[k].off, keys[k].len)) {
        if (keys_fix.empty()) keys_fix.assign(keys, keys + n_keys);
        keys_fix[k].off = UINT64_MAX;
      }
    for (uint32_t k = 0; k < n_tmpls; ++k)
      if (out(tmpls[k].prefix_off, tmpls[k].prefix_len) || out(tmpls[k].suffix_off, tmpls[k].suffix_len)) {
        if (tmpls_fix.empty()) tmpls_fix.assign(tmpls, tmpls + n_tmpls);
        tmpls_fix[k].prefix_off = UINT64_MAX;
      }
    if (!keys_fix.empty()) keys = keys_fix.data();
    if (!tmpls_fix.empty()) tmpls = tmpls_fix.data();
  }
  // a record's key index, either table (the count passes)
  auto key_at = [&](uint64_t i) -> uint32_t { return packed ? sigs12[i].key_idx : sigs[i].key_idx; };
  if (c->fault) return fail(CG_ERR_DEVICE, "cg_verify_tx_signatures: device fault (injected by cg_pool_inject_fault)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  // chunks: the device chunk, but at least CG_TXSIG_MIN_CHUNKS of them for a large call unless the
  // caller set cg_config.chunk_items (the first chunk's copy is the part nothing overlaps; measured on
  // the configs[4] shard: 2 chunks 190.7M, 3 200.8M, 4 207.7M, 6 190.0M sigs/s,
  // profiles/r03/chunks_v1)
  uint64_t per = chunk_of(c, n_sigs);
  if (!c->chunk_set && n_sigs >= CG_TXSIG_MIN_CHUNKS * (1ull << 20)) {
    const uint64_t alt = (n_sigs + CG_TXSIG_MIN_CHUNKS - 1) / CG_TXSIG_MIN_CHUNKS;
    if (alt < per) per = alt;
  }
  // chunk bounds: with a first-chunk divisor D > 1 (CG_TXSIG_FIRST_DIV, default 6; 0 or 1: equal
  // chunks of `per`) the first chunk is 1/D of the call and the rest is split into as many chunks as
  // the equal split would make: the first copy is the part nothing hides, and at 1/6 it lands as
  // the key-table builds finish (headline A/B, 4 pairs: 257.0 -> 262.9 M sigs/s; 1/5 neutral, 1/7
  // and 1/8 -3%: their fronts then share the chip with the builds; profiles/r03/env_fd15*)
  std::vector<uint64_t> bounds;
  {
    static const uint64_t first_div = [] {
      const char* v = getenv("CG_TXSIG_FIRST_DIV");
      return v ? (uint64_t)strtoull(v, nullptr, 10) : 6ull;
    }();
    const uint64_t k0 = (n_sigs + per - 1) / per;
    if (first_div > 1 && k0 > 1) {
      const uint64_t f0 = n_sigs / first_div, rest = n_sigs - f0, kr = k0;
      bounds.push_back(0);
      bounds.push_back(f0);
      for (uint64_t k = 1; k <= kr; ++k) bounds.push_back(f0 + rest * k / kr);
    } else {
      for (uint64_t k = 0; k <= k0; ++k) bounds.push_back(k == k0 ? n_sigs : k * per);
    }
    per = 0;
    for (size_t k = 0; k + 1 < bounds.size(); ++k) per = std::max(per, bounds[k + 1] - bounds[k]);
  }
  const uint64_t nch = bounds.size() - 1;
  // arena extents: key bytes + template bytes (the header), then each chunk's signature bytes
  Extent head, win;
  for (uint32_t k = 0; k < n_keys; ++k) head.add(keys[k].off, keys[k].len, caller_len);
  for (uint32_t k = 0; k < n_tmpls; ++k) {
    head.add(tmpls[k].prefix_off, tmpls[k].prefix_len, caller_len);
    head.add(tmpls[k].suffix_off, tmpls[k].suffix_len, caller_len);
  }
  // Key-use counts for the table modes from a 1-in-CG_TXSIG_COUNT_SAMPLE sample of the signature
  // table (16 host threads; the modes change only speed, never a verdict), every key at least 1 so
  // that each key an unsampled signature may use has its row-0 table. Each chunk's byte extents are
  // scanned just before its copy, while the device works on the chunks before it.
  std::vector<uint32_t> counts(n_keys ? n_keys : 1, 0u);
  // the budget's host threads (host_budget.h), on the context's pool (spawning 16 threads per scan
  // cost 0.35-0.5 ms a round)
  const uint64_t nt = host_threads_of(c, n_sigs);
  auto par = [&](uint64_t m, const std::function<void(uint64_t)>& fn) { host_par(c, m, fn); };
  auto sample_counts = [&] {
    // 1 in S signatures counted (CG_TXSIG_SAMPLE, a power of two, overrides): S = 32 when keys average
    // at least 256 uses (every key far above the 32-use full-table threshold), else 8: at S = 32 an
    // unsampled key could not be told from one at the threshold, and a long-tailed key mix (Zipf
    // over 1M keys) built full tables for every used key (125 -> 55 M sigs/s, profiles/r03/v12)
    static const uint32_t S_env = [] {
      const char* v = getenv("CG_TXSIG_SAMPLE");
      const uint32_t x = v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
      return x && (x & (x - 1)) == 0 ? x : 0u;
    }();
    // Round 4: 1 (exact counts) instead of 1 in 8 when keys are many. With the quarter mode from 3
    // uses, an unsampled key (unused, or used a few times) could not be given a mode: row 0 for all
    // of them left ~20% of the 2^20-distinct-key leg's keys (12 uses) on the Horner ladder, quarter
    // tables for all of them built tables for the Zipf leg's ~900k unused keys (125 -> 108 M sigs/s)
    const uint32_t S = S_env ? S_env : n_sigs >= 256ull * (n_keys ? n_keys : 1) ? CG_TXSIG_COUNT_SAMPLE : 1u;
    // CG_TXSIG_SAMPLE_BLOCK (A/B): consecutive records per sample. 8 reads an eighth of the table's
    // cache lines instead of all of them (every 8th 24-B record): the pass went 5.3 -> 2.8 ms on the
    // configs[4] shard, 218 -> 238 M sigs/s (profiles/r03/env_ec3); a key the block sampling
    // under-counts only lands in a smaller table mode, whose ladders run on the side streams
    static const uint32_t B = [] {
      const char* v = getenv("CG_TXSIG_SAMPLE_BLOCK");
      const uint32_t x = v ? (uint32_t)strtoul(v, nullptr, 10) : CG_TXSIG_SAMPLE_BLOCK;
      return x >= 1 && x <= 64 ? x : CG_TXSIG_SAMPLE_BLOCK;
    }();
    if (S == 1) {  // exact: byte counters per thread (1 MB for 2^20 keys, cache-resident), wraps logged
      c->cnt8.resize(nt);
      c->ovf.resize(nt);
      auto scan8 = [&](uint64_t t) {
        std::vector<uint8_t>& c8 = c->cnt8[t];
        if (c8.size() < n_keys) c8.resize(n_keys);
        memset(c8.data(), 0, n_keys);
        std::vector<uint32_t>& of = c->ovf[t];
        of.clear();
        uint8_t* cc = c8.data();
        auto run = [&](const auto* tab) {
          for (uint64_t i = n_sigs * t / nt; i < n_sigs * (t + 1) / nt; ++i) {
            const uint32_t k = tab[i].key_idx;
            if (k < n_keys && ++cc[k] == 0) of.push_back(k);
          }
        };
        if (packed) run(sigs12);
        else run(sigs);
      };
      par(nt, scan8);
      auto sum = [&](uint64_t t) {
        for (uint64_t k = n_keys * t / nt; k < n_keys * (t + 1) / nt; ++k) {
          uint32_t v = 0;
          for (uint64_t u = 0; u < nt; ++u) v += c->cnt8[u][k];
          counts[k] = v;
        }
      };
      par(nt, sum);
      for (uint64_t t = 0; t < nt; ++t)
        for (uint32_t k : c->ovf[t]) counts[k] += 256u;
      return;
    }
    const uint64_t Bs = B;
    const uint64_t ng = (n_sigs + (uint64_t)S * Bs - 1) / ((uint64_t)S * Bs);
    std::vector<std::vector<uint32_t>> pc(nt > 1 ? nt : 0, std::vector<uint32_t>(n_keys ? n_keys : 1, 0u));
    auto scan = [&](uint64_t t) {
      uint32_t* cnt = nt > 1 ? pc[t].data() : counts.data();
      for (uint64_t g = ng * t / nt; g < ng * (t + 1) / nt; ++g) {
        // B consecutive records per group of S B, the block at a hashed position (no aliasing with
        // a layout that cycles through the keys); B > 1 reads fewer cache lines per sample
        const uint64_t i0 = (g * S + (((uint32_t)g * 0x9E3779B1u) >> 24) % S) * Bs;
        for (uint64_t i = i0; i < i0 + Bs && i < n_sigs; ++i) {
          const uint32_t k = key_at(i);
          if (k < n_keys) ++cnt[k];
        }
      }
    };
    if (nt == 1) {
      scan(0);
    } else {
      par(nt, scan);
      par(nt, [&](uint64_t t) {  // sum the per-thread counts, key ranges in parallel
        for (uint64_t k = n_keys * t / nt; k < n_keys * (t + 1) / nt; ++k)
          for (uint64_t u = 0; u < nt; ++u) counts[k] += pc[u][k];
      });
    }
    // c sampled uses -> S (c + 3 sqrt(c) + 1): about three standard deviations above the unbiased
    // S c, so a key whose true count clears a mode threshold is not sampled below it (two were not
    // enough at 1 in 32: a few keys got full tables and a 0.18 ms full-table ladder per chunk,
    // profiles/r03/v14; on the
    // configs[4] shard the plain estimate put 2 of 4096 Ed25519 keys, true minimum 1 634 uses, under
    // the 1 536 wide threshold: full tables and a 170 us pf ladder per chunk, profiles/r03/v5); an
    // unsampled key counts min(S, 8): its row-0 table, so every key a signature may use has one
    // In a hot call (1 in 32: keys average 256+ uses) every sampled key is counted up to the wide
    // threshold: a few keys left in full-table mode cost a serial full-table launch per chunk (0.18
    // ms, ~1.4% of the headline, profiles/r03/ab_der), a wide table costs about 230 items' work.
    const cg::WidePool thr = c->eng->make_wide_pool(nullptr, n_keys, n_sigs, cg::kKeyWideMax);  // the wide thresholds
    const uint64_t floor_hot = S >= CG_TXSIG_COUNT_SAMPLE ? (uint64_t)std::max(thr.min_ed, thr.min_ec) : 0u;
    // The raised estimate only where it decides a wide table: below the wide threshold the plain
    // S c decides row 0 against full tables (a wrong full table costs ~230 ns, a wrong row 0 ~7 ns
    // per use; at 1 in 8 the raised estimate put every sampled key of the 2^20-distinct-key leg,
    // ~12 uses each, in full mode: 22-row builds for ~1M keys, profiles/r04/kd)
    for (uint32_t k = 0; k < n_keys; ++k) {
      const uint64_t c = counts[k];
      const uint64_t up = (uint64_t)S * (c + 3 * (uint64_t)std::ceil(std::sqrt((double)c)) + 1);
      const uint64_t wmin = keys[k].scheme == CG_EDDSA_ED25519_SHA512 ? thr.min_ed : thr.min_ec;
      uint64_t e = c ? (up >= wmin ? up : (uint64_t)S * c)
                     : (S < 8u ? S : 8u);  // unsampled: row-0 tables (below the 32-use threshold)
      if (c && e < floor_hot) e = floor_hot;
      counts[k] = e > 0xfffffff0ull ? 0xfffffff0u : (uint32_t)e;
    }
  };
  // chunk k's signature bytes and id bytes (exact: a threaded scan of its slice of the table). The
  // 12-byte table: the chunk's stream bytes (the sum of round_up(sig_len, 4)) in `span`, its extent
  // set once its stream offset is known (copy_table: the chunks before it summed)
  auto chunk_extents = [&](uint64_t k, Extent& ext, Extent& idx, uint64_t& span) {
    const uint64_t f = bounds[k], e = bounds[k + 1];
    const uint64_t m = (e - f) < (1u << 16) ? 1 : nt;
    std::vector<Extent> pe(m), pi(m);
    std::vector<uint64_t> ps(m, 0);
    auto scan = [&](uint64_t t) {
      Extent a, b;  // thread-local until the end (the vector slots share cache lines)
      uint64_t sp = 0;
      const uint64_t i0 = f + (e - f) * t / m, i1 = f + (e - f) * (t + 1) / m;
      if (packed) {
        for (uint64_t i = i0; i < i1; ++i) {
          sp += ((uint64_t)sigs12[i].sig_len + 3u) & ~(uint64_t)3;
          if (sigs12[i].tx_idx < n_ids) b.add(32ull * sigs12[i].tx_idx, 32, 32ull * n_ids);
        }
      } else {
        for (uint64_t i = i0; i < i1; ++i) {
          a.add(sigs[i].sig_off, sigs[i].sig_len, arena_len);
          if (sigs[i].tx_idx < n_ids) b.add(32ull * sigs[i].tx_idx, 32, 32ull * n_ids);
        }
      }
      pe[t] = a;
      pi[t] = b;
      ps[t] = sp;
    };
    par(m, scan);
    span = 0;
    for (uint64_t t = 0; t < m; ++t) {
      ext.merge(pe[t]);
      idx.merge(pi[t]);
      span += ps[t];
    }
  };
  // the 12-byte table: chunk k's first signature at stream offset cbase[k] (cbase[k + 1] is set when
  // chunk k's table slice is staged)
  std::vector<uint64_t> cbase(nch + 1, 0);
  // the device arena mirrors [0, arena_len) (only referenced bytes are copied)
  win.lo = 0;
  win.hi = arena_len;
  const uint64_t slot = tmpl_slot(tmpls, n_tmpls);
  HIP_TRY(c->keys.ensure(sizeof(cg_key) * (n_keys ? n_keys : 1)), "hipMalloc(keys)");
  HIP_TRY(c->h_sigs.ensure(rec_bytes * n_sigs), "hipMalloc(sigs)");
  if (packed) HIP_TRY(c->sig12ws.ensure(cg::tx_sig12_scratch_bytes(per)), "hipMalloc(signature offsets)");
  HIP_TRY(c->aux1.ensure(sizeof(uint32_t) * counts.size()), "hipMalloc(key use counts)");
  HIP_TRY(c->h_ids.ensure(32 * (n_ids ? n_ids : 1)), "hipMalloc(ids)");
  HIP_TRY(c->arena.ensure((win.hi - win.lo) + 16), "hipMalloc(arena window)");
  HIP_TRY(c->status.ensure(n_sigs), "hipMalloc(status)");
  HIP_TRY(ensure_txsig_ws(c, n_sigs, n_tmpls, slot), "hipMalloc(tx signature workspace)");
  HIP_TRY(ensure_ws(c, n_keys, per, n_sigs), "hipMalloc(workspace)");
  // CG_TXSIG_OVERLAP_PLAN=1 (A/B): sample the counts while chunk 0 copies. Measured slower on the
  // configs[4] shard (197 / 205 vs 213 / 220 M sigs/s, profiles/r03/ab_sc): the sample pass slows
  // 2x beside the pageable copy's staging and the late counts delay the key tables.
  static const bool overlap = [] {
    const char* v = getenv("CG_TXSIG_OVERLAP_PLAN");
    return v && v[0] == '1';
  }();
  if (overlap && c->pin_counts_cap < counts.size()) {
    if (c->pin_counts) HIP_TRY(hipHostFree(c->pin_counts), "hipHostFree");
    c->pin_counts = nullptr;
    c->pin_counts_cap = 0;
    HIP_TRY(hipHostMalloc((void**)&c->pin_counts, sizeof(uint32_t) * counts.size(), hipHostMallocDefault),
            "hipHostMalloc(key use counts)");
    c->pin_counts_cap = counts.size();
  }
  while (c->seg.size() < nch + 1) {
    hipEvent_t e;
    HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming), "hipEventCreate");
    c->seg.push_back(e);
  }
  hipStream_t s = c->stream;
  uint8_t* dwin = (uint8_t*)c->arena.p;
  const uint8_t* dbase = dwin - win.lo;  // kernels index the arena by absolute offsets
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(hipEventRecord(c->tev[0], s), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(c->copy, c->tev[0], 0), "hipStreamWaitEvent");
  HIP_TRY(hipStreamWaitEvent(c->copy2, c->tev[0], 0), "hipStreamWaitEvent");
  std::vector<std::pair<uint64_t, uint64_t>> have;
  if (n_keys)
    HIP_TRY(hipMemcpyAsync(c->keys.p, keys, sizeof(cg_key) * n_keys, hipMemcpyHostToDevice, c->copy), "H2D keys");
  HIP_TRY(copy_missing(have, head, arena, dwin, win.lo, c->copy), "H2D key / template bytes");
  std::vector<std::pair<uint64_t, uint64_t>> have_ids;  // id bytes already resident
  std::vector<std::pair<uint64_t, uint64_t>> have_sig;  // the 12-byte form's stream bytes already resident
  // chunk k: its slice of the signature table, the ids it references not yet resident (a caller that
  // lists each transaction's signatures together ships each id once, with its first chunk), then its
  // signature bytes, on copy stream cs; seg[k] marks the end
  // CG_HOST_TRACE=1: per-chunk host timings to stderr (extent scan, each copy call's return)
  static const bool htrace = [] {
    const char* v = getenv("CG_HOST_TRACE");
    return v && v[0] == '1';
  }();
  auto ms_since = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  c->htrace = htrace;
  for (int q = 0; q < 2 && htrace; ++q)
    if (!c->backt[q]) HIP_TRY(hipEventCreate(&c->backt[q]), "hipEventCreate");
  while (htrace && c->fbt.size() < 3 * nch) {
    hipEvent_t ev;
    HIP_TRY(hipEventCreate(&ev), "hipEventCreate");
    c->fbt.push_back(ev);
  }
  if (htrace) c->fbh.assign(nch, 0.0);
  // CG_SCAN_AHEAD=1 (A/B): chunk k+1's extent scan runs on the pool from a helper thread while this
  // thread stages chunk k's copies (round 4 measured scanning ahead neutral to -1%, the copies'
  // landing times did not move, profiles/r04/ahead; round 5's trace shows the main stream waiting
  // 0.33 ms for chunk 1's bytes)
  bool ct_active = false;  // the copy thread below issues the copies (it runs ahead: no scan-ahead helper)
  static const bool scan_ahead = [] {
    const char* v = getenv("CG_SCAN_AHEAD");
    return v && v[0] == '1';
  }();
  std::thread ahead_thr;
  uint64_t ahead_k = ~0ull, ahead_span = 0;
  Extent ahead_ek, ahead_ik;
  struct JoinAhead {  // every exit path joins the helper before the extents it writes go away
    std::thread& t;
    ~JoinAhead() {
      if (t.joinable()) t.join();
    }
  } join_ahead{ahead_thr};
  // chunk k's copies in two parts: the extent scan and the signature-table slice (all its plan
  // needs), then the ids and signature bytes (what its hashes need); seg[k] marks the end
  std::vector<Extent> ext_e(nch), ext_i(nch);
  std::vector<double> ht(3 * nch, 0.0);
  auto copy_table = [&](uint64_t k, hipStream_t cs) {
    Extent& ek = ext_e[k];
    Extent& ik = ext_i[k];
    const double h0 = htrace ? ms_since() : 0;
    uint64_t span = 0;
    if (ahead_k == k) {
      ahead_thr.join();
      ek = ahead_ek;
      ik = ahead_ik;
      span = ahead_span;
      ahead_k = ~0ull;
    } else {
      chunk_extents(k, ek, ik, span);
    }
    if (packed) {  // the chunk's stream bytes, clipped to the caller's buffer (past it: CG_NOT_RUN)
      cbase[k + 1] = cbase[k] + span;
      ek = Extent();
      ek.add(cbase[k], span, sig_bytes_len);
    }
    if (scan_ahead && !ct_active && k + 1 < nch) {
      ahead_k = k + 1;
      ahead_ek = Extent();
      ahead_ik = Extent();
      ahead_thr = std::thread([&, k] { chunk_extents(k + 1, ahead_ek, ahead_ik, ahead_span); });
    }
    const double h1 = htrace ? ms_since() : 0;
    const uint64_t first = bounds[k], cnt = bounds[k + 1] - bounds[k];
    const hipError_t e =
        packed ? hipMemcpyAsync((cg_txsig_packed*)c->h_sigs.p + first, sigs12 + first, rec_bytes * cnt,
                                hipMemcpyHostToDevice, cs)
               : hipMemcpyAsync((cg_txsig*)c->h_sigs.p + first, sigs + first, rec_bytes * cnt, hipMemcpyHostToDevice,
                                cs);
    ht[3 * k] = h0;
    ht[3 * k + 1] = h1 - h0;
    ht[3 * k + 2] = htrace ? ms_since() - h1 : 0;
    return e;
  };
  auto copy_bytes = [&](uint64_t k, hipStream_t cs) {
    const Extent& ek = ext_e[k];
    const double h2 = htrace ? ms_since() : 0;
    hipError_t e = copy_missing(have_ids, ext_i[k], ids, (uint8_t*)c->h_ids.p, 0, cs);
    const double h3 = htrace ? ms_since() : 0;
    if (e == hipSuccess && packed) e = copy_missing(have_sig, ek, sig_bytes, dwin + sig_region, 0, cs);
    else if (e == hipSuccess) e = copy_missing(have, ek, arena, dwin, win.lo, cs);
    if (e == hipSuccess) e = hipEventRecord(c->seg[k], cs);
    if (e == hipSuccess && htrace) {
      while (c->segt.size() <= k) {
        hipEvent_t ev;
        if (hipEventCreate(&ev) != hipSuccess) break;
        c->segt.push_back(ev);
      }
      if (c->segt.size() > k) e = hipEventRecord(c->segt[k], cs);
    }
    if (htrace)
      fprintf(stderr, "[cg host] chunk %llu at %.3f: scan %.3f sigs %.3f (%.1f MB) ids %.3f arena %.3f (%.1f MB) ms\n",
              (unsigned long long)k, ht[3 * k], ht[3 * k + 1], ht[3 * k + 2],
              rec_bytes * (bounds[k + 1] - bounds[k]) / 1e6, h3 - h2, ms_since() - h3,
              ek.empty() ? 0.0 : (ek.hi - ek.lo) / 1e6);
    return e;
  };
  auto copy_chunk = [&](uint64_t k, hipStream_t cs) {
    hipError_t e = copy_table(k, cs);
    if (e == hipSuccess) e = copy_bytes(k, cs);
    return e;
  };
  // The key-use counts gate only the key tables; chunk 0's bytes gate everything else. With
  // `overlap`, chunk 0's copy (its own thread, second copy stream) runs while this thread samples
  // the counts, which then go from the pinned buffer behind the key bytes on the first copy stream.
  hipError_t pre_err = hipSuccess;
  double ms_plan = 0;
  if (overlap) {
    std::thread pre([&] {
      pre_err = hipSetDevice(c->device);
      if (pre_err == hipSuccess) pre_err = copy_chunk(0, c->copy2);
    });
    sample_counts();
    ms_plan = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    memcpy(c->pin_counts, counts.data(), sizeof(uint32_t) * counts.size());
    const hipError_t e = hipMemcpyAsync(c->aux1.p, c->pin_counts, sizeof(uint32_t) * counts.size(),
                                        hipMemcpyHostToDevice, c->copy);
    pre.join();
    HIP_TRY(e, "H2D key use counts");
    HIP_TRY(pre_err, "H2D chunk 0");
  } else {
    sample_counts();
    ms_plan = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    HIP_TRY(hipMemcpyAsync(c->aux1.p, counts.data(), sizeof(uint32_t) * counts.size(), hipMemcpyHostToDevice,
                           c->copy),
            "H2D key use counts");
  }
  HIP_TRY(hipEventRecord(c->seg[nch], c->copy), "hipEventRecord");
  HIP_TRY(hipStreamWaitEvent(s, c->seg[nch], 0), "hipStreamWaitEvent");
  // Round 5: chunk k's front waits only for its signature-table slice; its item build and plan are
  // enqueued before the host stages the chunk's ids and signature bytes (launch_items_front runs the
  // hook between the plan and the hashes), so the plan overlaps the byte copy. Headline A/B, 10
  // interleaved pairs: 327.7 -> 330.5 M sigs/s, 7 of 10 pairs faster (profiles/r05/split);
  // CG_SPLIT_COPY=0 restores the whole-chunk wait.
  static const bool split = [] {
    const char* v = getenv("CG_SPLIT_COPY");
    return !(v && v[0] == '0');
  }();
  const bool split_on = split && !overlap;
  while (split_on && c->segtab.size() < nch) {
    hipEvent_t ev;
    HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming), "hipEventCreate");
    c->segtab.push_back(ev);
  }
  hipError_t copy_err = hipSuccess;
  uint64_t mid_k = 0;
  // the second half of chunk mid_k's before(): bytes copied, the front's stream ordered after them
  // Round 6 (CG_COPY_THREAD=1, A/B): a copy thread issues every chunk's table slice and bytes in
  // order, running ahead, while this thread enqueues the kernels. The pageable copies block the
  // issuing thread for the runtime's staging (~4 ms of a ~6-ms chunk on the headline) and the kernel
  // and event calls of a chunk take ~2 ms of host time more (CG_HOST_TRACE, profiles/r06/copy_thread):
  // in one thread the device waited ~0.3 ms per chunk for the host. This thread now waits (host
  // condition) only until the copier has recorded the event it orders the main stream after.
  static const bool copy_thread_env = [] {
    const char* v = getenv("CG_COPY_THREAD");
    return v && v[0] == '1';
  }();
  const bool ct = copy_thread_env && split_on && nch > 1;
  ct_active = ct;
  struct Feed {
    std::mutex m;
    std::condition_variable cv;
    uint64_t tab = 0, bytes = 0;  // chunks whose table slice / bytes the copier has issued
    hipError_t err = hipSuccess;
    bool stop = false;
  } feed;
  auto feed_wait = [&](bool bytes, uint64_t k) -> hipError_t {
    std::unique_lock<std::mutex> lk(feed.m);
    feed.cv.wait(lk, [&] { return feed.err != hipSuccess || (bytes ? feed.bytes : feed.tab) > k; });
    return (bytes ? feed.bytes : feed.tab) > k ? hipSuccess : feed.err;
  };
  std::thread copier;
  struct JoinCopier {  // every exit path stops and joins the copier before the locals it uses go away
    std::thread& t;
    Feed& f;
    ~JoinCopier() {
      {
        std::lock_guard<std::mutex> g(f.m);
        f.stop = true;
      }
      if (t.joinable()) t.join();
    }
  } join_copier{copier, feed};
  const std::function<hipError_t()> mid = [&]() -> hipError_t {
    c->fork.mid_front = nullptr;
    const uint64_t k = mid_k;
    hipError_t e = ct ? feed_wait(true, k) : copy_bytes(k, c->copy);
    if (e == hipSuccess) e = hipStreamWaitEvent(s, c->seg[k], 0);
    if (e == hipSuccess && htrace && 3 * k < c->fbt.size()) {
      c->fbh[k] = ms_since();
      e = hipEventRecord(c->fbt[3 * k], s);
    }
    if (e == hipSuccess && k == 0) e = hipEventRecord(c->tev[1], s);
    if (e != hipSuccess) copy_err = e;
    return e;
  };
  struct ClearHook {  // no hook outlives this call's locals, whatever the exit path
    cg_ctx* c;
    ~ClearHook() { c->fork.mid_front = nullptr; }
  } clear_hook{c};
  const std::function<hipError_t(uint64_t, uint64_t, uint64_t)> before = [&](uint64_t k, uint64_t, uint64_t) {
    if (split_on) {
      hipError_t e = c->fork.mid_front ? mid() : hipSuccess;  // a hook a front did not consume
      if (ct) {
        if (e == hipSuccess) e = feed_wait(false, k);  // the copier recorded segtab[k]
      } else {
        if (e == hipSuccess) e = copy_table(k, c->copy);
        if (e == hipSuccess) e = hipEventRecord(c->segtab[k], c->copy);
      }
      if (e == hipSuccess) e = hipStreamWaitEvent(s, c->segtab[k], 0);
      if (e == hipSuccess) {
        mid_k = k;
        c->fork.mid_front = &mid;
      }
      if (e != hipSuccess) copy_err = e;
      return e;
    }
    hipError_t e = overlap && k == 0 ? hipSuccess : copy_chunk(k, c->copy);
    const hipStream_t fs = s;  // the stream chunk k's front runs on
    if (e == hipSuccess) e = hipStreamWaitEvent(fs, c->seg[k], 0);
    if (e == hipSuccess && htrace && 3 * k < c->fbt.size()) {
      c->fbh[k] = ms_since();
      e = hipEventRecord(c->fbt[3 * k], fs);  // the front's stream reaches chunk k's front
    }
    if (e == hipSuccess && k == 0) e = hipEventRecord(c->tev[1], fs);
    if (e != hipSuccess) copy_err = e;
    return e;
  };
  uint8_t* ds = (uint8_t*)c->status.p;
  cg::KeyUses uses;
  uses.counts = (const uint32_t*)c->aux1.p;
  uses.n = n_sigs;
  uses.host_keys = keys;
  uses.host_counts = counts.data();
  Packed12 p12;
  if (packed) {
    p12.d_sigs = (const cg_txsig_packed*)c->h_sigs.p;
    p12.sig_region = sig_region;
    p12.sig_bytes_len = sig_bytes_len;
    p12.chunk_base = &cbase;
  }
  if (ct)
    copier = std::thread([&] {
      hipError_t e = hipSetDevice(c->device);
      for (uint64_t k = 0; k < nch && e == hipSuccess; ++k) {
        {
          std::lock_guard<std::mutex> g(feed.m);
          if (feed.stop) break;
        }
        e = copy_table(k, c->copy);
        if (e == hipSuccess) e = hipEventRecord(c->segtab[k], c->copy);
        if (e == hipSuccess) {
          std::lock_guard<std::mutex> g(feed.m);
          feed.tab = k + 1;
        }
        feed.cv.notify_all();
        if (e == hipSuccess) e = copy_bytes(k, c->copy);  // records seg[k]
        if (e == hipSuccess) {
          std::lock_guard<std::mutex> g(feed.m);
          feed.bytes = k + 1;
        }
        feed.cv.notify_all();
      }
      std::lock_guard<std::mutex> g(feed.m);
      if (e != hipSuccess) feed.err = e;
      else if (feed.bytes < nch) feed.err = hipErrorUnknown;  // stopped early: no waiter may hang
      feed.cv.notify_all();
    });
  const hipError_t le = launch_txsig(c, (const cg_key*)c->keys.p, n_keys, (const uint8_t*)c->h_ids.p, n_ids,
                                     packed ? nullptr : (const cg_txsig*)c->h_sigs.p, n_sigs, tmpls, n_tmpls, dbase,
                                     arena_len, mode, ds, s, slot, uses, &before, &bounds, packed ? &p12 : nullptr);
  if (le == hipSuccess && c->fork.mid_front) {  // the last front did not consume its hook
    const hipError_t me = mid();
    if (me != hipSuccess) copy_err = me;
  }
  if (copier.joinable()) {
    {
      std::lock_guard<std::mutex> g(feed.m);
      feed.stop = true;
    }
    copier.join();
    if (feed.err != hipSuccess && copy_err == hipSuccess && le == hipSuccess) copy_err = feed.err;
  }
  if (copy_err != hipSuccess) return hip_fail(copy_err, "H2D signature bytes");
  HIP_TRY(le, "launch_txsig");
  HIP_TRY(hipEventRecord(c->tev[2], s), "hipEventRecord");
  HIP_TRY(hipMemcpyAsync(status_out, ds, n_sigs, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipEventRecord(c->tev[3], s), "hipEventRecord");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  const double h_enq = htrace ? ms_since() : 0;
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  if (htrace) {
    fprintf(stderr, "[cg host] enqueued at %.3f, done at %.3f ms; copies landed (device ms after the call's first event):",
            h_enq, ms_since());
    for (uint64_t k = 0; k < nch && k < c->segt.size(); ++k) {
      float t = 0;
      hipEventElapsedTime(&t, c->tev[0], c->segt[k]);
      fprintf(stderr, " %.3f", t);
    }
    float t = 0, f0 = 0, tb = 0;
    hipEventElapsedTime(&t, c->tev[0], c->tev[2]);
    hipEventElapsedTime(&f0, c->tev[0], c->backt[0]);
    hipEventElapsedTime(&tb, c->tev[0], c->backt[1]);
    fprintf(stderr, "; chunk 0 front done %.3f, tables built %.3f, verify done %.3f\n", f0, tb, t);
    for (uint64_t k = 0; k < nch && 3 * k + 2 < c->fbt.size(); ++k) {
      float fs = 0, be = 0, bj = 0;
      hipEventElapsedTime(&fs, c->tev[0], c->fbt[3 * k]);
      hipEventElapsedTime(&bj, c->tev[0], c->fbt[3 * k + 2]);
      hipEventElapsedTime(&be, c->tev[0], c->fbt[3 * k + 1]);
      fprintf(stderr, "[cg host] chunk %llu: front enqueued (host) %.3f, front reached (device) %.3f, back's "
              "kernels done %.3f, joins done %.3f\n", (unsigned long long)k, c->fbh[k], fs, bj, be);
    }
  }
  if (stats) {
    float a = 0, b = 0, d = 0;
    hipEventElapsedTime(&a, c->tev[0], c->tev[1]);
    hipEventElapsedTime(&b, c->tev[1], c->tev[2]);
    hipEventElapsedTime(&d, c->tev[2], c->tev[3]);
    stats->n_items = n_sigs;
    stats->n_keys = n_keys;
    stats->ms_h2d = a;
    stats->ms_key_prep = ms_plan;  // host-side planning: the key-use sample pass
    stats->ms_verify = b;
    stats->ms_d2h = d;
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return CG_OK;
}

static int txsig_args(const char* fn, cg_ctx* c, uint32_t n_keys, const void* keys, uint64_t n_ids, const void* ids,
                      uint64_t n_sigs, const void* sigs, const void* status, uint32_t n_tmpls, const void* tmpls,
                      uint32_t mode) {
  if (!c) return fail(CG_ERR_ARG, "%s: ctx is NULL", fn);
  if (n_sigs && (!sigs || !status)) return fail(CG_ERR_ARG, "%s: NULL signature / status buffer", fn);
  if (n_keys && !keys) return fail(CG_ERR_ARG, "%s: keys is NULL", fn);
  if (n_ids && !ids) return fail(CG_ERR_ARG, "%s: ids is NULL", fn);
  if (n_tmpls && !tmpls) return fail(CG_ERR_ARG, "%s: templates is NULL", fn);
  if (n_tmpls > 0x10000u) return fail(CG_ERR_ARG, "%s: more than 65536 templates (cg_txsig.tmpl is 16-bit)", fn);
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "%s: bad mode", fn);
  return CG_OK;
}

int cg_verify_tx_signatures_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_ids,
                                   uint64_t n_ids, const cg_txsig* d_sigs, uint64_t n_sigs,
                                   const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* d_arena,
                                   uint64_t arena_len, uint32_t mode, uint8_t* d_status, void* hip_stream) {
  const int a = txsig_args("cg_verify_tx_signatures_device", c, n_keys, d_keys, n_ids, d_ids, n_sigs, d_sigs, d_status,
                           n_tmpls, tmpls, mode);
  if (a != CG_OK) return a;
  if (n_sigs == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->fault) return fail(CG_ERR_DEVICE, "cg_verify_tx_signatures_device: device fault (injected)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  const uint64_t slot = tmpl_slot(tmpls, n_tmpls);
  HIP_TRY(ensure_txsig_ws(c, n_sigs, n_tmpls, slot), "hipMalloc(tx signature workspace)");
  HIP_TRY(ensure_ws(c, n_keys, chunk_of(c, n_sigs), n_sigs), "hipMalloc(workspace)");
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  cg::KeyUses uses;
  uses.sigs = d_sigs;
  uses.n = n_sigs;
  HIP_TRY(launch_txsig(c, d_keys, n_keys, d_ids, n_ids, d_sigs, n_sigs, tmpls, n_tmpls, d_arena, arena_len, mode,
                       d_status, s, slot, uses, nullptr),
          "launch_txsig");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_verify_tx_signatures_packed_device(cg_ctx* c, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_ids,
                                          uint64_t n_ids, const cg_txsig_packed* d_sigs, uint64_t n_sigs,
                                          uint64_t sig_bytes_off, uint64_t sig_bytes_len,
                                          const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* d_arena,
                                          uint64_t arena_len, uint32_t mode, uint8_t* d_status, void* hip_stream) {
  const int a = txsig_args("cg_verify_tx_signatures_packed_device", c, n_keys, d_keys, n_ids, d_ids, n_sigs, d_sigs,
                           d_status, n_tmpls, tmpls, mode);
  if (a != CG_OK) return a;
  if (sig_bytes_off > arena_len || sig_bytes_len > arena_len - sig_bytes_off)
    return fail(CG_ERR_ARG, "cg_verify_tx_signatures_packed_device: the signature stream lies outside the arena");
  if (n_sigs == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  if (c->fault) return fail(CG_ERR_DEVICE, "cg_verify_tx_signatures_packed_device: device fault (injected)");
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  const uint64_t slot = tmpl_slot(tmpls, n_tmpls);
  // equal chunks rounded to the 256-record blocks whose stream offsets are computed once for the table
  uint64_t per = chunk_of(c, n_sigs);
  per = (per + 255) & ~(uint64_t)255;
  std::vector<uint64_t> bounds;
  for (uint64_t f = 0; f < n_sigs; f += per) bounds.push_back(f);
  bounds.push_back(n_sigs);
  // CG_DEV_FIRST_PCT=<p> (A/B): a two-chunk call's first chunk p% of the call instead of half; 50 / 60
  // / 67% measured 391.2 / 392.1 / 392.3 M sigs/s over 3 rounds, within the noise (profiles/r06/firstpct)
  static const uint64_t first_pct = [] {
    const char* v = getenv("CG_DEV_FIRST_PCT");
    const uint64_t x = v ? (uint64_t)strtoull(v, nullptr, 10) : 0ull;
    return x >= 10 && x <= 90 ? x : 0ull;
  }();
  if (first_pct && bounds.size() == 3) {
    bounds[1] = std::min<uint64_t>(((n_sigs * first_pct / 100) + 255) & ~(uint64_t)255, n_sigs);
    per = std::max(bounds[1], n_sigs - bounds[1]);
  }
  HIP_TRY(ensure_txsig_ws(c, n_sigs, n_tmpls, slot), "hipMalloc(tx signature workspace)");
  HIP_TRY(ensure_ws(c, n_keys, per, n_sigs), "hipMalloc(workspace)");
  HIP_TRY(c->sig12ws.ensure(cg::tx_sig12_scratch_bytes(n_sigs)), "hipMalloc(signature offsets)");
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(cg::launch_tx_sig12_bases(d_sigs, 0, n_sigs, 0, (uint64_t*)c->sig12ws.p, s), "launch_tx_sig12_bases");
  cg::KeyUses uses;
  uses.sigs12 = d_sigs;
  uses.n = n_sigs;
  Packed12 p12;
  p12.d_sigs = d_sigs;
  p12.sig_region = sig_bytes_off;
  p12.sig_bytes_len = sig_bytes_len;
  p12.d_bases = (const uint64_t*)c->sig12ws.p;
  HIP_TRY(launch_txsig(c, d_keys, n_keys, d_ids, n_ids, nullptr, n_sigs, tmpls, n_tmpls, d_arena, arena_len, mode,
                       d_status, s, slot, uses, nullptr, &bounds, &p12),
          "launch_txsig");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_verify_tx_signatures_packed(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const uint8_t* ids, uint64_t n_ids,
                                   const cg_txsig_packed* sigs, uint64_t n_sigs, const uint8_t* sig_bytes,
                                   uint64_t sig_bytes_len, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                                   const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out,
                                   cg_stats* stats) {
  const int a = txsig_args("cg_verify_tx_signatures_packed", c, n_keys, keys, n_ids, ids, n_sigs, sigs, status_out,
                           n_tmpls, tmpls, mode);
  if (a != CG_OK) return a;
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_verify_tx_signatures_packed: arena is NULL");
  if (sig_bytes_len && !sig_bytes) return fail(CG_ERR_ARG, "cg_verify_tx_signatures_packed: sig_bytes is NULL");
  if (n_sigs) memset(status_out, CG_NOT_RUN, n_sigs);
  if (n_sigs == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  const int rc = verify_txsig_host_locked(c, keys, n_keys, ids, n_ids, nullptr, n_sigs, tmpls, n_tmpls, arena,
                                          arena_len, mode, status_out, stats, sigs, sig_bytes, sig_bytes_len);
  if (rc != CG_OK) memset(status_out, CG_NOT_RUN, n_sigs);
  return rc;
}

int cg_verify_tx_signatures(cg_ctx* c, const cg_key* keys, uint32_t n_keys, const uint8_t* ids, uint64_t n_ids,
                            const cg_txsig* sigs, uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls,
                            const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out,
                            cg_stats* stats) {
  const int a = txsig_args("cg_verify_tx_signatures", c, n_keys, keys, n_ids, ids, n_sigs, sigs, status_out, n_tmpls,
                           tmpls, mode);
  if (a != CG_OK) return a;
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_verify_tx_signatures: arena is NULL");
  if (n_sigs) memset(status_out, CG_NOT_RUN, n_sigs);
  if (n_sigs == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  const int rc = verify_txsig_host_locked(c, keys, n_keys, ids, n_ids, sigs, n_sigs, tmpls, n_tmpls, arena, arena_len,
                                          mode, status_out, stats);
  if (rc != CG_OK) memset(status_out, CG_NOT_RUN, n_sigs);
  return rc;
}

int cg_verify_filtered_device(cg_ctx* c, const cg_filtered_tx* d_ftxs, uint64_t n_ftx, const cg_pmt_node* d_nodes,
                              uint64_t n_nodes, const cg_filtered_leaf* d_leaves, uint64_t n_leaves,
                              const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_status, void* hip_stream) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_filtered_device: ctx is NULL");
  if (n_ftx && (!d_ftxs || !d_status)) return fail(CG_ERR_ARG, "cg_verify_filtered_device: NULL buffer");
  if (n_ftx == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  if (c->ftxws.cap < cg::ftx_ws_bytes(n_leaves)) {
    HIP_TRY(hipDeviceSynchronize(), "hipDeviceSynchronize");
    HIP_TRY(c->ftxws.ensure(cg::ftx_ws_bytes(n_leaves)), "hipMalloc(filtered ws)");
  }
  hipStream_t s = stream_of(c, hip_stream);
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(cg::launch_filtered(d_ftxs, n_ftx, d_nodes, n_nodes, d_leaves, n_leaves, d_arena, arena_len, d_status,
                              (uint8_t*)c->ftxws.p, s), "launch_filtered");
  HIP_TRY(order_out(c, s), "hipEventRecord");
  return CG_OK;
}

int cg_verify_filtered(cg_ctx* c, const cg_filtered_tx* ftxs, uint64_t n_ftx, const cg_pmt_node* nodes,
                       uint64_t n_nodes, const cg_filtered_leaf* leaves, uint64_t n_leaves, const uint8_t* arena,
                       uint64_t arena_len, uint8_t* status_out) {
  if (!c) return fail(CG_ERR_ARG, "cg_verify_filtered: ctx is NULL");
  if (n_ftx && (!ftxs || !status_out)) return fail(CG_ERR_ARG, "cg_verify_filtered: NULL buffer");
  if ((n_nodes && !nodes) || (n_leaves && !leaves) || (arena_len && !arena))
    return fail(CG_ERR_ARG, "cg_verify_filtered: NULL table");
  if (n_ftx == 0) return CG_OK;
  std::lock_guard<std::mutex> g(c->mu);
  HIP_TRY(hipSetDevice(c->device), "hipSetDevice");
  hipStream_t s = c->stream;
  HIP_TRY(order_in(c, s), "hipStreamWaitEvent");
  HIP_TRY(c->h_txs.ensure(sizeof(cg_filtered_tx) * n_ftx), "hipMalloc(filtered txs)");
  HIP_TRY(c->h_comps.ensure(sizeof(cg_pmt_node) * (n_nodes ? n_nodes : 1)), "hipMalloc(nodes)");
  HIP_TRY(c->h_sigs.ensure(sizeof(cg_filtered_leaf) * (n_leaves ? n_leaves : 1)), "hipMalloc(leaves)");
  HIP_TRY(c->arena.ensure(((arena_len + 3) & ~(uint64_t)3) + 16), "hipMalloc(arena)");
  HIP_TRY(c->status.ensure(n_ftx), "hipMalloc(status)");
  HIP_TRY(c->ftxws.ensure(cg::ftx_ws_bytes(n_leaves)), "hipMalloc(filtered ws)");
  HIP_TRY(hipMemcpyAsync(c->h_txs.p, ftxs, sizeof(cg_filtered_tx) * n_ftx, hipMemcpyHostToDevice, s), "H2D ftxs");
  if (n_nodes)
    HIP_TRY(hipMemcpyAsync(c->h_comps.p, nodes, sizeof(cg_pmt_node) * n_nodes, hipMemcpyHostToDevice, s), "H2D nodes");
  if (n_leaves)
    HIP_TRY(hipMemcpyAsync(c->h_sigs.p, leaves, sizeof(cg_filtered_leaf) * n_leaves, hipMemcpyHostToDevice, s),
            "H2D leaves");
  if (arena_len) HIP_TRY(hipMemcpyAsync(c->arena.p, arena, arena_len, hipMemcpyHostToDevice, s), "H2D arena");
  HIP_TRY(cg::launch_filtered((const cg_filtered_tx*)c->h_txs.p, n_ftx, (const cg_pmt_node*)c->h_comps.p, n_nodes,
                              (const cg_filtered_leaf*)c->h_sigs.p, n_leaves, (const uint8_t*)c->arena.p, arena_len,
                              (uint8_t*)c->status.p, (uint8_t*)c->ftxws.p, s), "launch_filtered");
  HIP_TRY(hipMemcpyAsync(status_out, c->status.p, n_ftx, hipMemcpyDeviceToHost, s), "D2H status");
  HIP_TRY(hipStreamSynchronize(s), "hipStreamSynchronize");
  return CG_OK;
}

// ---------------------------------------------------------------- several devices (pool.h)
struct cg_pool {
  std::vector<cg_ctx*> ctx;
  std::vector<uint8_t> healthy;
  std::mutex mu;
};

int cg_pool_open(cg_pool** out, const int32_t* devices, uint32_t n_slots, const cg_config* cfg) {
  if (!out) return fail(CG_ERR_ARG, "cg_pool_open: out is NULL");
  *out = nullptr;
  if (n_slots == 0 || !devices) return fail(CG_ERR_ARG, "cg_pool_open: no devices");
  cg_pool* p = new cg_pool();
  for (uint32_t k = 0; k < n_slots; ++k) {
    cg_config c = cfg ? *cfg : cg_config{};
    c.device = devices[k];
    cg_ctx* x = nullptr;
    const int rc = cg_open(&x, &c);
    if (rc != CG_OK) {
      const std::string why = g_err;
      cg_pool_close(p);
      char buf[64];
      snprintf(buf, sizeof buf, "cg_pool_open: slot %u: ", k);
      g_err = buf + why;
      return rc;
    }
    p->ctx.push_back(x);
    p->healthy.push_back(1);
  }
  *out = p;
  return CG_OK;
}

void cg_pool_close(cg_pool* p) {
  if (!p) return;
  for (cg_ctx* c : p->ctx) cg_close(c);
  delete p;
}

uint32_t cg_pool_slots(const cg_pool* p) { return p ? (uint32_t)p->ctx.size() : 0; }

int cg_pool_slot_healthy(const cg_pool* p, uint32_t slot) {
  if (!p || slot >= p->ctx.size()) return -1;
  return p->healthy[slot] ? 1 : 0;
}

int cg_pool_inject_fault(cg_pool* p, uint32_t slot, int on) {
  if (!p || slot >= p->ctx.size()) return fail(CG_ERR_ARG, "cg_pool_inject_fault: bad slot");
  std::lock_guard<std::mutex> g(p->mu);
  std::lock_guard<std::mutex> gc(p->ctx[slot]->mu);
  p->ctx[slot]->fault = on != 0;
  if (!on) p->healthy[slot] = 1;
  return CG_OK;
}

// pool_run over one shard function; stats and the error message as cg_pool_verify_batch
static int pool_call(cg_pool* p, uint64_t n_items, uint8_t* status_out, cg_pool_stats* stats, const char* name,
                     const std::function<int(cg_ctx*, uint64_t, uint64_t)>& shard) {
  const auto t0 = std::chrono::steady_clock::now();
  std::lock_guard<std::mutex> g(p->mu);
  std::vector<std::string> errs(p->ctx.size());
  cg::PoolReport rep;
  const int rc = cg::pool_run(p->healthy, n_items, status_out,
                              [&](uint32_t slot, uint64_t first, uint64_t count) {
                                cg_ctx* c = p->ctx[slot];
                                std::lock_guard<std::mutex> gc(c->mu);
                                const int r = shard(c, first, count);
                                if (r != CG_OK) errs[slot] = g_err;  // g_err is this worker thread's
                                return r;
                              },
                              [&](uint32_t slot) {  // re-probe: no drill fault, the device answers
                                cg_ctx* c = p->ctx[slot];
                                std::lock_guard<std::mutex> gc(c->mu);
                                if (c->fault || hipSetDevice(c->device) != hipSuccess) return false;
                                const hipError_t q = hipStreamQuery(c->stream);
                                return q == hipSuccess || q == hipErrorNotReady;
                              },
                              &rep);
  if (stats) {
    stats->shards = rep.shards;
    stats->reruns = rep.reruns;
    stats->failed_slots = rep.failed_slots;
    stats->reserved = 0;
    stats->not_run = rep.not_run;
    stats->ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  if (rc != CG_OK) {
    std::string m = std::string(name) + (rc == CG_ERR_DEVICE ? ": no healthy slot could run every shard;"
                                                             : ": a shard failed (not a device fault);");
    for (size_t k = 0; k < errs.size(); ++k)
      if (!errs[k].empty()) m += " [slot " + std::to_string(k) + "] " + errs[k];
    g_err = m;
  }
  return rc;
}

int cg_pool_verify_tx_signatures(cg_pool* p, const cg_key* keys, uint32_t n_keys, const uint8_t* ids, uint64_t n_ids,
                                 const cg_txsig* sigs, uint64_t n_sigs, const cg_signable_tmpl* tmpls,
                                 uint32_t n_tmpls, const uint8_t* arena, uint64_t arena_len, uint32_t mode,
                                 uint8_t* status_out, cg_pool_stats* stats) {
  if (!p) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures: pool is NULL");
  if (p->ctx.empty()) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures: empty pool");
  const int a = txsig_args("cg_pool_verify_tx_signatures", p->ctx[0], n_keys, keys, n_ids, ids, n_sigs, sigs,
                           status_out, n_tmpls, tmpls, mode);
  if (a != CG_OK) return a;
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures: arena is NULL");
  return pool_call(p, n_sigs, status_out, stats, "cg_pool_verify_tx_signatures",
                   [&](cg_ctx* c, uint64_t first, uint64_t count) {
                     return verify_txsig_host_locked(c, keys, n_keys, ids, n_ids, sigs + first, count, tmpls, n_tmpls,
                                                     arena, arena_len, mode, status_out + first, nullptr);
                   });
}

// The whole call on one live slot (a signature may reference any transaction's id, so the call is not
// sharded): pool_run over a single unit, i.e. the first live slot, and on a device fault the next one.
int cg_pool_verify_transactions(cg_pool* p, const cg_tx* txs, uint64_t n_tx, const cg_component* comps,
                                uint64_t n_comps, const cg_key* keys, uint32_t n_keys, const cg_txsig* sigs,
                                uint64_t n_sigs, const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* arena,
                                uint64_t arena_len, uint32_t mode, uint8_t* ids_out, uint8_t* tx_status_out,
                                uint8_t* sig_status_out, cg_pool_stats* stats) {
  if (!p) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: pool is NULL");
  if (p->ctx.empty()) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: empty pool");
  if (n_tx && (!txs || !ids_out || !tx_status_out)) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: NULL tx buffer");
  if (n_sigs && (!sigs || !sig_status_out)) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: NULL sig buffer");
  if (n_comps && !comps) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: comps is NULL");
  if (n_keys && !keys) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: keys is NULL");
  if (n_tmpls && !tmpls) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: templates is NULL");
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: arena is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_pool_verify_transactions: bad mode");
  for (uint64_t i = 0; i < n_sigs; ++i) sig_status_out[i] = CG_NOT_RUN;
  if (n_tx == 0 && n_sigs == 0) return CG_OK;
  uint8_t unit = CG_NOT_RUN;
  const int rc = pool_call(p, 1, &unit, stats, "cg_pool_verify_transactions", [&](cg_ctx* c, uint64_t, uint64_t) {
    const int r = verify_transactions_host_locked(c, txs, n_tx, comps, n_comps, keys, n_keys, sigs, n_sigs, tmpls,
                                                  n_tmpls, arena, arena_len, mode, ids_out, tx_status_out,
                                                  sig_status_out);
    if (r != CG_OK)
      for (uint64_t i = 0; i < n_sigs; ++i) sig_status_out[i] = CG_NOT_RUN;
    return r;
  });
  if (stats) stats->not_run = rc == CG_OK ? 0 : n_sigs;
  return rc;
}

int cg_pool_verify_tx_signatures_packed(cg_pool* p, const cg_key* keys, uint32_t n_keys, const uint8_t* ids,
                                        uint64_t n_ids, const cg_txsig_packed* sigs, uint64_t n_sigs,
                                        const uint8_t* sig_bytes, uint64_t sig_bytes_len,
                                        const cg_signable_tmpl* tmpls, uint32_t n_tmpls, const uint8_t* arena,
                                        uint64_t arena_len, uint32_t mode, uint8_t* status_out,
                                        cg_pool_stats* stats) {
  if (!p) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures_packed: pool is NULL");
  if (p->ctx.empty()) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures_packed: empty pool");
  const int a = txsig_args("cg_pool_verify_tx_signatures_packed", p->ctx[0], n_keys, keys, n_ids, ids, n_sigs, sigs,
                           status_out, n_tmpls, tmpls, mode);
  if (a != CG_OK) return a;
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures_packed: arena is NULL");
  if (sig_bytes_len && !sig_bytes) return fail(CG_ERR_ARG, "cg_pool_verify_tx_signatures_packed: sig_bytes is NULL");
  // a shard [first, first + count) starts at the stream offset of record `first`: the sum of the spans
  // before it, in one threaded pass over the table (a prefix per 2^16-record block), looked up per shard
  const uint64_t B = 1u << 16, nb = (n_sigs + B - 1) / B;
  std::vector<uint64_t> blk(nb + 1, 0);
  {
    const unsigned nt = std::max(1u, std::min<unsigned>(16, (unsigned)nb));
    std::vector<std::thread> th;
    for (unsigned t = 0; t < nt; ++t)
      th.emplace_back([&, t] {
        for (uint64_t b = nb * t / nt; b < nb * (t + 1) / nt; ++b) {
          uint64_t sp = 0;
          for (uint64_t i = b * B; i < std::min(n_sigs, (b + 1) * B); ++i) sp += ((uint64_t)sigs[i].sig_len + 3u) & ~(uint64_t)3;
          blk[b + 1] = sp;
        }
      });
    for (std::thread& x : th) x.join();
    for (uint64_t b = 0; b < nb; ++b) blk[b + 1] += blk[b];
  }
  auto stream_at = [&](uint64_t i) {
    uint64_t o = blk[i / B];
    for (uint64_t j = (i / B) * B; j < i; ++j) o += ((uint64_t)sigs[j].sig_len + 3u) & ~(uint64_t)3;
    return o;
  };
  return pool_call(p, n_sigs, status_out, stats, "cg_pool_verify_tx_signatures_packed",
                   [&](cg_ctx* c, uint64_t first, uint64_t count) {
                     const uint64_t o = std::min(stream_at(first), sig_bytes_len);
                     return verify_txsig_host_locked(c, keys, n_keys, ids, n_ids, nullptr, count, tmpls, n_tmpls,
                                                     arena, arena_len, mode, status_out + first, nullptr, sigs + first,
                                                     sig_bytes + o, sig_bytes_len - o);
                   });
}

int cg_pool_verify_batch(cg_pool* p, const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items,
                         const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out,
                         cg_pool_stats* stats) {
  if (!p) return fail(CG_ERR_ARG, "cg_pool_verify_batch: pool is NULL");
  if (n_items && (!items || !status_out)) return fail(CG_ERR_ARG, "cg_pool_verify_batch: NULL buffer");
  if (n_keys && !keys) return fail(CG_ERR_ARG, "cg_pool_verify_batch: keys is NULL");
  if (arena_len && !arena) return fail(CG_ERR_ARG, "cg_pool_verify_batch: arena is NULL");
  if (mode > CG_MODE_ISVALID) return fail(CG_ERR_ARG, "cg_pool_verify_batch: bad mode");
  return pool_call(p, n_items, status_out, stats, "cg_pool_verify_batch", [&](cg_ctx* c, uint64_t first, uint64_t count) {
    return verify_host_locked(c, keys, n_keys, items + first, count, arena, arena_len, mode, status_out + first,
                              nullptr);
  });
}

}  // extern "C"
