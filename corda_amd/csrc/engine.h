// Internal interface between the C ABI host code (cordagpu.cpp) and the HIP kernels.
#pragma once
#include <functional>
#include <stdlib.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "../../include/cordagpu.h"

// Types shared by every build of the kernels. The radix-dependent translation units (verify.hip,
// verify_ed.hip, verify_ec.hip, plan_sort.hip) are compiled once per fixed-base table radix, the extra
// builds with `cg` renamed (Makefile VARIANTS: -Dcg=cg24 / -Dcg=cg22), so these types live in a
// namespace the rename does not touch and the C ABI layer hands the same objects to any build.
namespace cgt {


struct DeviceConsts;  // opaque
// The wide-table pools of a call (keyws.h EdWideSlot / EcWideSlot arrays; host-allocated), one per
// scheme family; caps 0 = no key gets wide tables.
struct WidePool {
  void* ed = nullptr;
  void* ec = nullptr;
  uint32_t cap_ed = 0, cap_ec = 0;
  uint32_t min_ed = 0, min_ec = 0;  // items per key from which a key gets wide tables, per family
};

// Side streams + events owned by a context. Key preparation forks off the caller's stream:
// the two ECDSA curves' tables and the Ed25519 row tables are built on side streams (each is a
// latency-bound chain of doublings on few waves), while the caller's stream goes on with the
// work that needs only decoded keys (the plan, the SHA-512 challenges). Each consumer waits
// for its `ready` event just before it reads tables: ready[0] secp256r1, [1] secp256k1,
// [2] Ed25519.
// Key prep fork: side[0] / side[1] build the secp256r1 / secp256k1 keys (decode -> chain -> tab),
// side[2] the Ed25519 keys; `start` orders them after the main stream's earlier work,
// ec_decoded[c] / ready[c] are what the item kernels on the main stream wait for.
// Item stages: the row-0 ladders (keys with few items, keyws.h) run on the side stream that
// built their class's tables, after `front` (the hashes / ECDSA prep on the main stream), while
// the main stream runs the full-table ladders; the main stream joins on row0[k]. A few row-0
// waves (long: 252 doublings) then overlap the full-table launch instead of trailing it.
// Per-stage timing (cg_config.flags & CG_FLAG_STAGE_TIMING): a pair of events around each stage's
// launches, recorded on the stream the stage runs on, so a stage's duration is measured where it
// ran even when other stages overlap it on other streams. Read (and reset) with cg_stage_times.
struct StageTimer {
  struct Rec {
    int stage;
    hipEvent_t a, b;
  };
  // At most kMaxRecs launches are recorded between two cg_stage_times calls (later launches are
  // not timed); event pairs are recycled through `spare`, so a context that never reads its stage
  // times holds a bounded number of events.
  static constexpr size_t kMaxRecs = 4096;
  std::vector<Rec> recs, spare;
  int mark(int stage, hipStream_t s) {
    if (recs.size() >= kMaxRecs) return -1;
    Rec r{stage, nullptr, nullptr};
    if (!spare.empty()) {
      r.a = spare.back().a;
      r.b = spare.back().b;
      spare.pop_back();
    } else {
      if (hipEventCreate(&r.a) != hipSuccess) return -1;
      if (hipEventCreate(&r.b) != hipSuccess) {
        (void)hipEventDestroy(r.a);
        return -1;
      }
    }
    (void)hipEventRecord(r.a, s);
    recs.push_back(r);
    return (int)recs.size() - 1;
  }
  void done(int idx, hipStream_t s) {
    if (idx >= 0) (void)hipEventRecord(recs[idx].b, s);
  }
};
#define CG_TIME(fork, stage, stream, launch)                                   \
  do {                                                                          \
    const int _t = (fork) && (fork)->timer ? (fork)->timer->mark((stage), (stream)) : -1; \
    launch;                                                                     \
    if (_t >= 0) (fork)->timer->done(_t, (stream));                            \
  } while (0)

// Key-table builds deferred by launch_keyprep until the first chunk's plan is sorted (the sort's
// decoupled look-back stalls when the table builds hold the SIMDs), then enqueued by launch_items.
struct PendingTabs {
  bool on = false;
  bool ec_front_side = false;  // this call's ECDSA fronts run on the side streams (launch_items_front)
  const cg_key* keys = nullptr;
  uint32_t n_keys = 0;
  void* keyprep = nullptr;
  WidePool wide;
  // per side stream (0 r1, 1 k1, 2 Ed25519): whether any key of the family gets row-0 / full
  // tables; false only when the host counts prove none does (KeyUses::host_counts), so the
  // near-empty table launch does not queue behind the wide builds for a slot
  bool need_full[3] = {true, true, true};
  uint32_t skip_mask = 0;  // bit f: !need_full[f] (k_key_classify checks it, k_mode_guard enforces it)
};

struct Fork {
  hipStream_t side[3];
  hipEvent_t start, ec_decoded[2], ready[3], front, row0[3];
  StageTimer* timer;  // null unless the ctx was opened with CG_FLAG_STAGE_TIMING
  hipEvent_t planned = nullptr, ed_tabs = nullptr;  // plan sorted (main); Ed25519 tables built (side[2])
  hipEvent_t chains[3] = {nullptr, nullptr, nullptr};  // each family's row-base chains done (side[k])
  // ECDSA fronts on side[k] (CG_EC_FRONT_SIDE): main's plan done / curve k's front done
  hipEvent_t ec_front_go = nullptr, ec_front_done[2] = {nullptr, nullptr};
  mutable PendingTabs pending;
  hipEvent_t mark = nullptr;  // CG_HOST_TRACE: recorded on the main stream before a back's final joins
  // Host hook launch_items_front runs once between a chunk's plan and its hashes (the host path's
  // CG_SPLIT_COPY: the chunk's signature bytes are copied there, after its plan is enqueued)
  const std::function<hipError_t()>* mid_front = nullptr;
};

// Dynamic LDS reserved by each row-base chain workgroup (CG_CHAIN_SPREAD=1: more than half a CU's
// 160 KB, so no two single-wave chain workgroups share a CU and their latency-bound walks never
// split one SIMD's issue; 0 otherwise). A/B knob.
inline uint32_t chain_spread_lds() {
  static const uint32_t b = [] {
    const char* v = getenv("CG_CHAIN_SPREAD");
    return v && v[0] == '1' ? 82u * 1024u : 0u;
  }();
  return b;
}


// Where the per-key use counts come from when there is no verify-item table yet: a cg_txsig table
// in HBM (sampled on the device) or exact counts (n_keys u32 in HBM, made by the host).
struct KeyUses {
  const cg_txsig* sigs = nullptr;
  const cg_txsig_packed* sigs12 = nullptr;  // or the 12-byte table (cg_verify_tx_signatures_packed_device)
  const uint32_t* counts = nullptr;
  uint64_t n = 0;  // signatures the counts cover (sizes the wide pools)
  // optional host copies of the key table and of `counts` (the host-buffer tx-signature path): the
  // host then knows, as k_key_classify will, which families need row-0 / full tables
  const cg_key* host_keys = nullptr;
  const uint32_t* host_counts = nullptr;
};

// One build of the radix-dependent kernels: the entry points cordagpu.cpp calls through a context's
// variant (cg_config.table_bytes_max picks it at cg_open). Each build defines cg::variant() (renamed
// cg24::variant() / cg22::variant() in the others).
struct EngineVariant {
  uint32_t fixed_base_bits;  // radix 2^bits of the constant B / G tables
  hipError_t (*upload_constants)();
  size_t (*keyprep_bytes)(uint32_t n_keys);
  size_t (*wide_bytes)(uint32_t n_keys, uint64_t n_items, uint32_t max_slots);
  size_t (*wide_slot_bytes)();
  WidePool (*make_wide_pool)(void* base, uint32_t n_keys, uint64_t n_items, uint32_t max_slots);
  size_t (*btab_bytes)();
  size_t (*btab_scratch_bytes)();
  hipError_t (*init_btab)(void* d_btab, void* d_scratch, hipStream_t stream);
  size_t (*item_ws_bytes)(uint64_t n_items);
  hipError_t (*launch_keyprep)(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                               void* d_keyprep, hipStream_t stream, const Fork* fork, const cg_item* d_items,
                               uint64_t n_items, const WidePool* wide, const KeyUses* src);
  hipError_t (*launch_key_tables)(const Fork* fork, hipStream_t stream);
  hipError_t (*launch_items)(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                             const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                             const void* d_keyprep, void* d_item_ws, const void* d_btab, hipStream_t stream,
                             const uint8_t* d_msgs, uint64_t msgs_len, const Fork* fork, const WidePool* wide);
  hipError_t (*launch_items_plan)(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                                  uint8_t* d_status, const void* d_keyprep, void* d_item_ws, hipStream_t stream,
                                  const Fork* fork, const WidePool* wide);
  hipError_t (*launch_items_front)(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                                   const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                                   const void* d_keyprep, void* d_item_ws, hipStream_t stream, const uint8_t* d_msgs,
                                   uint64_t msgs_len, const Fork* fork, const WidePool* wide, bool planned);
  hipError_t (*launch_items_back)(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                                  const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_status, const void* d_keyprep,
                                  void* d_item_ws, const void* d_btab, hipStream_t stream, const Fork* fork,
                                  const WidePool* wide);
};

}  // namespace cgt

namespace cg {

using cgt::EngineVariant;
using cgt::Fork;
using cgt::PendingTabs;
using cgt::StageTimer;
using cgt::WidePool;
using cgt::chain_spread_lds;

// this build's entry points (verify.hip)
const EngineVariant& variant();

// Upload the constant tables (curve constants, base-point tables) for the current device.
hipError_t upload_constants();

// Bytes of per-key workspace for n_keys keys.
size_t keyprep_bytes(uint32_t n_keys);
// Wide-table pools for a call of n_items over n_keys (keyws.h: keys with many items get one table
// row per radix-2^8 digit): bytes, and the pool view over `base` (caps 0 when nothing can be wide).
size_t wide_bytes(uint32_t n_keys, uint64_t n_items, uint32_t max_slots = 8192u);
size_t wide_slot_bytes();  // one Ed25519 + one ECDSA wide slot
constexpr uint32_t kKeyWideMax = 8192u;  // keyws.h KEY_WIDE_MAX (static_assert in verify.hip)
WidePool make_wide_pool(void* base, uint32_t n_keys, uint64_t n_items, uint32_t max_slots = 8192u);

// Enqueue the whole verify pipeline for one batch on `stream`:
//   key prep (one lane per key) -> per-scheme verify (one lane per item) -> status bytes.
hipError_t launch_verify(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                         const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                         void* d_keyprep, void* d_item_ws, const void* d_btab, hipStream_t stream,
                         const uint8_t* d_msgs = nullptr, uint64_t msgs_len = 0, const Fork* fork = nullptr,
                         const WidePool* wide = nullptr);
// Constant base-point row table: size and one-time initialisation (per context).
size_t btab_bytes();
size_t btab_scratch_bytes();  // temporary scratch of init_btab (free once it has run)
hipError_t init_btab(void* d_btab, void* d_scratch, hipStream_t stream);
// Bytes of per-item workspace (projective Ed25519 results awaiting the batched inversion).
size_t item_ws_bytes(uint64_t n_items);
using cgt::KeyUses;
// With `d_items` (or `src`), each key's table is sized by the number of items that use it
// (keyws.h); with neither (cg_prepare_keys_device), every key gets full tables.
hipError_t launch_keyprep(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                          void* d_keyprep, hipStream_t stream, const Fork* fork = nullptr,
                          const cg_item* d_items = nullptr, uint64_t n_items = 0, const WidePool* wide = nullptr,
                          const KeyUses* src = nullptr);
// Start the table builds launch_keyprep deferred (no-op if already started): a host-buffer call
// starts them before it blocks on the first chunk's arena copy, so they overlap that copy.
hipError_t launch_key_tables(const Fork* fork, hipStream_t stream);
// `d_msgs` (optional): the engine's spliced-message workspace, read by items flagged
// CG_ITEM_MSG_WS (keyws.h); caller items never carry that flag.
hipError_t launch_items(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                        const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                        const void* d_keyprep, void* d_item_ws, const void* d_btab, hipStream_t stream,
                        const uint8_t* d_msgs = nullptr, uint64_t msgs_len = 0, const Fork* fork = nullptr,
                        const WidePool* wide = nullptr);
// launch_items in two halves: the front (status checks, plan sort, challenge hashes, ECDSA prep and
// s^-1: needs only the decoded keys) and the back (ladders, finish: need the key tables). Between the
// two a caller with a second item workspace may enqueue the next chunk's front, so the first chunk's
// wait for the key tables is spent on the second chunk's fronts (cordagpu.cpp launch_chunked).
// The front's plan sort can be enqueued on its own first (`planned` = true then skips it in the
// front): onesweep's decoupled look-back stalls when the table builds hold the SIMDs, so a caller
// with two chunks sorts both before the first front starts the table builds.
hipError_t launch_items_plan(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                             uint8_t* d_status, const void* d_keyprep, void* d_item_ws, hipStream_t stream,
                             const Fork* fork, const WidePool* wide);
hipError_t launch_items_front(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                              const uint8_t* d_arena, uint64_t arena_len, uint32_t mode, uint8_t* d_status,
                              const void* d_keyprep, void* d_item_ws, hipStream_t stream, const uint8_t* d_msgs,
                              uint64_t msgs_len, const Fork* fork, const WidePool* wide, bool planned);
hipError_t launch_items_back(const cg_key* d_keys, uint32_t n_keys, const cg_item* d_items, uint64_t n_items,
                             const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_status, const void* d_keyprep,
                             void* d_item_ws, const void* d_btab, hipStream_t stream, const Fork* fork,
                             const WidePool* wide);

// Hashing kernels
hipError_t launch_sha256(const cg_span* d_spans, uint64_t n, const uint8_t* d_arena, uint64_t arena_len,
                         uint8_t* d_out, hipStream_t stream);
hipError_t launch_sha512(const cg_span* d_spans, uint64_t n, const uint8_t* d_arena, uint64_t arena_len,
                         uint8_t* d_out, hipStream_t stream);

// WireTransaction ids: leaf hashing + per-tx Merkle levels. `d_leaf_ws` must hold
// tx_ws_bytes(n_comps) bytes.
size_t tx_ws_bytes(uint64_t n_comps);
hipError_t launch_tx_ids(const cg_tx* d_txs, uint64_t n_tx, const cg_component* d_comps, uint64_t n_comps,
                         const uint8_t* d_arena, uint64_t arena_len, uint8_t* d_ids, uint8_t* d_status,
                         uint8_t* d_leaf_ws, hipStream_t stream);

// Transaction pipeline: per-signature verify items over SignableData splices. d_msgs (the message
// workspace, tx_msgs_head(n_tmpls, slot) bytes) holds the splice header, the templates' SHA-256
// midstates and their images (`slot` bytes each, a multiple of 16); no message is materialised.
uint64_t tx_msgs_head(uint32_t n_tmpls, uint64_t slot);
hipError_t launch_tx_sig_items(const cg_txsig* d_sigs, uint64_t n_sigs, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               const uint8_t* d_arena, uint64_t arena_len, uint64_t slot, cg_item* d_items,
                               uint8_t* d_msgs, hipStream_t stream);
// The same in two steps: the templates' midstates + images once per call (tx_sig_templates), then
// any contiguous range [first, first + n) of the signatures (tx_sig_range: its verify items and
// spliced messages; every signature keeps its own message slot).
hipError_t launch_tx_sig_templates(const cg_signable_tmpl* d_tmpls, uint32_t n_tmpls, const uint8_t* d_arena,
                                   uint64_t arena_len, uint64_t slot, const uint8_t* d_ids, uint64_t n_ids,
                                   uint8_t* d_msgs, hipStream_t stream);
hipError_t launch_tx_sig_range(const cg_txsig* d_sigs, uint64_t first, uint64_t n, const cg_signable_tmpl* d_tmpls,
                               uint32_t n_tmpls, const uint8_t* d_tx_status, uint64_t n_tx, const uint8_t* d_ids,
                               uint64_t arena_len, uint64_t slot, cg_item* d_items, uint8_t* d_msgs,
                               hipStream_t stream);

// The 12-byte signature table (cg_txsig_packed): records [first, first + n) become verify items like
// launch_tx_sig_range's, each signature's offset recovered by a prefix scan of round_up(sig_len, 4):
// per 256-record block sums, an exclusive scan of those, then each block's own scan in the item kernel.
// Signature j sits at sig_region + (offset of j in the signature stream) in the arena; one that runs
// past sig_bytes_len of the stream gets CG_NOT_RUN. Either
// `d_bases` holds the stream offset of every 256-record block of the whole table (tx_sig12_bases over
// [0, n_all); `first` must then be a multiple of 256), or the range's blocks are summed and scanned
// here, starting at stream offset `base`, into d_scratch (tx_sig12_scratch_bytes(n) bytes).
size_t tx_sig12_scratch_bytes(uint64_t n);
hipError_t launch_tx_sig12_bases(const cg_txsig_packed* d_sigs, uint64_t first, uint64_t n, uint64_t base,
                                 uint64_t* d_bases, hipStream_t stream);
hipError_t launch_tx_sig12_range(const cg_txsig_packed* d_sigs, uint64_t first, uint64_t n, uint64_t sig_region,
                                 uint64_t sig_bytes_len, uint64_t base, const uint64_t* d_bases,
                                 const cg_signable_tmpl* d_tmpls,
                                 uint32_t n_tmpls, uint64_t n_tx, uint64_t arena_len, cg_item* d_items,
                                 void* d_scratch, hipStream_t stream);

// Merkle roots over independent leaf lists.
hipError_t launch_merkle_roots(const uint8_t* d_leaves, const uint64_t* d_first, const uint32_t* d_count,
                               uint64_t n, uint8_t* d_roots, uint8_t* d_status, uint8_t* d_ws,
                               const uint64_t* d_wsoff, hipStream_t stream);

// Tear-offs (filtered.hip): leaf hashes, then one lane per filtered transaction. `d_ws` must
// hold ftx_ws_bytes(n_leaves) bytes.
size_t ftx_ws_bytes(uint64_t n_leaves);
hipError_t launch_filtered(const cg_filtered_tx* d_ftxs, uint64_t n_ftx, const cg_pmt_node* d_nodes, uint64_t n_nodes,
                           const cg_filtered_leaf* d_leaves, uint64_t n_leaves, const uint8_t* d_arena,
                           uint64_t arena_len, uint8_t* d_status, uint8_t* d_ws, hipStream_t stream);

}  // namespace cg
