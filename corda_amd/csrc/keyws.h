// Shared layout of the per-key and per-item device workspaces and the constant tables, used
// by the Ed25519 (verify_ed.hip), ECDSA (verify_ec.hip) and dispatch (verify.hip) units.
#pragma once
#include <hip/hip_runtime.h>

#include "ecdsa.h"
#include "ecdsa_rows.h"
#include "ed25519.h"
#include "ed25519_rows.h"
#include "engine.h"
#include "sha2.h"

namespace cg {

__device__ __forceinline__ uint64_t round4(uint64_t x) { return (x + 3) & ~(uint64_t)3; }

// Persistent, XCD-grouped walk over `n` work units starting at plan position `beg` (a unit is
// `per` consecutive positions: 1 for the one-lane-per-item stages, K for the batched
// inversions). Blocks b and b + 8 share an XCD (round-robin dealing, MI355X_MICROARCH.md
// "Workgroup dispatch"), so group g = b % 8 walks the contiguous g-th eighth of the range with
// its blocks strided by blockDim lanes: at any moment one XCD's lanes run adjacent, key-sorted
// positions and share that XCD's L2 for the key's rows. The grid is capped on the host
// (walk_grid), so a stage whose range is empty costs a few hundred exiting blocks, not
// n_items / 256 of them, and never competes for dispatch with a concurrent ladder.
#define CG_XCDS 8u
struct Walk {
  uint64_t u, end, step;
};
__device__ __forceinline__ Walk walk_units(uint64_t n) {
  const uint32_t groups = gridDim.x >= CG_XCDS ? CG_XCDS : 1u;
  const uint32_t g = blockIdx.x % groups;
  const uint32_t bpg = gridDim.x / groups;  // walk_grid makes gridDim.x a multiple of 8
  const uint64_t span = (n + groups - 1) / groups;
  const uint64_t lo = (uint64_t)g * span;
  const uint64_t hi = lo + span < n ? lo + span : n;
  Walk w;
  w.u = lo + (uint64_t)(blockIdx.x / groups) * blockDim.x + threadIdx.x;
  w.end = hi;
  w.step = (uint64_t)bpg * blockDim.x;
  return w;
}
// Grid for a walk: enough blocks for `units` (one lane each), at most `cap`, a multiple of 8.
static inline unsigned walk_grid(uint64_t units, uint32_t block, uint32_t cap) {
  uint64_t g = (units + block - 1) / block;
  if (g > cap) g = cap;
  g = (g + CG_XCDS - 1) / CG_XCDS * CG_XCDS;
  return (unsigned)(g ? g : CG_XCDS);
}
// Grid cap for a 256-lane-block stage at `waves_per_simd`: the resident blocks of the chip
// (256 CUs x 4 SIMDs x waves / 4 waves per block) times 2, so a block that finishes early
// (invalid items exit at once) is replaced. Resident blocks of one XCD still run one contiguous
// window of positions per iteration, so the cap does not cost L2 locality.
#define CG_CUS 256u
#define WALK_CAP(waves_per_simd) (CG_CUS * (waves_per_simd) * 2u)

__device__ __forceinline__ bool in_arena(uint64_t off, uint64_t len, uint64_t arena_len) {
  return off <= arena_len && len <= arena_len - off;
}

// Item flag (cg_item.reserved0, set only by the engine's own pipelines): the clear data lives
// in the engine's spliced-message workspace, not in the caller's arena. Launches without that
// workspace (every caller-facing entry point) pass msgs = nullptr, and the flag is ignored.
#define CG_ITEM_MSG_WS 1u
// With CG_ITEM_MSG_WS: the message is a SignableData splice of template reserved1, whose SHA-256
// midstate record (the template prefix's full 64-byte blocks) heads the message workspace.
#define CG_ITEM_TMPL 2u
// With CG_ITEM_MSG_WS | CG_ITEM_TMPL: the message is never materialised; msg_off is the tx index and
// the hash kernels read the splice through SpliceLd (sha2.h) from the workspace head below.
#define CG_ITEM_FUSED 4u
// Message workspace head (cg_verify_tx_signatures*, cg_verify_transactions*):
//   [SpliceHdr, 256 B][TmplMid x n_tmpls, 256-aligned][TmplW512 x n_tmpls][template images: n_tmpls x slot]
struct SpliceHdr {
  uint64_t ids;       // device address of the 32-byte ids
  uint64_t n_ids;
  uint64_t img_off;   // byte offset of the images in the workspace
  uint64_t slot;      // bytes per image: round16(longest prefix + 32 + suffix), zero-filled past the
                      // image (SpliceLd's aligned 16-byte reads past img_len see zeros)
  uint64_t w512_off;  // byte offset of the TmplW512 records
};
#define SPLICE_HDR_BYTES 256u
struct TmplMid {
  uint32_t state[8];
  uint32_t blocks;      // prefix blocks absorbed into state
  uint32_t prefix_len;  // the id's position in the message
  uint32_t ed_mid;      // 1: the template's TmplW512 record holds the Ed25519 challenge's block 1
  uint32_t pad;
};
static_assert(sizeof(TmplMid) == 48, "template midstate record");
// SHA-512(R || Abyte || M)'s block 1 is M[64, 192): with the id at prefix_len >= 192 it is template
// prefix for every signature of the template, so its message schedule, round constants folded in
// (wk[t] = W[t] + K[t]), is computed once per template (k_tmpl_prep) and k_ed_hash runs that block's
// 80 rounds without the schedule (sha512_compress_wk).
struct TmplW512 {
  uint64_t wk[80];
};
#define TMPL_ED_MID_MIN_PREFIX 192u
CG_HD uint64_t tmpl_w512_off(uint32_t n_tmpls) {
  return SPLICE_HDR_BYTES + (((uint64_t)n_tmpls * sizeof(TmplMid) + 255) & ~(uint64_t)255);
}
CG_HD uint64_t tmpl_mid_bytes(uint32_t n_tmpls) { return tmpl_w512_off(n_tmpls) + (uint64_t)n_tmpls * sizeof(TmplW512); }
__device__ __forceinline__ bool item_fused(const cg_item& it, const uint8_t* msgs) {
  return msgs && (it.reserved0 & (CG_ITEM_MSG_WS | CG_ITEM_TMPL | CG_ITEM_FUSED)) ==
                     (CG_ITEM_MSG_WS | CG_ITEM_TMPL | CG_ITEM_FUSED);
}
__device__ __forceinline__ const TmplMid* item_tmpl_mid(const cg_item& it, const uint8_t* msgs) {
  return (it.reserved0 & CG_ITEM_TMPL) && (it.reserved0 & CG_ITEM_MSG_WS) && msgs
             ? (const TmplMid*)(msgs + SPLICE_HDR_BYTES) + it.reserved1
             : nullptr;
}
// The splice of template `tmpl` with tx id `tx` (a fused item: tmpl = reserved1, tx = msg_off). With a
// wave-uniform tmpl the image address, length and id position are scalars, so SpliceLd's bounds and
// overlap tests are scalar branches; only the id words are per lane.
__device__ __forceinline__ SpliceLd tmpl_splice(uint32_t tmpl, uint64_t tx, const uint8_t* msgs) {
  const SpliceHdr* h = (const SpliceHdr*)msgs;
  const TmplMid* m = (const TmplMid*)(msgs + SPLICE_HDR_BYTES) + tmpl;
  SpliceLd ld;
  ld.img = msgs + h->img_off + (uint64_t)tmpl * h->slot;
  ld.img_len = h->slot;
  ld.id = (const uint32_t*)(uintptr_t)h->ids + 8ull * tx;
  ld.at = m->prefix_len;
  return ld;
}
__device__ __forceinline__ SpliceLd item_splice(const cg_item& it, const uint8_t* msgs) {
  return tmpl_splice(it.reserved1, it.msg_off, msgs);
}
__device__ __forceinline__ bool item_in_ws(const cg_item& it, const uint8_t* msgs) {
  return (it.reserved0 & CG_ITEM_MSG_WS) && msgs != nullptr;
}
__device__ __forceinline__ const uint8_t* item_msg_arena(const cg_item& it, const uint8_t* arena,
                                                         const uint8_t* msgs) {
  return item_in_ws(it, msgs) ? msgs : arena;
}
__device__ __forceinline__ uint64_t item_msg_len(const cg_item& it, uint64_t arena_len, uint64_t msgs_len,
                                                 const uint8_t* msgs) {
  return item_in_ws(it, msgs) ? msgs_len : arena_len;
}

// Row tables (ed25519_rows.h) with signed radix-64 digits: 43 digits in 11 rows of 4 windows.
typedef EdRowsCfg<ED_W, ED_K> EdCfg;
typedef EdRowTabW<ED_W, ED_K> EdTab;  // 22 x 32 affine niels = 84480 B
// The quarter tables (keys with KEY_QUARTER_MIN_USES .. ED_DIRECT_MAX_USES - 1 items): the same
// radix-2^6 digits in ED_QK windows per row, so 4 rows (row j = multiples of 2^{66 j} (-A)) and
// 60 doublings per item, stored in the first 4 rows of the key's EdTab (a key has one mode).
#ifndef ED_QK
#define ED_QK 11
#endif
typedef EdRowsCfg<ED_W, ED_QK> EdQCfg;
typedef EdRowTabW<ED_W, ED_QK> EdQTab;
static_assert(EdQCfg::kRows <= EdCfg::kRows && EdQCfg::kMult == EdCfg::kMult, "quarter rows fit the full table");
// base slots per key, one stride for both schemes (Ed25519 rows >= ECDSA rows)
#define KEY_BASES (EdCfg::kRows > EC_ROWS ? EdCfg::kRows : EC_ROWS)
static_assert(EC_QROWS <= EC_ROWS, "ECDSA quarter rows fit the full table");
typedef EdBCfg<ED_W, ED_K, ED_WB> EdBCfgT;
typedef EdBTabW<ED_W, ED_K, ED_WB> EdBTab;  // 26 x 512 affine niels = 1.6 MB, constant

// Row-base chains are latency-bound single waves (a key's doublings are one dependent sequence);
// beside the throughput-bound row builds they got a fraction of their SIMD's issue and ran ~4x
// slower (profiles/r03/env_copyq). CG_CHAIN_PRIO (default 1): the chain waves raise their issue
// priority, so a build wave on the same SIMD issues only in their stall cycles.
#ifndef CG_CHAIN_PRIO
#define CG_CHAIN_PRIO 1
#endif
__device__ __forceinline__ void chain_prio() {
#if CG_CHAIN_PRIO
  __builtin_amdgcn_s_setprio(3);
#endif
}

// CG_FRONT_PRIO (A/B): the per-chunk front kernels (item build, plan, challenge hashes, ECDSA prep
// and s^-1) raise their issue priority, so the first chunk's front is not slowed by the key-table
// builds it shares the chip with (its ladders wait for both).
#ifndef CG_FRONT_PRIO
#define CG_FRONT_PRIO 0
#endif
__device__ __forceinline__ void front_prio() {
#if CG_FRONT_PRIO
  __builtin_amdgcn_s_setprio(CG_FRONT_PRIO);
#endif
}

// Per-key header: status (0 = decoded) and, for Ed25519, the canonical Abyte i2p hashes.
struct EdKeyHdr {
  uint32_t status;
  uint32_t abyte[8];
  uint32_t pad[7];
};

// A key is either Ed25519 or ECDSA: its table and row-base slots are shared.
union TabSlot {
  EdTab ed;
  EcRowTab ec;
};
union BaseSlot {
  ge_p3 ed;
  Jac ec;
};

// Per-batch plan (plan_sort.hip): item indices sorted by (scheme class, key). Each scheme's
// kernels walk one dense range of `perm`, so no lane idles on another scheme's item; the
// per-item workspace is indexed by plan position.
#define PLAN_ED 0
#define PLAN_R1 1
#define PLAN_K1 2
#define PLAN_CLASSES 3
#define PLAN_FULL 4  // ranges[PLAN_FULL + c]: first item of class c whose key has full tables
#define PLAN_WIDE 7  // ranges[PLAN_WIDE + c]: first item of class c whose key has wide tables
#define PLAN_QUART 10  // ranges[PLAN_QUART + c]: first item of class c whose key has quarter tables
// Table-mode order inside a class (the plan's 2 mode bits): row 0, quarter, full, wide.
#define PLAN_MODE_ROW0 0u
#define PLAN_MODE_QUART 1u
#define PLAN_MODE_FULL 2u
#define PLAN_MODE_WIDE 3u
// Items whose clear data is longer than this sort after the short ones of their class and table
// mode (plan_sort.hip), so a wave hashes either short or long messages, never both.
#define ITEM_LONG_MIN 1024u
struct Plan {
  const uint32_t* perm;    // plan position -> item index
  const uint32_t* ranges;  // class c occupies positions [ranges[c], ranges[c + 1])
};
__device__ __forceinline__ int plan_class_of_curve(int curve) { return curve == 1 ? PLAN_R1 : PLAN_K1; }

// Key workspace, each region n_keys long (a key is either Ed25519 or ECDSA, so the table and
// base slots are shared: TabSlot / BaseSlot unions give one stride for both schemes):
//   hdr      EdKeyHdr (status [+ Abyte])                       64 B
//   tab      EdTab | EcRowTab                                  84 480 B
//   bases    KEY_BASES = 22 x (ge_p3 | Jac)                    3 520 B
// and, per family, the full / row-0 builds' park (ed_row_build_parked / ec_row_build_parked): one
// lane-interleaved region of min(n_keys x rows, TAB_PARK_LANES) lanes, the build kernels' grid
// (each lane loops over the compacted (key, row) tasks), 5 120 B (Ed25519) / 4 608 B (ECDSA) a lane.
static inline size_t al256(size_t x) { return (x + 255) & ~(size_t)255; }
#define TAB_PARK_LANES 131072u  // 2 waves per SIMD on 1024 SIMDs
static inline uint32_t tab_park_lanes(uint32_t n_keys, uint32_t rows) {
  uint64_t l = (uint64_t)(n_keys ? n_keys : 1) * rows;
  if (l > TAB_PARK_LANES) l = TAB_PARK_LANES;
  return (uint32_t)((l + 63) & ~(uint64_t)63);
}
#define ED_ROW_PARK_BYTES ((size_t)EdCfg::kMult * ED_PARK_DWORDS * 4)
#define EC_ROW_PARK_BYTES ((size_t)EC_MULT * EC_ROW_PARK * 4)
#define ROW0_COUNT_AT 8    // row0_count = full_count + 8 (the 256-B count block)
#define QUART_COUNT_AT 16  // quart_count = full_count + 16
// full_count[SKIP_MISMATCH_AT], bit f (0 secp256r1, 1 secp256k1, 2 Ed25519): k_key_classify put a
// key of family f in row-0 / quarter / full mode although the host's counts skipped that family's
// row-0 / quarter / full builds and ladders (families_needing_full): k_mode_guard then reports its
// items CG_NOT_RUN instead of verdicts from stale tables
#define SKIP_MISMATCH_AT 24
struct KeyWs {
  EdKeyHdr* hdr;
  TabSlot* tab;
  BaseSlot* bases;
  uint32_t* park_ed;     // full / row-0 build park, Ed25519 (park_lanes_ed lanes)
  uint32_t* park_ec[2];  // [CG_CURVE_K1], [CG_CURVE_R1] (park_lanes_ec lanes each)
  uint32_t park_lanes_ed, park_lanes_ec;
  uint32_t* uses;  // items per key in this batch, saturating at >= ED_DIRECT_MAX_USES
                   // (KEY_USES_ALL: unknown -> full tables)
  uint32_t* full;  // per scheme class c (PLAN_ED / PLAN_R1 / PLAN_K1): the keys that get full
                   // tables, full[c * n_keys + l] for l < full_count[c] (any order), so the
                   // chain / row kernels run dense lanes however few keys are hot
  uint32_t* full_count;
  uint32_t* row0;        // per class c: every used key without wide tables (its row 0 is built),
  uint32_t* row0_count;  // row0[c * n_keys + l] for l < row0_count[c] (= full_count + ROW0_COUNT_AT)
  uint32_t* quart;       // per class c: the keys with quarter tables (rows 1..3 built after row 0)
  uint32_t* quart_count;  // (= full_count + QUART_COUNT_AT)
  uint8_t* seen;   // 1 if any item of the batch uses the key (exact; uses is sampled)
  uint32_t* wide_idx;    // per key: its slot in the scheme's wide pool, or KEY_NOT_WIDE
  uint32_t* wide;        // per class c: the keys with wide tables, wide[c * n_keys + l]
  uint32_t* wide_count;  // [c] list lengths; [PLAN_CLASSES + 0 / 1] slots taken in the Ed / EC pool
  struct EdWideSlot* wed;  // wide pools (WidePool; empty: no key gets wide tables)
  struct EcWideSlot* wec;
  uint32_t cap_ed, cap_ec;
  uint32_t min_ed, min_ec;
  // the counting plan (plan_sort.hip): per key its ticket in its (class, mode, short / long) group
  // (2n), the per-chunk bucket counts and their exclusive scan by bucket rank (2n + 1 each, plus
  // one scan partial per 16k-bucket tile), and 64 words of group counts [0, 32) / group bases [32, 64)
  uint32_t* pl_tick;
  uint32_t* pl_cnt;
  uint32_t* pl_pos;
  uint32_t* pl_tile;
  uint32_t* pl_grp;
};
#define PL_TILE 16384u  // buckets per scan tile (1024 threads x 16)
static inline size_t pl_buckets(uint32_t n_keys) { return 2 * (size_t)(n_keys ? n_keys : 1) + 1; }
static inline size_t pl_tiles(uint32_t n_keys) { return (pl_buckets(n_keys) + PL_TILE - 1) / PL_TILE; }

// How much table a key gets, from the number of items that use it in the batch (one-shot entry
// points estimate it from a hashed 1-in-KEY_USES_SAMPLE sample of the items, plus an exact
// "used at all" flag;
// cg_prepare_keys_device cannot, and builds every key in full). The mode changes only speed,
// never a verdict: both ladders compute the same point.
//   0 uses                        decode only (Abyte, status), no rows
//   1 .. KEY_QUARTER_MIN_USES - 1 row 0 only (the 32 affine multiples of -A): the item runs the
//                                 252-doubling Horner ladder (ed_double_scalar_row0)
//   .. ED_DIRECT_MAX_USES - 1     quarter: 4 rows, 60 doublings per item (ed_double_scalar_fw over
//                                 EdQTab; ECDSA: EC_QROWS rows, ecdsa_ladder_check_w). Round 4: the
//                                 2^20-distinct-key leg (~12 uses a key) went 65 -> 90 M sigs/s
//                                 with quarter rows instead of row 0 (profiles/r04/kd)
//   more                          all 22 rows: 6 doublings per item (ed_double_scalar_wb)
// Break-even (measured on MI355X, 2^20 Ed25519 items): a key's full tables cost ~230 ns of
// GPU time, the row-0 ladder ~7 ns more per item than the full-table one -> ~32 items.
// A fourth mode, for keys with >= KEY_WIDE_MIN_USES_{ED,EC} items (and a free slot in the family's
// wide pool, sized by the host from the call's item count): one table row per signed radix-2^8
// digit (ed25519_rows.h / ecdsa_rows.h "wide tables"), 54 additions and no doublings per item.
// Break-even, measured on MI355X: a wide table costs ~1.2 us (Ed25519) / ~1 us
// (ECDSA) of chip time to build and saves ~0.64 ns (Ed25519) / ~2 ns (ECDSA) per item against the
// full tables, so ~1900 / ~500 items. (Environment CG_WIDE_MIN_USES_ED / _EC override, for A/B.)
#ifndef KEY_WIDE_MIN_USES_ED
#define KEY_WIDE_MIN_USES_ED 1536u
#endif
#ifndef KEY_WIDE_MIN_USES_EC
#define KEY_WIDE_MIN_USES_EC 512u
#endif
#define KEY_WIDE_MIN_USES (KEY_WIDE_MIN_USES_EC < KEY_WIDE_MIN_USES_ED ? KEY_WIDE_MIN_USES_EC : KEY_WIDE_MIN_USES_ED)
#define KEY_NOT_WIDE 0xffffffffu
#define KEY_WIDE_MAX 8192u  // wide slots per pool at most (Ed25519 9.4 GB / ECDSA 6.3 GB)
#define KEY_USES_ALL 0xffffffffu
#define KEY_USES_SAMPLE 4u  // k_key_uses samples by the top 2 bits of a 32-bit hash: 1 in 4
#ifndef KEY_QUARTER_MIN_USES
#define KEY_QUARTER_MIN_USES 3u
#endif
#ifndef ED_DIRECT_MAX_USES
#define ED_DIRECT_MAX_USES 32u
#endif
// Wide-table slot of one key: the table, its row bases and the row builds' scratch. The one-lane-
// per-row builds park every multiple's un-normalised coordinates between their two walks in
// `park`, lane-interleaved (dword d of entry i of row lane t at park[(i * fields + d) * lanes + t]:
// one store of a wave is 64 consecutive dwords, where parking in the entries themselves made every
// store touch 64 cache lines: the builds ran at about a third of their compute rate).
struct EdWideSlot {
  EdWideTab tab;
  ge_p3 bases[EdWideCfg::kRows];
  union {
    fe zpre[EdWideCfg::kRows][EdWideCfg::kMult];                       // three-pass build
    uint32_t park[EdWideCfg::kRows * EdWideCfg::kMult * ED_PARK_DWORDS];  // row-lane build
  };
};
struct EcWideSlot {
  EcWideTab tab;
  EcAff bases[EC_WIDE_DIGITS];  // 2^{8j} Q, affine (the row builds step by mixed additions)
  Jac jbases[EC_WIDE_DIGITS];   // the chain's Jacobian points
  union {
    EcWideScratch s[EC_WIDE_ROWS];                                 // three-pass build, the chain
    uint32_t park[EC_WIDE_ROWS * EC_WIDE_MULT * EC_PARK_DWORDS];   // row-lane build
  };
};
// Slots for a call of n_items over n_keys: no more keys can reach KEY_WIDE_MIN_USES.
// max_slots: the context's device-memory cap (cordagpu.cpp ensure_ws: ADVICE r3).
static inline uint32_t wide_cap(uint32_t n_keys, uint64_t n_items, uint32_t max_slots = KEY_WIDE_MAX,
                                uint32_t min_uses = KEY_WIDE_MIN_USES) {
  uint64_t c = n_items / min_uses;
  if (c > n_keys) c = n_keys;
  if (c > KEY_WIDE_MAX) c = KEY_WIDE_MAX;
  if (c > max_slots) c = max_slots;
  return (uint32_t)c;
}
static inline size_t wide_pool_bytes(uint32_t cap) {
  return cap ? al256((size_t)cap * sizeof(EdWideSlot)) + al256((size_t)cap * sizeof(EcWideSlot)) : 0;
}
static inline WidePool wide_pool(void* base, uint32_t cap) {
  WidePool p;
  p.min_ed = KEY_WIDE_MIN_USES_ED;
  p.min_ec = KEY_WIDE_MIN_USES_EC;
  if (!base || !cap) return p;
  p.ed = base;
  p.ec = (uint8_t*)base + al256((size_t)cap * sizeof(EdWideSlot));
  p.cap_ed = p.cap_ec = cap;
  return p;
}

static inline KeyWs key_ws(void* base, uint32_t n_keys, const WidePool* wp = nullptr) {
  const size_t n = n_keys ? n_keys : 1;
  uint8_t* p = (uint8_t*)base;
  KeyWs w;
  w.hdr = (EdKeyHdr*)p;
  p += al256(n * sizeof(EdKeyHdr));
  w.tab = (TabSlot*)p;
  p += al256(n * sizeof(TabSlot));
  w.bases = (BaseSlot*)p;
  p += al256(n * KEY_BASES * sizeof(BaseSlot));
  w.park_lanes_ed = tab_park_lanes(n_keys, EdCfg::kRows);
  w.park_lanes_ec = tab_park_lanes(n_keys, EC_ROWS);
  w.park_ed = (uint32_t*)p;
  p += al256(w.park_lanes_ed * ED_ROW_PARK_BYTES);
  for (int c = 0; c < 2; ++c) {
    w.park_ec[c] = (uint32_t*)p;
    p += al256(w.park_lanes_ec * EC_ROW_PARK_BYTES);
  }
  w.uses = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.full = (uint32_t*)p;
  p += al256(3 * n * sizeof(uint32_t));
  w.full_count = (uint32_t*)p;
  w.row0_count = w.full_count + ROW0_COUNT_AT;
  p += 256;
  w.quart_count = w.full_count + QUART_COUNT_AT;
  w.row0 = (uint32_t*)p;
  p += al256(3 * n * sizeof(uint32_t));
  w.quart = (uint32_t*)p;
  p += al256(3 * n * sizeof(uint32_t));
  w.seen = p;
  p += al256(n);
  w.wide_idx = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.wide = (uint32_t*)p;
  p += al256(3 * n * sizeof(uint32_t));
  w.wide_count = (uint32_t*)p;
  p += 256;
  w.pl_tick = (uint32_t*)p;
  p += al256(2 * n * sizeof(uint32_t));
  w.pl_cnt = (uint32_t*)p;
  p += al256(pl_buckets(n_keys) * sizeof(uint32_t));
  w.pl_pos = (uint32_t*)p;
  p += al256(pl_buckets(n_keys) * sizeof(uint32_t));
  w.pl_tile = (uint32_t*)p;
  p += al256(pl_tiles(n_keys) * sizeof(uint32_t));
  w.pl_grp = (uint32_t*)p;
  w.wed = wp ? (EdWideSlot*)wp->ed : nullptr;
  w.wec = wp ? (EcWideSlot*)wp->ec : nullptr;
  w.cap_ed = wp ? wp->cap_ed : 0;
  w.cap_ec = wp ? wp->cap_ec : 0;
  w.min_ed = wp && wp->min_ed ? wp->min_ed : KEY_WIDE_MIN_USES_ED;
  w.min_ec = wp && wp->min_ec ? wp->min_ec : KEY_WIDE_MIN_USES_EC;
  return w;
}
static inline size_t key_ws_bytes(uint32_t n_keys) {
  const size_t n = n_keys ? n_keys : 1;
  return al256(n * sizeof(EdKeyHdr)) + al256(n * sizeof(TabSlot)) + al256(n * KEY_BASES * sizeof(BaseSlot)) +
         al256(tab_park_lanes(n_keys, EdCfg::kRows) * ED_ROW_PARK_BYTES) +
         2 * al256(tab_park_lanes(n_keys, EC_ROWS) * EC_ROW_PARK_BYTES) + al256(n * sizeof(uint32_t)) +
         al256(3 * n * sizeof(uint32_t)) + 256 + 2 * al256(3 * n * sizeof(uint32_t)) + al256(n) +
         al256(n * sizeof(uint32_t)) + al256(3 * n * sizeof(uint32_t)) + 256 + al256(2 * n * sizeof(uint32_t)) +
         2 * al256(pl_buckets(n_keys) * sizeof(uint32_t)) + al256(pl_tiles(n_keys) * sizeof(uint32_t)) + 256;
}

// Per-item workspace slot (indexed by plan position, so the schemes never share one):
// projective Ed25519 R' awaiting the batched inversion, or the ECDSA stage hand-off.
constexpr size_t ITEM_SLOT = sizeof(ge_p2);
static_assert(sizeof(EcItemWs) == ITEM_SLOT, "ECDSA stage hand-off must fill one item slot");
// Item workspace: [slots: n x ITEM_SLOT, by plan position][perm: n x u32][ranges]
//                 [sort keys in/out, sort values in: 3 x n x u32][radix-sort temporary storage]
size_t plan_sort_temp_bytes(uint64_t n_items);  // plan_sort.hip
// Plan-ordered Ed25519 columns k_ed_hash writes for the ladders and the finish, so that they read
// coalesced instead of items[perm[p]] / status[perm[p]] / the signature's R in the arena (a cache
// line each per item: k_ed_finish moved 650 B per item at 0.48 of its issue rate,
// profiles/r03/v14/pmc_traffic.json): R's 8 words (word w of position p at r[w * n + p]), the
// pending flag, the key index.
struct EdCols {
  uint32_t* r;
  uint8_t* pend;
  uint32_t* key;
  uint64_t n;
};
struct ItemWs {
  void* slots;
  uint32_t* perm;
  uint32_t* ranges;
  uint32_t *skey_in, *skey_out, *sval_in;
  void* sort_temp;
  size_t sort_temp_bytes;
  EdCols ed;
};
static inline ItemWs item_ws(void* base, uint64_t n_items) {
  const size_t n = n_items ? n_items : 1;
  uint8_t* p = (uint8_t*)base;
  ItemWs w;
  w.slots = p;
  p += al256(n * ITEM_SLOT);
  w.perm = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.ranges = (uint32_t*)p;
  p += 256;
  w.skey_in = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.skey_out = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.sval_in = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.sort_temp = p;
  w.sort_temp_bytes = plan_sort_temp_bytes(n);
  p += al256(w.sort_temp_bytes);
  w.ed.n = n;
  w.ed.r = (uint32_t*)p;
  p += al256(8 * n * sizeof(uint32_t));
  w.ed.key = (uint32_t*)p;
  p += al256(n * sizeof(uint32_t));
  w.ed.pend = p;
  return w;
}
static inline size_t item_ws_total(uint64_t n_items) {
  const size_t n = n_items ? n_items : 1;
  return al256(n * ITEM_SLOT) + 4 * al256(n * sizeof(uint32_t)) + 256 + al256(plan_sort_temp_bytes(n)) +
         al256(8 * n * sizeof(uint32_t)) + al256(n * sizeof(uint32_t)) + al256(n);
}
hipError_t launch_plan(const cg_item* d_items, uint64_t n_items, const cg_key* d_keys, uint32_t n_keys,
                       const KeyWs& w, const ItemWs& iw, hipStream_t stream);

// Constant tables per context: [Ed25519 B rows (radix 2^10)][G rows k1][G rows r1]
// [Ed25519 B wide rows (radix 2^12)][G wide rows k1][G wide rows r1][row scratch]
#define EC_GTAB_LANES (EC_G_DIGITS * (EC_G_MULT / EC_MULT))  // one lane per (row, group of 32)
#define EC_GWIDE_LANES (EC_WIDE_GDIGITS * (EC_WIDE_GMULT / EC_MULT))
// the G-table builds run in batches of at most CONST_SCRATCH_LANES lanes over one scratch
#define CONST_SCRATCH_MAX 131072
#define CONST_SCRATCH_LANES                                                                        \
  ((EC_GWIDE_LANES < CONST_SCRATCH_MAX ? EC_GWIDE_LANES : CONST_SCRATCH_MAX) > EC_GTAB_LANES       \
       ? (EC_GWIDE_LANES < CONST_SCRATCH_MAX ? EC_GWIDE_LANES : CONST_SCRATCH_MAX)                 \
       : EC_GTAB_LANES)
static inline size_t const_tab_bytes() {
  return sizeof(EdBTab) + 2 * sizeof(EcGTab) + sizeof(EdBWideTab) + 2 * sizeof(EcGWideTab);
}
// scratch of the one-time builds: allocated by cg_open for init_btab only, then freed
static inline size_t const_scratch_bytes() { return (size_t)CONST_SCRATCH_LANES * sizeof(EcRowScratch); }
static inline const EcGTab* gtab(const void* d_btab, int curve) {
  return (const EcGTab*)((const uint8_t*)d_btab + sizeof(EdBTab)) + curve;
}
static inline const EdBWideTab* bwide(const void* d_btab) {
  return (const EdBWideTab*)((const uint8_t*)d_btab + sizeof(EdBTab) + 2 * sizeof(EcGTab));
}
static inline const EcGWideTab* gwide(const void* d_btab, int curve) {
  return (const EcGWideTab*)((const uint8_t*)bwide(d_btab) + sizeof(EdBWideTab)) + curve;
}

// Intermediate per-item status codes (never returned to the caller)
#define ED_PENDING 254u
#define EC_PENDING_BASE 250u  // + curve: parsed + hashed, awaiting the ladder

// Per-scheme halves (verify_ed.hip / verify_ec.hip)
hipError_t ed_upload_constants();
hipError_t ed_init_const(void* d_btab, void* d_scratch, hipStream_t stream);
void ed_launch_key_abyte(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                         const KeyWs& w, hipStream_t stream);
// decode -> chains (light), then the row tables (heavy)
void ed_launch_keyprep_chains(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                              const KeyWs& w, hipStream_t stream);
// the full / row-0 tables and / or the wide tables
void ed_launch_keyprep_tabs(const cg_key* d_keys, uint32_t n_keys, const KeyWs& w, hipStream_t stream, bool full,
                            bool wide);
// item stages (verify.hip launch_items orders them across the main and side streams)
void ed_launch_front(const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len,
                     uint32_t mode, uint8_t* d_status, const KeyWs& w, const uint8_t* d_msgs, uint64_t msgs_len,
                     const ItemWs& iw, hipStream_t stream);
void ed_launch_ladder(bool full, const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                      const ItemWs& iw, const void* d_btab, hipStream_t stream);
void ed_launch_ladder_wide(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                           const ItemWs& iw, const void* d_btab, hipStream_t stream);
void ed_launch_finish(const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len,
                      uint8_t* d_status, const ItemWs& iw, hipStream_t stream);
hipError_t ec_upload_constants();
hipError_t ec_init_const(void* d_btab, void* d_scratch, hipStream_t stream);
// per curve: decode (records `decoded`: k_ec_prep needs the key status) -> chains; then the tables
void ec_launch_keyprep_chains(int curve, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena,
                              uint64_t arena_len, const KeyWs& w, hipStream_t stream, hipEvent_t decoded);
void ec_launch_keyprep_tabs(int curve, const cg_key* d_keys, uint32_t n_keys, const KeyWs& w, hipStream_t stream,
                            bool full, bool wide);
void ec_launch_front(int curve, const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena,
                     uint64_t arena_len, uint32_t mode, uint8_t* d_status, const KeyWs& w, const uint8_t* d_msgs,
                     uint64_t msgs_len, const ItemWs& iw, hipStream_t stream);
void ec_launch_ladder(int curve, bool full, const cg_item* d_items, uint64_t n_items, uint8_t* d_status,
                      const KeyWs& w, const ItemWs& iw, const void* d_btab, hipStream_t stream);
void ec_launch_ladder_wide(int curve, const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                           const ItemWs& iw, const void* d_btab, hipStream_t stream);
// both curves' wide ladders in one launch (verify_ec.hip k_ec_ladder_wide2)
void ec_launch_ladder_wide_merged(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                                  const ItemWs& iw, const void* d_btab, hipStream_t stream);

}  // namespace cg
