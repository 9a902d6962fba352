// ECDSA (SHA256withECDSA) verification kernels on secp256r1 / secp256k1, BouncyCastle 1.57
// semantics (ecdsa.h header comment).
//   k_ec_keyprep_decode one lane per ECDSA key: decode + validate Q   (side stream of the curve;
//   k_ec_keyprep_chain one lane per ECDSA key: row bases 2^{24j} Q      prep waits for the decode,
//   k_ec_keyprep_tab   one lane per (key, row): 32 affine multiples     the ladder for the tab)
//   k_ec_prep          one lane per item: DER, range checks, SHA-256, e mod n
//   k_ec_inv           EC_INV_K items per lane: one shared inversion of s mod n -> u1, u2
//   k_ec_ladder        one lane per item: u1 G (radix-2^10 constant table) + u2 Q (key rows;
//                      row 0 and 252 doublings for a key with few items, keyws.h),
//                      BC's inversion-free x(R) == r check
// Replaces, per item, BC DSABase.engineVerify behind Crypto.isValid
// (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559, schemes :92-117).
#include "keyws.h"

namespace cg {

__constant__ EcConsts c_ec[2];  // [CG_CURVE_K1], [CG_CURVE_R1]


template <int C>
__device__ __forceinline__ uint8_t ec_scheme() {
  return C == CG_CURVE_R1 ? CG_ECDSA_SECP256R1_SHA256 : CG_ECDSA_SECP256K1_SHA256;
}

template <int C>
__global__ void __launch_bounds__(64) k_ec_keyprep_decode(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                        const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                        EdKeyHdr* __restrict__ hdr, BaseSlot* __restrict__ bases) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_keys) return;
  const cg_key k = keys[i];
  if (k.scheme != ec_scheme<C>()) return;
  EdKeyHdr h;
  for (int w = 0; w < 7; ++w) h.pad[w] = 0;
  for (int w = 0; w < 8; ++w) h.abyte[w] = 0;
  h.status = CG_KEY_INVALID;
  if (in_arena(k.off, k.len, arena_len)) {
    f29 xm, ym;
    if (ec_key_decode_bytes<C>(xm, ym, arena, round4(arena_len), k.off, k.len, k.fmt, c_ec[C]) == 0) {
      h.status = 0;
      bases[(size_t)i * KEY_BASES].ec = Jac{xm, ym, c_ec[C].one_p};
    }
  }
  hdr[i] = h;
}

// one lane per full-table key of this curve (keyws.h: the compacted list), then one per quarter key
template <int C>
__global__ void __launch_bounds__(64) k_ec_keyprep_chain(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                         const uint32_t* __restrict__ full,
                                                         const uint32_t* __restrict__ quart,
                                                         const uint32_t* __restrict__ full_count,
                                                         BaseSlot* __restrict__ bases) {
  chain_prio();
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = plan_class_of_curve(C);
  const uint32_t nf = full_count[c], nq = full_count[QUART_COUNT_AT + c];
  if (l >= nf + nq) return;
  const bool q = l >= nf;
  const uint32_t i = q ? quart[(size_t)c * n_keys + (l - nf)] : full[(size_t)c * n_keys + l];
  if (hdr[i].status != 0) return;
  Jac P = bases[(size_t)i * KEY_BASES].ec;
  const int rows = q ? EC_QROWS : EC_ROWS, step = EC_W * (q ? EC_QWINDOWS : EC_WINDOWS);
  for (int j = 1; j < rows; ++j) {
    jac_dbl_n<C>(P, P, step);
    bases[(size_t)i * KEY_BASES + j].ec = P;
  }
}

// The 32 affine multiples of a row base (ec_row_build_parked), for the compacted tasks: row 0 of
// every used key of this curve without wide tables, rows 1..10 of its full-table keys, rows 1..3 of
// its quarter keys; a grid
// of `lanes` lanes looping over the tasks, each parked in its own column (as k_ed_keyprep_tab).
template <int C>
__global__ void __launch_bounds__(64) k_ec_keyprep_tab(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                       const BaseSlot* __restrict__ bases,
                                                       const uint32_t* __restrict__ row0,
                                                       const uint32_t* __restrict__ full,
                                                       const uint32_t* __restrict__ quart,
                                                       const uint32_t* __restrict__ full_count,
                                                       TabSlot* __restrict__ tabs, uint32_t* __restrict__ park,
                                                       uint32_t lanes) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= lanes) return;
  const int c = plan_class_of_curve(C);
  const uint32_t n0 = full_count[ROW0_COUNT_AT + c], nf = full_count[c], nq = full_count[QUART_COUNT_AT + c];
  const uint64_t tf = n0 + (uint64_t)nf * (EC_ROWS - 1), tasks = tf + (uint64_t)nq * (EC_QROWS - 1);
  const EcRowParkLanes pk{park, p, lanes};
  for (uint64_t t = p; t < tasks; t += lanes) {
    uint32_t i, j;
    if (t < n0) {
      i = row0[(size_t)c * n_keys + t];
      j = 0;
    } else if (t < tf) {
      const uint64_t h = t - n0;
      j = 1 + (uint32_t)(h / nf);
      i = full[(size_t)c * n_keys + h % nf];
    } else {  // quarter rows 1..EC_QROWS - 1
      const uint64_t h = t - tf;
      j = 1 + (uint32_t)(h / nq);
      i = quart[(size_t)c * n_keys + h % nq];
    }
    if (hdr[i].status != 0) continue;
    ec_row_build_parked<C>(tabs[i].ec.t[j], bases[(size_t)i * KEY_BASES + j].ec, pk, c_ec[C]);
  }
}

// Wide tables (ecdsa_rows.h): one lane per wide key of this curve, the 32 row bases 2^{8j} Q
// (a chain of 248 doublings), then one lane per (wide key, row): 128 affine multiples, one
// inversion (row 32: the multiples 129..256 of the top row's base).
template <int C>
__global__ void __launch_bounds__(64) k_ec_wide_chain(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                      const uint32_t* __restrict__ wide,
                                                      const uint32_t* __restrict__ wide_count,
                                                      const uint32_t* __restrict__ wide_idx,
                                                      const BaseSlot* __restrict__ bases, EcWideSlot* __restrict__ wec) {
  chain_prio();
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = plan_class_of_curve(C);
  if (l >= wide_count[c]) return;
  const uint32_t i = wide[(size_t)c * n_keys + l];
  if (hdr[i].status != 0) return;
  EcWideSlot& ws = wec[wide_idx[i]];
  Jac P = bases[(size_t)i * KEY_BASES].ec;
  ws.jbases[0] = P;
  for (int j = 1; j < EC_WIDE_DIGITS; ++j) {
    jac_dbl_n<C>(P, P, EC_WIDE_W);
    ws.jbases[j] = P;
  }
  jac_batch_to_affine<C>(ws.bases, ws.jbases, EC_WIDE_DIGITS, ws.s[0].pre, c_ec[C]);
}

// The row tables in three passes over (wide key, row, group of 32) lanes, as the Ed25519 build
// (ecdsa_rows.h ec_wide_group_pass): chunk Z products, one inversion per row over its 64 chunk
// products (in the row's scratch z[0..63], prefixes in pre[0..63]), then the entries.
#define EC_WIDE_GROUP 32
#define EC_WIDE_GROUPS (EC_WIDE_MULT / EC_WIDE_GROUP)
struct EcWideLane {
  uint32_t l, j, g;
};
__device__ __forceinline__ EcWideLane ec_wide_lane(uint32_t rows, uint32_t groups) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  return EcWideLane{(uint32_t)(t / (rows * groups)), (uint32_t)(t / groups % rows), (uint32_t)(t % groups)};
}
#define EC_WIDE_KEY(C, L)                                  \
  const int c = plan_class_of_curve(C);                    \
  if ((L).l >= wide_count[c]) return;                      \
  const uint32_t i = wide[(size_t)c * n_keys + (L).l];     \
  if (hdr[i].status != 0) return;                          \
  EcWideSlot& ws = wec[wide_idx[i]]
static_assert(EC_WIDE_CHUNKS <= EC_WIDE_MULT, "chunk products fit a row's scratch");

template <int C>
__global__ void __launch_bounds__(64) k_ec_wide_fwd(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wide,
                                                    const uint32_t* __restrict__ wide_count,
                                                    const uint32_t* __restrict__ wide_idx, EcWideSlot* __restrict__ wec) {
  const EcWideLane L = ec_wide_lane(EC_WIDE_ROWS, EC_WIDE_GROUPS);
  EC_WIDE_KEY(C, L);
  constexpr int CPG = EC_WIDE_GROUP / EC_WIDE_CHUNK;
  ec_wide_group_pass<C, false>(nullptr, &ws.s[L.j].z[CPG * L.g],
                               ws.bases[L.j < EC_WIDE_DIGITS ? L.j : EC_WIDE_DIGITS - 1], (int)L.j, (int)L.g, c_ec[C]);
}

template <int C>
__global__ void __launch_bounds__(64) k_ec_wide_inv(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wide,
                                                    const uint32_t* __restrict__ wide_count,
                                                    const uint32_t* __restrict__ wide_idx, EcWideSlot* __restrict__ wec) {
  const EcWideLane L = ec_wide_lane(EC_WIDE_ROWS, 1);
  EC_WIDE_KEY(C, L);
  m29_invert_run<C, EC_WIDE_CHUNKS>(ws.s[L.j].z, ws.s[L.j].pre, c_ec[C]);
}

template <int C>
__global__ void __launch_bounds__(64) k_ec_wide_bwd(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wide,
                                                    const uint32_t* __restrict__ wide_count,
                                                    const uint32_t* __restrict__ wide_idx, EcWideSlot* __restrict__ wec) {
  const EcWideLane L = ec_wide_lane(EC_WIDE_ROWS, EC_WIDE_GROUPS);
  EC_WIDE_KEY(C, L);
  constexpr int CPG = EC_WIDE_GROUP / EC_WIDE_CHUNK;
  ec_wide_group_pass<C, true>(&ws.tab.t[L.j][EC_WIDE_GROUP * L.g], &ws.s[L.j].z[CPG * L.g],
                              ws.bases[L.j < EC_WIDE_DIGITS ? L.j : EC_WIDE_DIGITS - 1], (int)L.j, (int)L.g, c_ec[C]);
}

#ifndef EC_WIDE_ROWS_PRIO_R1
#define EC_WIDE_ROWS_PRIO_R1 0
#endif
// one lane per (wide key, row): the row's 128 affine multiples by co-Z additions, one launch
// (ecdsa_rows.h ec_wide_row_build; replaces the three passes above unless CG_EC_WIDE_COZ=0)
template <int C>
__global__ void __launch_bounds__(64) k_ec_wide_rows(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                     const uint32_t* __restrict__ wide,
                                                     const uint32_t* __restrict__ wide_count,
                                                     const uint32_t* __restrict__ wide_idx, EcWideSlot* __restrict__ wec) {
#if EC_WIDE_ROWS_PRIO_R1  // (A/B) secp256r1's rows (its first ladder comes before secp256k1's) above k1's
  if (C == CG_CURVE_R1) __builtin_amdgcn_s_setprio(EC_WIDE_ROWS_PRIO_R1);
#endif
  const EcWideLane L = ec_wide_lane(EC_WIDE_ROWS, EC_WIDE_ROW_LANES);
  EC_WIDE_KEY(C, L);
  constexpr int per = EC_WIDE_MULT / EC_WIDE_ROW_LANES;
  const EcParkLanes pk{ws.park, L.j * EC_WIDE_ROW_LANES + L.g, (uint32_t)(EC_WIDE_ROWS * EC_WIDE_ROW_LANES)};
  ec_wide_row_build<C>(ws.tab.t[L.j], pk, ws.bases[L.j < EC_WIDE_DIGITS ? L.j : EC_WIDE_DIGITS - 1],
                       L.j == EC_WIDE_DIGITS, per * (int)L.g, per * (int)L.g + per, c_ec[C]);
}
#ifndef CG_EC_WIDE_COZ
#define CG_EC_WIDE_COZ 1
#endif

// G wide rows: the row bases 2^{EC_WIDE_GW u} G first (one lane per row, into scratch slot 0),
// then one lane per (row u, group g of 32 multiples) in batches over scratch slots 1..
template <int C>
__global__ void __launch_bounds__(64) k_ec_gwide_bases(Jac* __restrict__ bases) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (uint32_t)EC_WIDE_GDIGITS) return;
  Jac P = {c_ec[C].gx, c_ec[C].gy, c_ec[C].one_p};
  if (u > 0) jac_dbl_n<C>(P, P, EC_WIDE_GW * (int)u);
  bases[u] = P;
}
#define EC_GWIDE_BATCH (CONST_SCRATCH_LANES - 1)
template <int C>
__global__ void __launch_bounds__(64) k_ec_gwide_init(EcGWideTab* __restrict__ out, EcRowScratch* __restrict__ scratch,
                                                      uint32_t lane0) {
  const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x, l = lane0 + s;
  if (s >= EC_GWIDE_BATCH || l >= EC_GWIDE_LANES) return;
  const int u = (int)(l / (EC_WIDE_GMULT / EC_MULT)), g = (int)(l % (EC_WIDE_GMULT / EC_MULT));
  ec_gwide_group_from<C>(&out->t[u][g * EC_MULT], ((const Jac*)scratch)[u], g, scratch[1 + s], c_ec[C]);
}

// one lane per (G row u, group g of 32 multiples)
template <int C>
__global__ void __launch_bounds__(64) k_ec_gtab_init(EcGTab* __restrict__ out, EcRowScratch* __restrict__ scratch) {
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= EC_GTAB_LANES) return;
  const int u = (int)(l / (EC_G_MULT / EC_MULT)), g = (int)(l % (EC_G_MULT / EC_MULT));
  ec_gtab_group<C>(&out->t[u][g * EC_MULT], u, g, scratch[l], c_ec[C]);
}

// Plan positions of curve C: [ranges[c], ranges[c + 1]), c = plan_class_of_curve(C)
#define EC_RANGE(C)                                   \
  const int cls = plan_class_of_curve(C);             \
  const uint32_t beg = ranges[cls], end = ranges[cls + 1]

#define EC_SIG_STAGED 80  // signature bytes k_ec_prep stages (DER for a 256-bit curve is at most 72)
template <int C, bool Fused>  // Fused: every message is a SignableData splice (the tx-signature paths)
__global__ void __launch_bounds__(256) k_ec_prep(const cg_item* __restrict__ items, const uint32_t* __restrict__ perm,
                                                 const uint32_t* __restrict__ ranges,
                                                 const EdKeyHdr* __restrict__ hdr,
                                                 const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                 const uint8_t* __restrict__ msgs, uint64_t msgs_len,
                                                 uint32_t mode, uint8_t* __restrict__ status,
                                                 EcItemWs* __restrict__ ws) {
  front_prio();
  EC_RANGE(C);
  // each lane's signature staged in LDS (21 dwords from its 4-aligned start: up to EC_SIG_STAGED
  // bytes) with six 16-byte loads, then parsed byte by byte from there (ecdsa.h DerStaged)
  __shared__ uint32_t sig_stage[256 * 21];
  uint32_t* my = sig_stage + 21 * threadIdx.x;  // odd stride: conflict-free dword accesses
  for (Walk wk = walk_units(end - beg); wk.u < wk.end; wk.u += wk.step) {
  const uint64_t p = beg + wk.u;
  const uint32_t i = perm[p];
  const cg_item it = items[i];
  uint8_t st;
  if (hdr[it.key_idx].status != 0) {
    st = CG_KEY_INVALID;
  } else if (mode == CG_MODE_DOVERIFY && (it.sig_len == 0 || it.msg_len == 0)) {
    st = CG_EMPTY;
  } else if (!in_arena(it.sig_off, it.sig_len, arena_len) ||
             (Fused ? !item_fused(it, msgs)
                    : !in_arena(it.msg_off, it.msg_len, item_msg_len(it, arena_len, msgs_len, msgs)))) {
    st = CG_NOT_RUN;
  } else {
    EcItemWs w;
    const TmplMid* mid = item_tmpl_mid(it, msgs);
    const uint64_t lr = round4(arena_len);
    uint32_t r;
    if (it.sig_len <= EC_SIG_STAGED) {
      const uint64_t a0 = it.sig_off & ~(uint64_t)3;
#pragma unroll
      for (int q = 0; q < 5; ++q) {
        uint32_t v[4];
        cg_ld_dwords4(v, arena, lr, a0 + 16 * q);
#pragma unroll
        for (int k = 0; k < 4; ++k) my[4 * q + k] = v[k];  // dword stores: a lane's image is only 4-aligned
      }
      my[20] = a0 + 80 < lr ? cg_ld32(arena + a0 + 80) : 0u;
      const DerStaged sig{(const uint8_t*)my + (it.sig_off & 3)};
      r = Fused ? ecdsa_prep_ld<C>(w, sig, it.sig_len, item_splice(it, msgs), 0, it.msg_len, mid->state, mid->blocks)
                : ecdsa_prep_ld<C>(w, sig, it.sig_len, ArenaLd{item_msg_arena(it, arena, msgs),
                                                               round4(item_msg_len(it, arena_len, msgs_len, msgs))},
                                   it.msg_off, it.msg_len, mid ? mid->state : nullptr, mid ? mid->blocks : 0u);
    } else {  // long (malformed or out-of-range) encodings: straight from the arena
      const DerArena sig{arena, lr, it.sig_off};
      r = Fused ? ecdsa_prep_ld<C>(w, sig, it.sig_len, item_splice(it, msgs), 0, it.msg_len, mid->state, mid->blocks)
                : ecdsa_prep_ld<C>(w, sig, it.sig_len, ArenaLd{item_msg_arena(it, arena, msgs),
                                                               round4(item_msg_len(it, arena_len, msgs_len, msgs))},
                                   it.msg_off, it.msg_len, mid ? mid->state : nullptr, mid ? mid->blocks : 0u);
    }
    if (r == 0) {
      ws[p] = w;
      st = (uint8_t)(EC_PENDING_BASE + C);
    } else {
      st = (uint8_t)r;
    }
  }
  status[i] = st;
  }
}

template <int C>
__global__ void __launch_bounds__(256) k_ec_inv(const uint32_t* __restrict__ perm, const uint32_t* __restrict__ ranges,
                                                const uint8_t* __restrict__ status, EcItemWs* __restrict__ ws) {
  front_prio();
  EC_RANGE(C);
  for (Walk wk = walk_units((end - beg + EC_INV_K - 1) / EC_INV_K); wk.u < wk.end; wk.u += wk.step) {
    const uint64_t base = beg + wk.u * EC_INV_K;
    const uint32_t cnt = (uint32_t)((end - base) < EC_INV_K ? (end - base) : EC_INV_K);
    uint32_t sel = 0;
    for (uint32_t k = 0; k < cnt; ++k) sel |= (uint32_t)(status[perm[base + k]] == EC_PENDING_BASE + C) << k;
    if (sel) ecdsa_batch_inv<C, EC_INV_K>(ws + base, cnt, sel, c_ec[C]);
  }
}

// One launch over the curve's range per table mode (the plan keeps the modes in separate waves, so
// a lane of another mode exits with its whole wave); separate kernels keep each ladder's register
// allocation free of the others'. Mode: PLAN_MODE_ROW0 / PLAN_MODE_QUART / PLAN_MODE_FULL.
template <int C, int Mode>
__global__ void __launch_bounds__(256) k_ec_ladder(const cg_item* __restrict__ items, const uint32_t* __restrict__ perm,
                                                   const uint32_t* __restrict__ ranges,
                                                   const TabSlot* __restrict__ tabs,
                                                   const EcGWideTab* __restrict__ gtab, uint8_t* __restrict__ status,
                                                   const EcItemWs* __restrict__ ws) {
  const int cls = plan_class_of_curve(C);  // the plan's mode split (plan_sort.hip)
  const uint32_t beg = Mode == PLAN_MODE_FULL    ? ranges[PLAN_FULL + cls]
                     : Mode == PLAN_MODE_QUART ? ranges[PLAN_QUART + cls]
                                               : ranges[cls];
  const uint32_t end = Mode == PLAN_MODE_FULL    ? ranges[PLAN_WIDE + cls]
                     : Mode == PLAN_MODE_QUART ? ranges[PLAN_FULL + cls]
                                               : ranges[PLAN_QUART + cls];
  for (Walk wk = walk_units(end - beg); wk.u < wk.end; wk.u += wk.step) {
    const uint64_t p = beg + wk.u;
    const uint32_t i = perm[p];
    if (status[i] != EC_PENDING_BASE + C) continue;
    const uint32_t key = items[i].key_idx;
    const EcItemWs w = ws[p];
    if (Mode == PLAN_MODE_FULL) {
      status[i] = (uint8_t)ecdsa_ladder_check<C>(w.a, w.b, w.r, *gtab, tabs[key].ec, c_ec[C]);
    } else if (Mode == PLAN_MODE_QUART) {  // the first rows of the table, 2^{66 j} Q (keyws.h)
      status[i] = (uint8_t)ecdsa_ladder_check_w<C, EC_QWINDOWS, EC_QROWS>(
          w.a, w.b, w.r, *gtab, *(const EcRowTabQ*)&tabs[key].ec, c_ec[C]);
    } else {  // a key with few items: row 0 only (keyws.h)
      status[i] = (uint8_t)ecdsa_ladder_check_row0<C>(w.a, w.b, w.r, *gtab, tabs[key].ec.t[0], c_ec[C]);
    }
  }
}

// The items of wide-table keys: ecdsa_ladder_check_wide's 32 Q rows then 12 G rows as one flat op
// sequence, each op's affine entry gathered straight into LDS one op ahead (global_load_lds, as
// k_ed_ladder_wide; the 1.8 GB G table's HBM latency and the Q rows' L2 latency leave the critical
// path; the plain-load form issued 0.86 / 0.93 of its time for r1 / k1). LDS image per wave: 4 x 16-B
// chunks then 2 x 4-B chunks of the 72-B entry, chunk c of lane l at wave_base + 64 * off_c +
// size_c * l (the DMA's lane-linear destination), 4608 B per wave.
typedef __attribute__((address_space(3))) void* ec_lds_ptr;
typedef __attribute__((address_space(1))) void* ec_gbl_ptr;
static_assert(sizeof(EcAff) == 72, "LDS chunking assumes 72-B affine entries");
#define EC_WAVE_LDS (64 * 72)
#define EC_WIDE_OPS (EC_WIDE_DIGITS + EC_WIDE_GDIGITS)

__device__ __forceinline__ ec_lds_ptr ec_lds_at(uint32_t wave_lds_off, uint32_t b) {
  return (ec_lds_ptr)(uintptr_t)(wave_lds_off + b);
}
__device__ __forceinline__ void ec_glds_aff(const EcAff* src, uint32_t wl) {
  const uint8_t* s = (const uint8_t*)src;
#pragma unroll
  for (int c = 0; c < 4; ++c)
    __builtin_amdgcn_global_load_lds((ec_gbl_ptr)(s + 16 * c), ec_lds_at(wl, 64 * 16 * c), 16, 0, 0);
  __builtin_amdgcn_global_load_lds((ec_gbl_ptr)(s + 64), ec_lds_at(wl, 64 * 64), 4, 0, 0);
  __builtin_amdgcn_global_load_lds((ec_gbl_ptr)(s + 68), ec_lds_at(wl, 64 * 68), 4, 0, 0);
}
__device__ __forceinline__ void ec_lds_aff(f29& x, f29& y, const uint8_t* wave_lds, uint32_t lane) {
  uint32_t d[18];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const uint4 v = *(const uint4*)(wave_lds + 64 * 16 * c + 16 * lane);
    d[4 * c] = v.x;
    d[4 * c + 1] = v.y;
    d[4 * c + 2] = v.z;
    d[4 * c + 3] = v.w;
  }
  d[16] = *(const uint32_t*)(wave_lds + 64 * 64 + 4 * lane);
  d[17] = *(const uint32_t*)(wave_lds + 64 * 68 + 4 * lane);
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    x.v[i] = d[i];
    y.v[i] = d[9 + i];
  }
}
// op o's digit and entry (Q row o, or row 32 for the top digit's 129..256; then G row o - 32)
__device__ __forceinline__ int ec_wide_digit(const uint32_t* dq, const uint32_t* dg, int o) {
  return o < EC_WIDE_DIGITS ? ec_digit10(dq, o) : ec_digit_at<EC_WIDE_GBITS>(dg, o - EC_WIDE_DIGITS);
}
__device__ __forceinline__ const void* ec_wide_src(const EcWideTab& TQ, const EcGWideTab& TG, int o, int d) {
  const int a = d < 0 ? -d : d;
  if (o < EC_WIDE_DIGITS) return a > EC_WIDE_MULT ? &TQ.t[EC_WIDE_DIGITS][a - EC_WIDE_MULT - 1] : &TQ.t[o][a > 0 ? a - 1 : 0];
  return &TG.t[o - EC_WIDE_DIGITS][a > 0 ? a - 1 : 0];
}
// op o's entry into / out of the wave's LDS image: the 72-B affine form, or (EC_GWIDE_PACK, G rows)
// the 64-B packed form, 4 x 16-B chunks unpacked to limbs
__device__ __forceinline__ void ec_wide_gather(const void* src, int o, uint32_t wl) {
  if (EC_GWIDE_PACK && o >= EC_WIDE_DIGITS) {
    const uint8_t* s = (const uint8_t*)src;
#pragma unroll
    for (int c = 0; c < 4; ++c)
      __builtin_amdgcn_global_load_lds((ec_gbl_ptr)(s + 16 * c), ec_lds_at(wl, 64 * 16 * c), 16, 0, 0);
  } else {
    ec_glds_aff((const EcAff*)src, wl);
  }
}
__device__ __forceinline__ void ec_wide_read(f29& x, f29& y, int o, const uint8_t* wave_lds, uint32_t lane) {
  if (EC_GWIDE_PACK && o >= EC_WIDE_DIGITS) {
    uint32_t w[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const uint4 v = *(const uint4*)(wave_lds + 64 * 16 * c + 16 * lane);
      w[4 * c] = v.x;
      w[4 * c + 1] = v.y;
      w[4 * c + 2] = v.z;
      w[4 * c + 3] = v.w;
    }
    ec_unpack256(x, w);
    ec_unpack256(y, w + 8);
  } else {
    ec_lds_aff(x, y, wave_lds, lane);
  }
}

#ifndef EC_LADDER_WIDE_WAVES  // waves per SIMD the wide ladders' registers must allow: 3 (168 VGPRs, 20 B of
#define EC_LADDER_WIDE_WAVES 3  // scratch for r1) against the compiler's 172 at 2: r1 1.73 -> 1.67 ms (profiles/r04/ecw3)
#endif
// One plan position of a wide-table ECDSA item: u1 G + u2 Q over the wide tables, then BC's x check.
template <int C>
__device__ __forceinline__ void ec_wide_item(uint64_t p, const cg_item* __restrict__ items,
                                             const uint32_t* __restrict__ perm, const uint32_t* __restrict__ wide_idx,
                                             const EcWideSlot* __restrict__ wec, const EcGWideTab* __restrict__ gw,
                                             uint8_t* __restrict__ status, const EcItemWs* __restrict__ ws,
                                             const uint8_t* wave_lds, uint32_t wl, uint32_t lane) {
  const EcConsts& K = c_ec[C];
  const uint32_t i = perm[p];
  if (status[i] != EC_PENDING_BASE + C) return;
  // every lane still here runs the same DMA sequence; lanes that left do not take part, and the
  // LDS image is per lane, so no barrier is needed
  const uint32_t key = items[i].key_idx;
  const EcItemWs w = ws[p];
  const EcWideTab& TQ = wec[wide_idx[key]].tab;
  uint32_t dg[EC_WIDE_GPACKED], dq[EC_WIDE_PACKED];
  ec_recode_wide<EC_WIDE_GW, EC_WIDE_GDIGITS, false, EC_WIDE_GBITS>(dg, w.a);
  ec_recode_wide<EC_WIDE_W, EC_WIDE_DIGITS, true>(dq, w.b);
  Jac R;
  jac_set_inf<C>(R, K);
  bool inf = true;
  int d_next = ec_wide_digit(dq, dg, 0);
  ec_wide_gather(ec_wide_src(TQ, *gw, 0, d_next), 0, wl);
#pragma unroll 1
  for (int o = 0; o < EC_WIDE_OPS; ++o) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // op o's entry
    f29 x, y;
    ec_wide_read(x, y, o, wave_lds, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before the next DMA lands
    const int d = d_next;
    if (o + 1 < EC_WIDE_OPS) {
      d_next = ec_wide_digit(dq, dg, o + 1);
      ec_wide_gather(ec_wide_src(TQ, *gw, o + 1, d_next), o + 1, wl);
    }
    if (d != 0) jac_madd9<C>(R, inf, x, y, d < 0, K);  // signed-limb form (ec9.h)
  }
  status[i] = (uint8_t)ecdsa_x_check9<C>(R, w.r, K);
}

template <int C>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EC_LADDER_WIDE_WAVES)))
k_ec_ladder_wide(const cg_item* __restrict__ items,
                                                        const uint32_t* __restrict__ perm,
                                                        const uint32_t* __restrict__ ranges,
                                                        const uint32_t* __restrict__ wide_idx,
                                                        const EcWideSlot* __restrict__ wec,
                                                        const EcGWideTab* __restrict__ gw, uint8_t* __restrict__ status,
                                                        const EcItemWs* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4 * EC_WAVE_LDS];
  const int cls = plan_class_of_curve(C);
  const uint32_t beg = ranges[PLAN_WIDE + cls], end = ranges[cls + 1];
  uint8_t* wave_lds = stage + (threadIdx.x >> 6) * EC_WAVE_LDS;
  const uint32_t wl = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(ec_lds_ptr)wave_lds);
  const uint32_t lane = __lane_id();
  for (Walk wk = walk_units(end - beg); wk.u < wk.end; wk.u += wk.step)
    ec_wide_item<C>(beg + wk.u, items, perm, wide_idx, wec, gw, status, ws, wave_lds, wl, lane);
}

// CG_EC_WIDE_MERGED (A/B): both curves' wide items in one launch, the secp256r1 range then the
// secp256k1 range walked as one (a curve's launch alone leaves a partial last round of waves: the
// k1 range is ~1.2 rounds of the resident lanes); a wave's items are of one curve except at the seam.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(EC_LADDER_WIDE_WAVES)))
k_ec_ladder_wide2(const cg_item* __restrict__ items, const uint32_t* __restrict__ perm,
                  const uint32_t* __restrict__ ranges, const uint32_t* __restrict__ wide_idx,
                  const EcWideSlot* __restrict__ wec, const EcGWideTab* __restrict__ gw_r1,
                  const EcGWideTab* __restrict__ gw_k1, uint8_t* __restrict__ status,
                  const EcItemWs* __restrict__ ws) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4 * EC_WAVE_LDS];
  const int c1 = plan_class_of_curve(CG_CURVE_R1), c0 = plan_class_of_curve(CG_CURVE_K1);
  const uint32_t b1 = ranges[PLAN_WIDE + c1], n1 = ranges[c1 + 1] - b1;
  const uint32_t b0 = ranges[PLAN_WIDE + c0], n0 = ranges[c0 + 1] - b0;
  uint8_t* wave_lds = stage + (threadIdx.x >> 6) * EC_WAVE_LDS;
  const uint32_t wl = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(ec_lds_ptr)wave_lds);
  const uint32_t lane = __lane_id();
  for (Walk wk = walk_units((uint64_t)n1 + n0); wk.u < wk.end; wk.u += wk.step) {
    if (wk.u < n1)
      ec_wide_item<CG_CURVE_R1>(b1 + wk.u, items, perm, wide_idx, wec, gw_r1, status, ws, wave_lds, wl, lane);
    else
      ec_wide_item<CG_CURVE_K1>(b0 + (wk.u - n1), items, perm, wide_idx, wec, gw_k1, status, ws, wave_lds, wl, lane);
  }
}

hipError_t ec_upload_constants() {
  EcConsts k[2];
  ec_consts_init<CG_CURVE_K1>(k[CG_CURVE_K1]);
  ec_consts_init<CG_CURVE_R1>(k[CG_CURVE_R1]);
  return hipMemcpyToSymbol(HIP_SYMBOL(c_ec), k, sizeof k, 0, hipMemcpyHostToDevice);
}

hipError_t ec_init_const(void* d_btab, void* d_scratch, hipStream_t stream) {
  const dim3 g((EC_GTAB_LANES + 63) / 64);
  hipLaunchKernelGGL(k_ec_gtab_init<CG_CURVE_K1>, g, dim3(64), 0, stream, (EcGTab*)gtab(d_btab, CG_CURVE_K1),
                     (EcRowScratch*)d_scratch);
  hipLaunchKernelGGL(k_ec_gtab_init<CG_CURVE_R1>, g, dim3(64), 0, stream, (EcGTab*)gtab(d_btab, CG_CURVE_R1),
                     (EcRowScratch*)d_scratch);
  // per curve: the row bases, then batches of EC_GWIDE_BATCH lanes over one scratch (stream order
  // serialises them)
  static_assert(EC_WIDE_GDIGITS * sizeof(Jac) <= sizeof(EcRowScratch), "G row bases fit scratch slot 0");
  const dim3 gw((EC_GWIDE_BATCH + 63) / 64);
  EcRowScratch* sc = (EcRowScratch*)d_scratch;
  hipLaunchKernelGGL(k_ec_gwide_bases<CG_CURVE_K1>, dim3(1), dim3(64), 0, stream, (Jac*)sc);
  for (uint32_t l0 = 0; l0 < (uint32_t)EC_GWIDE_LANES; l0 += EC_GWIDE_BATCH)
    hipLaunchKernelGGL(k_ec_gwide_init<CG_CURVE_K1>, gw, dim3(64), 0, stream, (EcGWideTab*)gwide(d_btab, CG_CURVE_K1),
                       sc, l0);
  hipLaunchKernelGGL(k_ec_gwide_bases<CG_CURVE_R1>, dim3(1), dim3(64), 0, stream, (Jac*)sc);
  for (uint32_t l0 = 0; l0 < (uint32_t)EC_GWIDE_LANES; l0 += EC_GWIDE_BATCH)
    hipLaunchKernelGGL(k_ec_gwide_init<CG_CURVE_R1>, gw, dim3(64), 0, stream, (EcGWideTab*)gwide(d_btab, CG_CURVE_R1),
                       sc, l0);
  return hipGetLastError();
}

template <int C>
static void launch_keyprep_chains(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                                  const KeyWs& w, hipStream_t stream, hipEvent_t decoded) {
  const uint32_t B = 64;
  const dim3 g((n_keys + B - 1) / B);
  hipLaunchKernelGGL(k_ec_keyprep_decode<C>, g, dim3(B), 0, stream, d_keys, n_keys, d_arena, arena_len, w.hdr,
                     w.bases);
  if (decoded) hipEventRecord(decoded, stream);
  hipLaunchKernelGGL(k_ec_keyprep_chain<C>, g, dim3(B), 0, stream, n_keys, w.hdr, (const uint32_t*)w.full,
                     (const uint32_t*)w.quart, (const uint32_t*)w.full_count, w.bases);
  if (w.cap_ec) {
    const uint32_t lds = chain_spread_lds();
    if (lds) hipFuncSetAttribute((const void*)k_ec_wide_chain<C>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k_ec_wide_chain<C>, dim3((w.cap_ec + B - 1) / B), dim3(B), lds, stream, n_keys, w.hdr,
                       (const uint32_t*)w.wide, (const uint32_t*)w.wide_count, (const uint32_t*)w.wide_idx,
                       (const BaseSlot*)w.bases, w.wec);
  }
}

template <int C>
static void launch_keyprep_tabs(const cg_key* d_keys, uint32_t n_keys, const KeyWs& w, hipStream_t stream, bool full,
                                bool wide) {
  const uint32_t B = 64;
  if (full)
    hipLaunchKernelGGL(k_ec_keyprep_tab<C>, dim3(w.park_lanes_ec / B), dim3(B), 0, stream, n_keys, w.hdr, w.bases,
                       (const uint32_t*)w.row0, (const uint32_t*)w.full, (const uint32_t*)w.quart,
                       (const uint32_t*)w.full_count, w.tab, w.park_ec[C], w.park_lanes_ec);
  if (wide && w.cap_ec) {
    const uint64_t gl = (uint64_t)w.cap_ec * EC_WIDE_ROWS * EC_WIDE_GROUPS, rl = (uint64_t)w.cap_ec * EC_WIDE_ROWS;
    const uint32_t* wl = (const uint32_t*)w.wide;
    const uint32_t* wc = (const uint32_t*)w.wide_count;
    const uint32_t* wi = (const uint32_t*)w.wide_idx;
    if (CG_EC_WIDE_COZ) {
      hipLaunchKernelGGL(k_ec_wide_rows<C>, dim3((unsigned)((rl * EC_WIDE_ROW_LANES + B - 1) / B)), dim3(B), 0, stream,
                         n_keys, w.hdr, wl, wc, wi, w.wec);
    } else {
      hipLaunchKernelGGL(k_ec_wide_fwd<C>, dim3((unsigned)((gl + B - 1) / B)), dim3(B), 0, stream, n_keys, w.hdr,
                         wl, wc, wi, w.wec);
      hipLaunchKernelGGL(k_ec_wide_inv<C>, dim3((unsigned)((rl + B - 1) / B)), dim3(B), 0, stream, n_keys, w.hdr,
                         wl, wc, wi, w.wec);
      hipLaunchKernelGGL(k_ec_wide_bwd<C>, dim3((unsigned)((gl + B - 1) / B)), dim3(B), 0, stream, n_keys, w.hdr,
                         wl, wc, wi, w.wec);
    }
  }
}

void ec_launch_keyprep_chains(int curve, const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena,
                              uint64_t arena_len, const KeyWs& w, hipStream_t stream, hipEvent_t decoded) {
  if (curve == CG_CURVE_R1) launch_keyprep_chains<CG_CURVE_R1>(d_keys, n_keys, d_arena, arena_len, w, stream, decoded);
  else launch_keyprep_chains<CG_CURVE_K1>(d_keys, n_keys, d_arena, arena_len, w, stream, decoded);
}

void ec_launch_keyprep_tabs(int curve, const cg_key* d_keys, uint32_t n_keys, const KeyWs& w, hipStream_t stream,
                            bool full, bool wide) {
  if (curve == CG_CURVE_R1) launch_keyprep_tabs<CG_CURVE_R1>(d_keys, n_keys, w, stream, full, wide);
  else launch_keyprep_tabs<CG_CURVE_K1>(d_keys, n_keys, w, stream, full, wide);
}

// Walk-grid caps of the front stages, in waves per SIMD (the kernels fit 5 and 6). Raising them to
// 5 / 6 was neutral on the headline (A/B 259.2 vs 259.0 M sigs/s, profiles/r02/cap_rejected): the
// r1 front slowed while the concurrent challenge hashes sped up.
#ifndef EC_PREP_CAP_WAVES
#define EC_PREP_CAP_WAVES 2
#endif
#ifndef EC_INV_CAP_WAVES
#define EC_INV_CAP_WAVES 2
#endif
template <int C>
static void launch_front(const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len,
                         uint32_t mode, uint8_t* d_status, const KeyWs& w, const uint8_t* d_msgs, uint64_t msgs_len,
                         const ItemWs& iw, hipStream_t stream) {
  const uint32_t B = 256;  // a curve's range is at most n_items long
  EcItemWs* ws = (EcItemWs*)iw.slots;
  static const uint32_t prep_waves = [] {  // CG_EC_PREP_WAVES (A/B): waves per SIMD of the prep grid
    const char* v = getenv("CG_EC_PREP_WAVES");
    const uint32_t x = v ? (uint32_t)strtoul(v, nullptr, 10) : 0u;
    return x ? x : (uint32_t)EC_PREP_CAP_WAVES;
  }();
  const dim3 pgrid(walk_grid(n_items, B, WALK_CAP(prep_waves)));
  if (d_msgs)
    hipLaunchKernelGGL((k_ec_prep<C, true>), pgrid, dim3(B), 0, stream, d_items, iw.perm, iw.ranges, w.hdr, d_arena,
                       arena_len, d_msgs, msgs_len, mode, d_status, ws);
  else
    hipLaunchKernelGGL((k_ec_prep<C, false>), pgrid, dim3(B), 0, stream, d_items, iw.perm, iw.ranges, w.hdr, d_arena,
                       arena_len, d_msgs, msgs_len, mode, d_status, ws);
  const unsigned igrid = walk_grid((n_items + EC_INV_K - 1) / EC_INV_K, B, WALK_CAP(EC_INV_CAP_WAVES));
  hipLaunchKernelGGL(k_ec_inv<C>, dim3(igrid), dim3(B), 0, stream, iw.perm, iw.ranges,
                     (const uint8_t*)d_status, ws);
}

void ec_launch_front(int curve, const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena,
                     uint64_t arena_len, uint32_t mode, uint8_t* d_status, const KeyWs& w, const uint8_t* d_msgs,
                     uint64_t msgs_len, const ItemWs& iw, hipStream_t stream) {
  if (curve == CG_CURVE_R1)
    launch_front<CG_CURVE_R1>(d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw, stream);
  else
    launch_front<CG_CURVE_K1>(d_items, n_items, d_arena, arena_len, mode, d_status, w, d_msgs, msgs_len, iw, stream);
}

template <int C, int Mode>
static void launch_ladder_m(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                            const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  const uint32_t B = 256;
  hipLaunchKernelGGL((k_ec_ladder<C, Mode>), dim3(walk_grid(n_items, B, WALK_CAP(2))), dim3(B), 0, stream, d_items,
                     iw.perm, iw.ranges, w.tab, gwide(d_btab, C), d_status, (const EcItemWs*)iw.slots);
}
// full: the full-table ladder; else the row-0 then the quarter-table one (the side streams)
template <int C, bool Full>
static void launch_ladder_t(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                            const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  if (Full) {
    launch_ladder_m<C, PLAN_MODE_FULL>(d_items, n_items, d_status, w, iw, d_btab, stream);
  } else {
    launch_ladder_m<C, PLAN_MODE_ROW0>(d_items, n_items, d_status, w, iw, d_btab, stream);
    launch_ladder_m<C, PLAN_MODE_QUART>(d_items, n_items, d_status, w, iw, d_btab, stream);
  }
}

void ec_launch_ladder(int curve, bool full, const cg_item* d_items, uint64_t n_items, uint8_t* d_status,
                      const KeyWs& w, const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  if (curve == CG_CURVE_R1) {
    if (full) launch_ladder_t<CG_CURVE_R1, true>(d_items, n_items, d_status, w, iw, d_btab, stream);
    else launch_ladder_t<CG_CURVE_R1, false>(d_items, n_items, d_status, w, iw, d_btab, stream);
  } else {
    if (full) launch_ladder_t<CG_CURVE_K1, true>(d_items, n_items, d_status, w, iw, d_btab, stream);
    else launch_ladder_t<CG_CURVE_K1, false>(d_items, n_items, d_status, w, iw, d_btab, stream);
  }
}

template <int C>
static void launch_ladder_wide_t(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                                 const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  const uint32_t B = 256;
  hipLaunchKernelGGL((k_ec_ladder_wide<C>), dim3(walk_grid(n_items, B, WALK_CAP(EC_LADDER_WIDE_WAVES))), dim3(B), 0,
                     stream, d_items,
                     iw.perm, iw.ranges, (const uint32_t*)w.wide_idx, (const EcWideSlot*)w.wec, gwide(d_btab, C),
                     d_status, (const EcItemWs*)iw.slots);
}

void ec_launch_ladder_wide(int curve, const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                           const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  if (curve == CG_CURVE_R1) launch_ladder_wide_t<CG_CURVE_R1>(d_items, n_items, d_status, w, iw, d_btab, stream);
  else launch_ladder_wide_t<CG_CURVE_K1>(d_items, n_items, d_status, w, iw, d_btab, stream);
}

void ec_launch_ladder_wide_merged(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                                  const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  const uint32_t B = 256;
  hipLaunchKernelGGL(k_ec_ladder_wide2, dim3(walk_grid(n_items, B, WALK_CAP(EC_LADDER_WIDE_WAVES))), dim3(B), 0, stream,
                     d_items, iw.perm, iw.ranges, (const uint32_t*)w.wide_idx, (const EcWideSlot*)w.wec,
                     gwide(d_btab, CG_CURVE_R1), gwide(d_btab, CG_CURVE_K1), d_status, (const EcItemWs*)iw.slots);
}

}  // namespace cg
