// Ed25519 (EDDSA_ED25519_SHA512) verification kernels, i2p 0.2.0 semantics.
//   k_ed_key_abyte       one lane per key (main stream): canonical Abyte without decoding
//   k_ed_keyprep_decode  one lane per key (side stream): decode A -> key status, -A
//   k_ed_keyprep_chain   one lane per key: row bases 2^{12j} (-A), j = 1..21
//   k_ed_keyprep_tab     one lane per (key, row): the 32 affine multiples of the row base
//   k_ed_hash            one lane per item: SHA-512 challenge, scalar prep, signed digits
//                        (needs only Abyte: overlaps the whole key decode + table build)
//   k_ed_ladder_pf       one lane per item of a full-table key: key status, then 2 windows x
//                        (~21.5 rows of -A + 13 rows of the radix-2^10 B table) mixed additions,
//                        6 doublings; each op's table entry gathered into LDS one op ahead
//   k_ed_ladder<false>   a key with few items in the batch: row 0 of -A and 252 doublings
//                        (keyws.h ED_DIRECT_MAX_USES)
//   k_ed_finish          16 items per lane: batch inversion, encode, byte compare
// Replaces, per item, i2p EdDSAEngine.engineVerify behind Crypto.isValid
// (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559, scheme :120-133).
#include "keyws.h"

namespace cg {

__constant__ Ed25519Consts c_ed;

static const uint8_t ED_SPKI_PREFIX[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};
// AlgorithmIdentifier with an explicit NULL parameter (46 bytes): Crypto.findSignatureScheme
// normalises DERNull away (Crypto.kt:219-228) and i2p 0.2.0 EdDSAPublicKey.decode accepts it.
static const uint8_t ED_SPKI_PREFIX_NULL[14] = {0x30, 0x2c, 0x30, 0x07, 0x06, 0x03, 0x2b,
                                                0x65, 0x70, 0x05, 0x00, 0x03, 0x21, 0x00};

// Offset of A's 32 bytes in the arena for a raw or SPKI Ed25519 key; false for a malformed
// encoding (wrong length / SPKI header / outside the arena).
__device__ __forceinline__ bool ed_key_locate(const cg_key& k, const uint8_t* arena, uint64_t arena_len,
                                              uint64_t& a_off) {
  const uint64_t lr = round4(arena_len);
  a_off = k.off;
  if (!in_arena(k.off, k.len, arena_len)) return false;
  if (k.fmt == CG_KEY_RAW) return k.len == 32;
  if (k.fmt != CG_KEY_SPKI) return false;
  if (k.len == 44) {
    for (int b = 0; b < 12; ++b)
      if ((cg_ld_bytes4(arena, lr, k.off + b) & 0xffu) != ED_SPKI_PREFIX[b]) return false;
    a_off = k.off + 12;
    return true;
  }
  if (k.len == 46) {
    for (int b = 0; b < 14; ++b)
      if ((cg_ld_bytes4(arena, lr, k.off + b) & 0xffu) != ED_SPKI_PREFIX_NULL[b]) return false;
    a_off = k.off + 14;
    return true;
  }
  return false;
}

// one lane per key, main stream: the canonical Abyte k_ed_hash needs, without the square root
// (ed_abyte_fast), so the challenge hashes run while the keys are still being decoded
__global__ void __launch_bounds__(64) k_ed_key_abyte(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                     const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                     EdKeyHdr* __restrict__ hdr) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_keys) return;
  const cg_key k = keys[i];
  if (k.scheme != CG_EDDSA_ED25519_SHA512) return;
  uint64_t a_off;
  uint32_t ab[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (ed_key_locate(k, arena, arena_len, a_off)) {
    const uint64_t lr = round4(arena_len);
    uint32_t aw[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) aw[w] = cg_ld_bytes4(arena, lr, a_off + 4 * w);
    ed_abyte_fast(ab, aw);
  }
#pragma unroll
  for (int w = 0; w < 8; ++w) hdr[i].abyte[w] = ab[w];
}

// one lane per key, side stream: decode A (i2p rules) -> key status, row base -A. Writes only
// hdr.status (k_ed_key_abyte owns hdr.abyte).
__global__ void __launch_bounds__(64) k_ed_keyprep_decode(const cg_key* __restrict__ keys, uint32_t n_keys,
                                                        const uint8_t* __restrict__ arena, uint64_t arena_len,
                                                        EdKeyHdr* __restrict__ hdr, BaseSlot* __restrict__ bases) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_keys) return;
  const cg_key k = keys[i];
  if (k.scheme != CG_EDDSA_ED25519_SHA512) return;
  uint64_t a_off;
  uint32_t st = CG_KEY_INVALID;
  if (ed_key_locate(k, arena, arena_len, a_off)) {
    const uint64_t lr = round4(arena_len);
    uint32_t aw[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) aw[w] = cg_ld_bytes4(arena, lr, a_off + 4 * w);
    ge_p3 A;
    if (ed_decode_point(A, aw, c_ed) == ED_ST_VALID) {
      st = 0;
      ge_p3 P;
      ed_neg_point(P, A);
      bases[(size_t)i * KEY_BASES].ed = P;
    }
  }
  hdr[i].status = st;
}

// one lane per full-table key (keyws.h: the compacted list): row bases 2^{12j} (-A), j = 1..21
// (a serial chain of 240 doublings)
__global__ void __launch_bounds__(64) k_ed_keyprep_chain(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                         const uint32_t* __restrict__ full,
                                                         const uint32_t* __restrict__ quart,
                                                         const uint32_t* __restrict__ full_count,
                                                         BaseSlot* __restrict__ bases) {
  chain_prio();
  // lanes [0, nf): full-table keys (21 x 12 doublings); [nf, nf + nq): quarter keys (3 x 66)
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t nf = full_count[PLAN_ED], nq = full_count[QUART_COUNT_AT + PLAN_ED];
  if (l >= nf + nq) return;
  const bool q = l >= nf;
  const uint32_t i = q ? quart[(size_t)PLAN_ED * n_keys + (l - nf)] : full[(size_t)PLAN_ED * n_keys + l];
  if (hdr[i].status != 0) return;
  ge_p3 P = bases[(size_t)i * KEY_BASES].ed;
  const int rows = q ? EdQCfg::kRows : EdCfg::kRows, step = q ? ED_W * ED_QK : ED_W * ED_K;
  for (int j = 1; j < rows; ++j) {
    ed_dbl_n(P, P, step);
    bases[(size_t)i * KEY_BASES + j].ed = P;
  }
}

// The 32 affine multiples of a row base, one inversion per row (ed_row_build_parked), for the
// compacted tasks: row 0 of every used key without wide tables (row0 list), then rows 1..21 of the
// full-table keys (full list), then rows 1..3 of the quarter-table keys (quart list). A grid of `lanes` lanes (keyws.h tab_park_lanes), each looping over
// tasks lane, lane + lanes, ... with its walk parked in its own lane-interleaved column of `park`.
#ifndef ED_TAB_WAVES  // waves per SIMD the row builds' registers must allow (255 VGPRs + 56 AGPRs left 1)
#define ED_TAB_WAVES 2
#endif
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ED_TAB_WAVES)))
k_ed_keyprep_tab(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                       const BaseSlot* __restrict__ bases,
                                                       const uint32_t* __restrict__ row0,
                                                       const uint32_t* __restrict__ full,
                                                       const uint32_t* __restrict__ quart,
                                                       const uint32_t* __restrict__ full_count,
                                                       TabSlot* __restrict__ tabs, uint32_t* __restrict__ park,
                                                       uint32_t lanes) {
  const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= lanes) return;
  const uint32_t n0 = full_count[ROW0_COUNT_AT + PLAN_ED], nf = full_count[PLAN_ED],
                 nq = full_count[QUART_COUNT_AT + PLAN_ED];
  const uint64_t tf = n0 + (uint64_t)nf * (EdCfg::kRows - 1), tasks = tf + (uint64_t)nq * (EdQCfg::kRows - 1);
  const EdParkLanes pk{park, p, lanes};
  for (uint64_t t = p; t < tasks; t += lanes) {
    uint32_t i, j;
    if (t < n0) {
      i = row0[(size_t)PLAN_ED * n_keys + t];
      j = 0;
    } else if (t < tf) {
      const uint64_t h = t - n0;
      j = 1 + (uint32_t)(h / nf);
      i = full[(size_t)PLAN_ED * n_keys + h % nf];
    } else {  // quarter rows 1..3 (their bases 2^{66 j} (-A) from the chain)
      const uint64_t h = t - tf;
      j = 1 + (uint32_t)(h / nq);
      i = quart[(size_t)PLAN_ED * n_keys + h % nq];
    }
    if (hdr[i].status != 0) continue;
    ed_row_build_parked<EdCfg::kMult>(tabs[i].ed.t[j], bases[(size_t)i * KEY_BASES + j].ed, c_ed.d2, pk);
  }
}

// Wide tables (ed25519_rows.h): one lane per wide key, the 32 row bases 2^{8j} (-A) (a chain of
// 248 doublings), then one lane per (wide key, row): the 128 affine multiples, one inversion.
__global__ void __launch_bounds__(64) k_ed_wide_chain(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                      const uint32_t* __restrict__ wide,
                                                      const uint32_t* __restrict__ wide_count,
                                                      const uint32_t* __restrict__ wide_idx,
                                                      const BaseSlot* __restrict__ bases, EdWideSlot* __restrict__ wed) {
  chain_prio();
  const uint32_t l = blockIdx.x * blockDim.x + threadIdx.x;
  if (l >= wide_count[PLAN_ED]) return;
  const uint32_t i = wide[(size_t)PLAN_ED * n_keys + l];
  if (hdr[i].status != 0) return;
  EdWideSlot& ws = wed[wide_idx[i]];
  ge_p3 P = bases[(size_t)i * KEY_BASES].ed;
  ws.bases[0] = P;
  for (int j = 1; j < EdWideCfg::kRows; ++j) {
    ed_dbl_n(P, P, ED_WIDE_W);
    ws.bases[j] = P;
  }
}

// The same chain with four lanes per key (ED_CHAIN_QUAD, default): the chain is one wave per SIMD
// on an otherwise idle chip at the start of a call, so its time is the dependent instruction
// stream of one lane (~9 cycles per instruction at one wave per SIMD, profiles/r04/ubench), not
// the chip's issue rate. A doubling's four squarings (X^2, Y^2, Z^2, (X+Y)^2) and its P1P1 -> P2/P3
// products (X T, Z Y, Z T, X Y) run one per lane of a quad; the quad then holds the point redundantly
// again after one DPP broadcast per limb and result. Same operations, operand order and bounds as
// ed_dbl_n (ge25519.h ge_p2_dbl, ge_p1p1_to_p2/p3), so every limb equals the one-lane chain's.
#ifndef ED_CHAIN_QUAD
#define ED_CHAIN_QUAD 0
#endif
template <int J>
__device__ __forceinline__ void fe_quad_bcast(fe& o, const fe& a) {  // lane J of each quad -> all four
#pragma unroll
  for (int k = 0; k < 10; ++k) o.v[k] = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.v[k], J * 0x55, 0xF, 0xF, false);
}
__device__ __forceinline__ void fe_pick4(fe& o, const fe& a, const fe& b, const fe& c, const fe& d, uint32_t q) {
#pragma unroll
  for (int k = 0; k < 10; ++k) {  // values, not lvalues: a select of addresses became a scratch array
    const uint32_t av = a.v[k], bv = b.v[k], cv = c.v[k], dv = d.v[k];
    const uint32_t lo = (q & 1u) ? bv : av, hi = (q & 1u) ? dv : cv;
    o.v[k] = (q & 2u) ? hi : lo;
  }
}
// 2^n P (n >= 1); every lane of the quad holds P and ends holding 2^n P
__device__ __forceinline__ void ed_dbl_n_quad(ge_p3& R, const ge_p3& P, int n, uint32_t q) {
  ge_p2 p;
  ge_p3_to_p2(p, P);
  for (int i = 0; i < n; ++i) {
    fe xy, in, s;
    fe_add(xy, p.X, p.Y);  // 2T
    fe_pick4(in, p.X, p.Y, p.Z, xy, q);
    fe_sq(s, in);
    fe xx, yy, zz, aa;
    fe_quad_bcast<0>(xx, s);
    fe_quad_bcast<1>(yy, s);
    fe_quad_bcast<2>(zz, s);
    fe_quad_bcast<3>(aa, s);
    ge_p1p1 t;  // ge_p2_dbl's outputs
    fe_add(t.T, zz, zz);  // fe_sq2: 2 Z^2, tight after the carry
    fe_carry(t.T);
    fe_add(t.Y, yy, xx);
    fe_sub(t.Z, yy, xx);
    fe_sub4(t.X, aa, t.Y);
    fe_sub4(t.T, t.T, t.Z);
    fe_carry(t.T);
    fe f, g, m;  // lane 0: X T, 1: Z Y, 2: Z T, 3: X Y (ge_p1p1_to_p3's operand order)
#pragma unroll
    for (int k = 0; k < 10; ++k) {
      f.v[k] = (q == 0 || q == 3) ? t.X.v[k] : t.Z.v[k];
      g.v[k] = (q == 0 || q == 2) ? t.T.v[k] : t.Y.v[k];
    }
    fe_mul(m, f, g);
    fe_quad_bcast<0>(p.X, m);
    fe_quad_bcast<1>(p.Y, m);
    fe_quad_bcast<2>(p.Z, m);
    if (i + 1 == n) fe_quad_bcast<3>(R.T, m);
  }
  fe_copy(R.X, p.X);
  fe_copy(R.Y, p.Y);
  fe_copy(R.Z, p.Z);
}
__global__ void __launch_bounds__(64) k_ed_wide_chain4(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                       const uint32_t* __restrict__ wide,
                                                       const uint32_t* __restrict__ wide_count,
                                                       const uint32_t* __restrict__ wide_idx,
                                                       const BaseSlot* __restrict__ bases, EdWideSlot* __restrict__ wed) {
  chain_prio();
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t l = t >> 2, q = t & 3u;  // the quad's key and this lane's part (quad-uniform exits)
  if (l >= wide_count[PLAN_ED]) return;
  const uint32_t i = wide[(size_t)PLAN_ED * n_keys + l];
  if (hdr[i].status != 0) return;
  EdWideSlot& ws = wed[wide_idx[i]];
  ge_p3 P = bases[(size_t)i * KEY_BASES].ed;
  fe* const out = &ws.bases[0].X + q;  // lane q stores coordinate q (X, Y, Z, T) of each base
  fe c;
  fe_pick4(c, P.X, P.Y, P.Z, P.T, q);
  *out = c;
  for (int j = 1; j < EdWideCfg::kRows; ++j) {
    ed_dbl_n_quad(P, P, ED_WIDE_W, q);
    fe_pick4(c, P.X, P.Y, P.Z, P.T, q);
    out[(size_t)j * 4] = c;
  }
}
static_assert(sizeof(ge_p3) == 4 * sizeof(fe), "ge_p3 is four consecutive field elements");

// The row tables in three passes (ed25519_rows.h "wide-table build"): chunk Z products per (wide
// key, row, group of 32) lane, one batch inversion per (wide key, row) lane over the row's 64 chunk
// products (kept in the slot's zpre[j][0..63], prefixes in zpre[j][64..127]), then the entries.
struct WideLane {
  uint32_t l, j, g;
};
__device__ __forceinline__ WideLane wide_lane(uint32_t rows, uint32_t groups) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  return WideLane{(uint32_t)(t / (rows * groups)), (uint32_t)(t / groups % rows), (uint32_t)(t % groups)};
}
static_assert(2 * ED_WIDE_CHUNKS <= EdWideCfg::kMult, "chunk products and prefixes fit a zpre row");

__global__ void __launch_bounds__(64) k_ed_wide_fwd(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wide,
                                                    const uint32_t* __restrict__ wide_count,
                                                    const uint32_t* __restrict__ wide_idx, EdWideSlot* __restrict__ wed) {
  const WideLane L = wide_lane(EdWideCfg::kRows, ED_WIDE_GROUPS);
  if (L.l >= wide_count[PLAN_ED]) return;
  const uint32_t i = wide[(size_t)PLAN_ED * n_keys + L.l];
  if (hdr[i].status != 0) return;
  EdWideSlot& ws = wed[wide_idx[i]];
  constexpr int CPG = ED_WIDE_GROUP / ED_WIDE_CHUNK;
  ed_wide_group_pass<false>((ge_niels*)nullptr, &ws.zpre[L.j][CPG * L.g], ws.bases[L.j], (int)L.g, c_ed.d2);
}

__global__ void __launch_bounds__(64) k_ed_wide_inv(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wide,
                                                    const uint32_t* __restrict__ wide_count,
                                                    const uint32_t* __restrict__ wide_idx, EdWideSlot* __restrict__ wed) {
  const WideLane L = wide_lane(EdWideCfg::kRows, 1);
  if (L.l >= wide_count[PLAN_ED]) return;
  const uint32_t i = wide[(size_t)PLAN_ED * n_keys + L.l];
  if (hdr[i].status != 0) return;
  fe* z = wed[wide_idx[i]].zpre[L.j];
  fe_invert_run<ED_WIDE_CHUNKS>(z, z + ED_WIDE_CHUNKS);
}

__global__ void __launch_bounds__(64) k_ed_wide_bwd(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                    const uint32_t* __restrict__ wide,
                                                    const uint32_t* __restrict__ wide_count,
                                                    const uint32_t* __restrict__ wide_idx, EdWideSlot* __restrict__ wed) {
  const WideLane L = wide_lane(EdWideCfg::kRows, ED_WIDE_GROUPS);
  if (L.l >= wide_count[PLAN_ED]) return;
  const uint32_t i = wide[(size_t)PLAN_ED * n_keys + L.l];
  if (hdr[i].status != 0) return;
  EdWideSlot& ws = wed[wide_idx[i]];
  constexpr int CPG = ED_WIDE_GROUP / ED_WIDE_CHUNK;
  ed_wide_group_pass<true>(&ws.tab.t[L.j][ED_WIDE_GROUP * L.g], &ws.zpre[L.j][CPG * L.g], ws.bases[L.j], (int)L.g,
                           c_ed.d2);
}

#ifndef ED_WIDE_ROWS9  // 1: the row walk in radix 2^29 (ed_wide_row_build9), 0: radix 2^25.5 (A/B)
#define ED_WIDE_ROWS9 1
#endif
#ifndef ED_WIDE_ROWS_WAVES  // waves per SIMD the register allocation must allow
#define ED_WIDE_ROWS_WAVES 2  // 3 spills 125 VGPRs
#endif
#ifndef ED_WIDE_ROWS_PRIO
#define ED_WIDE_ROWS_PRIO 2
#endif
// one lane per (wide key, row): the row's 128 multiples, one inversion, one launch
// (ed25519_rows.h ed_wide_row_build; replaces the three passes above unless CG_ED_WIDE_ROWS=0)
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ED_WIDE_ROWS_WAVES))) k_ed_wide_rows(uint32_t n_keys, const EdKeyHdr* __restrict__ hdr,
                                                     const uint32_t* __restrict__ wide,
                                                     const uint32_t* __restrict__ wide_count,
                                                     const uint32_t* __restrict__ wide_idx, EdWideSlot* __restrict__ wed) {
#if ED_WIDE_ROWS_PRIO  // (A/B) issue priority over the ECDSA row builds sharing the SIMDs
  __builtin_amdgcn_s_setprio(ED_WIDE_ROWS_PRIO);
#endif
  const WideLane L = wide_lane(EdWideCfg::kRows, ED_WIDE_ROW_LANES);
  if (L.l >= wide_count[PLAN_ED]) return;
  const uint32_t i = wide[(size_t)PLAN_ED * n_keys + L.l];
  if (hdr[i].status != 0) return;
  EdWideSlot& ws = wed[wide_idx[i]];
  constexpr int per = EdWideCfg::kMult / ED_WIDE_ROW_LANES;
  const uint32_t lane = L.j * ED_WIDE_ROW_LANES + L.g, lanes = (uint32_t)(EdWideCfg::kRows * ED_WIDE_ROW_LANES);
#if ED_WIDE_ROWS9
  ed_wide_row_build9(ws.tab.t[L.j], EdPark9Lanes{ws.park, lane, lanes}, ws.bases[L.j], per * (int)L.g,
                     per * (int)L.g + per, c_ed.d2);
#else
  ed_wide_row_build(ws.tab.t[L.j], EdParkLanes{ws.park, lane, lanes}, ws.bases[L.j], per * (int)L.g,
                    per * (int)L.g + per, c_ed.d2);
#endif
}
#ifndef CG_ED_WIDE_ROWS
#define CG_ED_WIDE_ROWS 1
#endif

// The base point B as an extended point (from the constant niels table entry 1*B)
__device__ void ed_base_point(ge_p3& B) {
  fe x, y, two_inv, t;
  fe_sub(x, c_ed.Btab[1].ypx, c_ed.Btab[1].ymx);
  fe_add(y, c_ed.Btab[1].ypx, c_ed.Btab[1].ymx);
  fe_0(t);
  t.v[0] = 2;
  fe_invert(two_inv, t);
  fe_mul(B.X, x, two_inv);
  fe_mul(B.Y, y, two_inv);
  fe_1(B.Z);
  fe_mul(B.T, B.X, B.Y);
}

// B rows (radix 2^ED_WB), built once per context: one lane per (row, group of 8 multiples)
__global__ void __launch_bounds__(64) k_ed_btab_init(EdBTab* __restrict__ out) {
  constexpr uint32_t G = EdBCfgT::kMult / 8;
  const uint32_t g = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t u = g / G, grp = g % G;
  if (u >= (uint32_t)EdBCfgT::kDigits) return;
  ge_p3 P;
  ed_base_point(P);
  if (EdBCfgT::shift(u) > 0) ed_dbl_n(P, P, EdBCfgT::shift(u));
  ge_p3 pts[8];
  ed_small_mul(pts[0], P, 8 * grp + 1, c_ed.d2);
  ge_cached c;
  ge_p3_to_cached(c, P, c_ed.d2);
  ge_p1p1 t;
  for (int k = 1; k < 8; ++k) {
    ge_add_cached(t, pts[k - 1], c);
    ge_p1p1_to_p3(pts[k], t);
  }
  ge_niels row[8];
  ed_niels_batch8(row, pts, c_ed.d2);
  for (int k = 0; k < 8; ++k) out->t[u][8 * grp + k] = row[k];
}

// Wide B rows (radix 2^ED_WIDE_BW, row u = multiples of 2^{ED_WIDE_BW u} B), built once per
// context: the row bases first (one lane per row, into the constant-table scratch), then one lane
// per (row, group of 8 multiples)
__global__ void __launch_bounds__(64) k_ed_bwide_bases(ge_p3* __restrict__ bases) {
  const uint32_t u = blockIdx.x * blockDim.x + threadIdx.x;
  if (u >= (uint32_t)EdWideCfg::kBDigits) return;
  ge_p3 P;
  ed_base_point(P);
  if (u > 0) ed_dbl_n(P, P, ED_WIDE_BW * (int)u);
  bases[u] = P;
}
__global__ void __launch_bounds__(64) k_ed_bwide_init(EdBWideTab* __restrict__ out, const ge_p3* __restrict__ bases) {
  constexpr uint32_t G = EdWideCfg::kBMult / 8;
  const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t u = (uint32_t)(g / G), grp = (uint32_t)(g % G);
  if (g == 0) ge9_niels_identity_half(out->ident);
  if (u >= (uint32_t)EdWideCfg::kBDigits) return;
  ed_bwide_group(&out->t[u][8 * grp], bases[u], 0, (int)grp, c_ed.d2);
}

__device__ __forceinline__ void ld_niels(ge_niels& n, const ge_niels* src) {
  const uint4* p = (const uint4*)src;
  uint32_t* d = (uint32_t*)&n;
#pragma unroll
  for (int q = 0; q < 7; ++q) {
    const uint4 v = p[q];
    d[4 * q] = v.x;
    d[4 * q + 1] = v.y;
    d[4 * q + 2] = v.z;
    d[4 * q + 3] = v.w;
  }
  const uint2 v = ((const uint2*)src)[14];
  d[28] = v.x;
  d[29] = v.y;
}

__device__ __forceinline__ void pick(ge_niels& out, const ge_niels* row, int d) {
  const int a = d < 0 ? -d : d;
  ld_niels(out, row + (a > 0 ? a - 1 : 0));
  if (a == 0) ge_niels_identity(out);
  ge_niels_cneg(out, d < 0);
}

// Digits handed from k_ed_hash to k_ed_ladder through the item slot (the ladder reads them
// before it writes R' into the same slot).
struct EdDigits {  // h in radix 2^6 (int8), S' in radix 2^ED_WIDE_BW (the wide B table's digits)
  uint32_t eh[EdCfg::kPackedWords], es[EdWideCfg::kBPackedWords];
  uint32_t pad[(ITEM_SLOT - 4 * (EdCfg::kPackedWords + EdWideCfg::kBPackedWords)) / 4];
};
static_assert(sizeof(EdDigits) == ITEM_SLOT, "digits must fill one item slot");
// the same hand-off for an item of a wide-table key: h in radix 2^8, S' in radix 2^12
struct EdDigitsWide {
  uint32_t eh[EdWideCfg::kPackedWords], es[EdWideCfg::kBPackedWords];
  uint32_t pad[(ITEM_SLOT - 4 * (EdWideCfg::kPackedWords + EdWideCfg::kBPackedWords)) / 4];
};
static_assert(sizeof(EdDigitsWide) == ITEM_SLOT, "digits must fill one item slot");

// One lane per Ed25519 plan position: item checks, h = SHA-512(R || Abyte || M) mod L,
// S' = i2p's slide value of S mod L, both recoded to signed radix-64 digits. Needs only the
// decoded keys (Abyte), so it runs while the key tables are still being built.
// 4 waves/SIMD (128 VGPRs, 52 B of scratch, no spill inside the SHA-512 round loops): the rounds
// are a dependent chain per lane, and at 3 waves (144 VGPRs) the SIMDs issued ~55% of the time;
// round 5: 5.55 -> 5.16 ms of k_ed_hash per headline step, with Ch as bitop3 5.0 ms (A/B, two
// rounds, profiles/r05/hash). (Round 1 went 2 -> 3 waves: 208 -> 214 M sigs/s.)
#ifndef ED_HASH_WAVES_PER_SIMD
#define ED_HASH_WAVES_PER_SIMD 4
#endif
#ifndef ED_HASH_STATUS_EARLY
#define ED_HASH_STATUS_EARLY 0
#endif
#ifndef ED_HASH_MID_SCHEDULE
#define ED_HASH_MID_SCHEDULE 1
#endif
template <bool Fused>
__device__ __forceinline__ void ed_hash_one(uint64_t p, const cg_item* __restrict__ items,
                                            const uint32_t* __restrict__ perm, const EdKeyHdr* __restrict__ hdr,
                                            const uint8_t* __restrict__ arena, uint64_t arena_len,
                                            const uint8_t* __restrict__ msgs, uint64_t msgs_len, uint32_t mode,
                                            uint8_t* __restrict__ status, EdDigits* __restrict__ dig, bool wide,
                                            const EdCols& ec) {
  const uint32_t i = perm[p];
  const cg_item it = items[i];
  ec.key[p] = it.key_idx;
  const EdKeyHdr* kh = hdr + it.key_idx;
  uint8_t st;  // a key that does not decode overrides this in k_ed_ladder
  if (mode == CG_MODE_DOVERIFY && (it.sig_len == 0 || it.msg_len == 0)) {
    st = CG_EMPTY;
  } else if (!in_arena(it.sig_off, it.sig_len, arena_len) ||
             (Fused ? !item_fused(it, msgs)
                    : !in_arena(it.msg_off, it.msg_len, item_msg_len(it, arena_len, msgs_len, msgs)))) {
    st = CG_NOT_RUN;
  } else if (it.sig_len != 64) {
    st = CG_SIG_MALFORMED;
  } else {
    const uint64_t lr = round4(arena_len);
    uint32_t sw[16];
#pragma unroll
    for (int w = 0; w < 16; ++w) sw[w] = cg_ld_bytes4(arena, lr, it.sig_off + 4 * w);
    uint32_t pre[16], hw[16], h[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      pre[w] = sw[w];
      pre[8 + w] = kh->abyte[w];
    }
    if (Fused) {
      // A wave whose items share one template (the plan groups a scheme's items; one template per
      // scheme in a notary batch) reads the image with scalar addresses and branches and runs block 1
      // from the template's precomputed schedule; a mixed wave takes the per-lane form.
      const uint32_t t0 = __builtin_amdgcn_readfirstlane(it.reserved1);
      if (__builtin_amdgcn_ballot_w64(it.reserved1 != t0) == 0 && ED_HASH_MID_SCHEDULE) {
        const TmplMid* m0 = (const TmplMid*)(msgs + SPLICE_HDR_BYTES) + t0;
        const uint64_t* wk1 =
            m0->ed_mid ? ((const TmplW512*)(msgs + ((const SpliceHdr*)msgs)->w512_off) + t0)->wk : nullptr;
        sha512_prefix64_splice(hw, pre, tmpl_splice(t0, it.msg_off, msgs), __builtin_amdgcn_readfirstlane(it.msg_len),
                               wk1);
      } else {
        sha512_prefix64_splice(hw, pre, item_splice(it, msgs), it.msg_len, (const uint64_t*)nullptr);
      }
    } else
      sha512_prefix64_msg(hw, pre, item_msg_arena(it, arena, msgs),
                          round4(item_msg_len(it, arena_len, msgs_len, msgs)), it.msg_off, it.msg_len);
    sc_reduce512(h, hw);
    uint32_t s[8], sr[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) s[w] = sw[8 + w];
    sc_reduce256(sr, s);
    if (s[7] >> 31) {
      if (sc_slide_escapes(s)) {
        uint32_t r1[8];
#pragma unroll
        for (int w = 0; w < 8; ++w) r1[w] = sc_R1w(w);
        sc_sub(sr, sr, r1);
      }
    }
    // only the digit words are stored (round 6): the whole 120-B slot store wrote its 48-B pad too,
    // ~48 B of HBM writes per item for nothing (profiles/r06/headline pmc_traffic.json)
    if (wide) {
      EdDigitsWide d;
      sc_recode_w<ED_WIDE_W>(d.eh, EdWideCfg::kPackedWords, h);
      sc_recode_wb<ED_WIDE_BW, EdWideCfg::kBBits>(d.es, EdWideCfg::kBPackedWords, sr);
      EdDigitsWide* o = (EdDigitsWide*)dig + p;
#pragma unroll
      for (int w = 0; w < EdWideCfg::kPackedWords; ++w) o->eh[w] = d.eh[w];
#pragma unroll
      for (int w = 0; w < EdWideCfg::kBPackedWords; ++w) o->es[w] = d.es[w];
    } else {
      EdDigits d;
      sc_recode_w<ED_W>(d.eh, EdCfg::kPackedWords, h);
      sc_recode_wb<ED_WIDE_BW, EdWideCfg::kBBits>(d.es, EdWideCfg::kBPackedWords, sr);
      EdDigits* o = dig + p;
#pragma unroll
      for (int w = 0; w < EdCfg::kPackedWords; ++w) o->eh[w] = d.eh[w];
#pragma unroll
      for (int w = 0; w < EdWideCfg::kBPackedWords; ++w) o->es[w] = d.es[w];
    }
    st = (uint8_t)ED_PENDING;
#pragma unroll
    for (int w = 0; w < 8; ++w) ec.r[(size_t)w * ec.n + p] = sw[w];
  }
  ec.pend[p] = st == ED_PENDING;
  // ED_HASH_STATUS_EARLY=0 (round 6): a pending item's status byte is left as k_misc_status set it
  // (CG_NOT_RUN) until k_ed_finish writes the verdict: nothing reads ED_PENDING, and a 1-byte store at
  // a random position (items are in plan order here) cost the kernel a whole written-back line per item
  if (!ED_HASH_STATUS_EARLY ? st != (uint8_t)ED_PENDING : true) status[i] = st;
}

template <bool Fused>  // Fused: every item's message is a SignableData splice (the tx-signature paths)
__global__ void __launch_bounds__(256, ED_HASH_WAVES_PER_SIMD) k_ed_hash(
    const cg_item* __restrict__ items, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ ranges,
    const EdKeyHdr* __restrict__ hdr, const uint8_t* __restrict__ arena, uint64_t arena_len,
    const uint8_t* __restrict__ msgs, uint64_t msgs_len, uint32_t mode, uint8_t* __restrict__ status,
    EdDigits* __restrict__ dig, EdCols ec) {
  front_prio();
  const uint32_t beg = ranges[PLAN_ED], wbeg = ranges[PLAN_WIDE + PLAN_ED];
  for (Walk w = walk_units(ranges[PLAN_ED + 1] - beg); w.u < w.end; w.u += w.step)
    ed_hash_one<Fused>(beg + w.u, items, perm, hdr, arena, arena_len, msgs, msgs_len, mode, status, dig,
                       beg + w.u >= wbeg, ec);
}

// One lane per pending Ed25519 plan position: R' = h (-A) + S' B over the row tables (B rows
// staged in LDS), left projective in the item slot.
struct PickGlobal {
  __device__ __forceinline__ void operator()(ge_niels& out, const ge_niels* row, int d) const { pick(out, row, d); }
};

#ifndef ED_LADDER_WAVES_PER_SIMD
#define ED_LADDER_WAVES_PER_SIMD 3  // 168 VGPRs: 3 waves/SIMD beat 2 (measured, r01)
#endif

// ---------------------------------------------------------------- pipelined full-table ladder
// The 55 mixed additions of ed_double_scalar_fw as one flat op sequence (window 1: 21 A rows;
// 6 doublings; window 0: 22 A rows, then the 12 radix-2^22 B rows). Op o+1's niels entry is
// gathered straight into LDS (global_load_lds, no VGPR destination) while op o's addition
// runs, and op o+2's digit word is loaded at the same time: the two dependent memory latencies
// per op (digit, then entry) leave the critical path. LDS image per wave: 7 x 16-B chunks then
// 2 x 4-B chunks, chunk c of lane l at wave_base + 64 * off_c + size_c * l (the DMA's
// lane-linear destination), 7680 B per wave. Only the 16-B and 4-B DMA forms are used: a
// first cut with 12-B chunks read back wrong entries.
typedef __attribute__((address_space(3))) void* cg_lds_ptr;
typedef __attribute__((address_space(1))) void* cg_gbl_ptr;

struct EdOps {
  static constexpr int kNa1 = (EdCfg::kDigits - 1 + ED_K - 1) / ED_K;  // A rows, window 1
  static constexpr int kNa0 = (EdCfg::kDigits + ED_K - 1) / ED_K;      // A rows, window 0
  static constexpr int kOps1 = kNa1;
  static constexpr int kOps = kNa1 + kNa0 + EdWideCfg::kBDigits;
  static constexpr uint32_t kWaveBytes = 64 * sizeof(ge_niels);
};
#ifndef ED_LADDER_PF  // -DED_LADDER_PF=0: the unpipelined full-table ladder (A/B; any ED_K)
#define ED_LADDER_PF 1
#endif
#if ED_LADDER_PF
static_assert(ED_K == 2, "the flat op sequence is written for 2 windows");
#endif
static_assert(sizeof(ge_niels) == 120, "LDS chunking assumes 120-B niels entries");

// op o -> (digit word index in EdDigits, shift, B?, row)
__device__ __forceinline__ void ed_op_info(int o, int& widx, int& sh, bool& is_b, int& row) {
  if (o < EdOps::kNa1 + EdOps::kNa0) {
    const bool w1 = o < EdOps::kOps1;
    const int k = w1 ? o : o - EdOps::kOps1;
    const int t = ED_K * k + (w1 ? 1 : 0);
    widx = t >> 2;
    sh = (t & 3) * 8;
    is_b = false;
    row = k;
  } else {
    constexpr int per = 32 / EdWideCfg::kBBits;
    const int u = o - EdOps::kNa1 - EdOps::kNa0;
    widx = EdCfg::kPackedWords + u / per;
    sh = (u % per) * EdWideCfg::kBBits;
    is_b = true;
    row = u;
  }
}

__device__ __forceinline__ int ed_op_digit(uint32_t w, int sh, bool is_b) {
  if (!is_b) return (int)(int8_t)(uint8_t)(w >> sh);
  return EdWideCfg::kBBits == 16 ? (int)(int16_t)(uint16_t)(w >> sh) : (int)w;
}

// wave_lds_off: the wave's LDS image as a wave-uniform LDS byte offset (readfirstlane'd once
// by the caller), so the per-chunk M0 values are scalar adds, not VALU readfirstlanes
__device__ __forceinline__ cg_lds_ptr ed_lds_at(uint32_t wave_lds_off, uint32_t b) {
  return (cg_lds_ptr)(uintptr_t)(wave_lds_off + b);
}
__device__ __forceinline__ void ed_glds_niels(const ge_niels* src, uint32_t wave_lds_off) {
  const uint8_t* s = (const uint8_t*)src;
#pragma unroll
  for (int c = 0; c < 7; ++c)
    __builtin_amdgcn_global_load_lds((cg_gbl_ptr)(s + 16 * c), ed_lds_at(wave_lds_off, 64 * 16 * c), 16, 0, 0);
  __builtin_amdgcn_global_load_lds((cg_gbl_ptr)(s + 112), ed_lds_at(wave_lds_off, 64 * 112), 4, 0, 0);
  __builtin_amdgcn_global_load_lds((cg_gbl_ptr)(s + 116), ed_lds_at(wave_lds_off, 64 * 116), 4, 0, 0);
}

__device__ __forceinline__ void ed_lds_niels(ge_niels& n, const uint8_t* wave_lds, uint32_t lane) {
  uint32_t* d = (uint32_t*)&n;
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    const uint4 v = *(const uint4*)(wave_lds + 64 * 16 * c + 16 * lane);
    d[4 * c] = v.x;
    d[4 * c + 1] = v.y;
    d[4 * c + 2] = v.z;
    d[4 * c + 3] = v.w;
  }
  d[28] = *(const uint32_t*)(wave_lds + 64 * 112 + 4 * lane);
  d[29] = *(const uint32_t*)(wave_lds + 64 * 116 + 4 * lane);
}

// the radix-2^29 wide-table entries (fe9.h, 112 B): 7 x 16-B chunks, the same lane-linear image
__device__ __forceinline__ void ed_glds_niels9(const ge9_niels* src, uint32_t wave_lds_off) {
  const uint8_t* s = (const uint8_t*)src;
#pragma unroll
  for (int c = 0; c < 7; ++c)
    __builtin_amdgcn_global_load_lds((cg_gbl_ptr)(s + 16 * c), ed_lds_at(wave_lds_off, 64 * 16 * c), 16, 0, 0);
}
__device__ __forceinline__ void ed_lds_niels9(ge9_niels& n, const uint8_t* wave_lds, uint32_t lane) {
  uint32_t* d = (uint32_t*)&n;
#pragma unroll
  for (int c = 0; c < 7; ++c) {
    const uint4 v = *(const uint4*)(wave_lds + 64 * 16 * c + 16 * lane);
    d[4 * c] = v.x;
    d[4 * c + 1] = v.y;
    d[4 * c + 2] = v.z;
    if (c < 6) d[4 * c + 3] = v.w;  // the pad dword stays unread
  }
}
static_assert(64 * 7 * 16 <= EdOps::kWaveBytes, "the LDS image (7 chunks a lane) holds either entry form");

__device__ __forceinline__ const ge_niels* ed_op_src(const EdTab& TA, int row, int d) {
  const int a = d < 0 ? -d : d;
  return &TA.t[row][a > 0 ? a - 1 : 0];
}
__device__ __forceinline__ const ge9_niels* ed_b_src(const EdBWideTab& TB, int row, int d) {
  const int a = d < 0 ? -d : d;
  return a > 0 ? &TB.t[row][a - 1] : &TB.ident;  // a zero digit adds the identity entry
}

// The 55 A additions in radix 2^25.5 (full-table entries), then the 12 B additions in radix 2^29
// (fe9.h, the wide B table's entry form), one entry gathered into LDS one op ahead throughout.
#if ED_LADDER_PF
__device__ __forceinline__ void ed_double_scalar_pf(ge_p2& out, const uint32_t* __restrict__ dw, const EdTab& TA,
                                                    const EdBWideTab& TB, uint8_t* wave_lds, uint32_t lane) {
  constexpr int N = EdOps::kOps, NA = EdOps::kNa1 + EdOps::kNa0;
  const uint32_t wl = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(cg_lds_ptr)wave_lds);
  int widx, sh, row;
  bool is_b;
  // prologue: op 0's digit and entry, op 1's digit word
  ed_op_info(0, widx, sh, is_b, row);
  int d_cur = ed_op_digit(dw[widx], sh, is_b);
  ed_glds_niels(ed_op_src(TA, row, d_cur), wl);
  ed_op_info(1, widx, sh, is_b, row);
  uint32_t w_next = dw[widx];
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int o = 0; o < NA; ++o) {
    if (o == EdOps::kOps1) {  // window 1 -> 0: W doublings while op o's entry is in flight
      for (int d = 0; d < ED_W - 1; ++d) {
        ge_p2_dbl(t, q);
        ge_p1p1_to_p2(q, t);
      }
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // op o's entry and op o+1's digit word
    ge_niels n;
    ed_lds_niels(n, wave_lds, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before the next DMA lands
    if (d_cur == 0) ge_niels_identity(n);
    const bool neg = d_cur < 0;  // the sign goes through the addition, not the entry
    ed_op_info(o + 1, widx, sh, is_b, row);
    d_cur = ed_op_digit(w_next, sh, is_b);
    if (is_b) ed_glds_niels9(ed_b_src(TB, row, d_cur), wl);
    else ed_glds_niels(ed_op_src(TA, row, d_cur), wl);
    ed_op_info(o + 2, widx, sh, is_b, row);
    w_next = dw[widx];
    ge_madd_signed(t, R, n, neg);
    if (o + 1 == EdOps::kOps1) ge_p1p1_to_p2(q, t);
    else ge_p1p1_to_p3(R, t);
  }
  ge9_p3 R9;
  ge9_from_p3(R9, R);
  for (int o = NA; o < N; ++o) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ge9_niels n;
    ed_lds_niels9(n, wave_lds, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const bool neg = d_cur < 0;
    if (o + 1 < N) {
      ed_op_info(o + 1, widx, sh, is_b, row);
      d_cur = ed_op_digit(w_next, sh, is_b);
      ed_glds_niels9(ed_b_src(TB, row, d_cur), wl);
      if (o + 2 < N) {
        ed_op_info(o + 2, widx, sh, is_b, row);
        w_next = dw[widx];
      }
      ge9_madd_half<true>(R9, R9, n, neg);
    } else {
      ge9_madd_half<false>(R9, R9, n, neg);
    }
  }
  ge9_to_p2(out, R9);
}

#endif
// A/B on one box (gpurun_out/ab_sw1, profiles/r01/ed25519_v9): the pipelined ladder at 2
// waves/SIMD (216 VGPRs, no scratch) against k_ed_ladder<true> at 3 waves/SIMD (168 VGPRs,
// digits and spills in scratch): item kernels 4.24 vs 4.28 ms per 2^20 items. The gain is
// small because the ladder is VALU-issue-bound, not latency-bound.
// -DED_LADDER_PF=0 builds the unpipelined ladder for A/B runs (tools/ab.sh).
#ifndef ED_LADDER_PF_WAVES
#define ED_LADDER_PF_WAVES 2
#endif
#if ED_LADDER_PF
__global__ void __launch_bounds__(256, ED_LADDER_PF_WAVES) k_ed_ladder_pf(
    const cg_item* __restrict__ items, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ ranges,
    const EdKeyHdr* __restrict__ hdr, const TabSlot* __restrict__ tabs, const EdBWideTab* __restrict__ btab,
    uint8_t* __restrict__ status, void* __restrict__ slots, EdCols ec) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4 * EdOps::kWaveBytes];
  const uint32_t beg = ranges[PLAN_FULL + PLAN_ED];
  uint8_t* wave_lds = stage + (threadIdx.x >> 6) * EdOps::kWaveBytes;
  for (Walk w = walk_units(ranges[PLAN_WIDE + PLAN_ED] - beg); w.u < w.end; w.u += w.step) {
    const uint64_t p = beg + w.u;
    const uint32_t key = ec.key[p];
    if (hdr[key].status != 0) {  // the key check comes first in i2p / Crypto.doVerify
      status[perm[p]] = CG_KEY_INVALID;
      ec.pend[p] = 0;
      continue;
    }
    if (!ec.pend[p]) continue;
    // every lane still here runs the same DMA sequence; lanes that left do not take part, and
    // the LDS image is per lane, so no barrier is needed
    ge_p2 q;
    ed_double_scalar_pf(q, (const uint32_t*)((const uint8_t*)slots + (size_t)p * ITEM_SLOT), tabs[key].ed, *btab,
                        wave_lds, __lane_id());
    ((ge_p2*)slots)[p] = q;
  }
}
#endif
// ---------------------------------------------------------------- wide-table ladder
// ed_double_scalar_wide as a flat sequence of 54 signed mixed additions (32 rows of the key's
// wide table, then the 22 radix-2^12 B rows), no doublings; each op's entry gathered into LDS
// one op ahead exactly as in ed_double_scalar_pf.
__device__ __forceinline__ void ed_wide_op(int o, int& widx, int& sh, bool& is_b, int& row) {
  is_b = o >= EdWideCfg::kRows;
  if (!is_b) {
    widx = o >> 2;
    sh = (o & 3) * 8;
    row = o;
  } else {
    constexpr int per = 32 / EdWideCfg::kBBits;
    const int u = o - EdWideCfg::kRows;
    widx = EdWideCfg::kPackedWords + u / per;
    sh = (u % per) * EdWideCfg::kBBits;
    row = u;
  }
}
__device__ __forceinline__ int ed_wide_digit(uint32_t w, int sh, bool is_b) {
  if (!is_b) return (int)(int8_t)(uint8_t)(w >> sh);
  return EdWideCfg::kBBits == 16 ? (int)(int16_t)(uint16_t)(w >> sh) : (int)w;
}

__device__ __forceinline__ const ge9_niels* ed_wide_src(const EdWideTab& TA, const EdBWideTab& TB, bool is_b, int row,
                                                        int d) {
  const int a = d < 0 ? -d : d;
  if (a == 0) return &TB.ident;  // a zero digit adds the identity entry (no select in the ladder)
  return is_b ? &TB.t[row][a - 1] : &TA.t[row][a - 1];
}

// 42 signed mixed additions (32 key rows + 10 B rows at radix 2^26) in the radix-2^29 arithmetic
// (fe9.h: ed_double_scalar_wide's form), the first entry folded into the second addition
__device__ __forceinline__ void ed_double_scalar_wide_pf(ge_p2& out, const uint32_t* __restrict__ dw,
                                                         const EdWideTab& TA, const EdBWideTab& TB, uint8_t* wave_lds,
                                                         uint32_t lane) {
  constexpr int N = EdWideCfg::kOps;
  const uint32_t wl = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(cg_lds_ptr)wave_lds);
  int widx, sh, row;
  bool is_b;
  ed_wide_op(0, widx, sh, is_b, row);
  int d_cur = ed_wide_digit(dw[widx], sh, is_b);
  ed_glds_niels9(ed_wide_src(TA, TB, is_b, row, d_cur), wl);
  ed_wide_op(1, widx, sh, is_b, row);
  uint32_t w_next = dw[widx];
  ge9_p3 R;
  // op o's entry from LDS into n, then op o + 1's gather and op o + 2's digit word issued
  auto next = [&](int o, ge9_niels& n, bool& neg) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // op o's entry and op o+1's digit word
    ed_lds_niels9(n, wave_lds, lane);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // slot read before the next DMA lands
    neg = d_cur < 0;
    ed_wide_op(o + 1, widx, sh, is_b, row);
    d_cur = ed_wide_digit(w_next, sh, is_b);
    ed_glds_niels9(ed_wide_src(TA, TB, is_b, row, d_cur), wl);
    if (o + 2 < N) {
      ed_wide_op(o + 2, widx, sh, is_b, row);
      w_next = dw[widx];
    }
  };
  // after next(o, ...), d_cur is op o + 1's digit: ED_SIGN_FOLD flips op o's output by the sign
  // change s_o s_{o+1} (fe9.h ge9_madd_half_flip), the last op's by s_{N-1}
  {  // op 0: identity + q0 (fe9.h ge9_from_niels_half: one product instead of an addition's seven)
    ge9_niels n;
    bool neg;
    next(0, n, neg);
    ge9_from_niels_half(R, n, ED_SIGN_FOLD ? neg != (d_cur < 0) : neg);
  }
  for (int o = 1; o + 1 < N; ++o) {
    ge9_niels n;
    bool neg;
    next(o, n, neg);
#if ED_SIGN_FOLD
    ge9_madd_half_flip<true>(R, R, n, neg != (d_cur < 0));
#else
    ge9_madd_half<true>(R, R, n, neg);
#endif
  }
  {  // the last addition: projective output
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    ge9_niels n;
    ed_lds_niels9(n, wave_lds, lane);
#if ED_SIGN_FOLD
    ge9_madd_half_flip<false>(R, R, n, d_cur < 0);
#else
    ge9_madd_half<false>(R, R, n, d_cur < 0);
#endif
  }
  ge9_to_p2(out, R);
}

// A/B (profiles/r02/w4_rejected): forcing 4 waves/SIMD (128 VGPRs, 52 B/lane of scratch) cost 4% of
// the kernel against the compiler's 144 VGPRs at 3 waves/SIMD (a cap of 2 waves/SIMD leaves the
// allocation at 144: the loop needs no more).
#ifndef ED_LADDER_WIDE_WAVES
#define ED_LADDER_WIDE_WAVES ED_LADDER_PF_WAVES
#endif
#ifndef ED_LADDER_WIDE_OCC  // the waves per SIMD the register use allows (the persistent grid's cap)
#define ED_LADDER_WIDE_OCC 4
#endif
__global__ void __launch_bounds__(256, ED_LADDER_WIDE_WAVES) k_ed_ladder_wide(
    const cg_item* __restrict__ items, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ ranges,
    const EdKeyHdr* __restrict__ hdr, const uint32_t* __restrict__ wide_idx, const EdWideSlot* __restrict__ wed,
    const EdBWideTab* __restrict__ btab, uint8_t* __restrict__ status, void* __restrict__ slots, EdCols ec) {
  __shared__ __attribute__((aligned(16))) uint8_t stage[4 * EdOps::kWaveBytes];
  const uint32_t beg = ranges[PLAN_WIDE + PLAN_ED];
  uint8_t* wave_lds = stage + (threadIdx.x >> 6) * EdOps::kWaveBytes;
  for (Walk w = walk_units(ranges[PLAN_ED + 1] - beg); w.u < w.end; w.u += w.step) {
    const uint64_t p = beg + w.u;
    const uint32_t key = ec.key[p];
    if (hdr[key].status != 0) {  // the key check comes first in i2p / Crypto.doVerify
      status[perm[p]] = CG_KEY_INVALID;
      ec.pend[p] = 0;
      continue;
    }
    if (!ec.pend[p]) continue;
    ge_p2 q;
    ed_double_scalar_wide_pf(q, (const uint32_t*)((const uint8_t*)slots + (size_t)p * ITEM_SLOT),
                             wed[wide_idx[key]].tab, *btab, wave_lds, __lane_id());
    ((ge_p2*)slots)[p] = q;
  }
}

// One lane per pending Ed25519 plan position: R' = h (-A) + S' B over the per-key rows and the
// constant radix-2^10 B table (both in global memory; the B table stays L2-resident), left
// projective in the item slot.
// One launch over the Ed25519 range per table mode (the plan keeps the modes in separate waves);
// separate kernels keep each ladder's registers free of the others'. Mode: PLAN_MODE_ROW0 /
// PLAN_MODE_QUART / PLAN_MODE_FULL (keyws.h).
template <int Mode>
__global__ void __launch_bounds__(256, ED_LADDER_WAVES_PER_SIMD) k_ed_ladder(
    const cg_item* __restrict__ items, const uint32_t* __restrict__ perm, const uint32_t* __restrict__ ranges,
    const EdKeyHdr* __restrict__ hdr, const TabSlot* __restrict__ tabs, const EdBWideTab* __restrict__ btab,
    uint8_t* __restrict__ status, void* __restrict__ slots, EdCols ec) {
  // the plan's mode split: row-0 keys' items, quarter-table keys', full-table keys' (plan_sort.hip)
  const uint32_t beg = Mode == PLAN_MODE_FULL    ? ranges[PLAN_FULL + PLAN_ED]
                     : Mode == PLAN_MODE_QUART ? ranges[PLAN_QUART + PLAN_ED]
                                               : ranges[PLAN_ED];
  const uint32_t end = Mode == PLAN_MODE_FULL    ? ranges[PLAN_WIDE + PLAN_ED]
                     : Mode == PLAN_MODE_QUART ? ranges[PLAN_FULL + PLAN_ED]
                                               : ranges[PLAN_QUART + PLAN_ED];
  for (Walk w = walk_units(end - beg); w.u < w.end; w.u += w.step) {
    const uint64_t p = beg + w.u;
    const uint32_t key = ec.key[p];
    if (hdr[key].status != 0) {  // the key check comes first in i2p / Crypto.doVerify
      status[perm[p]] = CG_KEY_INVALID;
      ec.pend[p] = 0;
      continue;
    }
    if (!ec.pend[p]) continue;
    const EdDigits d = ((const EdDigits*)slots)[p];
    ge_p2 q;
    if (Mode == PLAN_MODE_FULL) {
      ed_double_scalar_fw<ED_W, ED_K>(q, d.eh, d.es, tabs[key].ed, *btab, PickGlobal(), PickGlobal());
    } else if (Mode == PLAN_MODE_QUART) {  // the first rows of the table, 2^{66 j} (-A) (keyws.h)
      ed_double_scalar_fw<ED_W, ED_QK>(q, d.eh, d.es, *(const EdQTab*)&tabs[key].ed, *btab, PickGlobal(),
                                       PickGlobal());
    } else {  // a key with few items: row 0 only (keyws.h)
      ed_double_scalar_row0w<ED_W, ED_K>(q, d.eh, d.es, tabs[key].ed.t[0], *btab, PickGlobal(), PickGlobal());
    }
    ((ge_p2*)slots)[p] = q;
  }
}

// Encode + compare for ED_FINISH_K items per lane: one inversion per lane (Montgomery's trick)
// instead of one per item. A wave takes 64 x K consecutive plan positions, lane l the positions
// l, l + 64, ... of them, so the slot reads of a wave are contiguous (round 1 gave each lane K
// consecutive positions: every lane's 120-B slot reads were a separate pair of cache lines).
#ifndef ED_FINISH_K
#define ED_FINISH_K 16
#endif
__device__ __forceinline__ void ed_finish_one(uint64_t unit, uint32_t beg, uint32_t end,
                                              const uint32_t* __restrict__ perm, uint8_t* __restrict__ status,
                                              const ge_p2* __restrict__ rin, const EdCols& ec) {
  const uint64_t base = beg + (unit >> 6) * (64 * ED_FINISH_K) + (unit & 63);
  fe acc[ED_FINISH_K];
  fe run;
  fe_1(run);
  uint32_t pend = 0;
  for (uint32_t k = 0; k < ED_FINISH_K; ++k) {
    const uint64_t p = base + 64 * k;
    const bool pd = p < end && ec.pend[p];
    pend |= (uint32_t)pd << k;
    if (pd) fe_mul(run, run, rin[p].Z);
    fe_copy(acc[k], run);
  }
  if (!pend) return;
  fe inv;
  fe_invert(inv, run);
  for (int k = ED_FINISH_K - 1; k >= 0; --k) {
    if (!((pend >> k) & 1u)) continue;
    const uint64_t p = base + 64 * (uint32_t)k;
    const ge_p2 P = rin[p];
    fe zi, t;
    // acc[k - 1] = product of the pending Z before k (entries of non-pending items copy it forward)
    if (k > 0) fe_mul(zi, inv, acc[k - 1]);
    else fe_copy(zi, inv);
    fe_mul(t, inv, P.Z);
    fe_copy(inv, t);
    uint32_t rw[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) rw[w] = ec.r[(size_t)w * ec.n + p];
    status[perm[p]] = (uint8_t)ed_encode_cmp(P, zi, rw);
  }
}

__global__ void __launch_bounds__(256) k_ed_finish(const uint32_t* __restrict__ perm,
                                                   const uint32_t* __restrict__ ranges, uint8_t* __restrict__ status,
                                                   const ge_p2* __restrict__ rin, EdCols ec) {
  const uint32_t beg = ranges[PLAN_ED], end = ranges[PLAN_ED + 1];
  const uint64_t units = ((uint64_t)(end - beg) + 64 * ED_FINISH_K - 1) / (64 * ED_FINISH_K) * 64;
  for (Walk w = walk_units(units); w.u < w.end; w.u += w.step)
    ed_finish_one(w.u, beg, end, perm, status, rin, ec);
}

hipError_t ed_upload_constants() {
  Ed25519Consts h;
  ed_consts_init(h);
  return hipMemcpyToSymbol(HIP_SYMBOL(c_ed), &h, sizeof h, 0, hipMemcpyHostToDevice);
}

hipError_t ed_init_const(void* d_btab, void* d_scratch, hipStream_t stream) {
  const uint32_t lanes = EdBCfgT::kDigits * (EdBCfgT::kMult / 8);
  hipLaunchKernelGGL(k_ed_btab_init, dim3((lanes + 63) / 64), dim3(64), 0, stream, (EdBTab*)d_btab);
  static_assert(EdWideCfg::kBDigits * sizeof(ge_p3) <= sizeof(EcRowScratch), "B row bases fit the scratch");
  ge_p3* bases = (ge_p3*)d_scratch;  // free until ec_init_const's G builds (same stream)
  hipLaunchKernelGGL(k_ed_bwide_bases, dim3(1), dim3(64), 0, stream, bases);
  const uint64_t wlanes = (uint64_t)EdWideCfg::kBDigits * (EdWideCfg::kBMult / 8);
  hipLaunchKernelGGL(k_ed_bwide_init, dim3((unsigned)((wlanes + 63) / 64)), dim3(64), 0, stream,
                     (EdBWideTab*)bwide(d_btab), (const ge_p3*)bases);
  return hipGetLastError();
}

void ed_launch_key_abyte(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                         const KeyWs& w, hipStream_t stream) {
  const uint32_t B = 64;
  hipLaunchKernelGGL(k_ed_key_abyte, dim3((n_keys + B - 1) / B), dim3(B), 0, stream, d_keys, n_keys, d_arena,
                     arena_len, w.hdr);
}

// Light phase (decode, row-base chains: latency-bound, few waves) and heavy phase (the row tables:
// throughput-bound), so the host can start the heavy phase after the plan sort (keyws.h).
void ed_launch_keyprep_chains(const cg_key* d_keys, uint32_t n_keys, const uint8_t* d_arena, uint64_t arena_len,
                              const KeyWs& w, hipStream_t stream) {
  const uint32_t B = 64;  // one wave per block: keys are few, spread them over CUs
  hipLaunchKernelGGL(k_ed_keyprep_decode, dim3((n_keys + B - 1) / B), dim3(B), 0, stream, d_keys, n_keys, d_arena,
                     arena_len, w.hdr, w.bases);
  hipLaunchKernelGGL(k_ed_keyprep_chain, dim3((n_keys + B - 1) / B), dim3(B), 0, stream, n_keys, w.hdr,
                     (const uint32_t*)w.full, (const uint32_t*)w.quart, (const uint32_t*)w.full_count, w.bases);
  if (w.cap_ed) {
    const uint32_t lds = chain_spread_lds();
    static const bool quad = [] {  // CG_ED_CHAIN_QUAD=0 (A/B): the one-lane chain
      const char* v = getenv("CG_ED_CHAIN_QUAD");
      return v ? v[0] != '0' : ED_CHAIN_QUAD != 0;
    }();
    const auto kern = quad ? k_ed_wide_chain4 : k_ed_wide_chain;
    const uint64_t lanes = (uint64_t)w.cap_ed * (quad ? 4u : 1u);
    if (lds) hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)((lanes + B - 1) / B)), dim3(B), lds, stream, n_keys, w.hdr,
                       (const uint32_t*)w.wide, (const uint32_t*)w.wide_count, (const uint32_t*)w.wide_idx,
                       (const BaseSlot*)w.bases, w.wed);
  }
}

void ed_launch_keyprep_tabs(const cg_key* d_keys, uint32_t n_keys, const KeyWs& w, hipStream_t stream, bool full,
                            bool wide) {
  const uint32_t B = 64;
  if (full)
    hipLaunchKernelGGL(k_ed_keyprep_tab, dim3(w.park_lanes_ed / B), dim3(B), 0, stream, n_keys, w.hdr, w.bases,
                       (const uint32_t*)w.row0, (const uint32_t*)w.full, (const uint32_t*)w.quart,
                       (const uint32_t*)w.full_count, w.tab, w.park_ed, w.park_lanes_ed);
  if (wide && w.cap_ed) {
    const uint64_t gl = (uint64_t)w.cap_ed * EdWideCfg::kRows * ED_WIDE_GROUPS, rl = (uint64_t)w.cap_ed * EdWideCfg::kRows;
    const uint32_t* wl = (const uint32_t*)w.wide;
    const uint32_t* wc = (const uint32_t*)w.wide_count;
    const uint32_t* wi = (const uint32_t*)w.wide_idx;
    if (CG_ED_WIDE_ROWS) {
      hipLaunchKernelGGL(k_ed_wide_rows, dim3((unsigned)((rl * ED_WIDE_ROW_LANES + B - 1) / B)), dim3(B), 0, stream,
                         n_keys, w.hdr, wl, wc, wi, w.wed);
    } else {
      hipLaunchKernelGGL(k_ed_wide_fwd, dim3((unsigned)((gl + B - 1) / B)), dim3(B), 0, stream, n_keys, w.hdr, wl,
                         wc, wi, w.wed);
      hipLaunchKernelGGL(k_ed_wide_inv, dim3((unsigned)((rl + B - 1) / B)), dim3(B), 0, stream, n_keys, w.hdr, wl,
                         wc, wi, w.wed);
      hipLaunchKernelGGL(k_ed_wide_bwd, dim3((unsigned)((gl + B - 1) / B)), dim3(B), 0, stream, n_keys, w.hdr, wl,
                         wc, wi, w.wed);
    }
  }
}

void ed_launch_front(const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len,
                     uint32_t mode, uint8_t* d_status, const KeyWs& w, const uint8_t* d_msgs, uint64_t msgs_len,
                     const ItemWs& iw, hipStream_t stream) {
  const uint32_t B = 256;  // the Ed25519 range is at most n_items long
  const unsigned grid = walk_grid(n_items, B, WALK_CAP(ED_HASH_WAVES_PER_SIMD));
  if (d_msgs)
    hipLaunchKernelGGL(k_ed_hash<true>, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges, w.hdr, d_arena,
                       arena_len, d_msgs, msgs_len, mode, d_status, (EdDigits*)iw.slots, iw.ed);
  else
    hipLaunchKernelGGL(k_ed_hash<false>, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges, w.hdr, d_arena,
                       arena_len, d_msgs, msgs_len, mode, d_status, (EdDigits*)iw.slots, iw.ed);
}

void ed_launch_ladder(bool full, const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                      const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  const uint32_t B = 256;
  const unsigned grid = walk_grid(n_items, B, WALK_CAP(full && ED_LADDER_PF ? ED_LADDER_PF_WAVES : ED_LADDER_WAVES_PER_SIMD));
  // full: the full-table ladder; else the row-0 then the quarter-table one (the side streams)
#if ED_LADDER_PF
  if (full)
    hipLaunchKernelGGL(k_ed_ladder_pf, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges, w.hdr,
                       w.tab, bwide(d_btab), d_status, iw.slots, iw.ed);
  else
#endif
  if (full) {
    hipLaunchKernelGGL(k_ed_ladder<PLAN_MODE_FULL>, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges,
                       w.hdr, w.tab, bwide(d_btab), d_status, iw.slots, iw.ed);
  } else {
    hipLaunchKernelGGL(k_ed_ladder<PLAN_MODE_ROW0>, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges,
                       w.hdr, w.tab, bwide(d_btab), d_status, iw.slots, iw.ed);
    hipLaunchKernelGGL(k_ed_ladder<PLAN_MODE_QUART>, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges,
                       w.hdr, w.tab, bwide(d_btab), d_status, iw.slots, iw.ed);
  }
}

void ed_launch_ladder_wide(const cg_item* d_items, uint64_t n_items, uint8_t* d_status, const KeyWs& w,
                           const ItemWs& iw, const void* d_btab, hipStream_t stream) {
  const uint32_t B = 256;
  const unsigned grid = walk_grid(n_items, B, WALK_CAP(ED_LADDER_WIDE_OCC));  // fe9 ladder: 106 VGPRs, 4 waves/SIMD
  hipLaunchKernelGGL(k_ed_ladder_wide, dim3(grid), dim3(B), 0, stream, d_items, iw.perm, iw.ranges, w.hdr,
                     (const uint32_t*)w.wide_idx, (const EdWideSlot*)w.wed, bwide(d_btab), d_status, iw.slots, iw.ed);
}

void ed_launch_finish(const cg_item* d_items, uint64_t n_items, const uint8_t* d_arena, uint64_t arena_len,
                      uint8_t* d_status, const ItemWs& iw, hipStream_t stream) {
  const uint32_t B = 256;
  const uint64_t units = (n_items + 64 * ED_FINISH_K - 1) / (64 * ED_FINISH_K) * 64;
  const unsigned fgrid = walk_grid(units, B, WALK_CAP(2));
  (void)d_items;
  (void)d_arena;
  (void)arena_len;
  hipLaunchKernelGGL(k_ed_finish, dim3(fgrid), dim3(B), 0, stream, iw.perm, iw.ranges, d_status, (const ge_p2*)iw.slots,
                     iw.ed);
}

}  // namespace cg
