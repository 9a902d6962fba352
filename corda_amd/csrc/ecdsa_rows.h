// ECDSA double-scalar multiplication u1 G + u2 Q over "row" tables (signed radix-64 digits,
// the same row/window layout as the Ed25519 path in ed25519_rows.h), plus the split
// per-item pipeline pieces: parse+hash (prep), batched s^-1 (inv), ladder + x-check.
//
// A scalar k < 2^256 is recoded into 43 signed digits e_t in [-32, 32]; digit t = 4j + i
// belongs to row j (11 rows) and window i (4 windows):
//     [k] P = sum_{i<4} 2^{6i} sum_{j<11} e_{4j+i} P_j,   P_j = 2^{24j} P.
// Each row stores the affine multiples 1..32 of P_j (x, y in Montgomery form, 72 B each):
// 25 344 B per point. The G rows are built once per context; the Q rows once per key.
// The loop does 18 Jacobian doublings and one mixed addition per non-zero digit (<= 86),
// against BouncyCastle's ~256 doublings + wNAF additions (ECAlgorithms.sumOfTwoMultiplies).
// Exception cases (R = +-T, R = infinity) are handled inside jac_madd, so adversarial
// inputs stay exact; honest lanes never take those branches.
#pragma once
#include "ec9.h"
#include "ecdsa.h"

#define EC_W 6
#ifndef EC_WINDOWS  // windows per row; EC_ROWS = ceil(43 / EC_WINDOWS) (A/B builds: 11 and 4)
#define EC_WINDOWS 4
#endif
#define EC_DIGITS 43
#define EC_ROWS ((EC_DIGITS + EC_WINDOWS - 1) / EC_WINDOWS)
// quarter tables (keyws.h): EC_QWINDOWS windows per row, EC_QROWS rows (row j = 2^{66 j} Q), in
// the first EC_QROWS rows of the key's EcRowTab
#ifndef EC_QWINDOWS
#define EC_QWINDOWS 11
#endif
#define EC_QROWS ((EC_DIGITS + EC_QWINDOWS - 1) / EC_QWINDOWS)
#define EC_MULT 32
#define EC_PACKED 11

struct EcAff {
  f29 x, y;  // affine, Montgomery form
};

struct EcRowTab {
  EcAff t[EC_ROWS][EC_MULT];  // t[j][k-1] = k * 2^{24j} * P
};
struct EcRowTabQ {
  EcAff t[EC_QROWS][EC_MULT];  // t[j][k-1] = k * 2^{66j} * P (the quarter rows, same layout)
};

// Signed radix-64 digits of a < 2^256, 4 per word as signed bytes. The top digit covers
// bits 252..255 (+ carry <= 16), so no digit overflows.
CG_HD void ec_recode_w6(uint32_t packed[EC_PACKED], const u256w& a) {
#pragma unroll
  for (int w = 0; w < EC_PACKED; ++w) packed[w] = 0;
  int carry = 0;
#pragma unroll
  for (int t = 0; t < EC_DIGITS; ++t) {
    const int bit = t * EC_W;
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)a.w[wi] >> sh;
    if (sh + EC_W > 32 && wi + 1 < 8) x |= (uint64_t)a.w[wi + 1] << (32 - sh);
    int e = (int)((uint32_t)x & 63u) + carry;
    carry = (e + 32) >> 6;
    e -= carry << 6;
    packed[t >> 2] |= ((uint32_t)(e & 0xff)) << ((t & 3) * 8);
  }
}

CG_HD int ec_digit6(const uint32_t* packed, int t) {
  return (int)(int8_t)(uint8_t)(packed[t >> 2] >> ((t & 3) * 8));
}

// General Jacobian addition r = p + q (add-2007-bl), exception-complete.
template <int C>
CG_HD void jac_add(Jac& r, const Jac& p, const Jac& q, const EcConsts& K) {
  if (m29_iszero<C, 0>(p.Z)) {
    r = q;
    return;
  }
  if (m29_iszero<C, 0>(q.Z)) {
    r = p;
    return;
  }
  f29 Z1Z1, Z2Z2, U1, U2, S1, S2, H, rr, I, J, V, t;
  m29_sq<C, 0>(Z1Z1, p.Z);
  m29_sq<C, 0>(Z2Z2, q.Z);
  m29_mul<C, 0>(U1, p.X, Z2Z2);
  m29_mul<C, 0>(U2, q.X, Z1Z1);
  m29_mul<C, 0>(S1, p.Y, q.Z);
  m29_mul<C, 0>(S1, S1, Z2Z2);
  m29_mul<C, 0>(S2, q.Y, p.Z);
  m29_mul<C, 0>(S2, S2, Z1Z1);
  m29_sub<C, 0>(H, U2, U1);
  m29_sub<C, 0>(rr, S2, S1);
  if (m29_iszero<C, 0>(H)) {
    if (m29_iszero<C, 0>(rr)) {
      jac_dbl<C>(r, p);
    } else {
      jac_set_inf<C>(r, K);
    }
    return;
  }
  m29_add_lazy(I, H, H);
  m29_sq<C, 0>(I, I);
  m29_mul<C, 0>(J, H, I);
  m29_mul<C, 0>(V, U1, I);
  m29_add_lazy(rr, rr, rr);
  Jac o;
  m29_sq<C, 0>(o.X, rr);
  m29_sub<C, 0>(o.X, o.X, J);
  m29_add<C, 0>(t, V, V);
  m29_sub<C, 0>(o.X, o.X, t);
  m29_sub<C, 0>(t, V, o.X);
  m29_mul<C, 0>(o.Y, rr, t);
  m29_add_lazy(t, S1, S1);
  m29_mul<C, 0>(t, t, J);
  m29_sub<C, 0>(o.Y, o.Y, t);
  m29_add_lazy(t, p.Z, q.Z);
  m29_sq<C, 0>(t, t);
  m29_sub<C, 0>(t, t, Z1Z1);
  m29_sub<C, 0>(t, t, Z2Z2);
  m29_mul<C, 0>(o.Z, t, H);
  r = o;
}

// 2^n * P (the row-base chains: jac_dbl_w, fewer carry chains than jac_dbl, same point)
template <int C>
CG_HD void jac_dbl_n(Jac& r, const Jac& p, int n) {
  Jac t = p;
  for (int i = 0; i < n; ++i) jac_dbl_w<C>(t, t);
  r = t;
}

// One row: the affine multiples 1..32 of the (finite, prime-order) Jacobian point `base`.
// `scratch` holds 32 Jacobian points and 32 prefix products (the batch inversion runs
// through memory, not registers). One field inversion per row.
struct EcRowScratch {
  Jac p[EC_MULT];
  f29 pre[EC_MULT];
};

// A G wide-table entry packed into 64 B (EC_GWIDE_PACK, A/B): x and y as canonical 256-bit values
// (little-endian dwords), so a random gather is one 128-B line request instead of ~1.5 and the
// table is 21.5 instead of 24.2 GB per curve; the ladder unpacks the 29-bit limbs (ec_unpack256).
// Measured: ECDSA wide ladders 7.72 / 3.43 -> 7.79 / 3.46 ms per step (r1 / k1), headline within
// noise (profiles/r05/ec_pack): the unpacking costs what the bytes saved; the 72-B entries stay.
struct EcAffG64 {
  uint32_t w[16];
};
CG_HD void ec_pack256(uint32_t* w, const f29& a) {  // a canonical (< 2^256)
  uint64_t acc = 0;
  int bits = 0, j = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    acc |= (uint64_t)a.v[i] << bits;
    bits += 29;
    if (bits >= 32) {
      w[j++] = (uint32_t)acc;
      acc >>= 32;
      bits -= 32;
    }
  }
  FE_ASSERT(j == 8 && acc == 0);
}
CG_HD void ec_unpack256(f29& a, const uint32_t* w) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int b = 29 * i, j = b >> 5, sh = b & 31;
    const uint32_t lo = w[j], hi = j + 1 < 8 ? w[j + 1] : 0u;
    a.v[i] = (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & M29_MASK;
  }
}
template <int C>
CG_HD void ec_put(EcAff& o, const f29& x, const f29& y) {
  o.x = x;
  o.y = y;
}
template <int C>
CG_HD void ec_put(EcAffG64& o, const f29& x, const f29& y) {
  f29 c;
  m29_canon<C, 0>(c, x);
  ec_pack256(o.w, c);
  m29_canon<C, 0>(c, y);
  ec_pack256(o.w + 8, c);
}
CG_HD void ec_pick(f29& x, f29& y, const EcAffG64* row, int a) {
  ec_unpack256(x, row[a - 1].w);
  ec_unpack256(y, row[a - 1].w + 8);
}

// cnt (<= EC_MULT) affine points first + k step, k = 0..cnt-1, with one batched inversion.
template <int C, class Out>
CG_HD void ec_multiples(Out* out, const Jac& first, const Jac& step, int cnt, EcRowScratch& s, const EcConsts& K) {
  Jac acc = first;
  s.p[0] = acc;
  s.pre[0] = acc.Z;
  for (int k = 1; k < cnt; ++k) {
    jac_add<C>(acc, acc, step, K);  // acc == step goes through the doubling branch
    s.p[k] = acc;
    m29_mul<C, 0>(s.pre[k], s.pre[k - 1], acc.Z);
  }
  f29 inv;
  m29_inv<C, 0>(inv, s.pre[cnt - 1], K.one_p);
  for (int k = cnt - 1; k >= 0; --k) {
    f29 zi, zi2, zi3;
    if (k > 0) {
      m29_mul<C, 0>(zi, inv, s.pre[k - 1]);
      m29_mul<C, 0>(inv, inv, s.p[k].Z);
    } else {
      zi = inv;
    }
    m29_sq<C, 0>(zi2, zi);
    m29_mul<C, 0>(zi3, zi2, zi);
    f29 ox, oy;
    m29_mul<C, 0>(ox, s.p[k].X, zi2);
    m29_mul<C, 0>(oy, s.p[k].Y, zi3);
    ec_put<C>(out[k], ox, oy);
  }
}

// One row: the affine multiples 1..32 of the (finite, prime-order) Jacobian point `base`.
template <int C>
CG_HD void ec_row_build(EcAff* row, const Jac& base, EcRowScratch& s, const EcConsts& K) {
  ec_multiples<C>(row, base, base, EC_MULT, s, K);
}

// Row builds for many keys at once (k_ec_keyprep_tab): ec_row_build with the walk's points and
// running products parked lane-interleaved (dword d of field q of entry k at
// base[(k * EC_ROW_PARK + 9 q + d) * lanes + lane]), so one store of a wave is 64 consecutive
// dwords. The per-key EcRowScratch made every store and load of the two walks touch 64 cache
// lines: the 2^20-distinct-key leg's row-0 builds took 52 / 28 ms per call (profiles/r04/kd).
#define EC_ROW_PARK 36  // X, Y, Z and the running product: 4 x 9 limbs
struct EcRowParkLanes {
  uint32_t* base;
  uint32_t lane, lanes;
  CG_HDM void st(int k, int q, const f29& f) const {
    uint32_t* p = base + (size_t)(k * EC_ROW_PARK + q * 9) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 9; ++d) p[(size_t)d * lanes] = f.v[d];
  }
  CG_HDM void ld(int k, int q, f29& f) const {
    const uint32_t* p = base + (size_t)(k * EC_ROW_PARK + q * 9) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 9; ++d) f.v[d] = p[(size_t)d * lanes];
  }
};
template <int C>
CG_HD void ec_row_build_parked(EcAff* row, const Jac& base, const EcRowParkLanes& pk, const EcConsts& K) {
  Jac acc = base;
  f29 run = acc.Z;
  pk.st(0, 0, acc.X);
  pk.st(0, 1, acc.Y);
  pk.st(0, 2, acc.Z);
  pk.st(0, 3, run);
#pragma unroll 1
  for (int k = 1; k < EC_MULT; ++k) {
    jac_add<C>(acc, acc, base, K);  // k = 1: acc == base goes through the doubling branch
    m29_mul<C, 0>(run, run, acc.Z);
    pk.st(k, 0, acc.X);
    pk.st(k, 1, acc.Y);
    pk.st(k, 2, acc.Z);
    pk.st(k, 3, run);
  }
  f29 inv;
  m29_inv<C, 0>(inv, run, K.one_p);
#pragma unroll 1
  for (int k = EC_MULT - 1; k >= 0; --k) {
    f29 X, Y, zi, zi2, zi3;
    pk.ld(k, 0, X);
    pk.ld(k, 1, Y);
    if (k > 0) {
      f29 pr, Z;
      pk.ld(k - 1, 3, pr);
      pk.ld(k, 2, Z);
      m29_mul<C, 0>(zi, inv, pr);
      m29_mul<C, 0>(inv, inv, Z);
    } else {
      zi = inv;
    }
    m29_sq<C, 0>(zi2, zi);
    m29_mul<C, 0>(zi3, zi2, zi);
    m29_mul<C, 0>(row[k].x, X, zi2);
    m29_mul<C, 0>(row[k].y, Y, zi3);
  }
}

// The 11 row bases 2^{24j} P of an affine (Montgomery) point.
template <int C>
CG_HD void ec_row_bases(Jac bases[EC_ROWS], const f29& xm, const f29& ym, const EcConsts& K) {
  Jac P = {xm, ym, K.one_p};
  for (int j = 0; j < EC_ROWS; ++j) {
    bases[j] = P;
    if (j + 1 < EC_ROWS) jac_dbl_n<C>(P, P, EC_W * EC_WINDOWS);
  }
}

// Key decode (BC 1.57 semantics: SPKI / raw / SEC1, point validated on the curve) to the
// affine point in Montgomery form. Returns 0 ok / 3 KEY_INVALID.
template <int C>
CG_HD uint32_t ec_key_decode_xy(f29& xm, f29& ym, const u256w& x, const u256w& y, const EcConsts& K) {
  if (!u256_lt_mod<C, 0>(x) || !u256_lt_mod<C, 0>(y)) return 3;
  f29 l, rhs;
  m29_from_plain<C, 0>(xm, x, K.r2_p);
  m29_from_plain<C, 0>(ym, y, K.r2_p);
  m29_sq<C, 0>(l, ym);
  ec_rhs<C>(rhs, xm, K);
  return m29_eq<C, 0>(l, rhs) ? 0u : 3u;
}

template <int C>
CG_HD uint32_t ec_key_decode_bytes(f29& xm, f29& ym, const uint8_t* arena, uint64_t lr, uint64_t off,
                                   uint32_t len, uint32_t fmt, const EcConsts& K) {
  u256w x, y;
  uint64_t pt = off;
  uint32_t ptlen = len;
  if (fmt == 1) {  // SPKI: this scheme's id-ecPublicKey + named curve, then a 65- or 33-byte point
    const uint32_t pl = C == CG_CURVE_R1 ? 26 : 23;
    if (len == pl + 65) ptlen = 65;
    else if (len == pl + 33) ptlen = 33;
    else return 3;
    for (uint32_t i = 0; i < pl; ++i)
      if (der_byte(arena, lr, off + i) != ec_spki_header_byte(C, (int)i, ptlen)) return 3;
    pt = off + pl;
  } else if (fmt == 0) {  // RAW
    if (len != 64) return 3;
    ec_load_be32(x, arena, lr, off);
    ec_load_be32(y, arena, lr, off + 32);
    return ec_key_decode_xy<C>(xm, ym, x, y, K);
  } else if (fmt != 2) {
    return 3;
  }
  const uint32_t tag = ptlen ? der_byte(arena, lr, pt) : 0u;
  if (ptlen == 65 && (tag == 4 || tag == 6 || tag == 7)) {  // uncompressed / hybrid
    ec_load_be32(x, arena, lr, pt + 1);
    ec_load_be32(y, arena, lr, pt + 33);
    if (tag != 4 && (y.w[0] & 1u) != (tag & 1u)) return 3;  // hybrid tag carries y's parity
    return ec_key_decode_xy<C>(xm, ym, x, y, K);
  }
  if (ptlen == 33 && (tag == 2 || tag == 3)) {
    ec_load_be32(x, arena, lr, pt + 1);
    if (!ec_decompress<C>(y, x, tag & 1u, K)) return 3;
    return ec_key_decode_xy<C>(xm, ym, x, y, K);
  }
  return 3;
}

// ---------------------------------------------------------------- per-item pipeline
// Item workspace between the three stages: after prep {r, s, e}; after inv {r, u1, u2}.
// Padded to the 120-byte item slot (keyws.h), so every scheme's slot arrays share one stride.
struct EcItemWs {
  u256w r, a, b;
  uint32_t pad[6];
};

// Stage 1: DER, range checks, e = SHA-256(M) mod n. Returns 0 (pending: ws filled),
// 1 INVALID or 2 SIG_MALFORMED.
template <int C, class Ld = ArenaLd, class Src = DerArena>
CG_HD uint32_t ecdsa_prep_ld(EcItemWs& ws, const Src& sig, uint32_t sig_len, const Ld& mld, uint64_t msg_off,
                             uint64_t msg_len, const uint32_t* mid = nullptr, uint32_t mid_blocks = 0) {
  u256w r, s;
  bool range_ok = false;
  if (der_sig(sig, sig_len, r, s, &range_ok)) return 2;
  if (!range_ok) return 1;
  if (!u256_lt_mod<C, 1>(r) || !u256_lt_mod<C, 1>(s)) return 1;
  uint32_t h[8];
  sha256_ld_suffix(h, mld, msg_off, msg_len, nullptr, mid, mid_blocks);
  u256w e;
#pragma unroll
  for (int i = 0; i < 8; ++i) e.w[i] = h[7 - i];
  if (!u256_lt_mod<C, 1>(e)) {  // e < 2^256 < 2n
    uint32_t br = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const uint64_t x = (uint64_t)e.w[i] - Mod<C, 1>::w(i) - br;
      e.w[i] = (uint32_t)x;
      br = (uint32_t)(x >> 63);
    }
  }
  ws.r = r;
  ws.a = s;
  ws.b = e;
  return 0;
}

template <int C>
CG_HD uint32_t ecdsa_prep(EcItemWs& ws, const uint8_t* arena, uint64_t lr, uint64_t sig_off, uint32_t sig_len,
                          const uint8_t* marena, uint64_t mlr, uint64_t msg_off, uint64_t msg_len,
                          const uint32_t* mid = nullptr, uint32_t mid_blocks = 0) {
  return ecdsa_prep_ld<C>(ws, DerArena{arena, lr, sig_off}, sig_len, ArenaLd{marena, mlr}, msg_off, msg_len, mid,
                          mid_blocks);
}

// Items per lane of k_ec_inv, one inversion each (round 2: A/B 8 vs 16 vs 32 on MI355X,
// profiles/r02/sha_v2: 16 left ~1 wave per SIMD on a 1M-item curve range). Round 6: 16. Since round 4
// the inversions run on the side streams beside the ladders, so their latency is hidden and what
// counts is the issue slots they take from the ladders: half the inversion share per item, headline
// 338.5 -> 343.5 M sigs/s over 3 pairs, every pair faster (profiles/r06/inv16)
#ifndef EC_INV_K
#define EC_INV_K 16
#endif

// Stage 2 (per group): w = s^-1 by one shared inversion (Montgomery's trick); u1 = e w,
// u2 = r w as canonical plain words. `sel` marks the pending items of this curve among
// ws[0..cnt).
template <int C, int G>
CG_HD void ecdsa_batch_inv(EcItemWs* ws, uint32_t cnt, uint32_t sel, const EcConsts& K) {
  f29 pre[G];
  f29 run = K.one_n;
  for (uint32_t k = 0; k < cnt; ++k) {
    if ((sel >> k) & 1u) {
      f29 sm;
      m29_from_plain<C, 1>(sm, ws[k].a, K.r2_n);  // s R
      m29_mul<C, 1>(run, run, sm);
    }
    pre[k] = run;
  }
  if (!sel) return;
  f29 inv;
  m29_inv<C, 1>(inv, run, K.one_n);  // (prod s)^-1 R
  for (int k = (int)cnt - 1; k >= 0; --k) {
    if (!((sel >> k) & 1u)) continue;
    int prev = k - 1;
    while (prev >= 0 && !((sel >> prev) & 1u)) --prev;
    f29 wm, sm, t, u;
    if (prev >= 0) m29_mul<C, 1>(wm, inv, pre[prev]);  // s_k^-1 R
    else wm = inv;
    m29_from_plain<C, 1>(sm, ws[k].a, K.r2_n);
    m29_mul<C, 1>(inv, inv, sm);
    f29_from_words(t, ws[k].b.w);  // e (plain)
    m29_mul<C, 1>(u, t, wm);       // e w (plain)
    m29_to_words_canon<C, 1>(ws[k].a.w, u);
    f29_from_words(t, ws[k].r.w);  // r (plain)
    m29_mul<C, 1>(u, t, wm);       // r w (plain)
    m29_to_words_canon<C, 1>(ws[k].b.w, u);
  }
}

// ---------------------------------------------------------------- wide-radix G table
// u1 G with signed radix-2^10 digits over a constant table (G is the same for every item):
// 26 rows x 512 affine multiples (958 464 B per curve, global memory, L2-resident). G digit u
// is added in window i_u = floor(4u / 26) from a row pre-scaled by 2^(10u - 6 i_u), exactly
// as the Ed25519 B table (ed25519_rows.h). 43 + 26 = 69 mixed additions instead of 86.
#define EC_GB 10
#define EC_G_DIGITS 26
#define EC_G_MULT 512
#define EC_G_PACKED 13

struct EcGTab {
  EcAff t[EC_G_DIGITS][EC_G_MULT];  // t[u][k-1] = k * 2^(10u - 6 i_u) * G
};

CG_HD int ec_g_window(int u) { return (u * EC_WINDOWS) / EC_G_DIGITS; }
CG_HD int ec_g_shift(int u) { return EC_GB * u - EC_W * ec_g_window(u); }

// signed radix-2^10 digits of a < 2^256, packed 2 per word as int16
CG_HD void ec_recode_w10(uint32_t packed[EC_G_PACKED], const u256w& a) {
#pragma unroll
  for (int w = 0; w < EC_G_PACKED; ++w) packed[w] = 0;
  int carry = 0;
#pragma unroll
  for (int t = 0; t < EC_G_DIGITS; ++t) {
    const int bit = t * EC_GB;
    const int wi = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)a.w[wi] >> sh;
    if (sh + EC_GB > 32 && wi + 1 < 8) x |= (uint64_t)a.w[wi + 1] << (32 - sh);
    int e = (int)((uint32_t)x & 1023u) + carry;
    carry = (e + 512) >> 10;
    e -= carry << 10;
    packed[t >> 1] |= ((uint32_t)(e & 0xffff)) << ((t & 1) * 16);
  }
}

CG_HD int ec_digit10(const uint32_t* packed, int t) {
  return (int)(int16_t)(uint16_t)(packed[t >> 1] >> ((t & 1) * 16));
}

// G row u, multiples 32 g + 1 .. 32 g + 32 (one lane of the per-context table build)
template <int C>
CG_HD void ec_gtab_group(EcAff* out, int u, int g, EcRowScratch& s, const EcConsts& K) {
  Jac P = {K.gx, K.gy, K.one_p};
  if (ec_g_shift(u) > 0) jac_dbl_n<C>(P, P, ec_g_shift(u));
  const uint32_t m = 32u * (uint32_t)g + 1u;  // first multiple, by double-and-add
  Jac F = P;
  for (int b = 30 - __builtin_clz(m); b >= 0; --b) {
    jac_dbl<C>(F, F);
    if ((m >> b) & 1u) jac_add<C>(F, F, P, K);
  }
  ec_multiples<C>(out, F, P, EC_MULT, s, K);
}

// x(R) == r (mod n) for R = (X : Y : Z) by BC's inversion-free test (r Z^2 == X, or
// (r + n) Z^2 == X when r + n < p). Returns 0 VALID / 1 INVALID.
template <int C>
CG_HD uint32_t ecdsa_x_check(const Jac& R, const u256w& r, const EcConsts& K) {
  if (m29_iszero<C, 0>(R.Z)) return 1;
  f29 z2, t, rm;
  m29_sq<C, 0>(z2, R.Z);
  m29_from_plain<C, 0>(rm, r, K.r2_p);
  m29_mul<C, 0>(t, rm, z2);
  if (m29_eq<C, 0>(t, R.X)) return 0;
  u256w rn;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)r.w[i] + Mod<C, 1>::w(i);
    rn.w[i] = (uint32_t)c;
    c >>= 32;
  }
  if (c == 0 && u256_lt_mod<C, 0>(rn)) {
    m29_from_plain<C, 0>(rm, rn, K.r2_p);
    m29_mul<C, 0>(t, rm, z2);
    if (m29_eq<C, 0>(t, R.X)) return 0;
  }
  return 1;
}

// the same check on a wide-ladder result in ec9.h's signed form
template <int C>
CG_HD uint32_t ecdsa_x_check9(const Jac& R, const u256w& r, const EcConsts& K) {
  Jac q;
  ec9_to_m29<C>(q.X, R.X);
  ec9_to_m29<C>(q.Y, R.Y);
  ec9_to_m29<C>(q.Z, R.Z);
  return ecdsa_x_check<C>(q, r, K);
}

template <class Row>
CG_HD void ec_pick(f29& x, f29& y, const Row* row, int a) {
  const EcAff& e = row[a - 1];
  x = e.x;
  y = e.y;
}

// ---------------------------------------------------------------- wide tables (hot keys)
// A key with many items in the call (keyws.h KEY_WIDE_MIN_USES) gets one row per signed
// radix-2^8 digit of u2: row j holds the affine multiples 1..128 of 2^{8j} Q. The top digit
// (bits 248..255 plus the carry) is left in [0, 256] instead of carrying into a 33rd digit, so
// row 31 also holds the multiples 129..256, stored as a 33rd row of the table (304 128 B). G
// gets one row per signed radix-2^22 digit of u1 over a constant table built once per context
// (12 rows x 2^21 multiples of 2^{22u} G, 1.8 GB per curve in HBM; the last digit carries the
// recoding carry out of bit 255). R = one entry per row: 32 + 12 mixed additions, no doublings,
// against 69 additions + 18 doublings over the full tables. The fixed-base radix is an HBM-for-work
// trade: radix 2^12 / 2^16 / 2^20 / 2^22 took 22 / 17 / 13 / 12 G additions; the 2^22 table's
// gathers come from HBM, not MALL, and are still hidden (headline A/B on one MI355X: 2^16 227M,
// 2^20 238M, 2^22 246M sigs/s, profiles/r02/radix_v1).
#define EC_WIDE_W 8
#define EC_WIDE_DIGITS 32
#define EC_WIDE_ROWS 33   // row 32 = multiples 129..256 of row 31's base
#define EC_WIDE_MULT 128
#define EC_WIDE_PACKED 16  // int16 digits (the top one reaches 256)
#ifndef EC_WIDE_GW
#define EC_WIDE_GW 26
#endif
#define EC_WIDE_GDIGITS ((257 + EC_WIDE_GW - 1) / EC_WIDE_GW)  // radix 2^16: 17, the last the carry out of bit 255
#define EC_WIDE_GMULT (1 << (EC_WIDE_GW - 1))
#define EC_WIDE_GBITS (EC_WIDE_GW <= 16 ? 16 : 32)  // digit slot: int16 or int32
#define EC_WIDE_GPACKED ((EC_WIDE_GDIGITS * EC_WIDE_GBITS + 31) / 32)
static_assert(EC_WIDE_GDIGITS * EC_WIDE_GW > 256, "G digits: room for the recoding carry out of bit 255");

struct EcWideTab {
  EcAff t[EC_WIDE_ROWS][EC_WIDE_MULT];  // t[j][k-1] = k 2^{8j} Q; t[32][k-1] = (128 + k) 2^{248} Q
};
// G entries: EC_GWIDE_ENTRY_BYTES 128 (A/B) pads each 72-B entry to one 128-B line (a random
// gather then fetches one line instead of ~1.55, as the Ed25519 B entries, fe9.h GE9_NIELS_BYTES),
// at 42.9 instead of 24.2 GB per curve. Measured slower: 336.3 -> 332.4 M sigs/s over 4 pairs
// (profiles/r05/ecg128); the 72-B packing stays.
#ifndef EC_GWIDE_ENTRY_BYTES
#define EC_GWIDE_ENTRY_BYTES 72
#endif
#ifndef EC_GWIDE_PACK
#define EC_GWIDE_PACK 0
#endif
#if EC_GWIDE_PACK
typedef EcAffG64 EcAffG;
#elif EC_GWIDE_ENTRY_BYTES == 72
typedef EcAff EcAffG;
#else
struct EcAffG : EcAff {
  uint32_t pad[(EC_GWIDE_ENTRY_BYTES - 72) / 4];
};
static_assert(sizeof(EcAffG) == EC_GWIDE_ENTRY_BYTES, "padded G entry");
#endif
struct EcGWideTab {
  EcAffG t[EC_WIDE_GDIGITS][EC_WIDE_GMULT];  // t[u][k-1] = k 2^{EC_WIDE_GW u} G
};
// Batch-inversion scratch of one wide row (the Jacobian X, Y wait in the output entries)
struct EcWideScratch {
  f29 z[EC_WIDE_MULT], pre[EC_WIDE_MULT];
};

// Signed radix-2^W digits of a < 2^256 (D digits), packed as int16. TopUnsigned: the last digit
// keeps the carry (in [0, 2^W]) instead of being recentred.
template <int W, int D, bool TopUnsigned = false, int Bits = 16>
CG_HD void ec_recode_wide(uint32_t* packed, const u256w& a) {
  constexpr int per = 32 / Bits;
  for (int w = 0; w < (D + per - 1) / per; ++w) packed[w] = 0;
  int carry = 0;
#pragma unroll
  for (int t = 0; t < D; ++t) {
    const int bit = t * W;
    uint32_t v = 0;
    if (bit < 256) {
      const int wi = bit >> 5, sh = bit & 31;
      uint64_t x = (uint64_t)a.w[wi] >> sh;
      if (sh + W > 32 && wi + 1 < 8) x |= (uint64_t)a.w[wi + 1] << (32 - sh);
      v = (uint32_t)x & ((1u << W) - 1);
    }
    int e = (int)v + carry;
    if (!TopUnsigned || t + 1 < D) {
      carry = (e + (1 << (W - 1))) >> W;
      e -= carry << W;
    }
    if (Bits == 16) packed[t >> 1] |= ((uint32_t)(e & 0xffff)) << ((t & 1) * 16);
    else packed[t] = (uint32_t)e;
  }
}
template <int Bits>
CG_HD int ec_digit_at(const uint32_t* packed, int t) {
  return Bits == 16 ? (int)(int16_t)(uint16_t)(packed[t >> 1] >> ((t & 1) * 16)) : (int)packed[t];
}

// The affine multiples first + k step, k = 0..cnt-1, one field inversion for the whole run. The
// forward pass leaves X, Y in out[k], Z in z[k] and the running Z products in pre[k]; the backward
// pass starts from inv = 1 / pre[cnt-1]. `step` is affine (x, y), so each step is a mixed addition.
// The wide-table build runs the passes as separate kernels with one inversion per row between.
template <int C>
CG_HD void ec_multiples_fwd(EcAff* out, const Jac& first, const f29& sx, const f29& sy, int cnt, f29* z, f29* pre,
                            const EcConsts& K) {
  Jac acc = first;
  for (int k = 0; k < cnt; ++k) {
    if (k > 0) jac_madd<C>(acc, acc, sx, sy, K);  // acc == step goes through the doubling branch
    out[k].x = acc.X;
    out[k].y = acc.Y;
    z[k] = acc.Z;
    if (k == 0) pre[0] = acc.Z;
    else m29_mul<C, 0>(pre[k], pre[k - 1], acc.Z);
  }
}

template <int C>
CG_HD void ec_multiples_bwd(EcAff* out, const f29& inv_all, int cnt, const f29* z, const f29* pre) {
  f29 inv = inv_all;
  for (int k = cnt - 1; k >= 0; --k) {
    f29 zi, zi2, zi3;
    if (k > 0) {
      m29_mul<C, 0>(zi, inv, pre[k - 1]);
      m29_mul<C, 0>(inv, inv, z[k]);
    } else {
      zi = inv;
    }
    m29_sq<C, 0>(zi2, zi);
    m29_mul<C, 0>(zi3, zi2, zi);
    m29_mul<C, 0>(out[k].x, out[k].x, zi2);
    m29_mul<C, 0>(out[k].y, out[k].y, zi3);
  }
}

// m * (x, y) for a small m >= 1 and an affine (x, y) (double-and-add, MSB first)
template <int C>
CG_HD void jac_small_mul_aff(Jac& r, const f29& x, const f29& y, uint32_t m, const EcConsts& K) {
  Jac F = {x, y, K.one_p};
  for (int b = 30 - __builtin_clz(m); b >= 0; --b) {
    jac_dbl<C>(F, F);
    if ((m >> b) & 1u) jac_madd<C>(F, F, x, y, K);
  }
  r = F;
}

// Forward pass of multiples g * cnt + 1 .. (g + 1) * cnt of wide row j (row 32: 129..256 times the
// top row's base 2^{248} Q); `base` is affine (k_ec_wide_chain normalises the row bases).
template <int C>
CG_HD void ec_wide_group_fwd(EcAff* out, const EcAff& base, int j, int g, int cnt, f29* z, f29* pre,
                             const EcConsts& K) {
  const uint32_t m = (j < EC_WIDE_DIGITS ? 0u : (uint32_t)EC_WIDE_MULT) + (uint32_t)(g * cnt) + 1u;
  Jac F;
  jac_small_mul_aff<C>(F, base.x, base.y, m, K);
  ec_multiples_fwd<C>(out, F, base.x, base.y, cnt, z, pre, K);
}

// ---- wide-table build (as ed25519_rows.h "wide-table build"): one lane per (wide key, row j, group g
// of 32 multiples), walked twice in chunks of EC_WIDE_CHUNK = 2 points: pass 1 stores each chunk's Z
// product, one lane per row batch-inverts the row's 64 chunk products, pass 3 recomputes the points
// and writes the affine entries. Nothing but the chunk products goes through memory between passes.
#define EC_WIDE_CHUNK 2
#define EC_WIDE_CHUNKS (EC_WIDE_MULT / EC_WIDE_CHUNK)  // 64 per row

static_assert(EC_WIDE_CHUNK == 2, "ec_wide_chunk_out is written for chunks of 2");
template <int C>
CG_HD void ec_aff_from(EcAff& e, const Jac& p, const f29& zi) {
  f29 zi2, zi3;
  m29_sq<C, 0>(zi2, zi);
  m29_mul<C, 0>(zi3, zi2, zi);
  m29_mul<C, 0>(e.x, p.X, zi2);
  m29_mul<C, 0>(e.y, p.Y, zi3);
}
// the chunk's affine entries from zinv = 1 / (Z_0 Z_1) (straight-line, as ed_wide_chunk_out)
template <int C>
CG_HD void ec_wide_chunk_out(EcAff* out, const Jac pts[EC_WIDE_CHUNK], const f29& zinv) {
  f29 z1i, z0i;
  m29_mul<C, 0>(z1i, zinv, pts[0].Z);
  m29_mul<C, 0>(z0i, zinv, pts[1].Z);
  EcAff e0, e1;
  ec_aff_from<C>(e0, pts[0], z0i);
  ec_aff_from<C>(e1, pts[1], z1i);
  out[0] = e0;
  out[1] = e1;
}

// Pass 1 (Out = false): zc[c] = chunk c's Z product; pass 3 (Out = true): the group's 32 entries.
// Multiples g * 32 + 1 .. (g + 1) * 32 of the row's affine base (row 32: 129.. of the top row's).
template <int C, bool Out>
CG_HD void ec_wide_group_pass(EcAff* out, f29* zc, const EcAff& base, int j, int g, const EcConsts& K) {
  const uint32_t m = (j < EC_WIDE_DIGITS ? 0u : (uint32_t)EC_WIDE_MULT) + 32u * (uint32_t)g + 1u;
  Jac F;
  jac_small_mul_aff<C>(F, base.x, base.y, m, K);
#pragma unroll 1
  for (int ch = 0; ch < 32 / EC_WIDE_CHUNK; ++ch) {
    Jac pts[EC_WIDE_CHUNK];
    f29 zp;
    if (ch > 0) jac_madd<C>(F, F, base.x, base.y, K);  // the chunk's first point (F == base: doubling branch)
    if (Out) pts[0] = F;
    else zp = F.Z;
#pragma unroll
    for (int k = 1; k < EC_WIDE_CHUNK; ++k) {
      jac_madd<C>(F, F, base.x, base.y, K);
      if (Out) pts[k] = F;
      else m29_mul<C, 0>(zp, zp, F.Z);
    }
    if (Out) ec_wide_chunk_out<C>(out + EC_WIDE_CHUNK * ch, pts, zc[ch]);
    else zc[ch] = zp;
  }
}

// ---- wide-table rows by co-Z additions (round 3): one lane per (wide key, row j) walks the row's
// multiples k B of its affine base B with Meloni's ZADDU, the co-Z addition with update (T + B' and
// B' re-expressed at the sum's Z, 4M + 2S; "New point addition formulae for ECC applications",
// WAIFI 2007). The new Z is the old one times lambda = X_B' - X_T, so only the lambdas are kept; one
// inversion per row then normalises every entry walking back (Z_{k-1}^-1 = lambda_k Z_k^-1, 4
// products per entry): ~14 products per entry against the three-pass form's ~37, no group-start
// scalar multiplications, and one launch. The un-normalised X, Y wait in the row's output
// entries, the lambdas in its scratch. A valid key has prime order n > 256, so T = +-B' never
// happens (lambda != 0).
// (T, B') <- (B' + T, B' at the sum's Z); lam = X_B' - X_T
template <int C>
CG_HD void ec_zaddu(f29& XT, f29& YT, f29& XB, f29& YB, f29& lam) {
  f29 c, w1, w2, t, d, a1, u;
  m29_sub<C, 0>(lam, XB, XT);
  m29_sq<C, 0>(c, lam);
  m29_mul<C, 0>(w1, XB, c);
  m29_mul<C, 0>(w2, XT, c);
  m29_sub2<C, 0>(t, YB, YT);  // product operand only
  m29_sq<C, 0>(d, t);
  m29_sub2<C, 0>(u, w1, w2);
  m29_mul<C, 0>(a1, YB, u);
  m29_sub<C, 0>(XT, d, w1);
  m29_sub<C, 0>(XT, XT, w2);
  m29_sub2<C, 0>(u, w1, XT);
  m29_mul<C, 0>(YT, t, u);
  m29_sub<C, 0>(YT, YT, a1);
  XB = w1;
  YB = a1;
}

// 2B (X, Y at Z = 2y) and B at the same Z from an affine B = (x, y): DBLU, 2M + 4S
template <int C>
CG_HD void ec_dblu_aff(f29& XT, f29& YT, f29& XB, f29& YB, f29& Z, const f29& x, const f29& y, const EcConsts& K) {
  f29 xx, yy, s, l, m, t;
  m29_sq<C, 0>(xx, x);
  m29_sq<C, 0>(yy, y);
  m29_mul<C, 0>(s, x, yy);
  m29_add<C, 0>(s, s, s);
  m29_add<C, 0>(s, s, s);  // S = 4 x y^2
  m29_sq<C, 0>(l, yy);
  m29_add<C, 0>(l, l, l);
  m29_add<C, 0>(l, l, l);
  m29_add<C, 0>(l, l, l);  // 8 y^4
  if (C == CG_CURVE_R1) {  // M = 3 x^2 + a, a = -3
    m29_sub<C, 0>(t, xx, K.one_p);
    m29_add<C, 0>(m, t, t);
    m29_add<C, 0>(m, m, t);
  } else {  // a = 0
    m29_add<C, 0>(m, xx, xx);
    m29_add<C, 0>(m, m, xx);
  }
  m29_sq<C, 0>(XT, m);
  m29_sub<C, 0>(XT, XT, s);
  m29_sub<C, 0>(XT, XT, s);  // M^2 - 2S
  m29_sub2<C, 0>(t, s, XT);
  m29_mul<C, 0>(YT, m, t);
  m29_sub<C, 0>(YT, YT, l);  // M (S - X) - 8 y^4
  XB = s;
  YB = l;
  m29_add<C, 0>(Z, y, y);
}

// Where a row lane parks its entries' X, Y and lambdas between the walks (k = entry index relative
// to the lane's first): EcParkRow in the entries + lam[] (host build), EcParkLanes lane-interleaved
// (the device build, keyws.h EcWideSlot::park).
#define EC_PARK_DWORDS 27  // X, Y and lambda: 3 x 9 limbs
struct EcParkRow {
  EcAff* out;
  f29* lam;
  CG_HDM void put(int k, const f29& X, const f29& Y, const f29& l) const {
    out[k].x = X;
    out[k].y = Y;
    lam[k] = l;
  }
  CG_HDM void get(int k, f29& X, f29& Y, f29& l) const {
    X = out[k].x;
    Y = out[k].y;
    l = lam[k];
  }
};
struct EcParkLanes {
  uint32_t* base;
  uint32_t lane, lanes;
  CG_HDM void st(int k, int q, const f29& f) const {
    uint32_t* p = base + (size_t)(k * EC_PARK_DWORDS + q * 9) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 9; ++d) p[(size_t)d * lanes] = f.v[d];
  }
  CG_HDM void ld(int k, int q, f29& f) const {
    const uint32_t* p = base + (size_t)(k * EC_PARK_DWORDS + q * 9) * lanes + lane;
#pragma unroll
    for (int d = 0; d < 9; ++d) f.v[d] = p[(size_t)d * lanes];
  }
  CG_HDM void put(int k, const f29& X, const f29& Y, const f29& l) const {
    st(k, 0, X);
    st(k, 1, Y);
    st(k, 2, l);
  }
  CG_HDM void get(int k, f29& X, f29& Y, f29& l) const {
    ld(k, 0, X);
    ld(k, 1, Y);
    ld(k, 2, l);
  }
};

// Entries [e0, e1) of row j into out[] (entry e = multiple (top ? 128 : 0) + e + 1; top = row 32,
// the multiples 129..256 of the top row's base). A lane that does not start at entry 0 starts from
// its first multiple's predecessor by a scalar multiplication.
template <int C, class Park>
CG_HD void ec_wide_row_build(EcAff* out, const Park& pk, const EcAff& base, bool top, int e0, int e1,
                             const EcConsts& K) {
  f29 XT, YT, XB, YB, Z, l;
  int e_first, e_lo;  // the first entry ZADDU produces; the first entry the walk back normalises
  const uint32_t m0 = (top ? (uint32_t)EC_WIDE_MULT : 0u) + (uint32_t)e0;  // the multiple before entry e0
  if (m0 == 0) {
    out[0] = base;
    ec_dblu_aff<C>(XT, YT, XB, YB, Z, base.x, base.y, K);
    f29_zero(l);
    pk.put(1 - e0, XT, YT, l);  // Z_1 = 2y: no lambda
    e_first = 2;
    e_lo = 1;
  } else {
    Jac F;
    jac_small_mul_aff<C>(F, base.x, base.y, m0, K);
    f29 z2, z3;
    m29_sq<C, 0>(z2, F.Z);
    m29_mul<C, 0>(z3, z2, F.Z);
    m29_mul<C, 0>(XB, base.x, z2);
    m29_mul<C, 0>(YB, base.y, z3);
    XT = F.X;
    YT = F.Y;
    Z = F.Z;
    e_first = e_lo = e0;
  }
#pragma unroll 1
  for (int e = e_first; e < e1; ++e) {
    ec_zaddu<C>(XT, YT, XB, YB, l);  // Z_e = Z_{e-1} l
    m29_mul<C, 0>(Z, Z, l);
    pk.put(e - e0, XT, YT, l);
  }
  f29 inv;
  m29_inv<C, 0>(inv, Z, K.one_p);
  // the walk back, each entry's parked X, Y and lambda loaded one entry ahead
  f29 X, Y;
  pk.get(e1 - 1 - e0, X, Y, l);
#pragma unroll 1
  for (int e = e1 - 1; e >= e_lo; --e) {
    f29 Xn = X, Yn = Y, ln = l;
    if (e > e_lo) pk.get(e - 1 - e0, Xn, Yn, ln);
    f29 zi2, zi3, x, y;
    m29_sq<C, 0>(zi2, inv);
    m29_mul<C, 0>(zi3, zi2, inv);
    m29_mul<C, 0>(x, X, zi2);
    m29_mul<C, 0>(y, Y, zi3);
    out[e].x = x;
    out[e].y = y;
    if (e > e_lo) m29_mul<C, 0>(inv, inv, l);  // 1 / Z_{e-1}
    X = Xn;
    Y = Yn;
    l = ln;
  }
}
// lanes per row (each walks 128 / EC_WIDE_ROW_LANES entries with its own inversion): more waves for
// a latency-bound walk against one more scalar multiplication and inversion per extra lane
#ifndef EC_WIDE_ROW_LANES
#define EC_WIDE_ROW_LANES 2  // A/B 1 / 2 / 4 lanes: 218.6 / 226.7 / 226.6 and 222.7 / 234.8 / 223.4 M sigs/s (profiles/r03/ab_lanes)
#endif
static_assert(EC_WIDE_MULT % EC_WIDE_ROW_LANES == 0 && EC_WIDE_MULT / EC_WIDE_ROW_LANES >= 2, "row split");

// in place: z[g] <- 1 / z[g] mod p for the NG products of one row (prefix products in pre[])
template <int C, int NG>
CG_HD void m29_invert_run(f29* z, f29* pre, const EcConsts& K) {
  f29 run = z[0];
  pre[0] = run;
  for (int g = 1; g < NG; ++g) {
    m29_mul<C, 0>(run, run, z[g]);
    pre[g] = run;
  }
  f29 inv;
  m29_inv<C, 0>(inv, run, K.one_p);
  for (int g = NG - 1; g > 0; --g) {
    const f29 zg = z[g];
    m29_mul<C, 0>(z[g], inv, pre[g - 1]);
    m29_mul<C, 0>(inv, inv, zg);
  }
  z[0] = inv;
}

// Affine x, y of n finite Jacobian points in place (one inversion; `pre` holds n products).
template <int C>
CG_HD void jac_batch_to_affine(EcAff* out, const Jac* P, int n, f29* pre, const EcConsts& K) {
  pre[0] = P[0].Z;
  for (int k = 1; k < n; ++k) m29_mul<C, 0>(pre[k], pre[k - 1], P[k].Z);
  f29 inv;
  m29_inv<C, 0>(inv, pre[n - 1], K.one_p);
  for (int k = n - 1; k >= 0; --k) {
    f29 zi, zi2, zi3;
    if (k > 0) {
      m29_mul<C, 0>(zi, inv, pre[k - 1]);
      m29_mul<C, 0>(inv, inv, P[k].Z);
    } else {
      zi = inv;
    }
    m29_sq<C, 0>(zi2, zi);
    m29_mul<C, 0>(zi3, zi2, zi);
    m29_mul<C, 0>(out[k].x, P[k].X, zi2);
    m29_mul<C, 0>(out[k].y, P[k].Y, zi3);
  }
}

// Inverses of G group products (one inversion): out[g] = 1 / t_g.
template <int C, int G>
CG_HD void m29_batch_invert_small(f29* out, const f29* t, const EcConsts& K) {
  f29 pre[G];
  pre[0] = t[0];
  for (int g = 1; g < G; ++g) m29_mul<C, 0>(pre[g], pre[g - 1], t[g]);
  f29 inv;
  m29_inv<C, 0>(inv, pre[G - 1], K.one_p);
  for (int g = G - 1; g > 0; --g) {
    m29_mul<C, 0>(out[g], inv, pre[g - 1]);
    m29_mul<C, 0>(inv, inv, t[g]);
  }
  out[0] = inv;
}

// u1 G over the constant radix-2^EC_WIDE_GW table (no doublings needed: added after the Q part)
template <int C, class TabG>
CG_HD void ec_add_g_wide(Jac& R, bool& inf, const u256w& u1, const TabG& TG, const EcConsts& K) {
  uint32_t dg[EC_WIDE_GPACKED];
  ec_recode_wide<EC_WIDE_GW, EC_WIDE_GDIGITS, false, EC_WIDE_GBITS>(dg, u1);
#pragma unroll 1
  for (int u = 0; u < EC_WIDE_GDIGITS; ++u) {
    const int a = ec_digit_at<EC_WIDE_GBITS>(dg, u);
    if (a != 0) {
      f29 x, y;
      ec_pick(x, y, TG.t[u], a < 0 ? -a : a);
      jac_madd_w<C>(R, inf, x, y, a < 0, K);
    }
  }
}

// Stage 3: R = u2 Q + u1 G (Q over the per-key radix-64 rows in EC_WINDOWS windows, then G over
// the constant wide table: 43 + 12 mixed additions, 18 doublings; the round-1 radix-2^10 G table
// spread 26 additions over the windows), then the x-check. Returns 0 VALID / 1 INVALID.
// NW windows over NR rows (NW NR >= 43): the full tables (EC_WINDOWS, EC_ROWS) or the quarter ones
// (EC_QWINDOWS, EC_QROWS: (NW - 1) 6 = 60 doublings)
template <int C, int NW, int NR, class TabG, class TabQ>
CG_HD uint32_t ecdsa_ladder_check_w(const u256w& u1, const u256w& u2, const u256w& r, const TabG& TG, const TabQ& TQ,
                                    const EcConsts& K) {
  static_assert(NW * NR >= EC_DIGITS, "every digit has a row");
  uint32_t dq[EC_PACKED];
  ec_recode_w6(dq, u2);
  Jac R;
  jac_set_inf<C>(R, K);
  bool inf = true;  // R = infinity: doublings skipped, the next addition loads the point
  for (int i = NW - 1; i >= 0; --i) {
    if (i != NW - 1 && !inf) {
#pragma unroll 1
      for (int d = 0; d < EC_W; ++d) jac_dbl_w<C>(R, R);
    }
#pragma unroll 1
    for (int j = 0; j < NR; ++j) {
      const int t = NW * j + i;
      if (t >= EC_DIGITS) continue;
      const int b = ec_digit6(dq, t);
      if (b != 0) {
        f29 x, y;
        ec_pick(x, y, TQ.t[j], b < 0 ? -b : b);
        jac_madd_w<C>(R, inf, x, y, b < 0, K);
      }
    }
  }
  ec_add_g_wide<C>(R, inf, u1, TG, K);
  return ecdsa_x_check<C>(R, r, K);
}
template <int C, class TabG, class TabQ>
CG_HD uint32_t ecdsa_ladder_check(const u256w& u1, const u256w& u2, const u256w& r, const TabG& TG, const TabQ& TQ,
                                  const EcConsts& K) {
  return ecdsa_ladder_check_w<C, EC_WINDOWS, EC_ROWS>(u1, u2, r, TG, TQ, K);
}

// The same check for a key that has only row 0 of its table (few items in the batch,
// keyws.h): Horner over u2's 43 signed radix-64 digits (252 doublings), then u1 G as above.
template <int C, class TabG>
CG_HD uint32_t ecdsa_ladder_check_row0(const u256w& u1, const u256w& u2, const u256w& r, const TabG& TG,
                                       const EcAff* row0, const EcConsts& K) {
  uint32_t dq[EC_PACKED];
  ec_recode_w6(dq, u2);
  Jac R;
  jac_set_inf<C>(R, K);
  bool inf = true;
#pragma unroll 1
  for (int t = EC_DIGITS - 1; t >= 0; --t) {
    if (t != EC_DIGITS - 1 && !inf) {
#pragma unroll 1
      for (int d = 0; d < EC_W; ++d) jac_dbl_w<C>(R, R);
    }
    const int b = ec_digit6(dq, t);
    if (b != 0) {
      f29 x, y;
      ec_pick(x, y, row0, b < 0 ? -b : b);
      jac_madd_w<C>(R, inf, x, y, b < 0, K);
    }
  }
  ec_add_g_wide<C>(R, inf, u1, TG, K);
  return ecdsa_x_check<C>(R, r, K);
}

// R = u1 G + u2 Q over the wide tables, then BC's x-check. Returns 0 VALID / 1 INVALID.
template <int C, class TabG, class TabQ>
CG_HD uint32_t ecdsa_ladder_check_wide(const u256w& u1, const u256w& u2, const u256w& r, const TabG& TG,
                                       const TabQ& TQ, const EcConsts& K) {
  uint32_t dg[EC_WIDE_GPACKED], dq[EC_WIDE_PACKED];
  ec_recode_wide<EC_WIDE_GW, EC_WIDE_GDIGITS, false, EC_WIDE_GBITS>(dg, u1);
  ec_recode_wide<EC_WIDE_W, EC_WIDE_DIGITS, true>(dq, u2);
  Jac R;
  jac_set_inf<C>(R, K);
  bool inf = true;
#pragma unroll 1
  for (int j = 0; j < EC_WIDE_DIGITS; ++j) {
    const int b = ec_digit10(dq, j);  // int16 digits
    if (b != 0) {
      f29 x, y;
      const int a = b < 0 ? -b : b;  // the top digit alone reaches 129..256: row 32
      if (a > EC_WIDE_MULT) ec_pick(x, y, TQ.t[EC_WIDE_DIGITS], a - EC_WIDE_MULT);
      else ec_pick(x, y, TQ.t[j], a);
      jac_madd9<C>(R, inf, x, y, b < 0, K);
    }
  }
#pragma unroll 1
  for (int u = 0; u < EC_WIDE_GDIGITS; ++u) {
    const int a = ec_digit_at<EC_WIDE_GBITS>(dg, u);
    if (a != 0) {
      f29 x, y;
      ec_pick(x, y, TG.t[u], a < 0 ? -a : a);
      jac_madd9<C>(R, inf, x, y, a < 0, K);
    }
  }
  return ecdsa_x_check9<C>(R, r, K);
}

// G wide row u, multiples 32 g + 1 .. 32 g + 32 (one lane of the per-context table build)
// (the group from the row's base P = 2^{EC_WIDE_GW u} G: the host tests build only the groups their digits touch)
template <int C, class Out>
CG_HD void ec_gwide_group_from(Out* out, const Jac& P, int g, EcRowScratch& s, const EcConsts& K) {
  const uint32_t m = 32u * (uint32_t)g + 1u;
  Jac F = P;
  for (int b = 30 - __builtin_clz(m); b >= 0; --b) {
    jac_dbl<C>(F, F);
    if ((m >> b) & 1u) jac_add<C>(F, F, P, K);
  }
  ec_multiples<C>(out, F, P, EC_MULT, s, K);
}

template <int C, class Out>
CG_HD void ec_gwide_group(Out* out, int u, int g, EcRowScratch& s, const EcConsts& K) {
  Jac P = {K.gx, K.gy, K.one_p};
  if (u > 0) jac_dbl_n<C>(P, P, EC_WIDE_GW * u);
  ec_gwide_group_from<C>(out, P, g, s, K);
}
