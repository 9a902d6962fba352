// Ed25519 verification with i2p-eddsa-0.2.0 verdict semantics, one signature per lane.
//
// Reference path: Crypto.isValid -> JCA -> i2p EdDSAEngine.engineVerify
// (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559, scheme Crypto.kt:120-133).
// The verdict rule reproduced here (oracle/ed25519_i2p.py restates it):
//   sig.length != 64                        -> SIG_MALFORMED
//   h = SHA-512(R || Abyte || M) mod L       (Abyte = canonical re-encoding of decoded A)
//   S' = slide(S) value = S - 2^256 * escape (no S < L check; the carry i2p's slide()
//        drops past bit 255 is reproduced by sc_slide_escapes)
//   accept iff encode(h*(-A) + S'*B) == sig[0..32] byte for byte
// The arithmetic is our own: signed radix-16 fixed windows (uniform control flow across the
// 64 lanes of a wave) over a per-key table of 8 multiples of -A and a constant table of 8
// multiples of B, instead of i2p's vartime sliding window. Same group element, same bytes.
#pragma once
#include "ge25519.h"
#include "sc25519.h"
#include "sha2.h"

struct Ed25519Consts {
  fe d, d2, sqrtm1;
  ge_niels Btab[9];  // index k: k*B (k = 0 is the identity)
};

// Per-key precomputation (device workspace), produced once per distinct key (the JVM
// decodes a PublicKey object once: EdDSAPublicKeySpec -> GroupElement + Aneg precompute).
struct EdKeyPrep {
  uint32_t status;      // 0 ok, else CG_KEY_INVALID / CG_UNSUPPORTED
  uint32_t abyte[8];    // canonical encoding of A (hashed into h)
  uint32_t pad[7];
  ge_cached tab[9];     // index k: k*(-A) (k = 0 is the identity)
};

#define ED_ST_VALID 0
#define ED_ST_INVALID 1
#define ED_ST_SIG_MALFORMED 2
#define ED_ST_KEY_INVALID 3

CG_HD void ge_cached_identity(ge_cached& c) {
  fe_1(c.YpX);
  fe_1(c.YmX);
  fe_1(c.Z);
  fe_0(c.T2d);
}

CG_HD void ge_niels_identity(ge_niels& c) {
  fe_1(c.ypx);
  fe_1(c.ymx);
  fe_0(c.xy2d);
}
// the identity as a half-scaled entry (ge_madd_half_signed)
CG_HD void ge_niels_identity_half(ge_niels& c) {
  fe_half(c.ypx);
  fe_half(c.ymx);
  fe_0(c.xy2d);
}

// i2p GroupElement(curve, byte[] s): y = s with bit 255 masked (y >= p accepted), x from
// u/v; no square root -> KEY_INVALID; sign fix-up (x = 0 with sign bit 1 is accepted).
CG_HD int ed_decode_point(ge_p3& A, const uint32_t aw[8], const Ed25519Consts& C) {
  fe y, yy, u, v, v3, x, vxx, chk;
  fe_frombytes_words(y, aw);
  fe_sq(yy, y);
  fe one;
  fe_1(one);
  fe_sub(u, yy, one);
  fe_carry(u);
  fe_mul(v, yy, C.d);
  fe_add(v, v, one);
  fe_sq(v3, v);
  fe_mul(v3, v3, v);        // v^3
  fe_sq(x, v3);
  fe_mul(x, x, v);          // v^7
  fe_mul(x, x, u);          // u v^7
  fe_pow22523(x, x);        // (u v^7)^((p-5)/8)
  fe_mul(x, x, v3);
  fe_mul(x, x, u);          // u v^3 (u v^7)^((p-5)/8)
  fe_sq(vxx, x);
  fe_mul(vxx, vxx, v);
  fe_sub(chk, vxx, u);
  if (!fe_iszero(chk)) {
    fe_add(chk, vxx, u);
    if (!fe_iszero(chk)) return ED_ST_KEY_INVALID;
    fe_mul(x, x, C.sqrtm1);
  }
  if ((uint32_t)fe_isnegative(x) != (aw[7] >> 31)) {
    fe_neg(x, x);
    fe_carry(x);
  }
  fe_copy(A.X, x);
  fe_copy(A.Y, y);
  fe_1(A.Z);
  fe_mul(A.T, x, y);
  return ED_ST_VALID;
}

// Abyte = A.toByteArray() of the point ed_decode_point would return, without the square root:
// the canonical y (bit 255 masked, reduced mod p) and x's sign bit, which the decode's sign
// fix-up makes equal to the encoded bit unless x = 0 (y = +-1, where the fix-up leaves 0).
// Meaningful only for keys that decode (the caller checks the decode status separately).
CG_HD void ed_abyte_fast(uint32_t out[8], const uint32_t aw[8]) {
  fe y;
  fe_frombytes_words(y, aw);
  fe_tobytes_words(out, y);
  uint32_t one = out[0] ^ 1u, m1 = out[0] ^ 0xffffffecu;
#pragma unroll
  for (int i = 1; i < 7; ++i) {
    one |= out[i];
    m1 |= out[i] ^ 0xffffffffu;
  }
  one |= out[7];
  m1 |= out[7] ^ 0x7fffffffu;
  const uint32_t x_zero = (one == 0u) | (m1 == 0u);
  out[7] |= (aw[7] >> 31 & ~x_zero & 1u) << 31;
}

CG_HD void ed_encode_affine(uint32_t out[8], const fe& X, const fe& Y, const fe& Z) {
  fe zi, x, y;
  fe_invert(zi, Z);
  fe_mul(x, X, zi);
  fe_mul(y, Y, zi);
  fe_tobytes_words(out, y);
  out[7] |= (uint32_t)fe_isnegative(x) << 31;
}

// key bytes (raw A, 32 bytes) -> EdKeyPrep
CG_HD void ed_key_prep(EdKeyPrep& kp, const uint32_t aw[8], const Ed25519Consts& C) {
  ge_p3 A;
  kp.status = (uint32_t)ed_decode_point(A, aw, C);
#pragma unroll
  for (int i = 0; i < 7; ++i) kp.pad[i] = 0;
  if (kp.status != ED_ST_VALID) {
#pragma unroll
    for (int i = 0; i < 8; ++i) kp.abyte[i] = 0;
    return;
  }
  ed_encode_affine(kp.abyte, A.X, A.Y, A.Z);
  // -A
  ge_p3 N;
  fe_neg(N.X, A.X);
  fe_carry(N.X);
  fe_copy(N.Y, A.Y);
  fe_copy(N.Z, A.Z);
  fe_neg(N.T, A.T);
  fe_carry(N.T);
  ge_cached_identity(kp.tab[0]);
  ge_cached c1;
  ge_p3_to_cached(c1, N, C.d2);
  kp.tab[1] = c1;
  ge_p3 P = N;
  ge_p1p1 t;
  for (int k = 2; k <= 8; ++k) {
    ge_add_cached(t, P, c1);
    ge_p1p1_to_p3(P, t);
    ge_p3_to_cached(kp.tab[k], P, C.d2);
  }
}

// One signature. sig words: R = sw[0..7], S = sw[8..15] (little-endian).
CG_HD int ed_verify_core(const EdKeyPrep& kp, const ge_cached* ktab, const uint32_t sw[16], const uint8_t* arena,
                         uint64_t len_rounded, uint64_t msg_off, uint64_t msg_len, const Ed25519Consts& C,
                         const ge_niels* btab) {
  // h = SHA-512(R || Abyte || M) mod L
  uint32_t pre[16], hw[16], h[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];
    pre[8 + i] = kp.abyte[i];
  }
  sha512_prefix64_msg(hw, pre, arena, len_rounded, msg_off, msg_len);
  sc_reduce512(h, hw);
  // S' = slide value of S, reduced mod L
  uint32_t s[8], sr[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s[i] = sw[8 + i];
  sc_reduce256(sr, s);
  if (s[7] >> 31) {
    if (sc_slide_escapes(s)) {
      uint32_t r1[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) r1[i] = sc_R1w(i);
      sc_sub(sr, sr, r1);
    }
  }
  uint32_t eh[16], es[16];
  sc_recode16(eh, h);
  sc_recode16(es, sr);
  // R' = h*(-A) + S'*B, fixed signed radix-16 windows, most significant first
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int i = 63; i >= 0; --i) {
    if (i != 63) {
      ge_p3_to_p2(q, R);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    const int da = sc_digit(eh, i);
    const int db = sc_digit(es, i);
    const uint32_t ia = (uint32_t)(da < 0 ? -da : da);
    const uint32_t ib = (uint32_t)(db < 0 ? -db : db);
    ge_cached ca = ktab[ia];
    ge_cached_cneg(ca, da < 0);
    ge_add_cached(t, R, ca);
    ge_p1p1_to_p3(R, t);
    ge_niels nb = btab[ib];
    ge_niels_cneg(nb, db < 0);
    ge_madd(t, R, nb);
    ge_p1p1_to_p3(R, t);
  }
  uint32_t enc[8];
  ed_encode_affine(enc, R.X, R.Y, R.Z);
  uint32_t diff = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) diff |= enc[i] ^ sw[i];
  return diff == 0 ? ED_ST_VALID : ED_ST_INVALID;
}

// Host-side constant construction (also used by the host test build).
CG_HD void ed_consts_init(Ed25519Consts& C) {
  fe a, b, t;
  fe_0(a);
  a.v[0] = 121665;
  fe_0(b);
  b.v[0] = 121666;
  fe_invert(t, b);
  fe_mul(C.d, a, t);
  fe_neg(C.d, C.d);
  fe_carry(C.d);
  fe_add(C.d2, C.d, C.d);
  fe_carry(C.d2);
  // sqrt(-1) = 2^((p-1)/4): compute as 2^((p-5)/8 * 2 + 1) ... use pow22523: x^((p-5)/8)
  // with x = 4: sqrt(-1) = 2^((p-1)/4) = (2^2)^((p-5)/8) * 2
  fe four, two;
  fe_0(four);
  four.v[0] = 4;
  fe_0(two);
  two.v[0] = 2;
  fe_pow22523(t, four);
  fe_mul(C.sqrtm1, t, two);
  // base point: y = 4/5, x even
  fe five, y;
  fe_0(five);
  five.v[0] = 5;
  fe_invert(t, five);
  fe_mul(y, four, t);
  uint32_t yw[8];
  fe_tobytes_words(yw, y);
  ge_p3 B;
  ed_decode_point(B, yw, C);
  ge_niels_identity(C.Btab[0]);
  ge_p3 P = B;
  ge_cached cb;
  ge_p3_to_cached(cb, B, C.d2);
  ge_p1p1 tt;
  for (int k = 1; k <= 8; ++k) {
    if (k > 1) {
      ge_add_cached(tt, P, cb);
      ge_p1p1_to_p3(P, tt);
    }
    fe zi, x, yy, xy;
    fe_invert(zi, P.Z);
    fe_mul(x, P.X, zi);
    fe_mul(yy, P.Y, zi);
    fe_add(C.Btab[k].ypx, yy, x);
    fe_carry(C.Btab[k].ypx);
    fe_sub(C.Btab[k].ymx, yy, x);
    fe_carry(C.Btab[k].ymx);
    fe_mul(xy, x, yy);
    fe_mul(C.Btab[k].xy2d, xy, C.d2);
  }
}

// ====================================================================== v2: row tables
// [k]P for a 253-bit k is computed as sum_i 16^i sum_j e_{8j+i} (2^{32j} P) where e are the
// 64 signed radix-16 digits of k: 8 "rows" P_j = 2^{32j} P, each with the affine multiples
// 1..8 * P_j. 7 x 4 doublings replace 63 x 4; the same table shape serves -A (per key) and
// B (constant, staged in LDS).
struct EdRowTab {
  ge_niels t[8][8];  // t[j][k-1] = k * 2^{32j} * P, affine niels, tight
};

struct Ed25519Rows {
  EdRowTab B;
};

// Normalise 8 extended points to affine niels with one inversion (Montgomery's trick). Half:
// half-scaled entries ((y+x)/2, (y-x)/2, x y d): the inverse carries the 1/2, so x and y come out
// halved and x y d = (x/2)(y/2) 4d.
template <bool Half = false>
CG_HD void ed_niels_batch8(ge_niels out[8], const ge_p3 P[8], const fe& d2_in) {
  fe acc[8], inv, t, d2;
  fe_copy(acc[0], P[0].Z);
  for (int k = 1; k < 8; ++k) fe_mul(acc[k], acc[k - 1], P[k].Z);
  fe_invert(inv, acc[7]);
  if (Half) {
    fe h;
    fe_half(h);
    fe_mul(inv, inv, h);
    fe_add(d2, d2_in, d2_in);
    fe_carry(d2);
  } else {
    fe_copy(d2, d2_in);
  }
  for (int k = 7; k >= 0; --k) {
    fe zi;
    if (k > 0) {
      fe_mul(zi, inv, acc[k - 1]);
      fe_mul(t, inv, P[k].Z);
      fe_copy(inv, t);
    } else {
      fe_copy(zi, inv);
    }
    fe x, y, xy;
    fe_mul(x, P[k].X, zi);
    fe_mul(y, P[k].Y, zi);
    fe_add(out[k].ypx, y, x);
    fe_carry(out[k].ypx);
    fe_sub(out[k].ymx, y, x);
    fe_carry(out[k].ymx);
    fe_mul(xy, x, y);
    fe_mul(out[k].xy2d, xy, d2);
  }
}

// 2^32 * P (32 doublings)
CG_HD void ed_dbl32(ge_p3& R, const ge_p3& P) {
  ge_p2 q;
  ge_p1p1 t;
  ge_p3_to_p2(q, P);
  for (int i = 0; i < 31; ++i) {
    ge_p2_dbl(t, q);
    ge_p1p1_to_p2(q, t);
  }
  ge_p2_dbl(t, q);
  ge_p1p1_to_p3(R, t);
}

// multiples 1..8 of P -> niels row
CG_HD void ed_row_from_point(ge_niels row[8], const ge_p3& P, const fe& d2) {
  ge_p3 M[8];
  M[0] = P;
  ge_cached c;
  ge_p3_to_cached(c, P, d2);
  ge_p1p1 t;
  for (int k = 1; k < 8; ++k) {
    ge_add_cached(t, M[k - 1], c);
    ge_p1p1_to_p3(M[k], t);
  }
  ed_niels_batch8(row, M, d2);
}

CG_HD void ed_rows_init(EdRowTab& T, const ge_p3& P, const fe& d2) {
  ge_p3 Pj = P;
  for (int j = 0; j < 8; ++j) {
    ed_row_from_point(T.t[j], Pj, d2);
    if (j < 7) ed_dbl32(Pj, Pj);
  }
}

// -A as an extended point from a decoded key prep status (host/tests)
CG_HD void ed_neg_point(ge_p3& N, const ge_p3& A) {
  fe_neg(N.X, A.X);
  fe_carry(N.X);
  fe_copy(N.Y, A.Y);
  fe_copy(N.Z, A.Z);
  fe_neg(N.T, A.T);
  fe_carry(N.T);
}

// Select row entry |d| (d in [-8, 8]) with sign; d == 0 gives the identity.
CG_HD void ed_row_pick(ge_niels& out, const ge_niels* row, int d) {
  const int a = d < 0 ? -d : d;
  const ge_niels& src = row[a > 0 ? a - 1 : 0];
  out = src;
  if (a == 0) ge_niels_identity(out);
  ge_niels_cneg(out, d < 0);
}

// Prologue shared by v2: challenge, S' and digits. Returns false if nothing to compute.
CG_HD void ed_scalars(uint32_t eh[16], uint32_t es[16], const uint32_t abyte[8], const uint32_t sw[16],
                      const uint8_t* arena, uint64_t len_rounded, uint64_t msg_off, uint64_t msg_len) {
  uint32_t pre[16], hw[16], h[8];
  for (int i = 0; i < 8; ++i) {
    pre[i] = sw[i];
    pre[8 + i] = abyte[i];
  }
  sha512_prefix64_msg(hw, pre, arena, len_rounded, msg_off, msg_len);
  sc_reduce512(h, hw);
  uint32_t s[8], sr[8];
  for (int i = 0; i < 8; ++i) s[i] = sw[8 + i];
  sc_reduce256(sr, s);
  if (s[7] >> 31) {
    if (sc_slide_escapes(s)) {
      uint32_t r1[8];
      for (int i = 0; i < 8; ++i) r1[i] = sc_R1w(i);
      sc_sub(sr, sr, r1);
    }
  }
  sc_recode16(eh, h);
  sc_recode16(es, sr);
}

// R' = h*(-A) + S'*B with row tables; result left projective (X:Y:Z).
CG_HD void ed_double_scalar_rows(ge_p2& out, const uint32_t eh[16], const uint32_t es[16], const EdRowTab& TA,
                                 const EdRowTab& TB) {
  ge_p3 R;
  ge_p3_0(R);
  ge_p1p1 t;
  ge_p2 q;
  for (int i = 7; i >= 0; --i) {
    if (i != 7) {
      ge_p3_to_p2(q, R);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p2(q, t);
      ge_p2_dbl(t, q);
      ge_p1p1_to_p3(R, t);
    }
    for (int j = 0; j < 8; ++j) {
      ge_niels n;
      ed_row_pick(n, TA.t[j], sc_digit(eh, 8 * j + i));
      ge_madd(t, R, n);
      ge_p1p1_to_p3(R, t);
      ed_row_pick(n, TB.t[j], sc_digit(es, 8 * j + i));
      ge_madd(t, R, n);
      if (i == 0 && j == 7) {
        ge_p1p1_to_p2(out, t);
        return;
      }
      ge_p1p1_to_p3(R, t);
    }
  }
}

// encode (X:Y:Z) given zi = 1/Z, compare with R bytes
CG_HD int ed_encode_cmp(const ge_p2& P, const fe& zi, const uint32_t rw[8]) {
  fe x, y;
  fe_mul(x, P.X, zi);
  fe_mul(y, P.Y, zi);
  uint32_t enc[8];
  fe_tobytes_words(enc, y);
  enc[7] |= (uint32_t)fe_isnegative(x) << 31;
  uint32_t diff = 0;
  for (int i = 0; i < 8; ++i) diff |= enc[i] ^ rw[i];
  return diff == 0 ? ED_ST_VALID : ED_ST_INVALID;
}
