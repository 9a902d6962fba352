// ECDSA (SHA256withECDSA) verification on secp256r1 and secp256k1, one signature per lane,
// with BouncyCastle 1.57 verdict semantics (oracle/ecdsa_bc.py restates them):
//   DER: exactly SEQUENCE{INTEGER r, INTEGER s}, minimal definite lengths, minimal
//        non-empty two's-complement INTEGERs, no trailing bytes, else SIG_MALFORMED
//        (StdDSAEncoder.decode -> SignatureException("error decoding signature bytes."))
//   r, s in [1, n-1] else INVALID (negative INTEGERs included); high-S accepted
//   e = SHA-256(M) (no truncation, 256-bit n); w = s^-1; u1 = e w; u2 = r w (mod n)
//   R = u1 G + u2 Q; infinity -> INVALID; accept iff x(R) == r (mod n), tested as
//   r Z^2 == X or, when r + n < p, (r + n) Z^2 == X (BC's inversion-free test)
// Reference call site: Crypto.isValid (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559),
// schemes ECDSA_SECP256K1_SHA256 (Crypto.kt:92-103) / ECDSA_SECP256R1_SHA256 (:106-117).
//
// This header: plain 256-bit words (u256w) for everything byte-level (DER, hashes, range
// checks); the field / scalar arithmetic in Montgomery form with 29-bit limbs (mont29.h);
// Jacobian point arithmetic; curve constants; key decoding helpers. The double-scalar
// multiplication and the per-item stages are in ecdsa_rows.h.
#pragma once
#include "fe25519.h"
#include "mont29.h"
#include "sha2.h"

#define CG_CURVE_K1 0
#define CG_CURVE_R1 1

struct u256w {
  uint32_t w[8];
};

// ---- moduli ----
template <int C, int N>  // N = 0: field p, N = 1: group order n (plain 32-bit words)
struct Mod {
  CG_HDS uint32_t w(int i) { return m29_w32(C, N, i); }
};

CG_HD void u256_zero(u256w& a) {
#pragma unroll
  for (int i = 0; i < 8; ++i) a.w[i] = 0;
}

CG_HD bool u256_iszero(const u256w& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.w[i];
  return o == 0;
}

CG_HD bool u256_eq(const u256w& a, const u256w& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) o |= a.w[i] ^ b.w[i];
  return o == 0;
}

template <int C, int N>
CG_HD bool u256_lt_mod(const u256w& a) {
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t x = (uint64_t)a.w[i] - Mod<C, N>::w(i) - br;
    br = (uint32_t)(x >> 63);
  }
  return br != 0;
}

// ------------------------------------------------------------------ curve constants
// 8 little-endian words -> plain f29 / Montgomery f29 (value < m)
template <int C, int N>
CG_HD void m29_from_plain(f29& r, const u256w& a, const f29& r2) {
  f29 t;
  f29_from_words(t, a.w);
  m29_mul<C, N>(r, t, r2);
}

// Montgomery -> canonical plain words
template <int C, int N>
CG_HD void m29_to_plain(u256w& r, const f29& a) {
  f29 one, t;
  f29_zero(one);
  one.v[0] = 1;
  m29_mul<C, N>(t, a, one);
  m29_to_words_canon<C, N>(r.w, t);
}

// ------------------------------------------------------------------ curve constants
struct EcConsts {
  f29 one_p, r2_p, one_n, r2_n;  // Montgomery 1 (R mod m) and R^2 mod m, R = 2^261
  f29 b_m;                       // curve b (Montgomery)
  f29 gx, gy;                    // G, affine Montgomery
};

struct Jac {
  f29 X, Y, Z;  // Montgomery, reduced; Z == 0 (mod p) <=> infinity
};

template <int C>
CG_HD void jac_set_inf(Jac& r, const EcConsts& K) {
  f29_zero(r.X);
  r.Y = K.one_p;
  f29_zero(r.Z);
}

template <int C>
CG_HD void jac_dbl(Jac& r, const Jac& p) {
  f29 t1, t2, t3, X3, Y3, Z3;
  if (C == CG_CURVE_R1) {  // a = -3 : dbl-2001-b
    f29 delta, gamma, beta, alpha;
    m29_sq<C, 0>(delta, p.Z);
    m29_sq<C, 0>(gamma, p.Y);
    m29_mul<C, 0>(beta, p.X, gamma);
    m29_sub<C, 0>(t1, p.X, delta);
    m29_add_lazy(t2, p.X, delta);
    m29_mul<C, 0>(alpha, t1, t2);
    m29_add<C, 0>(t1, alpha, alpha);
    m29_add<C, 0>(alpha, alpha, t1);  // 3 (X - delta)(X + delta)
    m29_sq<C, 0>(X3, alpha);
    m29_add<C, 0>(t1, beta, beta);
    m29_add<C, 0>(t1, t1, t1);  // 4 beta
    m29_add<C, 0>(t2, t1, t1);  // 8 beta
    m29_sub<C, 0>(X3, X3, t2);
    m29_add_lazy(t3, p.Y, p.Z);
    m29_sq<C, 0>(Z3, t3);
    m29_sub<C, 0>(Z3, Z3, gamma);
    m29_sub<C, 0>(Z3, Z3, delta);
    m29_sub<C, 0>(t1, t1, X3);
    m29_mul<C, 0>(Y3, alpha, t1);
    m29_add_lazy(t3, gamma, gamma);
    m29_sq<C, 0>(t2, t3);      // 4 gamma^2
    m29_add<C, 0>(t2, t2, t2);  // 8 gamma^2
    m29_sub<C, 0>(Y3, Y3, t2);
  } else {  // a = 0 : dbl-2009-l
    f29 A, B, Cc, D, E, F;
    m29_sq<C, 0>(A, p.X);
    m29_sq<C, 0>(B, p.Y);
    m29_sq<C, 0>(Cc, B);
    m29_add_lazy(t1, p.X, B);
    m29_sq<C, 0>(t1, t1);
    m29_sub<C, 0>(t1, t1, A);
    m29_sub<C, 0>(t1, t1, Cc);
    m29_add<C, 0>(D, t1, t1);
    m29_add<C, 0>(E, A, A);
    m29_add<C, 0>(E, E, A);
    m29_sq<C, 0>(F, E);
    m29_add<C, 0>(t2, D, D);
    m29_sub<C, 0>(X3, F, t2);
    m29_sub<C, 0>(t3, D, X3);
    m29_mul<C, 0>(Y3, E, t3);
    m29_add<C, 0>(t2, Cc, Cc);
    m29_add<C, 0>(t2, t2, t2);
    m29_add<C, 0>(t2, t2, t2);  // 8 C
    m29_sub<C, 0>(Y3, Y3, t2);
    m29_add_lazy(t3, p.Y, p.Y);
    m29_mul<C, 0>(Z3, t3, p.Z);
  }
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// r = p + (x2, y2) affine (madd-2007-bl), exception-complete (infinity, doubling, inverse).
template <int C>
CG_HD void jac_madd(Jac& r, const Jac& p, const f29& x2, const f29& y2, const EcConsts& K) {
  if (m29_iszero<C, 0>(p.Z)) {
    r.X = x2;
    r.Y = y2;
    r.Z = K.one_p;
    return;
  }
  f29 Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
  m29_sq<C, 0>(Z1Z1, p.Z);
  m29_mul<C, 0>(U2, x2, Z1Z1);
  m29_mul<C, 0>(S2, y2, p.Z);
  m29_mul<C, 0>(S2, S2, Z1Z1);
  m29_sub<C, 0>(H, U2, p.X);
  m29_sub<C, 0>(rr, S2, p.Y);
  if (m29_iszero<C, 0>(H)) {
    if (m29_iszero<C, 0>(rr)) {
      jac_dbl<C>(r, p);
    } else {
      jac_set_inf<C>(r, K);
    }
    return;
  }
  m29_sq<C, 0>(HH, H);
  m29_add<C, 0>(I, HH, HH);
  m29_add_lazy(I, I, I);      // 4 HH (< 4m: multiply operand only)
  m29_mul<C, 0>(J, H, I);
  m29_mul<C, 0>(V, p.X, I);
  m29_add_lazy(rr, rr, rr);   // 2 (S2 - Y1) (multiply operand only)
  Jac o;
  m29_sq<C, 0>(o.X, rr);
  m29_sub<C, 0>(o.X, o.X, J);
  m29_add<C, 0>(t, V, V);
  m29_sub<C, 0>(o.X, o.X, t);
  m29_sub<C, 0>(t, V, o.X);
  m29_mul<C, 0>(o.Y, rr, t);
  m29_add_lazy(t, p.Y, p.Y);
  m29_mul<C, 0>(t, t, J);
  m29_sub<C, 0>(o.Y, o.Y, t);
  m29_add_lazy(t, p.Z, H);
  m29_sq<C, 0>(o.Z, t);
  m29_sub<C, 0>(o.Z, o.Z, Z1Z1);
  m29_sub<C, 0>(o.Z, o.Z, HH);
  r = o;
}

// r = 2p with fewer carry chains (the ladders' doublings; p finite or Z = 0, reduced coordinates):
// X - delta and the Y3 / a = 0 D - X3 factors are semi-reduced (m29_sub2), used only as products'
// operands; secp256r1's Z3 = 2 Y Z is one product instead of (Y + Z)^2 - gamma - delta. Same point
// as jac_dbl.
#ifndef CG_EC_DBL_LAZY  // 0: the round-3 v16 chains (A/B)
#define CG_EC_DBL_LAZY 1
#endif
template <int C>
CG_HD void jac_dbl_w(Jac& r, const Jac& p) {
  f29 t1, t2, t3, X3, Y3, Z3;
  if (C == CG_CURVE_R1) {  // a = -3 : dbl-2001-b
    f29 delta, gamma, beta, alpha;
    m29_sq<C, 0>(delta, p.Z);
    m29_sq<C, 0>(gamma, p.Y);
    m29_mul<C, 0>(beta, p.X, gamma);
    m29_sub2<C, 0>(t1, p.X, delta);   // < 4m
    m29_add_lazy(t2, p.X, delta);     // < 4m
    m29_mul<C, 0>(alpha, t1, t2);
#if CG_EC_DBL_LAZY
    // 3 (X - delta)(X + delta) as 2t (reduced) + t lazily: < 4m, a product operand only; 8 beta and
    // 8 gamma^2 as lazy sums of reduced 4 beta / 4 gamma^2, taken off in m29_sub_lazy3
    m29_add<C, 0>(t1, alpha, alpha);
    m29_add_lazy(alpha, alpha, t1);
    m29_sq<C, 0>(X3, alpha);
    m29_add<C, 0>(t1, beta, beta);
    m29_add<C, 0>(t1, t1, t1);  // 4 beta
    m29_add_lazy(t2, t1, t1);   // 8 beta < 4m, limbs < 2^30
    m29_sub_lazy3<C, 0>(X3, X3, t2);
    m29_add_lazy(t3, p.Z, p.Z);       // 2Z < 4m
    m29_mul<C, 0>(Z3, p.Y, t3);       // 2 Y Z
    m29_sub2<C, 0>(t1, t1, X3);       // 4 beta - X3, < 4m
    m29_mul<C, 0>(Y3, alpha, t1);
    m29_add_lazy(t3, gamma, gamma);
    m29_sq<C, 0>(t2, t3);       // 4 gamma^2
    m29_add_lazy(t2, t2, t2);   // 8 gamma^2 < 4m
    m29_sub_lazy3<C, 0>(Y3, Y3, t2);
#else
    m29_add<C, 0>(t1, alpha, alpha);
    m29_add<C, 0>(alpha, alpha, t1);  // 3 (X - delta)(X + delta)
    m29_sq<C, 0>(X3, alpha);
    m29_add<C, 0>(t1, beta, beta);
    m29_add<C, 0>(t1, t1, t1);  // 4 beta
    m29_add<C, 0>(t2, t1, t1);  // 8 beta
    m29_sub<C, 0>(X3, X3, t2);
    m29_add_lazy(t3, p.Z, p.Z);       // 2Z < 4m
    m29_mul<C, 0>(Z3, p.Y, t3);       // 2 Y Z
    m29_sub2<C, 0>(t1, t1, X3);       // 4 beta - X3, < 4m
    m29_mul<C, 0>(Y3, alpha, t1);
    m29_add_lazy(t3, gamma, gamma);
    m29_sq<C, 0>(t2, t3);      // 4 gamma^2
    m29_add<C, 0>(t2, t2, t2);  // 8 gamma^2
    m29_sub<C, 0>(Y3, Y3, t2);
#endif
  } else {  // a = 0 : dbl-2009-l
    f29 A, B, Cc, D, E, F;
    m29_sq<C, 0>(A, p.X);
    m29_sq<C, 0>(B, p.Y);
    m29_sq<C, 0>(Cc, B);
    m29_add_lazy(t1, p.X, B);
    m29_sq<C, 0>(t1, t1);
    m29_sub<C, 0>(t1, t1, A);
    m29_sub<C, 0>(t1, t1, Cc);
    m29_add<C, 0>(D, t1, t1);
#if CG_EC_DBL_LAZY
    // E = 3A as 2A (reduced) + A lazily (< 4m: F = E^2 and E (D - X3) stay under 16 m^2); 2D and 8C
    // as lazy sums of reduced values, taken off in m29_sub_lazy3
    m29_add<C, 0>(E, A, A);
    m29_add_lazy(E, E, A);
    m29_sq<C, 0>(F, E);
    m29_add_lazy(t2, D, D);
    m29_sub_lazy3<C, 0>(X3, F, t2);
    m29_sub2<C, 0>(t3, D, X3);        // < 4m
    m29_mul<C, 0>(Y3, E, t3);
    m29_add<C, 0>(t2, Cc, Cc);
    m29_add<C, 0>(t2, t2, t2);  // 4 C
    m29_add_lazy(t2, t2, t2);   // 8 C < 4m
    m29_sub_lazy3<C, 0>(Y3, Y3, t2);
#else
    m29_add<C, 0>(E, A, A);
    m29_add<C, 0>(E, E, A);
    m29_sq<C, 0>(F, E);
    m29_add<C, 0>(t2, D, D);
    m29_sub<C, 0>(X3, F, t2);
    m29_sub2<C, 0>(t3, D, X3);        // < 4m
    m29_mul<C, 0>(Y3, E, t3);
    m29_add<C, 0>(t2, Cc, Cc);
    m29_add<C, 0>(t2, t2, t2);
    m29_add<C, 0>(t2, t2, t2);  // 8 C
    m29_sub<C, 0>(Y3, Y3, t2);
#endif
    m29_add_lazy(t3, p.Y, p.Y);
    m29_mul<C, 0>(Z3, t3, p.Z);
  }
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// r = p + (x2, +-y2) affine for the wide ladder: madd-2007-bl with fewer carry chains.
//  * `inf` flags p = infinity (the ladder's start, or an exceptional P + (-P)) instead of testing Z;
//  * the sign rides on S2 = +-y2 Z1^3 (m29_neg2: one chain);
//  * H = U2 - X1 and V - X3 are semi-reduced (m29_sub2: one chain), both used only as
//    multiplication operands against values < 4m;
//  * Z3 = Z1 * 2H (one product) instead of (Z1 + H)^2 - Z1Z1 - HH (a square and two subtractions);
//  * H == 0 (mod p), i.e. the exceptional cases, behind a limb-0 filter that honest inputs fail
//    with probability ~3 / 2^29, so the wave skips the exact test.
// Same point as jac_madd (the exceptional cases included: doubling, P + (-P) -> infinity).
#ifndef CG_EC_MADD_LAZY  // 0: round-3 v15 chains, 1: lazy 4HH + three-chain X3, 2: madd-2004-hmv (A/B)
#define CG_EC_MADD_LAZY 2
#endif
template <int C>
CG_HD void jac_madd_w(Jac& r, bool& inf, const f29& x2, const f29& y2, bool neg, const EcConsts& K) {
  if (inf) {
    r.X = x2;
    if (neg) m29_neg2<C, 0>(r.Y, y2);
    else r.Y = y2;
    r.Z = K.one_p;
    inf = false;
    return;
  }
  f29 Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
  m29_sq<C, 0>(Z1Z1, r.Z);
  m29_mul<C, 0>(U2, x2, Z1Z1);
  m29_mul<C, 0>(S2, y2, r.Z);
  m29_mul<C, 0>(S2, S2, Z1Z1);
  if (neg) m29_neg2<C, 0>(S2, S2);
  m29_sub2<C, 0>(H, U2, r.X);
#if CG_EC_MADD_LAZY == 2
  // madd-2004-hmv: r = S2 - Y1 undoubled, so it may stay semi-reduced (r^2 < 16 m^2); no 4HH, 2Y1
  // or 2H: HHH = H HH, V = X1 HH, X3 = r^2 - HHH - 2V, Y3 = r (V - X3) - Y1 HHH, Z3 = Z1 H (the
  // same point as madd-2007-bl's, another Jacobian representative)
  m29_sub2<C, 0>(rr, S2, r.Y);
  if (m29_maybe_zero_semi<C, 0>(H)) {
    if (m29_zero_semi<C, 0>(H)) {
      if (m29_zero_semi<C, 0>(rr)) {
        jac_dbl<C>(r, r);
      } else {
        jac_set_inf<C>(r, K);
        inf = true;
      }
      return;
    }
  }
  {
    f29 HHH;
    m29_sq<C, 0>(HH, H);
    m29_mul<C, 0>(HHH, H, HH);
    m29_mul<C, 0>(V, r.X, HH);
    Jac o;
    m29_sq<C, 0>(o.X, rr);
    m29_add_lazy(t, HHH, V);  // HHH + 2V < 6m, limbs < 3 * 2^29
    m29_add_lazy(t, t, V);
    m29_sub_lazy3<C, 0>(o.X, o.X, t);
    m29_sub2<C, 0>(t, V, o.X);
    m29_mul<C, 0>(o.Y, rr, t);
    m29_mul<C, 0>(t, r.Y, HHH);
    m29_sub<C, 0>(o.Y, o.Y, t);
    m29_mul<C, 0>(o.Z, r.Z, H);
    r = o;
    return;
  }
#endif
  m29_sub<C, 0>(rr, S2, r.Y);
  if (m29_maybe_zero_semi<C, 0>(H)) {
    if (m29_zero_semi<C, 0>(H)) {
      if (m29_iszero<C, 0>(rr)) {
        jac_dbl<C>(r, r);
      } else {
        jac_set_inf<C>(r, K);
        inf = true;
      }
      return;
    }
  }
  m29_sq<C, 0>(HH, H);
#if CG_EC_MADD_LAZY
  // 4 HH as lazy sums (< 8m, limbs < 2^31): its products are with H (< 4m) and X1 (< 2m), so
  // a b < 32 m^2 < m R (m < 2^256), and a column stays below 9 * 2^60 + 9 * 2^58 + 2^35
  m29_add_lazy(I, HH, HH);
  m29_add_lazy(I, I, I);
#else
  m29_add<C, 0>(I, HH, HH);
  m29_add_lazy(I, I, I);      // 4 HH (< 4m: multiply operand only)
#endif
  m29_mul<C, 0>(J, H, I);
  m29_mul<C, 0>(V, r.X, I);
  m29_add_lazy(rr, rr, rr);   // 2 (S2 - Y1) (multiply operand only)
  Jac o;
  m29_sq<C, 0>(o.X, rr);
#if CG_EC_MADD_LAZY
  m29_add_lazy(t, J, V);  // J + 2V < 6m, limbs < 3 * 2^29
  m29_add_lazy(t, t, V);
  m29_sub_lazy3<C, 0>(o.X, o.X, t);
#else
  m29_sub<C, 0>(o.X, o.X, J);
  m29_add<C, 0>(t, V, V);
  m29_sub<C, 0>(o.X, o.X, t);
#endif
  m29_sub2<C, 0>(t, V, o.X);
  m29_mul<C, 0>(o.Y, rr, t);
  m29_add_lazy(t, r.Y, r.Y);
  m29_mul<C, 0>(t, t, J);
  m29_sub<C, 0>(o.Y, o.Y, t);
  m29_add_lazy(H, H, H);      // 2H < 8m, limbs < 2^30: times Z1 < 2m
  m29_mul<C, 0>(o.Z, r.Z, H);
  r = o;
}

// affine (Montgomery) of a finite Jacobian point
template <int C>
CG_HD void jac_to_affine(f29& x, f29& y, const Jac& p, const EcConsts& K) {
  f29 zi, zi2, zi3;
  m29_inv<C, 0>(zi, p.Z, K.one_p);
  m29_sq<C, 0>(zi2, zi);
  m29_mul<C, 0>(zi3, zi2, zi);
  m29_mul<C, 0>(x, p.X, zi2);
  m29_mul<C, 0>(y, p.Y, zi3);
}

// R^2 mod m (R = 2^261) by 522 modular doublings of 1 -- init only
template <int C, int N>
CG_HD void m29_r2(f29& r) {
  f29 x;
  f29_zero(x);
  x.v[0] = 1;
  if (m29_plain(C, N)) {  // plain form (mont29.h): R = 1
    r = x;
    return;
  }
  for (int i = 0; i < 522; ++i) m29_add<C, N>(x, x, x);
  m29_canon<C, N>(r, x);
}

template <int C>
CG_HD void ec_consts_init(EcConsts& K) {
  m29_r2<C, 0>(K.r2_p);
  m29_r2<C, 1>(K.r2_n);
  f29 one;
  f29_zero(one);
  one.v[0] = 1;
  m29_mul<C, 0>(K.one_p, one, K.r2_p);
  m29_mul<C, 1>(K.one_n, one, K.r2_n);
  u256w b, gx, gy;
  u256_zero(b);
  if (C == CG_CURVE_R1) {
    const uint32_t B[8] = {0x27d2604bu, 0x3bce3c3eu, 0xcc53b0f6u, 0x651d06b0u,
                           0x769886bcu, 0xb3ebbd55u, 0xaa3a93e7u, 0x5ac635d8u};
    const uint32_t GX[8] = {0xd898c296u, 0xf4a13945u, 0x2deb33a0u, 0x77037d81u,
                            0x63a440f2u, 0xf8bce6e5u, 0xe12c4247u, 0x6b17d1f2u};
    const uint32_t GY[8] = {0x37bf51f5u, 0xcbb64068u, 0x6b315eceu, 0x2bce3357u,
                            0x7c0f9e16u, 0x8ee7eb4au, 0xfe1a7f9bu, 0x4fe342e2u};
    for (int i = 0; i < 8; ++i) {
      b.w[i] = B[i];
      gx.w[i] = GX[i];
      gy.w[i] = GY[i];
    }
  } else {
    b.w[0] = 7;
    const uint32_t GX[8] = {0x16f81798u, 0x59f2815bu, 0x2dce28d9u, 0x029bfcdbu,
                            0xce870b07u, 0x55a06295u, 0xf9dcbbacu, 0x79be667eu};
    const uint32_t GY[8] = {0xfb10d4b8u, 0x9c47d08fu, 0xa6855419u, 0xfd17b448u,
                            0x0e1108a8u, 0x5da4fbfcu, 0x26a3c465u, 0x483ada77u};
    for (int i = 0; i < 8; ++i) {
      gx.w[i] = GX[i];
      gy.w[i] = GY[i];
    }
  }
  m29_from_plain<C, 0>(K.b_m, b, K.r2_p);
  m29_from_plain<C, 0>(K.gx, gx, K.r2_p);
  m29_from_plain<C, 0>(K.gy, gy, K.r2_p);
}

// y^2 = x^3 + a x + b (Montgomery), a = -3 (r1) or 0 (k1)
template <int C>
CG_HD void ec_rhs(f29& rhs, const f29& xm, const EcConsts& K) {
  m29_sq<C, 0>(rhs, xm);
  m29_mul<C, 0>(rhs, rhs, xm);
  if (C == CG_CURVE_R1) {
    f29 t;
    m29_add<C, 0>(t, xm, xm);
    m29_add<C, 0>(t, t, xm);
    m29_sub<C, 0>(rhs, rhs, t);
  }
  m29_add<C, 0>(rhs, rhs, K.b_m);
}

// Decompress x (plain, < p) with y parity `odd` (SEC1 02/03); p = 3 mod 4 for both curves.
// Returns false if x is not on the curve.
template <int C>
CG_HD bool ec_decompress(u256w& y, const u256w& x, uint32_t odd, const EcConsts& K) {
  if (!u256_lt_mod<C, 0>(x)) return false;
  f29 xm, rhs, ym, chk;
  m29_from_plain<C, 0>(xm, x, K.r2_p);
  ec_rhs<C>(rhs, xm, K);
  uint32_t e[8];  // (p + 1) / 4
  uint64_t c = 1;
  for (int i = 0; i < 8; ++i) {
    c += Mod<C, 0>::w(i);
    e[i] = (uint32_t)c;
    c >>= 32;
  }
  const uint32_t top = (uint32_t)c;
  for (int i = 0; i < 8; ++i) e[i] = (e[i] >> 2) | ((i < 7 ? e[i + 1] : top) << 30);
  m29_pow<C, 0>(ym, rhs, e, K.one_p);
  m29_sq<C, 0>(chk, ym);
  if (!m29_eq<C, 0>(chk, rhs)) return false;
  m29_to_plain<C, 0>(y, ym);
  if ((y.w[0] & 1u) != odd && !u256_iszero(y)) {  // y := p - y
    uint32_t br = 0;
    for (int i = 0; i < 8; ++i) {
      const uint64_t d = (uint64_t)Mod<C, 0>::w(i) - y.w[i] - br;
      y.w[i] = (uint32_t)d;
      br = (uint32_t)(d >> 63);
    }
  }
  return true;
}

// ------------------------------------------------------------------ DER (StdDSAEncoder)
// The parser reads the signature through a byte source: DerArena straight from the arena (each byte
// a dword load: the host build and long signatures), DerStaged from a copy the caller staged (the
// device stage copies a signature's dwords into LDS with a few 16-byte loads first: read byte by
// byte from the arena, 64 lanes' scattered signatures cost ~140 loads per item, k_ec_prep ran at
// 0.15 of its issue rate moving 2.4 KB per item, profiles/r03/v14/pmc_traffic.json).
// One byte of the arena (key decoding, DerArena)
CG_HD uint32_t der_byte(const uint8_t* arena, uint64_t lr, uint64_t off) {
  return cg_ld_bytes4(arena, lr, off) & 0xffu;
}
struct DerArena {
  const uint8_t* arena;
  uint64_t lr, off;
  CG_HDM uint32_t byte(uint32_t i) const { return der_byte(arena, lr, off + i); }
};
struct DerStaged {
  const uint8_t* p;  // the signature's first byte
  CG_HDM uint32_t byte(uint32_t i) const { return p[i]; }
};

// DER length at position *i (within [0, n)); returns false if malformed / not minimal.
template <class Src>
CG_HD bool der_len(const Src& b, uint32_t n, uint32_t* i, uint32_t* out) {
  if (*i >= n) return false;
  const uint32_t l0 = b.byte((*i)++);
  if (l0 < 0x80u) {
    *out = l0;
    return true;
  }
  const uint32_t nb = l0 & 0x7fu;
  if (nb == 0 || nb > 4 || *i + nb > n) return false;
  uint32_t v = 0;
  for (uint32_t k = 0; k < nb; ++k) v = (v << 8) | b.byte((*i)++);
  if (v < 0x80u) return false;
  if (nb > 1 && (v >> (8 * (nb - 1))) == 0) return false;
  *out = v;
  return true;
}

// INTEGER at *i: validates strict DER; value (if 0 < v < 2^256) -> out (little-endian words),
// *in_range = false if negative, zero or >= 2^256.
template <class Src>
CG_HD bool der_int(const Src& b, uint32_t n, uint32_t* i, u256w& out, bool* in_range) {
  if (*i >= n || b.byte(*i) != 0x02u) return false;
  (*i)++;
  uint32_t ln;
  if (!der_len(b, n, i, &ln)) return false;
  if (ln == 0 || *i + ln > n) return false;
  const uint32_t c0 = b.byte(*i);
  const uint32_t c1 = ln > 1 ? b.byte(*i + 1) : 0;
  if (ln > 1 && ((c0 == 0 && c1 < 0x80u) || (c0 == 0xffu && c1 >= 0x80u))) return false;
  u256_zero(out);
  uint32_t start = *i, len = ln;
  *i += ln;
  if (c0 & 0x80u) {
    *in_range = false;
    return true;
  }
  if (c0 == 0 && len > 1) {
    start++;
    len--;
  }
  if (len > 32) {
    *in_range = false;
    return true;
  }
  // word by word with static indices (a per-lane byte position into out.w[] put it in scratch)
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint32_t w = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t pos = 4 * j + q;  // little-endian byte index
      if (pos < len) w |= b.byte(start + len - 1 - pos) << (8 * q);
    }
    out.w[j] = w;
  }
  *in_range = !u256_iszero(out);
  return true;
}

// returns 0 ok, 2 malformed; *range_ok false => INVALID
template <class Src>
CG_HD uint32_t der_sig(const Src& b, uint32_t n, u256w& r, u256w& s, bool* range_ok) {
  if (n < 2 || b.byte(0) != 0x30u) return 2;
  uint32_t i = 1, sl;
  if (!der_len(b, n, &i, &sl)) return 2;
  if (i + sl != n) return 2;
  bool ok1 = false, ok2 = false;
  if (!der_int(b, n, &i, r, &ok1)) return 2;
  if (i >= n) return 2;
  if (!der_int(b, n, &i, s, &ok2)) return 2;
  if (i != n) return 2;
  *range_ok = ok1 && ok2;
  return 0;
}
CG_HD uint32_t der_sig(const uint8_t* arena, uint64_t lr, uint64_t off, uint32_t n, u256w& r, u256w& s,
                       bool* range_ok) {
  return der_sig(DerArena{arena, lr, off}, n, r, s, range_ok);
}

// ------------------------------------------------------------------ key bytes
// Formats (include/cordagpu.h): RAW 64 B X||Y; SPKI (PublicKey.getEncoded(), 91 B r1 /
// 88 B k1, or the 59 / 56 B form around a compressed point); SEC1 04||X||Y, 06/07||X||Y (hybrid)
// or 02/03||X.
CG_HD void ec_load_be32(u256w& v, const uint8_t* arena, uint64_t lr, uint64_t off) {
#pragma unroll
  for (int i = 0; i < 8; ++i) v.w[7 - i] = CG_BSWAP32(cg_ld_bytes4(arena, lr, off + 4 * i));
}

CG_HD uint32_t ec_spki_prefix_byte(int curve, int i) {
  const uint8_t R1[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                          0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
  const uint8_t K1[23] = {0x30, 0x56, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02,
                          0x01, 0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a, 0x03, 0x42, 0x00};
  return curve == CG_CURVE_R1 ? R1[i] : K1[i];
}

// SPKI header byte i for a point of ptlen bytes (65 or 33): only the outer SEQUENCE length
// (byte 1) and the BIT STRING length (byte pl - 2) depend on the point's length.
CG_HD uint32_t ec_spki_header_byte(int curve, int i, uint32_t ptlen) {
  const int pl = curve == CG_CURVE_R1 ? 26 : 23;
  const uint32_t b = ec_spki_prefix_byte(curve, i);
  return (i == 1 || i == pl - 2) ? b - (65u - ptlen) : b;
}

