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
// Arithmetic: 8 x 32-bit limbs, Montgomery multiplication in product-scanning form (FIPS):
// both the a*b and the m*p column products go through one 96-bit column accumulator
// (v_mad_u64_u32 + carry). The moduli are compile-time constants, so the P-256 zero and
// one words fold away. Scalar multiplication: signed radix-16 fixed windows (65 windows),
// Shamir-interleaved over an 8-entry affine table of G (constant) and of Q (per key).
#pragma once
#include "fe25519.h"
#include "sha2.h"

struct u256w {
  uint32_t w[8];
};

// ---- moduli ----
#define CG_CURVE_K1 0
#define CG_CURVE_R1 1

template <int C, int N>  // N = 0: field p, N = 1: group order n
struct Mod {
  CG_HDS uint32_t w(int i) {
    if (C == CG_CURVE_R1 && N == 0) {
      const uint32_t P[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};
      return P[i];
    } else if (C == CG_CURVE_R1 && N == 1) {
      const uint32_t P[8] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                             0xffffffffu, 0xffffffffu, 0u, 0xffffffffu};
      return P[i];
    } else if (C == CG_CURVE_K1 && N == 0) {
      const uint32_t P[8] = {0xfffffc2fu, 0xfffffffeu, 0xffffffffu, 0xffffffffu,
                             0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
      return P[i];
    } else {
      const uint32_t P[8] = {0xd0364141u, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u,
                             0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
      return P[i];
    }
  }
  // -m^-1 mod 2^32
  CG_HDS uint32_t inv() {
    if (C == CG_CURVE_R1 && N == 0) return 1u;
    if (C == CG_CURVE_R1 && N == 1) return 0xee00bc4fu;
    if (C == CG_CURVE_K1 && N == 0) return 0xd2253531u;
    return 0x5588b13fu;
  }
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

// 96-bit column accumulator (hi:lo)
struct Acc {
  uint64_t lo;
  uint32_t hi;
};

CG_HD void acc_mac(Acc& a, uint32_t x, uint32_t y) {
  const uint64_t p = (uint64_t)x * y;
  uint64_t s;
  const bool c = __builtin_add_overflow(a.lo, p, &s);
  a.lo = s;
  a.hi += (uint32_t)c;
}

CG_HD void acc_add(Acc& a, uint32_t x) {
  uint64_t s;
  const bool c = __builtin_add_overflow(a.lo, (uint64_t)x, &s);
  a.lo = s;
  a.hi += (uint32_t)c;
}

CG_HD void acc_shr32(Acc& a) {
  a.lo = (a.lo >> 32) | ((uint64_t)a.hi << 32);
  a.hi = 0;
}

// r = a - m if a >= m (a given as 8 words + carry bit) -> fully reduced
template <int C, int N>
CG_HD void mod_final(u256w& r, const uint32_t t[8], uint32_t carry) {
  uint32_t d[8];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t x = (uint64_t)t[i] - Mod<C, N>::w(i) - br;
    d[i] = (uint32_t)x;
    br = (uint32_t)(x >> 63);
  }
  const bool take = carry || !br;
#pragma unroll
  for (int i = 0; i < 8; ++i) r.w[i] = take ? d[i] : t[i];
}

// Montgomery product a * b * 2^-256 mod m (inputs < m, output < m)
template <int C, int N>
CG_HD void mm_mul(u256w& r, const u256w& a, const u256w& b) {
  uint32_t m[8], out[8];
  Acc acc = {0, 0};
#pragma unroll
  for (int k = 0; k < 16; ++k) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 8) acc_mac(acc, a.w[i], b.w[j]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 8) {
        const uint32_t pw = Mod<C, N>::w(j);
        if (pw == 1u) acc_add(acc, m[i]);
        else if (pw != 0u) acc_mac(acc, m[i], pw);
      }
    }
    if (k < 8) {
      m[k] = (uint32_t)acc.lo * Mod<C, N>::inv();
      const uint32_t p0 = Mod<C, N>::w(0);
      if (p0 == 1u) acc_add(acc, m[k]);
      else acc_mac(acc, m[k], p0);
    } else {
      out[k - 8] = (uint32_t)acc.lo;
    }
    acc_shr32(acc);
  }
  mod_final<C, N>(r, out, (uint32_t)acc.lo);
}

template <int C, int N>
CG_HD void mm_sq(u256w& r, const u256w& a) {
  mm_mul<C, N>(r, a, a);
}

template <int C, int N>
CG_HD void mm_add(u256w& r, const u256w& a, const u256w& b) {
  uint32_t t[8];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)a.w[i] + b.w[i];
    t[i] = (uint32_t)c;
    c >>= 32;
  }
  mod_final<C, N>(r, t, (uint32_t)c);
}

template <int C, int N>
CG_HD void mm_sub(u256w& r, const u256w& a, const u256w& b) {
  uint32_t t[8];
  uint32_t br = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint64_t x = (uint64_t)a.w[i] - b.w[i] - br;
    t[i] = (uint32_t)x;
    br = (uint32_t)(x >> 63);
  }
  // if borrow: add m
  const uint32_t mask = 0u - br;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)t[i] + (Mod<C, N>::w(i) & mask);
    r.w[i] = (uint32_t)c;
    c >>= 32;
  }
}

template <int C, int N>
CG_HD void mm_neg(u256w& r, const u256w& a) {
  u256w z;
  u256_zero(z);
  mm_sub<C, N>(r, z, a);
}

// R^2 mod m, computed (host or device) by 512 modular doublings of 1 -- only used at init
template <int C, int N>
CG_HD void mm_r2(u256w& r) {
  u256w x;
  u256_zero(x);
  x.w[0] = 1;
  for (int i = 0; i < 512; ++i) mm_add<C, N>(x, x, x);
  r = x;
}

// a^e (Montgomery domain, e plain, MSB first, square-and-multiply)
template <int C, int N>
CG_HD void mm_pow(u256w& r, const u256w& a, const u256w& e, const u256w& one_m) {
  u256w acc = one_m;
  for (int i = 255; i >= 0; --i) {
    mm_sq<C, N>(acc, acc);
    if ((e.w[i >> 5] >> (i & 31)) & 1u) mm_mul<C, N>(acc, acc, a);
  }
  r = acc;
}

// a^(m-2)
template <int C, int N>
CG_HD void mm_inv(u256w& r, const u256w& a, const u256w& one_m) {
  u256w e;
#pragma unroll
  for (int i = 0; i < 8; ++i) e.w[i] = Mod<C, N>::w(i);
  e.w[0] -= 2;  // low words of every modulus here are >= 2
  mm_pow<C, N>(r, a, e, one_m);
}

CG_HD int u256_cmp(const u256w& a, const u256w& b) {
  for (int i = 7; i >= 0; --i) {
    if (a.w[i] != b.w[i]) return a.w[i] < b.w[i] ? -1 : 1;
  }
  return 0;
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
struct EcConsts {
  u256w one_p, r2_p, one_n, r2_n;  // Montgomery 1 and R^2 for p and n
  u256w b_m;                       // curve b (Montgomery form)
  u256w gx[9], gy[9];              // k*G affine, Montgomery form (index 0 unused)
};

struct EcKeyPrep {
  uint32_t status;
  uint32_t pad[7];
  u256w qx[9], qy[9];              // k*Q affine, Montgomery form (index 0 unused)
};

struct Jac {
  u256w X, Y, Z;  // Z == 0 <=> infinity
};

template <int C>
CG_HD void jac_dbl(Jac& r, const Jac& p) {
  u256w t1, t2, t3, t4, X3, Y3, Z3;
  if (C == CG_CURVE_R1) {  // a = -3 : dbl-2001-b
    u256w delta, gamma, beta, alpha;
    mm_sq<C, 0>(delta, p.Z);
    mm_sq<C, 0>(gamma, p.Y);
    mm_mul<C, 0>(beta, p.X, gamma);
    mm_sub<C, 0>(t1, p.X, delta);
    mm_add<C, 0>(t2, p.X, delta);
    mm_mul<C, 0>(alpha, t1, t2);
    mm_add<C, 0>(t1, alpha, alpha);
    mm_add<C, 0>(alpha, alpha, t1);
    mm_sq<C, 0>(X3, alpha);
    mm_add<C, 0>(t1, beta, beta);
    mm_add<C, 0>(t1, t1, t1);  // 4 beta
    mm_add<C, 0>(t2, t1, t1);  // 8 beta
    mm_sub<C, 0>(X3, X3, t2);
    mm_add<C, 0>(t3, p.Y, p.Z);
    mm_sq<C, 0>(Z3, t3);
    mm_sub<C, 0>(Z3, Z3, gamma);
    mm_sub<C, 0>(Z3, Z3, delta);
    mm_sub<C, 0>(t1, t1, X3);
    mm_mul<C, 0>(Y3, alpha, t1);
    mm_sq<C, 0>(t4, gamma);
    mm_add<C, 0>(t4, t4, t4);
    mm_add<C, 0>(t4, t4, t4);
    mm_add<C, 0>(t4, t4, t4);
    mm_sub<C, 0>(Y3, Y3, t4);
  } else {  // a = 0 : dbl-2009-l
    u256w A, B, Cc, D, E, F;
    mm_sq<C, 0>(A, p.X);
    mm_sq<C, 0>(B, p.Y);
    mm_sq<C, 0>(Cc, B);
    mm_add<C, 0>(t1, p.X, B);
    mm_sq<C, 0>(t1, t1);
    mm_sub<C, 0>(t1, t1, A);
    mm_sub<C, 0>(t1, t1, Cc);
    mm_add<C, 0>(D, t1, t1);
    mm_add<C, 0>(E, A, A);
    mm_add<C, 0>(E, E, A);
    mm_sq<C, 0>(F, E);
    mm_add<C, 0>(t2, D, D);
    mm_sub<C, 0>(X3, F, t2);
    mm_sub<C, 0>(t3, D, X3);
    mm_mul<C, 0>(Y3, E, t3);
    mm_add<C, 0>(t4, Cc, Cc);
    mm_add<C, 0>(t4, t4, t4);
    mm_add<C, 0>(t4, t4, t4);
    mm_sub<C, 0>(Y3, Y3, t4);
    mm_mul<C, 0>(Z3, p.Y, p.Z);
    mm_add<C, 0>(Z3, Z3, Z3);
  }
  r.X = X3;
  r.Y = Y3;
  r.Z = Z3;
}

// r = p + (x2, y2) affine, exception-complete (infinity, doubling, inverse points)
template <int C>
CG_HD void jac_madd(Jac& r, const Jac& p, const u256w& x2, const u256w& y2, const EcConsts& K) {
  if (u256_iszero(p.Z)) {
    r.X = x2;
    r.Y = y2;
    r.Z = K.one_p;
    return;
  }
  u256w Z1Z1, U2, S2, H, HH, I, J, rr, V, t;
  mm_sq<C, 0>(Z1Z1, p.Z);
  mm_mul<C, 0>(U2, x2, Z1Z1);
  mm_mul<C, 0>(S2, y2, p.Z);
  mm_mul<C, 0>(S2, S2, Z1Z1);
  mm_sub<C, 0>(H, U2, p.X);
  mm_sub<C, 0>(rr, S2, p.Y);
  if (u256_iszero(H)) {
    if (u256_iszero(rr)) {
      jac_dbl<C>(r, p);
    } else {
      u256_zero(r.X);
      r.Y = K.one_p;
      u256_zero(r.Z);
    }
    return;
  }
  mm_sq<C, 0>(HH, H);
  mm_add<C, 0>(I, HH, HH);
  mm_add<C, 0>(I, I, I);
  mm_mul<C, 0>(J, H, I);
  mm_add<C, 0>(rr, rr, rr);
  mm_mul<C, 0>(V, p.X, I);
  Jac o;
  mm_sq<C, 0>(o.X, rr);
  mm_sub<C, 0>(o.X, o.X, J);
  mm_add<C, 0>(t, V, V);
  mm_sub<C, 0>(o.X, o.X, t);
  mm_sub<C, 0>(t, V, o.X);
  mm_mul<C, 0>(o.Y, rr, t);
  mm_mul<C, 0>(t, p.Y, J);
  mm_add<C, 0>(t, t, t);
  mm_sub<C, 0>(o.Y, o.Y, t);
  mm_add<C, 0>(t, p.Z, H);
  mm_sq<C, 0>(o.Z, t);
  mm_sub<C, 0>(o.Z, o.Z, Z1Z1);
  mm_sub<C, 0>(o.Z, o.Z, HH);
  r = o;
}

template <int C>
CG_HD void jac_to_affine(u256w& x, u256w& y, const Jac& p, const EcConsts& K) {
  u256w zi, zi2, zi3;
  mm_inv<C, 0>(zi, p.Z, K.one_p);
  mm_sq<C, 0>(zi2, zi);
  mm_mul<C, 0>(zi3, zi2, zi);
  mm_mul<C, 0>(x, p.X, zi2);
  mm_mul<C, 0>(y, p.Y, zi3);
}

// Fill tab[1..8] = k*P (affine, Montgomery) from affine P
template <int C>
CG_HD void ec_table8(u256w tx[9], u256w ty[9], const u256w& px, const u256w& py, const EcConsts& K) {
  tx[1] = px;
  ty[1] = py;
  Jac Pj = {px, py, K.one_p};
  Jac acc;
  jac_dbl<C>(acc, Pj);
  jac_to_affine<C>(tx[2], ty[2], acc, K);
  for (int k = 3; k <= 8; ++k) {
    jac_madd<C>(acc, acc, px, py, K);
    jac_to_affine<C>(tx[k], ty[k], acc, K);
  }
  u256_zero(tx[0]);
  u256_zero(ty[0]);
}

template <int C>
CG_HD void ec_consts_init(EcConsts& K) {
  mm_r2<C, 0>(K.r2_p);
  mm_r2<C, 1>(K.r2_n);
  u256w one;
  u256_zero(one);
  one.w[0] = 1;
  mm_mul<C, 0>(K.one_p, one, K.r2_p);
  mm_mul<C, 1>(K.one_n, one, K.r2_n);
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
  mm_mul<C, 0>(K.b_m, b, K.r2_p);
  u256w gxm, gym;
  mm_mul<C, 0>(gxm, gx, K.r2_p);
  mm_mul<C, 0>(gym, gy, K.r2_p);
  ec_table8<C>(K.gx, K.gy, gxm, gym, K);
}

// ------------------------------------------------------------------ key decode
// Validates a plain (x, y) < p on the curve; fills the per-key table. Returns 0 / 3.
template <int C>
CG_HD uint32_t ec_key_prep_xy(EcKeyPrep& kp, const u256w& x, const u256w& y, const EcConsts& K) {
  if (!u256_lt_mod<C, 0>(x) || !u256_lt_mod<C, 0>(y)) return 3;
  u256w xm, ym, l, rr;
  mm_mul<C, 0>(xm, x, K.r2_p);
  mm_mul<C, 0>(ym, y, K.r2_p);
  mm_sq<C, 0>(l, ym);
  mm_sq<C, 0>(rr, xm);
  if (C == CG_CURVE_R1) {  // x^3 - 3x + b
    u256w t;
    mm_mul<C, 0>(rr, rr, xm);
    mm_add<C, 0>(t, xm, xm);
    mm_add<C, 0>(t, t, xm);
    mm_sub<C, 0>(rr, rr, t);
  } else {
    mm_mul<C, 0>(rr, rr, xm);
  }
  mm_add<C, 0>(rr, rr, K.b_m);
  if (!u256_eq(l, rr)) return 3;
  ec_table8<C>(kp.qx, kp.qy, xm, ym, K);
  return 0;
}

// Decompress x (plain, < p) with y parity `odd`; p = 3 mod 4 for both curves.
template <int C>
CG_HD bool ec_decompress(u256w& y, const u256w& x, uint32_t odd, const EcConsts& K) {
  if (!u256_lt_mod<C, 0>(x)) return false;
  u256w xm, rhs, e, ym, chk;
  mm_mul<C, 0>(xm, x, K.r2_p);
  mm_sq<C, 0>(rhs, xm);
  mm_mul<C, 0>(rhs, rhs, xm);
  if (C == CG_CURVE_R1) {
    u256w t;
    mm_add<C, 0>(t, xm, xm);
    mm_add<C, 0>(t, t, xm);
    mm_sub<C, 0>(rhs, rhs, t);
  }
  mm_add<C, 0>(rhs, rhs, K.b_m);
  // e = (p + 1) / 4
  uint64_t c = 1;
  for (int i = 0; i < 8; ++i) {
    c += Mod<C, 0>::w(i);
    e.w[i] = (uint32_t)c;
    c >>= 32;
  }
  const uint32_t top = (uint32_t)c;
  for (int i = 0; i < 8; ++i) e.w[i] = (e.w[i] >> 2) | ((i < 7 ? e.w[i + 1] : top) << 30);
  mm_pow<C, 0>(ym, rhs, e, K.one_p);
  mm_sq<C, 0>(chk, ym);
  if (!u256_eq(chk, rhs)) return false;
  u256w one;
  u256_zero(one);
  one.w[0] = 1;
  mm_mul<C, 0>(y, ym, one);  // from Montgomery
  if ((y.w[0] & 1u) != odd) {
    u256w z;
    u256_zero(z);
    if (!u256_iszero(y)) mm_sub<C, 0>(y, z, y);
  }
  return true;
}

// ------------------------------------------------------------------ DER (StdDSAEncoder)
// Reads one byte of the signature
CG_HD uint32_t der_byte(const uint8_t* arena, uint64_t lr, uint64_t off) {
  return cg_ld_bytes4(arena, lr, off) & 0xffu;
}

// DER length at position *i (within [0, n)); returns false if malformed / not minimal.
CG_HD bool der_len(const uint8_t* arena, uint64_t lr, uint64_t base, uint32_t n, uint32_t* i, uint32_t* out) {
  if (*i >= n) return false;
  const uint32_t l0 = der_byte(arena, lr, base + (*i)++);
  if (l0 < 0x80u) {
    *out = l0;
    return true;
  }
  const uint32_t nb = l0 & 0x7fu;
  if (nb == 0 || nb > 4 || *i + nb > n) return false;
  uint32_t v = 0;
  for (uint32_t k = 0; k < nb; ++k) v = (v << 8) | der_byte(arena, lr, base + (*i)++);
  if (v < 0x80u) return false;
  if (nb > 1 && (v >> (8 * (nb - 1))) == 0) return false;
  *out = v;
  return true;
}

// INTEGER at *i: validates strict DER; value (if 0 < v < 2^256) -> out (little-endian words),
// *in_range = false if negative, zero or >= 2^256.
CG_HD bool der_int(const uint8_t* arena, uint64_t lr, uint64_t base, uint32_t n, uint32_t* i, u256w& out,
                   bool* in_range) {
  if (*i >= n || der_byte(arena, lr, base + *i) != 0x02u) return false;
  (*i)++;
  uint32_t ln;
  if (!der_len(arena, lr, base, n, i, &ln)) return false;
  if (ln == 0 || *i + ln > n) return false;
  const uint32_t c0 = der_byte(arena, lr, base + *i);
  const uint32_t c1 = ln > 1 ? der_byte(arena, lr, base + *i + 1) : 0;
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
  for (uint32_t k = 0; k < len; ++k) {
    const uint32_t byte = der_byte(arena, lr, base + start + k);
    const uint32_t pos = len - 1 - k;  // little-endian byte index
    out.w[pos >> 2] |= byte << (8 * (pos & 3));
  }
  *in_range = !u256_iszero(out);
  return true;
}

// returns 0 ok, 2 malformed; *range_ok false => INVALID
CG_HD uint32_t der_sig(const uint8_t* arena, uint64_t lr, uint64_t off, uint32_t n, u256w& r, u256w& s,
                       bool* range_ok) {
  if (n < 2 || der_byte(arena, lr, off) != 0x30u) return 2;
  uint32_t i = 1, sl;
  if (!der_len(arena, lr, off, n, &i, &sl)) return 2;
  if (i + sl != n) return 2;
  bool ok1 = false, ok2 = false;
  if (!der_int(arena, lr, off, n, &i, r, &ok1)) return 2;
  if (i >= n) return 2;
  if (!der_int(arena, lr, off, n, &i, s, &ok2)) return 2;
  if (i != n) return 2;
  *range_ok = ok1 && ok2;
  return 0;
}

// signed radix-16 recoding of a < 2^256 into 65 digits in [-8, 8], packed 4 per word
CG_HD void ec_recode16(uint32_t packed[17], const u256w& a) {
  int carry = 0;
#pragma unroll
  for (int w = 0; w < 17; ++w) packed[w] = 0;
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    int e = (int)((a.w[i >> 3] >> ((i & 7) * 4)) & 15u) + carry;
    carry = (e + 8) >> 4;
    e -= carry << 4;
    packed[i >> 2] |= ((uint32_t)(e & 0xff)) << ((i & 3) * 8);
  }
  packed[16] = (uint32_t)carry;
}

CG_HD int ec_digit(const uint32_t packed[17], int i) {
  return (int)(int8_t)(uint8_t)(packed[i >> 2] >> ((i & 3) * 8));
}

// ------------------------------------------------------------------ verify
// Returns 0 VALID, 1 INVALID, 2 SIG_MALFORMED. Key already prepared (status 0).
template <int C>
CG_HD uint32_t ecdsa_verify_core(const EcKeyPrep& kp, const uint8_t* arena, uint64_t lr, uint64_t sig_off,
                                 uint32_t sig_len, uint64_t msg_off, uint64_t msg_len, const EcConsts& K) {
  u256w r, s;
  bool range_ok = false;
  if (der_sig(arena, lr, sig_off, sig_len, r, s, &range_ok)) return 2;
  // e = SHA-256(M), big-endian -> little-endian words
  uint32_t h[8];
  sha256_arena_suffix(h, arena, lr, msg_off, msg_len, nullptr);
  if (!range_ok) return 1;
  if (!u256_lt_mod<C, 1>(r) || !u256_lt_mod<C, 1>(s)) return 1;
  u256w e;
#pragma unroll
  for (int i = 0; i < 8; ++i) e.w[i] = h[7 - i];
  if (!u256_lt_mod<C, 1>(e)) {  // e < 2^256 < 2n
    uint32_t br = 0;
    for (int i = 0; i < 8; ++i) {
      const uint64_t x = (uint64_t)e.w[i] - Mod<C, 1>::w(i) - br;
      e.w[i] = (uint32_t)x;
      br = (uint32_t)(x >> 63);
    }
  }
  // w = s^-1 (Montgomery), u1 = e w, u2 = r w (plain)
  u256w sm, wm, u1, u2;
  mm_mul<C, 1>(sm, s, K.r2_n);
  mm_inv<C, 1>(wm, sm, K.one_n);
  mm_mul<C, 1>(u1, e, wm);
  mm_mul<C, 1>(u2, r, wm);
  uint32_t d1[17], d2[17];
  ec_recode16(d1, u1);
  ec_recode16(d2, u2);
  Jac R;
  u256_zero(R.X);
  R.Y = K.one_p;
  u256_zero(R.Z);
  for (int i = 64; i >= 0; --i) {
    if (i != 64) {
      jac_dbl<C>(R, R);
      jac_dbl<C>(R, R);
      jac_dbl<C>(R, R);
      jac_dbl<C>(R, R);
    }
    const int a = i == 64 ? (int)d1[16] : ec_digit(d1, i);
    const int b = i == 64 ? (int)d2[16] : ec_digit(d2, i);
    if (a != 0) {
      const int ia = a < 0 ? -a : a;
      u256w y = K.gy[ia];
      if (a < 0) mm_neg<C, 0>(y, y);
      jac_madd<C>(R, R, K.gx[ia], y, K);
    }
    if (b != 0) {
      const int ib = b < 0 ? -b : b;
      u256w y = kp.qy[ib];
      if (b < 0) mm_neg<C, 0>(y, y);
      jac_madd<C>(R, R, kp.qx[ib], y, K);
    }
  }
  if (u256_iszero(R.Z)) return 1;
  // x(R) == r mod n  <=>  r Z^2 == X  or  (r + n < p and (r + n) Z^2 == X)
  u256w z2, t, rm;
  mm_sq<C, 0>(z2, R.Z);
  mm_mul<C, 0>(rm, r, K.r2_p);
  mm_mul<C, 0>(t, rm, z2);
  if (u256_eq(t, R.X)) return 0;
  u256w rn;
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (uint64_t)r.w[i] + Mod<C, 1>::w(i);
    rn.w[i] = (uint32_t)c;
    c >>= 32;
  }
  if (c == 0 && u256_lt_mod<C, 0>(rn)) {
    mm_mul<C, 0>(rm, rn, K.r2_p);
    mm_mul<C, 0>(t, rm, z2);
    if (u256_eq(t, R.X)) return 0;
  }
  return 1;
}

// ------------------------------------------------------------------ key bytes -> prep
// Formats (include/cordagpu.h): RAW 64 B X||Y; SPKI (PublicKey.getEncoded(), 91 B r1 /
// 88 B k1) ending in an uncompressed point; SEC1 04||X||Y or 02/03||X.
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

template <int C>
CG_HD uint32_t ec_key_prep_bytes(EcKeyPrep& kp, const uint8_t* arena, uint64_t lr, uint64_t off, uint32_t len,
                                 uint32_t fmt, const EcConsts& K) {
  u256w x, y;
  uint64_t pt = off;
  uint32_t ptlen = len;
  if (fmt == 1) {  // SPKI
    const uint32_t pl = C == CG_CURVE_R1 ? 26 : 23;
    if (len != pl + 65) return 3;
    for (uint32_t i = 0; i < pl; ++i)
      if (der_byte(arena, lr, off + i) != ec_spki_prefix_byte(C, (int)i)) return 3;
    pt = off + pl;
    ptlen = 65;
  } else if (fmt == 0) {  // RAW
    if (len != 64) return 3;
    ec_load_be32(x, arena, lr, off);
    ec_load_be32(y, arena, lr, off + 32);
    return ec_key_prep_xy<C>(kp, x, y, K);
  } else if (fmt != 2) {
    return 3;
  }
  const uint32_t tag = ptlen ? der_byte(arena, lr, pt) : 0u;
  if (ptlen == 65 && tag == 4) {
    ec_load_be32(x, arena, lr, pt + 1);
    ec_load_be32(y, arena, lr, pt + 33);
    return ec_key_prep_xy<C>(kp, x, y, K);
  }
  if (ptlen == 33 && (tag == 2 || tag == 3)) {
    ec_load_be32(x, arena, lr, pt + 1);
    if (!ec_decompress<C>(y, x, tag & 1u, K)) return 3;
    return ec_key_prep_xy<C>(kp, x, y, K);
  }
  return 3;
}
