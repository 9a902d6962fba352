// Montgomery arithmetic modulo a 256-bit prime in 9 unsaturated 29-bit limbs, one element per
// lane in VGPRs (secp256r1 / secp256k1: field p and group order n).
//
// Why 29-bit limbs: with 32-bit limbs every 32x32->64 product added into a column needs its
// own carry detection (the compiler emits v_mad_u64_u32 + 64-bit add + compare + add-carry,
// ~4.5 instructions per product: 457 VALU per 8x8 Montgomery product on gfx950). With 29-bit
// limbs a column of up to 18 products (9 of a*b, 9 of q*m) stays below 2^64, so every product
// is ONE v_mad_u64_u32 accumulating in place, and the carry is one shift per column.
//
// Representation (R = 2^261):
//   "normalized"  every limb < 2^29
//   "reduced"     normalized and value < 2m (the Montgomery product's output range)
//   m29_mul accepts limbs < 2^30 and values < 4m, so the lazy sum of two reduced values can be
//   multiplied without reducing it first: a column is <= 9*2^60 + 9*2^58 + 2^35 < 2^64, and
//   (a b + q m) / R < (16 m^2 + R m) / R < 2m because 16 m < R.
// Equality and zero tests go through m29_canon (value in [0, m)).
#pragma once
#include <stdint.h>

#include "fe25519.h"  // CG_HD, fe_acc_t, FE_ASSERT

#define M29_MASK 0x1fffffffu

// Host-build op counter (tests/native/host_kernels.cpp): Montgomery products per (curve, modulus),
// the executed-work figure bench.py prices the ECDSA kernels with. Compiled out of the device build.
#ifdef FE_OP_COUNT
extern uint64_t g_m29_nmul[2][2];
#define M29_COUNT(C, N) (++g_m29_nmul[C][N])
#else
#define M29_COUNT(C, N) ((void)0)
#endif

struct f29 {
  uint32_t v[9];
};

// 32-bit little-endian words of the moduli. C: 0 = secp256k1, 1 = secp256r1; N: 0 = p, 1 = n.
constexpr uint32_t m29_w32(int C, int N, int i) {
  constexpr uint32_t R1P[8] = {0xffffffffu, 0xffffffffu, 0xffffffffu, 0u, 0u, 0u, 1u, 0xffffffffu};
  constexpr uint32_t R1N[8] = {0xfc632551u, 0xf3b9cac2u, 0xa7179e84u, 0xbce6faadu,
                               0xffffffffu, 0xffffffffu, 0u, 0xffffffffu};
  constexpr uint32_t K1P[8] = {0xfffffc2fu, 0xfffffffeu, 0xffffffffu, 0xffffffffu,
                               0xffffffffu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  constexpr uint32_t K1N[8] = {0xd0364141u, 0xbfd25e8cu, 0xaf48a03bu, 0xbaaedce6u,
                               0xfffffffeu, 0xffffffffu, 0xffffffffu, 0xffffffffu};
  return i < 0 || i >= 8 ? 0u : (C == 1 ? (N == 0 ? R1P[i] : R1N[i]) : (N == 0 ? K1P[i] : K1N[i]));
}

// word i (0..9) of k * m, k = 1 or 2
constexpr uint32_t m29_wk(int C, int N, int k, int i) {
  return k == 1 ? m29_w32(C, N, i)
                : (uint32_t)((m29_w32(C, N, i) << 1) | (i > 0 ? (m29_w32(C, N, i - 1) >> 31) : 0u));
}

// 29-bit limb i (0..8) of k * m
constexpr uint32_t m29_limb(int C, int N, int k, int i) {
  return (uint32_t)((((uint64_t)m29_wk(C, N, k, (29 * i) >> 5) >> ((29 * i) & 31)) |
                     ((uint64_t)m29_wk(C, N, k, ((29 * i) >> 5) + 1) << (32 - ((29 * i) & 31)))) &
                    M29_MASK);
}

// 29-bit limb i (0..8) of k * m for a small k (k m < 2^261)
constexpr uint32_t m29_limb_k(int C, int N, uint32_t k, int i) {
  uint64_t carry = 0;
  uint32_t w[9] = {};
  for (int j = 0; j < 9; ++j) {
    const uint64_t x = (uint64_t)m29_w32(C, N, j) * k + carry;
    w[j] = (uint32_t)x;
    carry = x >> 32;
  }
  const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
  const uint64_t x = ((uint64_t)w[wi] >> sh) | (wi + 1 < 9 ? (uint64_t)w[wi + 1] << (32 - sh) : 0u);
  return (uint32_t)x & M29_MASK;
}

// -m^-1 mod 2^29 (Newton iteration for m^-1 mod 2^32)
constexpr uint32_t m29_ninv(int C, int N) {
  uint32_t inv = 1;
  for (int k = 0; k < 5; ++k) inv *= 2u - m29_w32(C, N, 0) * inv;
  return (0u - inv) & M29_MASK;
}

CG_HD void f29_zero(f29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) a.v[i] = 0;
}

CG_HD bool f29_iszero_raw(const f29& a) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) o |= a.v[i];
  return o == 0;
}

CG_HD bool f29_eq_raw(const f29& a, const f29& b) {
  uint32_t o = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) o |= a.v[i] ^ b.v[i];
  return o == 0;
}

// 8 little-endian 32-bit words (value < 2^256) -> normalized limbs
CG_HD void f29_from_words(f29& r, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)w[wi] >> sh;
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    r.v[i] = (uint32_t)x & M29_MASK;
  }
}

// normalized limbs, value < 2^256 -> 8 words
CG_HD void f29_to_words(uint32_t w[8], const f29& a) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int bit = 32 * k, li = bit / 29, sh = bit % 29;  // sh <= 21: two limbs cover 32 bits
    const uint64_t x = ((uint64_t)a.v[li] >> sh) | ((uint64_t)a.v[li + 1] << (29 - sh));
    w[k] = (uint32_t)x;
  }
}

// A modulus limb as a multiply operand. A power-of-two limb (secp256r1 p: 2^18) would otherwise be
// folded into a 64-bit shift and two masks (3 VALU, ~4 ns of issue) instead of one v_mad_u64_u32
// (~2.4 ns): hide it in an SGPR the compiler cannot see through (SALU, off the VALU path).
#ifndef CG_M29_OPAQUE_POW2  // 0: let the compiler fold power-of-two limbs (A/B builds)
#define CG_M29_OPAQUE_POW2 1
#endif
constexpr bool m29_pow2(uint32_t v) { return CG_M29_OPAQUE_POW2 && v != 0 && (v & (v - 1)) == 0; }
CG_HD uint32_t m29_opaque(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(v));
#endif
  return v;
}

// r = a b R^-1 mod m, product scanning (bounds: header). r is reduced.
template <int C, int N>
CG_HD void m29_mul(f29& r, const f29& a, const f29& b) {
  M29_COUNT(C, N);
  uint32_t q[9], out[9];
  fe_acc_t acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (j >= 0 && j < 9) acc += (fe_acc_t)((uint64_t)a.v[i] * b.v[j]);
    }
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      const int j = k - i;
      if (i < k && j >= 0 && j < 9 && m29_limb(C, N, 1, j) != 0)
        acc += (fe_acc_t)((uint64_t)q[i] *
                          (m29_pow2(m29_limb(C, N, 1, j)) ? m29_opaque(m29_limb(C, N, 1, j)) : m29_limb(C, N, 1, j)));
    }
    if (k < 9) {
      const uint32_t qk = m29_ninv(C, N) == 1u ? ((uint32_t)acc & M29_MASK)
                                                : (((uint32_t)acc * m29_ninv(C, N)) & M29_MASK);
      q[k] = qk;
      acc += (fe_acc_t)((uint64_t)qk * m29_limb(C, N, 1, 0));
      FE_ASSERT(((uint64_t)acc & M29_MASK) == 0);
    } else {
      out[k - 9] = (uint32_t)acc & M29_MASK;
    }
    FE_ASSERT(acc < ((fe_acc_t)1 << 64));
    acc >>= 29;
  }
  out[8] = (uint32_t)acc;
#ifdef FE_BOUNDS_CHECK
  {  // the output is reduced (< 2m): the inputs respected a b < m R
    int32_t br = 0;
    for (int i = 0; i < 9; ++i) {
      const int32_t d = (int32_t)out[i] - (int32_t)m29_limb(C, N, 2, i) + br;
      br = d >> 29;
    }
    FE_ASSERT(br < 0);
  }
#endif
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = out[i];
}

template <int C, int N>
CG_HD void m29_sq(f29& r, const f29& a) {
  m29_mul<C, N>(r, a, a);
}

// r = a - K m if a >= K m (a normalized, K = 1 or 2)
template <int C, int N, int K>
CG_HD void m29_csub(f29& r, const f29& a) {
  uint32_t d[9];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t s = (int32_t)a.v[i] - (int32_t)m29_limb(C, N, K, i) + br;
    d[i] = (uint32_t)s & M29_MASK;
    br = s >> 29;
  }
  const bool take = br == 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = take ? d[i] : a.v[i];
}

// canonical representative in [0, m) of a reduced value
template <int C, int N>
CG_HD void m29_canon(f29& r, const f29& a) {
  m29_csub<C, N, 1>(r, a);
}

template <int C, int N>
CG_HD bool m29_iszero(const f29& a) {
  f29 c;
  m29_canon<C, N>(c, a);
  return f29_iszero_raw(c);
}

template <int C, int N>
CG_HD bool m29_eq(const f29& a, const f29& b) {
  f29 x, y;
  m29_canon<C, N>(x, a);
  m29_canon<C, N>(y, b);
  return f29_eq_raw(x, y);
}

// reduced + reduced -> reduced
template <int C, int N>
CG_HD void m29_add(f29& r, const f29& a, const f29& b) {
  f29 t;
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t s = a.v[i] + b.v[i] + c;
    t.v[i] = s & M29_MASK;
    c = s >> 29;
  }
  m29_csub<C, N, 2>(r, t);
}

// reduced + reduced -> limbs < 2^30, value < 4m: only as an m29_mul operand
CG_HD void m29_add_lazy(f29& r, const f29& a, const f29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
}

// reduced - reduced -> reduced (a - b, plus 2m when negative)
template <int C, int N>
CG_HD void m29_sub(f29& r, const f29& a, const f29& b) {
  uint32_t t[9];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t s = (int32_t)a.v[i] - (int32_t)b.v[i] + br;
    t[i] = (uint32_t)s & M29_MASK;
    br = s >> 29;
  }
  const uint32_t mask = (uint32_t)br;  // 0 or all ones
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t s = t[i] + (m29_limb(C, N, 2, i) & mask) + c;
    r.v[i] = s & M29_MASK;
    c = s >> 29;
  }
}

// "Semi-reduced": normalized limbs, value < 4m. A valid m29_mul operand when the other operand is
// < 4m (16 m^2 < m R), not a valid m29_sub / m29_add input.
// r = a + 2m - b (a, b reduced): ONE signed carry chain instead of m29_sub's two; r semi-reduced,
// r in (0, 4m).
template <int C, int N>
CG_HD void m29_sub2(f29& r, const f29& a, const f29& b) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t s = (int32_t)(a.v[i] + m29_limb(C, N, 2, i)) - (int32_t)b.v[i] + c;
    r.v[i] = (uint32_t)s & M29_MASK;
    c = s >> 29;
  }
  FE_ASSERT(c == 0);
}

// r = 2m - a for a reduced and a != 0 (as a value): r in (0, 2m), reduced; one carry chain.
template <int C, int N>
CG_HD void m29_neg2(f29& r, const f29& a) {
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t s = (int32_t)m29_limb(C, N, 2, i) - (int32_t)a.v[i] + c;
    r.v[i] = (uint32_t)s & M29_MASK;
    c = s >> 29;
  }
  FE_ASSERT(c == 0);
}

// Can a semi-reduced a (value < 4m) be 0 mod m, i.e. one of 0, m, 2m, 3m? A filter on limb 0 (false
// positives ~3 in 2^29); m29_zero_semi decides.
template <int C, int N>
CG_HD bool m29_maybe_zero_semi(const f29& a) {
  const uint32_t x = a.v[0];
  return x == 0u || x == m29_limb_k(C, N, 1, 0) || x == m29_limb_k(C, N, 2, 0) || x == m29_limb_k(C, N, 3, 0);
}
template <int C, int N>
CG_HD bool m29_zero_semi(const f29& a) {
  bool z = false;
#pragma unroll
  for (uint32_t k = 0; k < 4; ++k) {
    uint32_t o = 0;
#pragma unroll
    for (int i = 0; i < 9; ++i) o |= a.v[i] ^ m29_limb_k(C, N, k, i);
    z |= o == 0;
  }
  return z;
}

template <int C, int N>
CG_HD void m29_neg(f29& r, const f29& a) {
  f29 z;
  f29_zero(z);
  m29_sub<C, N>(r, z, a);
}

// a^e (a Montgomery, e plain little-endian words), MSB first
template <int C, int N>
CG_HD void m29_pow(f29& r, const f29& a, const uint32_t e[8], const f29& one_m) {
  f29 acc = one_m;
  for (int i = 255; i >= 0; --i) {
    m29_sq<C, N>(acc, acc);
    if ((e[i >> 5] >> (i & 31)) & 1u) m29_mul<C, N>(acc, acc, a);
  }
  r = acc;
}

// a^(m-2) = a^-1 (Fermat; a != 0)
template <int C, int N>
CG_HD void m29_inv(f29& r, const f29& a, const f29& one_m) {
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = m29_w32(C, N, i);
  e[0] -= 2;  // the low word of every modulus here is >= 2
  m29_pow<C, N>(r, a, e, one_m);
}

// plain (reduced, Montgomery-free) value -> canonical 8 words
template <int C, int N>
CG_HD void m29_to_words_canon(uint32_t w[8], const f29& a) {
  f29 c;
  m29_canon<C, N>(c, a);
  f29_to_words(w, c);
}
