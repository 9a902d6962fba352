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
extern uint64_t g_m29_nsqr[2];  // of the mod-p products, the squares (ec9.h: 45 a*a MACs, not 81)
#define M29_COUNT(C, N) (++g_m29_nmul[C][N])
#define M29_COUNT_SQR(C) (++g_m29_nsqr[C])
#else
#define M29_COUNT(C, N) ((void)0)
#define M29_COUNT_SQR(C) ((void)0)
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

// secp256k1's field prime p = 2^256 - 2^32 - 977 is pseudo-Mersenne: its elements are kept in
// PLAIN form (R = 1 in everything below: m29_r2 gives 1, so the "Montgomery" conversions are
// identities) and a product is folded instead of Montgomery-reduced. The fold uses
// 2^261 = 32 * 2^256 = 2^37 + 31264 (mod p): 81 + 11 MACs per product instead of 162.
#ifndef CG_M29_K1_PLAIN  // 0: secp256k1 p in Montgomery form like the other moduli (A/B builds)
#define CG_M29_K1_PLAIN 1
#endif
constexpr bool m29_plain(int C, int N) { return CG_M29_K1_PLAIN && C == 0 && N == 0; }

// r = a b mod p (p = 2^256 - 2^32 - 977) for limbs < 2^30 (a b < 2^524); r reduced (< 2p). The low nine product columns stay raw 64-bit sums (no carries); the high eight
// are product-scanned into 29-bit limbs H, folded into the low columns (H_m 31264 into column m,
// H_m 2^8 into column m + 1), then one carry chain; bits >= 256 fold once more (x 977, x 2^32).
CG_HD void m29_mul_k1p(f29& r, const f29& a, const f29& b) {
  fe_acc_t c[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    fe_acc_t s = 0;
#pragma unroll
    for (int i = 0; i <= k; ++i) s += (fe_acc_t)((uint64_t)a.v[i] * b.v[k - i]);
    c[k] = s;
  }
  uint32_t H[9];
  fe_acc_t acc = 0;
#pragma unroll
  for (int k = 9; k < 17; ++k) {
#pragma unroll
    for (int i = k - 8; i < 9; ++i) acc += (fe_acc_t)((uint64_t)a.v[i] * b.v[k - i]);
    FE_ASSERT(acc < ((fe_acc_t)1 << 64));
    H[k - 9] = (uint32_t)acc & M29_MASK;
    acc >>= 29;
  }
  FE_ASSERT(acc < ((fe_acc_t)1 << 31));  // a b < 2^524
  H[8] = (uint32_t)acc;
  // 2^261 = 2^37 + 31264 (mod p): H_m 2^{29m} 2^261 -> H_m 31264 (column m) + H_m 2^8 (column m + 1)
  const uint32_t k31264 = m29_opaque(31264u), k256 = m29_opaque(256u);  // MACs, not shift pairs
#pragma unroll
  for (int m = 0; m < 9; ++m) {
    c[m] += (fe_acc_t)((uint64_t)H[m] * k31264);
    if (m < 8) c[m + 1] += (fe_acc_t)((uint64_t)H[m] * k256);
  }
  uint32_t M[9];
  acc = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    acc += c[j];
    FE_ASSERT(acc >= c[j]);  // no 64-bit wrap
    M[j] = (uint32_t)acc & M29_MASK;
    acc >>= 29;
  }
  acc += (fe_acc_t)H[8] << 8;  // H_8's 2^8 term: weight 2^261 again
  FE_ASSERT(acc < ((fe_acc_t)1 << 40));
  // bits >= 256: top 2^261 (31264 into limb 0, 2^8 into limb 1) and M[8] >> 24 (977, 2^3)
  const fe_acc_t top = acc;
  const uint32_t t = M[8] >> 24;
  M[8] &= 0xffffffu;
  acc = top * 31264u + (fe_acc_t)(t * 977u) + M[0];
  uint32_t out[9];
  out[0] = (uint32_t)acc & M29_MASK;
  acc >>= 29;
  acc += ((fe_acc_t)top << 8) + (fe_acc_t)(t << 3) + M[1];
  out[1] = (uint32_t)acc & M29_MASK;
  uint32_t cy = (uint32_t)(acc >> 29);  // < 2^19: the rest of the chain in 32 bits
#pragma unroll
  for (int j = 2; j < 9; ++j) {
    const uint32_t x = M[j] + cy;
    out[j] = j < 8 ? x & M29_MASK : x;
    cy = x >> 29;
  }
  FE_ASSERT(out[8] < (1u << 29));
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = out[i];
}

// secp256r1's p = 2^256 - 2^224 + 2^192 + 2^96 - 1 in 29-bit limbs is (2^29-1, 2^29-1, 2^29-1,
// 2^9-1, 0, 0, 2^18, 2^29-2^21, 2^24-1): the run of all-ones limbs telescopes, limbs 0..3 being
// 2^96 - 1. With -p^-1 = 1 (mod 2^29) the Montgomery digit q is the column's low 29 bits, so the -q
// term only clears bits the column shift drops: q p costs four MACs (2^9, 2^18, limbs 7 and 8)
// instead of seven.
#ifndef CG_M29_R1_TELESCOPE  // 0: seven MACs per digit (A/B builds)
#define CG_M29_R1_TELESCOPE 1
#endif
constexpr bool m29_r1p_tel(int C, int N) { return CG_M29_R1_TELESCOPE && C == 1 && N == 0; }
static_assert(m29_limb(1, 0, 1, 0) == M29_MASK && m29_limb(1, 0, 1, 1) == M29_MASK && m29_limb(1, 0, 1, 2) == M29_MASK &&
                  m29_limb(1, 0, 1, 3) == 0x1ffu && m29_limb(1, 0, 1, 4) == 0 && m29_limb(1, 0, 1, 5) == 0 &&
                  m29_limb(1, 0, 1, 6) == (1u << 18) && m29_ninv(1, 0) == 1u,
              "secp256r1 p limbs as the telescoped reduction assumes");

// r = a b R^-1 mod m, product scanning (bounds: header). r is reduced.
template <int C, int N>
CG_HD void m29_mul(f29& r, const f29& a, const f29& b) {
  M29_COUNT(C, N);
  if constexpr (m29_plain(C, N)) {
    m29_mul_k1p(r, a, b);
#ifdef FE_BOUNDS_CHECK
    int32_t br = 0;
    for (int i = 0; i < 9; ++i) {
      const int32_t d = (int32_t)r.v[i] - (int32_t)m29_limb(C, N, 2, i) + br;
      br = d >> 29;
    }
    FE_ASSERT(br < 0);
#endif
    return;
  }
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
      if (!(i < k && j >= 0 && j < 9)) continue;
      if (m29_r1p_tel(C, N)) {  // q p = q (2^96 - 1 + 2^192 + p7 2^203 + p8 2^232): see m29_r1p_tel
        if (j == 3) acc += (fe_acc_t)((uint64_t)q[i] * m29_opaque(1u << 9));  // one MAC, not shift + masks
        if (j == 6) acc += (fe_acc_t)((uint64_t)q[i] * m29_opaque(1u << 18));
        if (j >= 7) acc += (fe_acc_t)((uint64_t)q[i] * m29_limb(C, N, 1, j));
      } else if (m29_limb(C, N, 1, j) != 0) {
        acc += (fe_acc_t)((uint64_t)q[i] *
                          (m29_pow2(m29_limb(C, N, 1, j)) ? m29_opaque(m29_limb(C, N, 1, j)) : m29_limb(C, N, 1, j)));
      }
    }
    if (k < 9) {
      const uint32_t qk = m29_ninv(C, N) == 1u ? ((uint32_t)acc & M29_MASK)
                                                : (((uint32_t)acc * m29_ninv(C, N)) & M29_MASK);
      q[k] = qk;
      // telescoped: the -q term clears the low 29 bits, which the shift below drops anyway
      if (!m29_r1p_tel(C, N)) acc += (fe_acc_t)((uint64_t)qk * m29_limb(C, N, 1, 0));
      FE_ASSERT(m29_r1p_tel(C, N) || ((uint64_t)acc & M29_MASK) == 0);
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

// r = a - K m if a >= K m (a normalized, K any small multiple: m29_limb_k)
template <int C, int N, uint32_t K>
CG_HD void m29_csub_k(f29& r, const f29& a) {
  uint32_t d[9];
  int32_t br = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int32_t s = (int32_t)a.v[i] - (int32_t)m29_limb_k(C, N, K, i) + br;
    d[i] = (uint32_t)s & M29_MASK;
    br = s >> 29;
  }
  const bool take = br == 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = take ? d[i] : a.v[i];
}

// r = a - b reduced, for a reduced and b a lazy sum of three normalized values below 6m in all
// (limbs < 3 * 2^29): one signed chain a + 6m - b, in (0, 8m), then the conditional subtractions
// of 4m and 2m. Three carry chains where sub(sub(a, b1), add(b2, b3)) takes six.
template <int C, int N>
CG_HD void m29_sub_lazy3(f29& r, const f29& a, const f29& b) {
  f29 t;
  int32_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE_ASSERT(b.v[i] < 3u * (1u << 29));
    const int32_t s = (int32_t)(a.v[i] + m29_limb_k(C, N, 6, i)) - (int32_t)b.v[i] + c;
    t.v[i] = (uint32_t)s & M29_MASK;
    c = s >> 29;
  }
  FE_ASSERT(c == 0);
  m29_csub_k<C, N, 4>(t, t);
  m29_csub_k<C, N, 2>(r, t);
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

// a^(m-2) = a^-1 (Fermat; a != 0) by a 4-bit sliding window over the constant exponent: the odd
// powers a, a^3, .., a^15 (8 products), then per window its squarings and one product. The windows
// are laid out at compile time (M29InvSched: squarings and table index per window, scalar loads in
// the loop); the table entry is picked by a uniform switch, so every product has static operands.
// secp256r1 n - 2 has 160 one bits: 416 products by square-and-multiply, ~315 here.
struct M29InvSched {
  uint32_t n, tail;  // windows; squarings after the last one
  uint8_t sq[96];    // squarings before window w's product (w >= 1)
  uint8_t idx[96];   // window w's odd power a^(2 idx + 1)
};
constexpr M29InvSched m29_make_inv_sched(int C, int N) {
  M29InvSched s{};
  uint32_t e[8] = {};
  for (int i = 0; i < 8; ++i) e[i] = m29_w32(C, N, i);
  e[0] -= 2;  // the low word of every modulus here is >= 2
  int i = 255;
  while (i > 0 && !((e[i >> 5] >> (i & 31)) & 1u)) --i;
  uint32_t zeros = 0;
  while (i >= 0) {
    if (!((e[i >> 5] >> (i & 31)) & 1u)) {
      ++zeros;
      --i;
      continue;
    }
    int l = i - 3 > 0 ? i - 3 : 0;
    while (!((e[l >> 5] >> (l & 31)) & 1u)) ++l;
    uint32_t v = 0;
    for (int j = i; j >= l; --j) v = (v << 1) | ((e[j >> 5] >> (j & 31)) & 1u);
    s.sq[s.n] = (uint8_t)(s.n == 0 ? 0u : zeros + (uint32_t)(i - l + 1));
    s.idx[s.n] = (uint8_t)(v >> 1);
    ++s.n;
    zeros = 0;
    i = l - 1;
  }
  s.tail = zeros;
  return s;
}
#if defined(__HIP_DEVICE_COMPILE__)
static __constant__ const M29InvSched CG_M29_INV_SCHED[2][2] = {
    {m29_make_inv_sched(0, 0), m29_make_inv_sched(0, 1)}, {m29_make_inv_sched(1, 0), m29_make_inv_sched(1, 1)}};
#else
static const M29InvSched CG_M29_INV_SCHED[2][2] = {
    {m29_make_inv_sched(0, 0), m29_make_inv_sched(0, 1)}, {m29_make_inv_sched(1, 0), m29_make_inv_sched(1, 1)}};
#endif
static_assert(m29_make_inv_sched(1, 1).n < 96 && m29_make_inv_sched(0, 1).n < 96 && m29_make_inv_sched(1, 0).n < 96 &&
                  m29_make_inv_sched(0, 0).n < 96,
              "inversion windows fit the schedule");

#ifndef CG_M29_INV_WINDOW  // 0: square-and-multiply (A/B)
#define CG_M29_INV_WINDOW 1
#endif
// Windowed for the group order only (k_ec_inv's s^-1, ~1 wave per SIMD: latency-bound, registers
// to spare); the field inversions of the table builds keep square-and-multiply, whose register
// footprint keeps those kernels at 3 waves per SIMD (the 8-entry table took k_ec_wide_rows from 155
// to 216 VGPRs).
template <int C, int N>
CG_HD void m29_inv(f29& r, const f29& a, const f29& one_m) {
  if constexpr (CG_M29_INV_WINDOW && N == 1) {
  (void)one_m;
  const M29InvSched& S = CG_M29_INV_SCHED[C][N];
  // eight named values, not an array: an array of them stayed in scratch for secp256r1
  f29 a2, t0 = a, t1, t2, t3, t4, t5, t6, t7;
  m29_sq<C, N>(a2, a);
  m29_mul<C, N>(t1, t0, a2);
  m29_mul<C, N>(t2, t1, a2);
  m29_mul<C, N>(t3, t2, a2);
  m29_mul<C, N>(t4, t3, a2);
  m29_mul<C, N>(t5, t4, a2);
  m29_mul<C, N>(t6, t5, a2);
  m29_mul<C, N>(t7, t6, a2);
  f29 acc;
  switch (S.idx[0]) {
    case 0: acc = t0; break;
    case 1: acc = t1; break;
    case 2: acc = t2; break;
    case 3: acc = t3; break;
    case 4: acc = t4; break;
    case 5: acc = t5; break;
    case 6: acc = t6; break;
    default: acc = t7; break;
  }
#pragma unroll 1
  for (uint32_t w = 1; w < S.n; ++w) {
#pragma unroll 1
    for (uint32_t j = 0; j < S.sq[w]; ++j) m29_sq<C, N>(acc, acc);
    switch (S.idx[w]) {  // uniform: the schedule is the same for every lane
      case 0: m29_mul<C, N>(acc, acc, t0); break;
      case 1: m29_mul<C, N>(acc, acc, t1); break;
      case 2: m29_mul<C, N>(acc, acc, t2); break;
      case 3: m29_mul<C, N>(acc, acc, t3); break;
      case 4: m29_mul<C, N>(acc, acc, t4); break;
      case 5: m29_mul<C, N>(acc, acc, t5); break;
      case 6: m29_mul<C, N>(acc, acc, t6); break;
      default: m29_mul<C, N>(acc, acc, t7); break;
    }
  }
#pragma unroll 1
  for (uint32_t j = 0; j < S.tail; ++j) m29_sq<C, N>(acc, acc);
  r = acc;
  } else {
  uint32_t e[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) e[i] = m29_w32(C, N, i);
  e[0] -= 2;  // the low word of every modulus here is >= 2
  m29_pow<C, N>(r, a, e, one_m);
  }
}

// plain (reduced, Montgomery-free) value -> canonical 8 words
template <int C, int N>
CG_HD void m29_to_words_canon(uint32_t w[8], const f29& a) {
  f29 c;
  m29_canon<C, N>(c, a);
  f29_to_words(w, c);
}
