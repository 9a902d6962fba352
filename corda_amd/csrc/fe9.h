// GF(2^255 - 19) in nine 29-bit limbs, for the wide-table Ed25519 ladders (k_ed_ladder_wide and the
// fixed-base B part of the other ladders): one element per lane in VGPRs.
//
// Why a second representation (fe25519.h keeps radix 2^25.5 for everything else): the wide ladder
// is VALU-issue-bound and on gfx950 every VALU instruction of a MAC-heavy stream costs ~4 cycles
// whatever it is (profiles/r04/ubench: a MAC + v_add_u32 mix issues at 15-16 instruction-lanes per
// clock per SIMD, the same as MACs alone), so the instruction COUNT sets the time. Radix 2^25.5
// spends 100 MACs, ten x19 multiplies, five doublings and twelve three-instruction 64-bit carries
// per product, and two instructions per limb per subtraction. Nine 29-bit limbs take 81 MACs; the
// columns of weight >= 2^261 fold back with 2^261 = 19 * 2^6 = 1216 (mod p) split at their 32-bit
// halves (lo * 1216 into column k - 9, hi * 1216 * 2^3 = hi * 9728 into column k - 8: two MACs per
// column and no carries), and the nine low columns are product-scanned (a column's carry is the
// next column's initial accumulator: two instructions per column). ~121 instructions per product
// against ~150, and a subtraction is one instruction per limb.
//
// The price is headroom: a column of nine 58-bit products is 2^61.2, leaving 2.8 bits below 2^64
// (1.8 below 2^63 signed). So limbs may be SIGNED (a difference is a plain limb-wise subtraction)
// and there are two products, both exact for the operand classes below (FE_BOUNDS_CHECK asserts
// every column on the host, tests/test_host_kernels.py):
//   fe9_mul<false> (uu): non-negative limbs, unsigned MACs; operand limbs a_i b_j < 2^60.6.
//   fe9_mul<true>  (ss): signed limbs, signed MACs; |a_i b_j| < 2^59.6. The product may be negative,
//       so the low columns carry B = 2^40 p = 2^295 - 19 2^40 (2^63 in column 8, -19 2^40 in column
//       0): column 8's total lies in (0, 2^64) and its carry-out is non-negative, so the output is
//       non-negative like uu's.
// Operand classes (limb bounds):
//   T  (tight: any product's output)   limb_i in [0, 2^29), limb_1 in [0, 2^29 + 2^17)
//   A2 (T + T)                          [0, 2^30 + 2^18)
//   S  (T - T, fe9_sub)                 (-2^29 - 2^17, 2^29 + 2^17)
//   V  (T + 128 p - T, fe9_subk)        [2^28, 2^30 + 2^29 + 2^17)
//   uu: T x T, A2 x T, A2 x A2, A2 x V (2^60.59 per term, 9 terms 2^63.76 < 2^64)
//   ss: S x T, S x A2, S x V           (2^59.59 per term, 9 terms 2^62.76 < 2^63)
#pragma once
#include <stdint.h>

#include <type_traits>

#include "fe25519.h"
#include "ge25519.h"

#define FE9_M 0x1fffffffu

struct fe9 {
  uint32_t v[9];
};

#ifdef FE_OP_COUNT
extern uint64_t g_fe9_nmul;
#define FE9_COUNT() (++g_fe9_nmul)
#else
#define FE9_COUNT() ((void)0)
#endif

// A constant multiplier as an SGPR the compiler cannot fold into shifts (mont29.h m29_opaque).
CG_HD uint32_t fe9_opaque(uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+s"(v));
#endif
  return v;
}

// a b + c as one MAC whose result the compiler may not re-associate (an empty asm pins it): product
// scanning keeps the carry inside the column's MAC chain instead of a 64-bit add per column. (The
// MAC itself as inline asm made the hazard recognizer put an s_nop after every one: 313 per addition.)
CG_HD uint64_t fe9_mac_u(uint32_t a, uint32_t b, uint64_t c) {
  uint64_t r = (uint64_t)a * b + c;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(r));
#endif
  return r;
}
CG_HD int64_t fe9_mac_i(uint32_t a, uint32_t b, int64_t c) {
  int64_t r = (int64_t)(int32_t)a * (int32_t)b + c;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(r));
#endif
  return r;
}

CG_HD void fe9_0(fe9& h) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = 0;
}
CG_HD void fe9_1(fe9& h) {
  fe9_0(h);
  h.v[0] = 1;
}
// 1/2 = (p + 1) / 2 = 2^254 - 9 (tight)
CG_HD void fe9_half(fe9& h) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = FE9_M;
  h.v[0] = FE9_M - 8u;
  h.v[8] = (1u << 22) - 1u;
}

CG_HD void fe9_add(fe9& h, const fe9& f, const fe9& g) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = f.v[i] + g.v[i];
}
// signed difference (class S when f, g are T)
CG_HD void fe9_sub(fe9& h, const fe9& f, const fe9& g) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = f.v[i] - g.v[i];
}
// f + 128 p - g, non-negative limbs for tight g (class V): 128 p = 2 * (2^261 - 1216) with every
// 29-bit limb of 64 p doubled, limbs >= 2^30 - 2432 > any tight limb
CG_HD void fe9_subk(fe9& h, const fe9& f, const fe9& g) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const uint32_t k = i == 0 ? (1u << 30) - 2432u : (1u << 30) - 2u;
    FE_ASSERT(g.v[i] <= k);
    h.v[i] = (f.v[i] + k) - g.v[i];
  }
}
// Non-negative limbs below 2^31 (classes A2, V) -> tight (class T): one carry pass, the bits of
// weight >= 2^261 folded back as 1216 into limb 0 and its carry into limb 1
CG_HD void fe9_carry(fe9& h, const fe9& f) {
  uint32_t n[9];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    FE_ASSERT(f.v[i] < (1u << 31));
    c += f.v[i];
    n[i] = (uint32_t)c & FE9_M;
    c >>= 29;
  }
  const uint64_t x0 = (uint64_t)n[0] + c * 1216u;
  h.v[0] = (uint32_t)x0 & FE9_M;
  h.v[1] = n[1] + (uint32_t)(x0 >> 29);
  FE_ASSERT(h.v[1] < (1u << 29) + (1u << 17));
#pragma unroll
  for (int i = 2; i < 9; ++i) h.v[i] = n[i];
}
CG_HD void fe9_cmov(fe9& h, const fe9& a, const fe9& b, bool take_b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) h.v[i] = take_b ? b.v[i] : a.v[i];
}

#ifdef FE_BOUNDS_CHECK
typedef __int128 fe9_acc;
#define FE9_IN_RANGE(x, lo, hi) FE_ASSERT((x) >= (fe9_acc)(lo) && (x) < (fe9_acc)(hi))
#endif

// out = a b mod p, tight. Signed: limbs of a and b are int32 (class S operands), else uint32.
// Pin (default FE9_PIN_ACC): the column sums as one opaque chain from the carry (the ladders: issue-
// bound, 2-3 waves per SIMD hide the chain's latency). Pin = false: the compiler's independent column
// chains, for latency-bound callers with few waves per SIMD (the wide-row builds of phase 1,
// round 6: FE9_ROWS_ILP).
// Copy = false: no opaque operand copies (round 6: operands used twice, whose copies are v_movs)
template <bool Signed, bool Pin = true, bool Copy = true>
CG_HD void fe9_mul(fe9& out, const fe9& a, const fe9& b) {
  FE9_COUNT();
  const uint32_t k1216 = fe9_opaque(1216u), k9728 = fe9_opaque(9728u);
  (void)k9728;
#ifdef FE_BOUNDS_CHECK
  // exact model with 128-bit integers: every column of the 64-bit device arithmetic must be exact
  auto prod = [&](int i, int j) -> fe9_acc {
    return Signed ? (fe9_acc)(int32_t)a.v[i] * (int32_t)b.v[j] : (fe9_acc)a.v[i] * b.v[j];
  };
  const fe9_acc lim = Signed ? ((fe9_acc)1 << 63) : ((fe9_acc)1 << 64);
  fe9_acc hc[8];
  for (int k = 9; k < 17; ++k) {
    fe9_acc s = 0;
    for (int i = k - 8; i < 9; ++i) {
      FE9_IN_RANGE(prod(i, k - i), Signed ? -((fe9_acc)1 << 60) : 0, Signed ? ((fe9_acc)1 << 60) : ((fe9_acc)1 << 61));
      s += prod(i, k - i);
    }
    FE9_IN_RANGE(s, Signed ? -lim : 0, lim);
    hc[k - 9] = s;
  }
  uint32_t d[9];
  fe9_acc acc = Signed ? -(fe9_acc)19 * ((fe9_acc)1 << 40) : 0;
  for (int m = 0; m < 9; ++m) {
    for (int i = 0; i <= m; ++i) acc += prod(i, m - i);
    if (m <= 7) acc += (fe9_acc)(uint32_t)(uint64_t)hc[m] * 1216;  // lo half (two's complement)
    if (m >= 1) {
      const fe9_acc h = Signed ? (fe9_acc)(int32_t)(uint32_t)((uint64_t)hc[m - 1] >> 32)
                               : (fe9_acc)(uint32_t)((uint64_t)hc[m - 1] >> 32);
      acc += h * 9728;
    }
    if (m == 8 && Signed) acc += (fe9_acc)1 << 63;
    if (m < 8) FE9_IN_RANGE(acc, Signed ? -lim : 0, lim);
    else FE9_IN_RANGE(acc, 0, (fe9_acc)1 << 64);  // column 8 (ss: biased) is non-negative
    d[m] = (uint32_t)(acc & FE9_M);
    acc >>= 29;  // floor division, exact in 128 bits
  }
  const uint64_t T = (uint64_t)acc;
  FE_ASSERT(acc >= 0 && T < (1ull << 35));
#else
  typedef typename std::conditional<Signed, int64_t, uint64_t>::type acc_t;
#ifndef FE9_PIN_COPIES
#define FE9_PIN_COPIES 1
#endif
#if defined(__HIP_DEVICE_COMPILE__) && FE9_PIN_COPIES
  // opaque 32-bit operands: in the ladder loop the compiler otherwise widened loop-carried
  // differences to 64 bits and emitted 64 x 64-bit multiplies (3 MACs + moves each)
  fe9 a_ = a, b_ = b;
  if (Copy) {
#pragma unroll
    for (int i = 0; i < 9; ++i) asm volatile("" : "+v"(a_.v[i]), "+v"(b_.v[i]));
  }
#define a a_
#define b b_
#endif
  acc_t hc[8];
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    acc_t s = 0;
#pragma unroll
    for (int i = k - 8; i < 9; ++i) {
      if (Signed) s += (acc_t)(int64_t)(int32_t)a.v[i] * (int64_t)(int32_t)b.v[k - i];
      else s += (acc_t)((uint64_t)a.v[i] * b.v[k - i]);
    }
    hc[k - 9] = s;
  }
  uint32_t d[9];
  acc_t acc = Signed ? (acc_t)(-(int64_t)19 * ((int64_t)1 << 40)) : 0;
#pragma unroll
  for (int m = 0; m < 9; ++m) {
#ifndef FE9_PIN_ACC  // round 4: 2326 -> 2217 VALU per two additions (v_lshl_add_u64 126 -> 22, plus
#define FE9_PIN_ACC 1  // 333 s_nop the other waves fill), k_ed_ladder_wide 2.80 -> 2.68 ms (profiles/r04/pin)
#endif
#ifndef FE9_SCAN_ASM  // 1: pinned MACs (fe9_mac_*): 1004 -> 993 VALU per addition, but 176 s_nop (rejected)
#define FE9_SCAN_ASM 0
#endif
#pragma unroll
    for (int i = 0; i <= m; ++i) {
      if (FE9_SCAN_ASM && m > 0) {  // every MAC of the chain (an asm one among C adds is re-associated anyway);
                                   // column 0 stays C: its constant addend then needs no VGPR copy
        if (Signed) acc = (acc_t)fe9_mac_i(a.v[i], b.v[m - i], (int64_t)acc);
        else acc = (acc_t)fe9_mac_u(a.v[i], b.v[m - i], (uint64_t)acc);
      } else if (Signed) {
        acc += (acc_t)(int64_t)(int32_t)a.v[i] * (int64_t)(int32_t)b.v[m - i];
      } else {
        acc += (acc_t)((uint64_t)a.v[i] * b.v[m - i]);
      }
#if defined(__HIP_DEVICE_COMPILE__) && FE9_PIN_ACC
      // the running column sum as an opaque value after every MAC: the carry-in then stays the
      // first MAC's addend instead of being re-associated into a separate 64-bit add
      if (Pin) asm volatile("" : "+v"(acc));
#endif
    }
    if (m <= 7) acc = (acc_t)fe9_mac_u((uint32_t)hc[m], k1216, (uint64_t)acc);
    if (m >= 1) {
      const uint32_t hi = (uint32_t)((uint64_t)hc[m - 1] >> 32);
      if (Signed) acc = (acc_t)fe9_mac_i(hi, k9728, (int64_t)acc);
      else acc = (acc_t)fe9_mac_u(hi, k9728, (uint64_t)acc);
    }
    d[m] = (uint32_t)acc & FE9_M;
    if (m < 8) {
      acc = Signed ? (acc_t)((int64_t)acc >> 29) : (acc_t)((uint64_t)acc >> 29);
    } else {
      // column 8: ss adds 2^63 (bit 63 flipped), after which the total is read as unsigned
      uint64_t c8 = (uint64_t)acc;
      if (Signed) c8 ^= 1ull << 63;
      d[8] = (uint32_t)c8 & FE9_M;
      acc = (acc_t)(c8 >> 29);
    }
  }
  const uint64_t T = (uint64_t)acc;
#if defined(__HIP_DEVICE_COMPILE__) && FE9_PIN_COPIES
#undef a
#undef b
#endif
#endif
  // T 2^261 = 1216 T: T_lo 1216 into limb 0, T_hi 2^32 1216 = T_hi 9728 2^29 into limb 1
  const uint64_t x0 = (uint64_t)d[0] + (uint64_t)(uint32_t)T * k1216;
  out.v[0] = (uint32_t)x0 & FE9_M;
  out.v[1] = d[1] + (uint32_t)(T >> 32) * 9728u + (uint32_t)(x0 >> 29);
  FE_ASSERT(out.v[1] < (1u << 29) + (1u << 17));
#pragma unroll
  for (int i = 2; i < 9; ++i) out.v[i] = d[i];
}

// Little-endian 32 bytes (value < 2^256) -> tight limbs
CG_HD void fe9_from_words(fe9& h, const uint32_t w[8]) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int bit = 29 * i, wi = bit >> 5, sh = bit & 31;
    uint64_t x = (uint64_t)w[wi] >> sh;
    if (wi + 1 < 8) x |= (uint64_t)w[wi + 1] << (32 - sh);
    h.v[i] = (uint32_t)x & FE9_M;
  }
}

CG_HD void fe9_from_fe(fe9& h, const fe& f) {
  uint32_t w[8];
  fe_tobytes_words(w, f);
  fe9_from_words(h, w);
}

// Non-negative limbs (any class but S) -> 8 words of a value < 2^255 congruent mod p (not always
// canonical: fe_frombytes_words takes it as is)
CG_HD void fe9_to_words255(uint32_t w[8], const fe9& f) {
  uint32_t n[9];
  uint64_t c = 0;
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    c += f.v[i];
    n[i] = (uint32_t)c & FE9_M;
    c >>= 29;
  }
  // bits >= 255: n_8 >> 23 and c (weight 2^261 = 2^255 2^6); 2^255 = 19
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const uint64_t t = (uint64_t)(n[8] >> 23) + (c << 6);
    n[8] &= (1u << 23) - 1u;
    c = 0;
    uint64_t x = (uint64_t)n[0] + 19u * t;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      if (i > 0) x = (uint64_t)n[i] + (x >> 29);
      n[i] = (uint32_t)x & FE9_M;
    }
    c = x >> 29;  // 0: n_8 < 2^23 + small
  }
  FE_ASSERT(n[8] < (1u << 23));
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int bit = 32 * k, li = bit / 29, sh = bit % 29;
    const uint64_t x = ((uint64_t)n[li] >> sh) | ((uint64_t)n[li + 1] << (29 - sh)) |
                       (li + 2 < 9 && sh > 26 ? (uint64_t)n[li + 2] << (58 - sh) : 0ull);
    w[k] = (uint32_t)x;
  }
}

CG_HD void fe_from_fe9(fe& h, const fe9& f) {
  uint32_t w[8];
  fe9_to_words255(w, f);
  fe_frombytes_words(h, w);
}

// ---------------------------------------------------------------- points
struct ge9_p3 {
  fe9 X, Y, Z, T;
};
// A half-scaled wide-table entry ((y+x)/2, (y-x)/2, x y d), tight: 108 B of limbs, gathered as
// 7 x 16-B LDS DMA chunks. Padded to one 128-B line (round 5; GE9_NIELS_BYTES 112 = the round-4
// packing): a random gather into the fixed-base table then fetches one line instead of 1.9 (every
// HBM read request is a 128-B line on gfx950, profiles/r05/calib). The B table grows 37.6 -> 42.9 GB;
// headline A/B 326.9 -> 332.5 M sigs/s over 4 pairs (Ed25519 ladder 13.06 -> 12.75 ms per step,
// profiles/r05/n128).
#ifndef GE9_NIELS_BYTES
#define GE9_NIELS_BYTES 128
#endif
struct ge9_niels {
  fe9 ypx, ymx, xy2d;
  uint32_t pad[(GE9_NIELS_BYTES - 108) / 4];
};
static_assert(sizeof(ge9_niels) == GE9_NIELS_BYTES && (GE9_NIELS_BYTES == 112 || GE9_NIELS_BYTES == 128),
              "ge9_niels layout");

CG_HD void ge9_niels_from(ge9_niels& o, const ge_niels& n) {
  fe9_from_fe(o.ypx, n.ypx);
  fe9_from_fe(o.ymx, n.ymx);
  fe9_from_fe(o.xy2d, n.xy2d);
  for (uint32_t& w : o.pad) w = 0;
}
// store overloads for the table builders (the host tests also build fe tables)
CG_HD void ed_niels_store(ge_niels* dst, const ge_niels& n) { *dst = n; }
CG_HD void ed_niels_store(ge9_niels* dst, const ge_niels& n) { ge9_niels_from(*dst, n); }

CG_HD void ge9_niels_identity_half(ge9_niels& n) {
  fe9_half(n.ypx);
  fe9_half(n.ymx);
  fe9_0(n.xy2d);
}

CG_HD void ge9_p3_0(ge9_p3& h) {
  fe9_0(h.X);
  fe9_1(h.Y);
  fe9_1(h.Z);
  fe9_0(h.T);
}

CG_HD void ge9_from_p3(ge9_p3& r, const ge_p3& p) {
  fe9_from_fe(r.X, p.X);
  fe9_from_fe(r.Y, p.Y);
  fe9_from_fe(r.Z, p.Z);
  fe9_from_fe(r.T, p.T);
}

// r = p + (-1)^neg q for a half-scaled entry q (HWCD mixed addition; the sums come out halved, so
// D = Z). The sign goes through the entry: -q swaps (y+x)/2 and (y-x)/2 and negates xyd, i.e.
// C -> -C, which swaps F = Z - C and G = Z + C. Every product's operand classes (header):
//   B' = (Y+X) sp   uu A2 x T      A' = (Y-X) sm   ss S x T      C = T xyd   uu T x T
//   E = B' - A' (S), H = B' + A' (A2), u = Z + C (A2), v = Z + 128p - C (V)
//   X3 = E F  ss S x {A2, V}   Y3 = G H  uu {V, A2} x A2   Z3 = u v (= F G)  uu   T3 = E H  ss S x A2
// WithT = false leaves T unset (the last addition of a ladder: projective output).
template <bool WithT>
CG_HD void ge9_madd_half(ge9_p3& r, const ge9_p3& p, const ge9_niels& q, bool neg) {
  fe9 sp, sm;
  fe9_cmov(sp, q.ypx, q.ymx, neg);
  fe9_cmov(sm, q.ymx, q.ypx, neg);
  fe9 a, b;
  fe9_add(a, p.Y, p.X);
  fe9_sub(b, p.Y, p.X);
  fe9 Bp, Ap, C;
  fe9_mul<false>(Bp, a, sp);
  fe9_mul<true>(Ap, b, sm);
  fe9_mul<false>(C, p.T, q.xy2d);
  fe9 E, H, u, v;
  fe9_sub(E, Bp, Ap);
  fe9_add(H, Bp, Ap);
  fe9_add(u, p.Z, C);
  fe9_subk(v, p.Z, C);
  fe9 F, G;
  fe9_cmov(F, v, u, neg);
  fe9_cmov(G, u, v, neg);
  fe9_mul<true>(r.X, E, F);
  fe9_mul<false>(r.Y, G, H);
  fe9_mul<false>(r.Z, u, v);
  if (WithT) fe9_mul<true>(r.T, E, H);
}

// r = (-1)^flip (p + q) for a half-scaled entry q taken as stored (round 6, ED_SIGN_FOLD): a ladder
// keeps its running point as s_k R_k, s_k the sign of op k's digit, so every op adds the entry of
// |digit| and the sign change s_k s_{k+1} rides on the output. -P = (-X, Y, Z, -T), and X3 = E F,
// T3 = E H share E: negating E alone negates the point. That is 9 multiplies of E's limbs by +-1
// (E is class S, symmetric, so -E is too) against ge9_madd_half's 36 selects of the entry halves
// and of F / G.
#ifndef ED_SIGN_FOLD
#define ED_SIGN_FOLD 1
#endif
#ifndef ED_FLIP_COPY  // which of the four output products copy their operands (bit 0: X3 ... bit 3: T3)
#define ED_FLIP_COPY 1  // X3 only: 2471 -> 2430 VALU per two loop additions (15: 2457, 0: 2674)
#endif
CG_HD uint32_t fe9_sign_mask(bool flip) {
  uint32_t s = flip ? ~0u : 1u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(s));  // a multiply by an opaque +-1, not a select of -x and x (two ops a limb)
#endif
  return s;
}
template <bool WithT>
CG_HD void ge9_madd_half_flip(ge9_p3& r, const ge9_p3& p, const ge9_niels& q, bool flip) {
  fe9 a, b;
  fe9_add(a, p.Y, p.X);
  fe9_sub(b, p.Y, p.X);
  fe9 Bp, Ap, C;
  fe9_mul<false>(Bp, a, q.ypx);
  fe9_mul<true>(Ap, b, q.ymx);
  fe9_mul<false>(C, p.T, q.xy2d);
  fe9 E, H, u, v;
  fe9_sub(E, Bp, Ap);
  const uint32_t s = fe9_sign_mask(flip);
#pragma unroll
  for (int i = 0; i < 9; ++i) E.v[i] *= s;
  fe9_add(H, Bp, Ap);
  fe9_add(u, p.Z, C);
  fe9_subk(v, p.Z, C);
  fe9_mul<true, true, (ED_FLIP_COPY & 1) != 0>(r.X, E, v);
  fe9_mul<false, true, (ED_FLIP_COPY & 2) != 0>(r.Y, u, H);
  fe9_mul<false, true, (ED_FLIP_COPY & 4) != 0>(r.Z, u, v);
  if (WithT) fe9_mul<true, true, (ED_FLIP_COPY & 8) != 0>(r.T, E, H);
}

// r = (-1)^neg q as an extended point (the first entry of a ladder, added to the identity): x =
// (y+x)/2 - (y-x)/2 and y = (y+x)/2 + (y-x)/2 carried tight, Z = 1, T = x y. One product and two
// carry passes instead of ge9_madd_half's seven products (-x swaps the two halves: -q).
CG_HD void ge9_from_niels_half(ge9_p3& r, const ge9_niels& q, bool neg) {
  fe9 sp, sm, t;
  fe9_cmov(sp, q.ypx, q.ymx, neg);
  fe9_cmov(sm, q.ymx, q.ypx, neg);
  fe9_subk(t, sp, sm);  // class V
  fe9_carry(r.X, t);
  fe9_add(t, sp, sm);   // class A2
  fe9_carry(r.Y, t);
  fe9_1(r.Z);
  fe9_mul<false>(r.T, r.X, r.Y);
}

CG_HD void ge9_to_p2(ge_p2& o, const ge9_p3& r) {
  fe_from_fe9(o.X, r.X);
  fe_from_fe9(o.Y, r.Y);
  fe_from_fe9(o.Z, r.Z);
}
