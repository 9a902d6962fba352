// Signed-limb field arithmetic for the ECDSA wide ladders (k_ec_ladder_wide): the mixed addition
// without carry chains in its additions and subtractions.
//
// mont29.h keeps every value reduced (normalized 29-bit limbs, < 2m), so each subtraction of the
// madd-2004-hmv addition is a signed carry chain (m29_sub2: ~5 instructions per limb) and X3 takes
// three chains and two conditional subtractions: ~440 of a ~2100-instruction addition (the ladder is
// issue-bound, profiles/r03 SQ pass, and every VALU instruction costs ~4 cycles in a MAC stream,
// profiles/r04/ubench). Here a field element is nine SIGNED 32-bit limbs (value = sum l_i 2^{29 i}),
// differences are limb-wise (one instruction per limb), and every product takes signed limbs
// (v_mad_i64_i32) and returns "tight" limbs: digits 0..7 in [0, 2^29) and a small signed top
// (r1), or digits with limb 2 off by < 2^16 (k1):
//   tight T   |limb| <= 2^29 + 2^16              S = T - T   |limb| <= 2^29 + 2^17
//   every operand of every product in jac_madd9 is T or S (|term| <= 2^58.001), so a column of nine
//   terms (eighteen in ec9_mul2) plus the reduction terms stays below 2^62.6 < 2^63.
// The three forms:
//   ec9_mul<C>   (a b)          ec9_mul_add<C> (a b + e, e limb-wise, |e_i| < 2^31)
//   ec9_mul2<C>  (a b + c d, one reduction)
// secp256r1 (Montgomery, R = 2^261, telescoped p as in mont29.h): signed T through REDC gives
// (T + Q p) / R, Q in [0, R); e joins at column 9 + i (added after the division). Values stay
// below ~6p in magnitude along a ladder: every product divides by R ~ 32 p, so |X3| <= |rr|^2/32p +
// p + |HHH| + 2|V| converges (~5.8p; FE_BOUNDS_CHECK asserts each column on the host).
// secp256k1 (plain, 2^261 = 2^37 + 31264 mod p): mont29.h's fold with signed columns; e joins the
// low columns before the scan, so X3 comes out folded like any product (< 2^261 + small).
// Exact tests (H = 0 mod p, the final x-check) go through ec9_to_m29 (back to mont29.h's reduced form).
#pragma once
#include "ecdsa.h"

#ifdef FE_BOUNDS_CHECK
typedef __int128 ec9_acc;
#define EC9_CHK(x) FE_ASSERT((x) > -((ec9_acc)1 << 63) && (x) < ((ec9_acc)1 << 63))
#else
typedef int64_t ec9_acc;
#define EC9_CHK(x) ((void)0)
#endif

// signed 32 x 32 -> 64 term (v_mad_i64_i32 when accumulated)
CG_HD ec9_acc ec9_t(uint32_t a, uint32_t b) { return (ec9_acc)((int64_t)(int32_t)a * (int64_t)(int32_t)b); }

// opaque copies (round 5: every product pinned copies of its operands, because in a ladder loop the
// compiler had widened loop-carried limb differences to 64 bits, as fe9.h saw). Round 6: the copies
// cost a v_mov per limb whenever the operand stayed live (~110 per addition) and hid a square's
// symmetry from the compiler; the products read their operands directly (EC9_PIN_COPIES restores the
// copies for A/B: 329.9 vs 334.8 M sigs/s over 3 pairs, profiles/r06/ec_acc) and the ISA shows no
// 64 x 64 multiply (tools/microbench/ec9_probe.hip)
CG_HD void ec9_pin(f29& o, const f29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    o.v[i] = a.v[i];
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(o.v[i]));
#endif
  }
}

// EC9_PIN_ACC (round 6, default 1): the running column sum made opaque after each term, so a
// column's chain starts from the carry instead of being summed from 0 and joined by a separate 64-bit
// add (fe9.h's FE9_PIN_ACC, adopted for the Ed25519 ladder in round 4); secp256k1's low columns then
// run after the high ones as one chain with the fold terms first. Per addition 1790 -> 1661 (r1) /
// 1786 -> 1657 (k1) static VALU (tools/microbench/ec9_probe.hip), ~1000 hazard s_nop 0 the other
// waves fill; headline A/B over 3 pairs 334.8 -> 341.7 M sigs/s, r1 ladder 7.44 -> 7.14, k1 3.38 ->
// 3.12 ms per step (profiles/r06/ec_acc). 0: the independent column sums (A/B).
#ifndef EC9_PIN_ACC
#define EC9_PIN_ACC 1
#endif
#ifndef EC9_SIGN_MUL
#define EC9_SIGN_MUL 1
#endif
// EC9_SQR=1: squares as 45 MACs against a doubled copy (ec9_col); 0: as general products (A/B)
#ifndef EC9_SQR
#define EC9_SQR 1
#endif
CG_HD void ec9_opaque(ec9_acc& x) {
#if defined(__HIP_DEVICE_COMPILE__)
  if (EC9_PIN_ACC) asm volatile("" : "+v"(x));
#else
  (void)x;
#endif
}

CG_HD void ec9_add(f29& r, const f29& a, const f29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] + b.v[i];
}
CG_HD void ec9_sub(f29& r, const f29& a, const f29& b) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = a.v[i] - b.v[i];
}
CG_HD void ec9_neg(f29& r, const f29& a) {
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = 0u - a.v[i];
}

// Column k's product terms (i + j = k, 0 <= i, j < 9) of a b (+ c d), added to acc. Sq: a b is a
// square, b = 2a (the caller's doubled copy): each pair i < j once as a_i (2 a_j), plus a_i^2 on
// the diagonal -- 45 MACs instead of 81 (|2 a_j| < 2^31 for every limb class of ec9.h).
template <bool Two, bool Sq>
CG_HD void ec9_col(ec9_acc& acc, int k, const f29& a, const f29& b, const f29& c, const f29& d) {
#pragma unroll
  for (int i = 0; i < 9; ++i) {
    const int j = k - i;
    if (j < 0 || j > 8) continue;
    if (Sq && i > j) continue;
    acc += Sq && i == j ? ec9_t(a.v[i], a.v[i]) : ec9_t(a.v[i], b.v[j]);
    ec9_opaque(acc);
    if (Two) {
      acc += ec9_t(c.v[i], d.v[j]);
      ec9_opaque(acc);
    }
  }
}

// ---------------------------------------------------------------- secp256r1: Montgomery
template <bool Two, bool Add, bool Sq = false>
CG_HD void ec9_mul_r1(f29& out, const f29& a0, const f29& b0, const f29& c0, const f29& d0, const f29& e) {
  constexpr uint32_t P7 = m29_limb(1, 0, 1, 7), P8 = m29_limb(1, 0, 1, 8);
  const uint32_t k9 = m29_opaque(1u << 9), k18 = m29_opaque(1u << 18);  // MACs, not shift pairs
#ifdef EC9_PIN_COPIES
  f29 a, b, c, d;
  ec9_pin(a, a0);
  ec9_pin(b, b0);
  if (Two) {
    ec9_pin(c, c0);
    ec9_pin(d, d0);
  }
#else
  const f29 &a = a0, &b = b0, &c = c0, &d = d0;
#endif
  uint32_t q[9];
  ec9_acc acc = 0;
#pragma unroll
  for (int k = 0; k < 17; ++k) {
    ec9_col<Two, Sq>(acc, k, a, b, c, d);
#pragma unroll
    for (int i = 0; i < 9; ++i) {  // q p = q (2^96 - 1 + 2^192 + p7 2^203 + p8 2^232) (mont29.h)
      const int j = k - i;
      if (!(i < k && j >= 0 && j < 9)) continue;
      if (j == 3) acc += ec9_t(q[i], k9);
      if (j == 6) acc += ec9_t(q[i], k18);
      if (j == 7) acc += ec9_t(q[i], P7);
      if (j == 8) acc += ec9_t(q[i], P8);
      if (j == 3 || j >= 6) ec9_opaque(acc);
    }
    if (Add && k >= 9) acc += (ec9_acc)(int32_t)e.v[k - 9];
    EC9_CHK(acc);
    if (k < 9) q[k] = (uint32_t)acc & M29_MASK;  // -p^-1 = 1 (mod 2^29): the -q term clears these bits
    else out.v[k - 9] = (uint32_t)acc & M29_MASK;
    acc >>= 29;  // arithmetic: floor
  }
  if (Add) acc += (ec9_acc)(int32_t)e.v[8];  // e's top limb joins the output's (column 17)
  FE_ASSERT(acc > -((ec9_acc)1 << 29) && acc < ((ec9_acc)1 << 29));
  out.v[8] = (uint32_t)(int32_t)acc;
}

// ---------------------------------------------------------------- secp256k1: plain form, folded
template <bool Two, bool Add, bool Sq = false>
CG_HD void ec9_mul_k1(f29& out, const f29& a0, const f29& b0, const f29& c0, const f29& d0, const f29& e) {
  const uint32_t k31264 = m29_opaque(31264u), k256 = m29_opaque(256u);
#ifdef EC9_PIN_COPIES
  f29 a, b, c, d;
  ec9_pin(a, a0);
  ec9_pin(b, b0);
  if (Two) {
    ec9_pin(c, c0);
    ec9_pin(d, d0);
  }
#else
  const f29 &a = a0, &b = b0, &c = c0, &d = d0;
#endif
#if !EC9_PIN_ACC
  ec9_acc col[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    ec9_acc s = Add ? (ec9_acc)(int32_t)e.v[k] : 0;
    ec9_col<Two, Sq>(s, k, a, b, c, d);
    col[k] = s;
  }
#endif
  uint32_t H[8];
  ec9_acc acc = 0;
#pragma unroll
  for (int k = 9; k < 17; ++k) {
    ec9_col<Two, Sq>(acc, k, a, b, c, d);
    EC9_CHK(acc);
    H[k - 9] = (uint32_t)acc & M29_MASK;
    acc >>= 29;
  }
  FE_ASSERT(acc > -((ec9_acc)1 << 31) && acc < ((ec9_acc)1 << 31));
  const uint32_t H8 = (uint32_t)(int32_t)acc;
  // H_m 2^{29 m} 2^261 = H_m 31264 (column m) + H_m 2^8 (column m + 1)
  uint32_t M[9];
#if EC9_PIN_ACC
  // the low columns after the high ones: one chain from the carry, the fold terms and e first
  acc = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    if (Add) acc += (ec9_acc)(int32_t)e.v[j];
    acc += ec9_t(j < 8 ? H[j] : H8, k31264);
    ec9_opaque(acc);
    if (j >= 1) {
      acc += ec9_t(H[j - 1], k256);
      ec9_opaque(acc);
    }
    ec9_col<Two, Sq>(acc, j, a, b, c, d);
    EC9_CHK(acc);
    M[j] = (uint32_t)acc & M29_MASK;
    acc >>= 29;
  }
#else
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    col[m] += ec9_t(H[m], k31264);
    col[m + 1] += ec9_t(H[m], k256);
  }
  col[8] += ec9_t(H8, k31264);
  acc = 0;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    acc += col[j];
    EC9_CHK(acc);
    M[j] = (uint32_t)acc & M29_MASK;
    acc >>= 29;
  }
#endif
  // top (weight 2^261) = acc + H8 2^8, folded as (2^37 + 31264) at its 32-bit halves
  const ec9_acc top = acc + (ec9_acc)(int32_t)H8 * 256;
  FE_ASSERT(top > -((ec9_acc)1 << 40) && top < ((ec9_acc)1 << 40));
  const uint32_t tlo = (uint32_t)(uint64_t)top;
  const int32_t thi = (int32_t)(top >> 32);
  const uint64_t x0 = (uint64_t)M[0] + (uint64_t)tlo * k31264;                 // tlo 31264
  const int64_t x1 = (int64_t)M[1] + (int64_t)((uint64_t)tlo * k256) +          // tlo 2^37
                     (int64_t)thi * 250112 + (int64_t)(x0 >> 29);               // thi 2^32 31264
  out.v[0] = (uint32_t)x0 & M29_MASK;
  out.v[1] = (uint32_t)x1 & M29_MASK;
  out.v[2] = M[2] + (uint32_t)(int32_t)(x1 >> 29) + (uint32_t)(thi * 2048);     // thi 2^69
#pragma unroll
  for (int i = 3; i < 9; ++i) out.v[i] = M[i];
}

template <int C>
CG_HD void ec9_mul(f29& out, const f29& a, const f29& b) {
  M29_COUNT(C, 0);
  if (C == CG_CURVE_R1) ec9_mul_r1<false, false>(out, a, b, a, b, a);
  else ec9_mul_k1<false, false>(out, a, b, a, b, a);
}
// a b + e (e limb-wise, |e_i| < 2^31)
template <int C>
CG_HD void ec9_mul_add(f29& out, const f29& a, const f29& b, const f29& e) {
  M29_COUNT(C, 0);
  if (C == CG_CURVE_R1) ec9_mul_r1<false, true>(out, a, b, a, b, e);
  else ec9_mul_k1<false, true>(out, a, b, a, b, e);
}
// a^2 (+ e): the pairs i < j once against a doubled copy (ec9_col)
template <int C, bool Add>
CG_HD void ec9_sqr_impl(f29& out, const f29& a, const f29& e) {
  M29_COUNT(C, 0);
  M29_COUNT_SQR(C);
  f29 a2;
#pragma unroll
  for (int i = 0; i < 9; ++i) a2.v[i] = a.v[i] << 1;
  if (C == CG_CURVE_R1) ec9_mul_r1<false, Add, true>(out, a, a2, a, a, e);
  else ec9_mul_k1<false, Add, true>(out, a, a2, a, a, e);
}
template <int C>
CG_HD void ec9_sqr(f29& out, const f29& a) {
#if EC9_SQR
  ec9_sqr_impl<C, false>(out, a, a);
#else
  ec9_mul<C>(out, a, a);
#endif
}
template <int C>
CG_HD void ec9_sqr_add(f29& out, const f29& a, const f29& e) {
#if EC9_SQR
  ec9_sqr_impl<C, true>(out, a, e);
#else
  ec9_mul_add<C>(out, a, a, e);
#endif
}
// a b + c d, one reduction
template <int C>
CG_HD void ec9_mul2(f29& out, const f29& a, const f29& b, const f29& c, const f29& d) {
  M29_COUNT(C, 0);
  M29_COUNT(C, 0);
  if (C == CG_CURVE_R1) ec9_mul_r1<true, false>(out, a, b, c, d, a);
  else ec9_mul_k1<true, false>(out, a, b, c, d, a);
}

// ---------------------------------------------------------------- back to mont29.h's reduced form
// signed limbs -> digits 0..7 in [0, 2^29) and a signed top (weight 2^232) in d8
CG_HD void ec9_carry(int64_t d[9], const f29& a) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += (int32_t)a.v[i];
    d[i] = c & M29_MASK;
    c >>= 29;
  }
  d[8] = c + (int32_t)a.v[8];
}
CG_HD void ec9_carry64(int64_t d[9]) {
  int64_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    c += d[i];
    d[i] = c & M29_MASK;
    c >>= 29;
  }
  d[8] += c;
}
// any value of the ladder (|v| < 2^262) -> reduced (normalized limbs, value in [0, 2m)), the same
// residue mod p
template <int C>
CG_HD void ec9_to_m29(f29& r, const f29& a) {
  int64_t d[9];
  ec9_carry(d, a);
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    // bits >= 256: t = d8 >> 24 (signed), 2^256 = 2^32 + 977 (k1) or 2^224 - 2^192 - 2^96 + 1 (r1)
    const int64_t t = d[8] >> 24;
    d[8] -= t * (1 << 24);
    if (C == CG_CURVE_R1) {
      d[0] += t;
      d[3] -= t * (1 << 9);
      d[6] -= t * (1 << 18);
      d[7] += t * (1 << 21);
    } else {
      d[0] += t * 977;
      d[1] += t * 8;
    }
    ec9_carry64(d);
  }
  // now -small <= v < 2^256 + small: add 2m when negative (d8 < 0), then v in [0, 2m)
  if (d[8] < 0) {
#pragma unroll
    for (int i = 0; i < 9; ++i) d[i] += m29_limb(C, 0, 2, i);
    ec9_carry64(d);
  }
  FE_ASSERT(d[8] >= 0 && d[8] < (1 << 29));
#pragma unroll
  for (int i = 0; i < 9; ++i) r.v[i] = (uint32_t)d[i];
  m29_csub<C, 0, 2>(r, r);  // < 2m (v < 2^256 + small can exceed 2m only for k1 never; cheap)
}

// Can H be 0 mod p? A filter on the value's low 29 bits (= limb 0's): |H| < 64 p, so H = k p with
// |k| <= 64 and H mod 2^29 = k p mod 2^29: -k (r1, p = -1 mod 2^29) or -977 k (k1). False
// positives ~2^-24 (k1) / ~2^-25 (r1) per lane; ec9_to_m29 + m29_iszero decide.
template <int C>
CG_HD bool ec9_maybe_zero(const f29& a) {
  const uint32_t x = (0u - a.v[0]) & M29_MASK;
  if (C == CG_CURVE_R1) return ((x + 64u) & M29_MASK) <= 128u;
  return x <= 977u * 64u || x >= (1u << 29) - 977u * 64u;
}

// ---------------------------------------------------------------- the wide ladder's addition
// R += (-1)^neg (x2, y2), madd-2004-hmv as jac_madd_w (ecdsa.h), in the signed-limb form: R's
// coordinates are tight (or reduced) values, (x2, y2) a reduced table entry. H = 0 mod p (doubling,
// or P + (-P): adversarial inputs only) and the filter's false positives take jac_madd_w's exact path
// on the reduced form.
template <int C>
CG_HD void jac_madd9(Jac& r, bool& inf, const f29& x2, const f29& y2, bool neg, const EcConsts& K) {
  if (inf) {
    jac_madd_w<C>(r, inf, x2, y2, neg, K);  // R = (x2, +-y2, 1), reduced
    return;
  }
  f29 Z1Z1, U2, ys, S2, H;
  ec9_sqr<C>(Z1Z1, r.Z);
  ec9_mul<C>(U2, x2, Z1Z1);
#if EC9_SIGN_MUL
  // S2 = +-y2 Z1^3: each limb times an opaque +-1 (one v_mul_lo_u32 a limb, as fe9.h's
  // fe9_sign_mask) instead of a negation and a select (two)
  uint32_t sg = neg ? ~0u : 1u;
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("" : "+v"(sg));
#endif
#pragma unroll
  for (int i = 0; i < 9; ++i) ys.v[i] = y2.v[i] * sg;
#else
#pragma unroll
  for (int i = 0; i < 9; ++i) ys.v[i] = neg ? 0u - y2.v[i] : y2.v[i];  // S2 = +-y2 Z1^3
#endif
  ec9_mul<C>(S2, ys, r.Z);
  ec9_mul<C>(S2, S2, Z1Z1);
  ec9_sub(H, U2, r.X);
#ifndef EC9_NO_EXACT  // (defined only by the instruction-count probe: the exact path compiled out)
  if (ec9_maybe_zero<C>(H)) {
    Jac q;
    ec9_to_m29<C>(q.X, r.X);
    ec9_to_m29<C>(q.Y, r.Y);
    ec9_to_m29<C>(q.Z, r.Z);
    jac_madd_w<C>(q, inf, x2, y2, neg, K);
    r = q;
    return;
  }
#endif
  f29 rr, HH, HHH, V, E, t, nY;
  ec9_sub(rr, S2, r.Y);
  ec9_sqr<C>(HH, H);
  ec9_mul<C>(HHH, H, HH);
  ec9_mul<C>(V, r.X, HH);
#pragma unroll
  for (int i = 0; i < 9; ++i) E.v[i] = 0u - HHH.v[i] - 2u * V.v[i];  // X3 = rr^2 - HHH - 2V
  Jac o;
  ec9_sqr_add<C>(o.X, rr, E);
  ec9_sub(t, V, o.X);
  ec9_neg(nY, r.Y);
  ec9_mul2<C>(o.Y, rr, t, nY, HHH);  // Y3 = rr (V - X3) - Y1 HHH
  ec9_mul<C>(o.Z, r.Z, H);
  r = o;
}
