// Edwards25519 group operations (twisted Edwards, a = -1) for one point per lane.
//
// Extended coordinates (Hisil-Wong-Carter-Dawson 2008); the completed "P1P1" form and the
// cached/niels operand forms are the usual ones. All addition formulas used are the
// unified ones, which are complete on edwards25519 (d non-square), so small-order and
// mixed-order public keys (class A9) need no special cases.
//
// Bounds (fe25519.h): every P1P1 producer leaves X <= 5 tight and Y, Z, T <= 3 tight, so
// p1p1_to_p2/p3 may feed (X, Y, Z, T) as the f operand and (T, Z, T, Y) as the g operand.
#pragma once
#include "fe25519.h"

struct ge_p2 {
  fe X, Y, Z;
};
struct ge_p3 {
  fe X, Y, Z, T;
};
struct ge_p1p1 {
  fe X, Y, Z, T;
};
struct ge_cached {  // (Y+X, Y-X, Z, 2dT), all tight
  fe YpX, YmX, Z, T2d;
};
struct ge_niels {  // affine (y+x, y-x, 2dxy), all tight
  fe ypx, ymx, xy2d;
};

// Operand order shares work between the products: fe_mul(f, g) scales g by 19 and doubles
// f's odd limbs, so Y = Z * Y and Z = Z * T share f = Z, and X = X * T shares g = T with it.
CG_HD void ge_p1p1_to_p2(ge_p2& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
}

// (shared operands: g = T for X and Z, g = Y for Y and T, f = X for X and T, f = Z for Y and Z)
CG_HD void ge_p1p1_to_p3(ge_p3& r, const ge_p1p1& p) {
  fe_mul(r.X, p.X, p.T);
  fe_mul(r.Y, p.Z, p.Y);
  fe_mul(r.Z, p.Z, p.T);
  fe_mul(r.T, p.X, p.Y);
}

CG_HD void ge_p3_to_p2(ge_p2& r, const ge_p3& p) {
  fe_copy(r.X, p.X);
  fe_copy(r.Y, p.Y);
  fe_copy(r.Z, p.Z);
}

// r = 2p.  XX=X^2, YY=Y^2, B=2Z^2, AA=(X+Y)^2; X3=AA-(YY+XX), Y3=YY+XX, Z3=YY-XX, T3=B-Z3
CG_HD void ge_p2_dbl(ge_p1p1& r, const ge_p2& p) {
  fe xx, a, aa;
  fe_sq(xx, p.X);
  fe_sq(r.Z, p.Y);     // YY
  fe_sq2(r.T, p.Z);    // 2 Z^2 (tight)
  fe_add(a, p.X, p.Y); // 2T
  fe_sq(aa, a);
  fe_add(r.Y, r.Z, xx);  // YY + XX  (2T)
  fe_sub(r.Z, r.Z, xx);  // YY - XX  (3T)
  fe_sub4(r.X, aa, r.Y); // 5T
  fe_sub4(r.T, r.T, r.Z);
  fe_carry(r.T);         // tight
}

CG_HD void ge_p3_dbl(ge_p1p1& r, const ge_p3& p) {
  ge_p2 q;
  ge_p3_to_p2(q, p);
  ge_p2_dbl(r, q);
}

// r = p + q (q cached); sign != 0 adds -q instead
CG_HD void ge_add_cached(ge_p1p1& r, const ge_p3& p, const ge_cached& q) {
  fe a, b, c, d;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul(r.X, a, q.YpX);   // A
  fe_mul(r.Y, b, q.YmX);   // B
  fe_mul(c, q.T2d, p.T);   // C
  fe_mul(d, p.Z, q.Z);
  fe_add(d, d, d);         // D = 2 Z1 Z2 (2T)
  fe_sub(r.Z, r.X, r.Y);   // tmp: A - B (3T)
  fe_add(r.Y, r.X, r.Y);   // A + B (2T)
  fe_copy(r.X, r.Z);       // X3 = A - B
  fe_add(r.Z, d, c);       // Z3 = D + C (3T)
  fe_sub(r.T, d, c);       // T3 = D - C (4T)
  fe_carry(r.T);
}

// r = p + q (q niels, affine)
CG_HD void ge_madd(ge_p1p1& r, const ge_p3& p, const ge_niels& q) {
  fe a, b, c, d;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
  fe_mul(r.X, a, q.ypx);
  fe_mul(r.Y, b, q.ymx);
  fe_mul(c, q.xy2d, p.T);
  fe_add(d, p.Z, p.Z);
  fe_sub(r.Z, r.X, r.Y);
  fe_add(r.Y, r.X, r.Y);
  fe_copy(r.X, r.Z);
  fe_add(r.Z, d, c);
  fe_sub(r.T, d, c);
  fe_carry(r.T);
}

// r = p + (-1)^neg q for an affine niels q, without negating q (ge_niels_cneg costs a negation,
// a carry pass and 30 swaps). With neg, a = Y+X and b = Y-X trade multiplicands, which
// leaves (Y'-X', X'+Y') for the negated sum's (X'-Y', X'+Y'); the sign goes to Z instead
// (x = X/Z), and the xy2d product's sign flips Z and T:
//   neg = 0: (X'-Y', X'+Y', d + c, d - c)     neg = 1: (Y'-X' = -(X'-Y'), X'+Y', c - d, d + c)
// Bounds: Z <= 5 tight (c + 4p - d), so the next product must take Z as its first operand
// (ge_p1p1_to_p2 / _p3 do); T is carried (tight).
CG_HD void ge_madd_signed(ge_p1p1& r, const ge_p3& p, const ge_niels& q, bool neg) {
  fe a, b, c, d;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t ai = a.v[i], bi = b.v[i];
    a.v[i] = neg ? bi : ai;
    b.v[i] = neg ? ai : bi;
  }
  fe_mul(r.X, a, q.ypx);
  fe_mul(r.Y, b, q.ymx);
  fe_mul(c, q.xy2d, p.T);
  fe_add(d, p.Z, p.Z);
  fe_sub(r.Z, r.X, r.Y);
  fe_add(r.Y, r.X, r.Y);
  fe_copy(r.X, r.Z);
  fe s, e, ne;
  fe_add(s, d, c);
  fe_sub(e, d, c);
  fe_sub4(ne, c, d);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.Z.v[i] = neg ? ne.v[i] : s.v[i];
    r.T.v[i] = neg ? s.v[i] : e.v[i];
  }
  fe_carry(r.T);
}

// ge_madd_signed for a half-scaled niels entry q = ((y+x)/2, (y-x)/2, x y d) (the wide tables):
// the sum comes out as ge_madd_signed's divided by 2, so D = Z instead of 2Z, and with Z and T of
// p tight every output stays <= 3 tight: no doubling of Z, no sub4, no carry pass.
//   neg = 0: (X'-Y', X'+Y', Z + c, Z - c)     neg = 1: (Y'-X', X'+Y', c - Z, Z + c)
CG_HD void ge_madd_half_signed(ge_p1p1& r, const ge_p3& p, const ge_niels& q, bool neg) {
  fe a, b, c;
  fe_add(a, p.Y, p.X);
  fe_sub(b, p.Y, p.X);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t ai = a.v[i], bi = b.v[i];
    a.v[i] = neg ? bi : ai;
    b.v[i] = neg ? ai : bi;
  }
  fe_mul(r.X, a, q.ypx);
  fe_mul(r.Y, b, q.ymx);
  fe_mul(c, q.xy2d, p.T);
  fe_sub(r.Z, r.X, r.Y);
  fe_add(r.Y, r.X, r.Y);
  fe_copy(r.X, r.Z);
  fe s, e, ne;
  fe_add(s, p.Z, c);
  fe_sub(e, p.Z, c);
  fe_sub(ne, c, p.Z);
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    r.Z.v[i] = neg ? ne.v[i] : s.v[i];
    r.T.v[i] = neg ? s.v[i] : e.v[i];
  }
}

// Conditionally negate a cached point in place: (YpX, YmX, Z, T2d) -> (YmX, YpX, Z, -T2d)
CG_HD void ge_cached_cneg(ge_cached& q, uint32_t neg) {
  fe t;
  fe_neg(t, q.T2d);
  fe_carry(t);
  const uint32_t m = 0u - neg;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t x = (q.YpX.v[i] ^ q.YmX.v[i]) & m;
    q.YpX.v[i] ^= x;
    q.YmX.v[i] ^= x;
    q.T2d.v[i] ^= (q.T2d.v[i] ^ t.v[i]) & m;
  }
}

CG_HD void ge_niels_cneg(ge_niels& q, uint32_t neg) {
  fe t;
  fe_neg(t, q.xy2d);
  fe_carry(t);
  const uint32_t m = 0u - neg;
#pragma unroll
  for (int i = 0; i < 10; ++i) {
    const uint32_t x = (q.ypx.v[i] ^ q.ymx.v[i]) & m;
    q.ypx.v[i] ^= x;
    q.ymx.v[i] ^= x;
    q.xy2d.v[i] ^= (q.xy2d.v[i] ^ t.v[i]) & m;
  }
}

CG_HD void ge_p3_0(ge_p3& h) {
  fe_0(h.X);
  fe_1(h.Y);
  fe_1(h.Z);
  fe_0(h.T);
}

CG_HD void ge_p3_to_cached(ge_cached& r, const ge_p3& p, const fe& d2) {
  fe_add(r.YpX, p.Y, p.X);
  fe_carry(r.YpX);
  fe_sub(r.YmX, p.Y, p.X);
  fe_carry(r.YmX);
  fe_copy(r.Z, p.Z);
  fe_mul(r.T2d, p.T, d2);
}
