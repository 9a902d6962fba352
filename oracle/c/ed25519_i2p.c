/* C restatement of Ed25519 verification as net.i2p.crypto:eddsa:0.2.0 performs it.
 * TEST INFRASTRUCTURE ONLY (oracle / CPU "port" baseline).
 *
 * Called by the reference at core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559
 * (scheme EDDSA_ED25519_SHA512, Crypto.kt:120-133). The loop structure, point
 * representations (P2/P3/P1P1/PRECOMP/CACHED) and tables follow i2p's GroupElement so the
 * field-operation counts (or_counters) are the reference's algorithmic work:
 *   EdDSAPublicKeySpec(A): GroupElement(curve, A) decode; Aneg = A.negate();
 *                          Aneg.precompute(false) -> 8 odd multiples as PRECOMP, one
 *                          inversion each                                  (per key)
 *   EdDSAEngine.engineVerify: len check; h = SHA-512(R||Abyte||M) mod L; slide(h),
 *                          slide(S); 256-step Shamir loop (dbl, madd/msub); toByteArray;
 *                          32-byte compare                                 (per signature)
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "bn.h"
#include "oracle.h"

static mont_ctx FP, SL; /* field p = 2^255-19 ; scalar L */
static u256 FE_D, FE_D2, FE_SQRTM1, FE_ONE, FE_ZERO;
static int g_init = 0;

typedef struct { u256 X, Y, Z; } ge_p2;
typedef struct { u256 X, Y, Z, T; } ge_p3;
typedef struct { u256 X, Y, Z, T; } ge_p1p1;
typedef struct { u256 yplusx, yminusx, xy2d; } ge_precomp;
typedef struct { u256 YplusX, YminusX, Z, T2d; } ge_cached;

struct or_ed_key {
  ge_p3 A;
  uint8_t abyte[32];
  ge_precomp negA_tab[8]; /* (2i+1) * (-A), i2p dblPrecmp */
};

static ge_precomp B_TAB[8];

size_t or_ed_key_size(void) { return sizeof(or_ed_key); }
const uint8_t* or_ed_key_abyte(const or_ed_key* k) { return k->abyte; }

/* ---- field helpers (Montgomery domain) ---- */
#define fmul(r, a, b) mont_mul(&FP, r, a, b)
#define fsq(r, a) mont_sq(&FP, r, a)
#define fadd(r, a, b) mont_add(&FP, r, a, b)
#define fsub(r, a, b) mont_sub(&FP, r, a, b)

static void fe_frombytes(u256* r, const uint8_t s[32]) {
  /* Ed25519FieldElement.fromByteArray: bit 255 masked, value may be >= p (reduced mod p) */
  uint8_t b[32];
  memcpy(b, s, 32);
  b[31] &= 0x7f;
  u256 x;
  u256_from_le(&x, b);
  u256_mod(&FP, &x, &x);
  mont_to(&FP, r, &x);
}
static void fe_tobytes(uint8_t s[32], const u256* a) {
  u256 x;
  mont_from(&FP, &x, a);
  u256_to_le(s, &x);
}
static int fe_isneg(const u256* a) {
  uint8_t s[32];
  fe_tobytes(s, a);
  return s[0] & 1;
}
static int fe_iszero(const u256* a) { return u256_is_zero(a); }
static void fe_invert(u256* r, const u256* a) { mont_inv(&FP, r, a); }
static void fe_pow22523(u256* r, const u256* a) {
  /* a^((p-5)/8) */
  u256 e;
  /* (p-5)/8 = 2^252 - 3 */
  e.v[0] = 0xFFFFFFFFFFFFFFFDULL; e.v[1] = ~0ULL; e.v[2] = ~0ULL; e.v[3] = 0x0FFFFFFFFFFFFFFFULL;
  mont_pow(&FP, r, a, &e);
}

/* ---- group ops (ref10 / i2p GroupElement formulas) ---- */
static void p1p1_to_p2(ge_p2* r, const ge_p1p1* p) {
  fmul(&r->X, &p->X, &p->T);
  fmul(&r->Y, &p->Y, &p->Z);
  fmul(&r->Z, &p->Z, &p->T);
}
static void p1p1_to_p3(ge_p3* r, const ge_p1p1* p) {
  fmul(&r->X, &p->X, &p->T);
  fmul(&r->Y, &p->Y, &p->Z);
  fmul(&r->Z, &p->Z, &p->T);
  fmul(&r->T, &p->X, &p->Y);
}
static void p2_dbl(ge_p1p1* r, const ge_p2* p) {
  u256 t0;
  fsq(&r->X, &p->X);
  fsq(&r->Z, &p->Y);
  fsq(&r->T, &p->Z);
  fadd(&r->T, &r->T, &r->T);
  fadd(&r->Y, &p->X, &p->Y);
  fsq(&t0, &r->Y);
  fadd(&r->Y, &r->Z, &r->X);
  fsub(&r->Z, &r->Z, &r->X);
  fsub(&r->X, &t0, &r->Y);
  fsub(&r->T, &r->T, &r->Z);
}
static void p3_to_p2(ge_p2* r, const ge_p3* p) { r->X = p->X; r->Y = p->Y; r->Z = p->Z; }
static void p3_to_cached(ge_cached* r, const ge_p3* p) {
  fadd(&r->YplusX, &p->Y, &p->X);
  fsub(&r->YminusX, &p->Y, &p->X);
  r->Z = p->Z;
  fmul(&r->T2d, &p->T, &FE_D2);
}
static void ge_add(ge_p1p1* r, const ge_p3* p, const ge_cached* q) {
  u256 t0;
  fadd(&r->X, &p->Y, &p->X);
  fsub(&r->Y, &p->Y, &p->X);
  fmul(&r->Z, &r->X, &q->YplusX);
  fmul(&r->Y, &r->Y, &q->YminusX);
  fmul(&r->T, &q->T2d, &p->T);
  fmul(&r->X, &p->Z, &q->Z);
  fadd(&t0, &r->X, &r->X);
  fsub(&r->X, &r->Z, &r->Y);
  fadd(&r->Y, &r->Z, &r->Y);
  fadd(&r->Z, &t0, &r->T);
  fsub(&r->T, &t0, &r->T);
}
static void ge_sub(ge_p1p1* r, const ge_p3* p, const ge_cached* q) {
  u256 t0;
  fadd(&r->X, &p->Y, &p->X);
  fsub(&r->Y, &p->Y, &p->X);
  fmul(&r->Z, &r->X, &q->YminusX);
  fmul(&r->Y, &r->Y, &q->YplusX);
  fmul(&r->T, &q->T2d, &p->T);
  fmul(&r->X, &p->Z, &q->Z);
  fadd(&t0, &r->X, &r->X);
  fsub(&r->X, &r->Z, &r->Y);
  fadd(&r->Y, &r->Z, &r->Y);
  fsub(&r->Z, &t0, &r->T);
  fadd(&r->T, &t0, &r->T);
}
static void ge_madd(ge_p1p1* r, const ge_p3* p, const ge_precomp* q) {
  u256 t0;
  fadd(&r->X, &p->Y, &p->X);
  fsub(&r->Y, &p->Y, &p->X);
  fmul(&r->Z, &r->X, &q->yplusx);
  fmul(&r->Y, &r->Y, &q->yminusx);
  fmul(&r->T, &q->xy2d, &p->T);
  fadd(&t0, &p->Z, &p->Z);
  fsub(&r->X, &r->Z, &r->Y);
  fadd(&r->Y, &r->Z, &r->Y);
  fadd(&r->Z, &t0, &r->T);
  fsub(&r->T, &t0, &r->T);
}
static void ge_msub(ge_p1p1* r, const ge_p3* p, const ge_precomp* q) {
  u256 t0;
  fadd(&r->X, &p->Y, &p->X);
  fsub(&r->Y, &p->Y, &p->X);
  fmul(&r->Z, &r->X, &q->yminusx);
  fmul(&r->Y, &r->Y, &q->yplusx);
  fmul(&r->T, &q->xy2d, &p->T);
  fadd(&t0, &p->Z, &p->Z);
  fsub(&r->X, &r->Z, &r->Y);
  fadd(&r->Y, &r->Z, &r->Y);
  fsub(&r->Z, &t0, &r->T);
  fadd(&r->T, &t0, &r->T);
}

/* GroupElement.precompute(false): odd multiples P, 3P, ..., 15P as affine PRECOMP */
static void precompute_dbl(ge_precomp tab[8], const ge_p3* P) {
  ge_p3 Bi = *P;
  ge_cached c;
  ge_p1p1 t;
  ge_p3 t3;
  for (int i = 0; i < 8; ++i) {
    u256 recip, x, y, xy;
    fe_invert(&recip, &Bi.Z);
    fmul(&x, &Bi.X, &recip);
    fmul(&y, &Bi.Y, &recip);
    fadd(&tab[i].yplusx, &y, &x);
    fsub(&tab[i].yminusx, &y, &x);
    fmul(&xy, &x, &y);
    fmul(&tab[i].xy2d, &xy, &FE_D2);
    /* Bi = P + (P + Bi) */
    p3_to_cached(&c, &Bi);
    ge_add(&t, P, &c);
    p1p1_to_p3(&t3, &t);
    p3_to_cached(&c, &t3);
    ge_add(&t, P, &c);
    p1p1_to_p3(&Bi, &t);
  }
}

/* GroupElement(curve, bytes): returns 0 or CG_KEY_INVALID */
static int ge_frombytes(ge_p3* h, const uint8_t s[32]) {
  u256 u, v, v3, vxx, check, x, y, yy;
  fe_frombytes(&y, s);
  fsq(&yy, &y);
  fsub(&u, &yy, &FE_ONE);
  fmul(&v, &yy, &FE_D);
  fadd(&v, &v, &FE_ONE);
  fsq(&v3, &v);
  fmul(&v3, &v3, &v);
  fsq(&x, &v3);
  fmul(&x, &x, &v);
  fmul(&x, &x, &u);
  fe_pow22523(&x, &x);
  fmul(&x, &x, &v3);
  fmul(&x, &x, &u);
  fsq(&vxx, &x);
  fmul(&vxx, &vxx, &v);
  fsub(&check, &vxx, &u);
  if (!fe_iszero(&check)) {
    fadd(&check, &vxx, &u);
    if (!fe_iszero(&check)) return CG_KEY_INVALID;
    fmul(&x, &x, &FE_SQRTM1);
  }
  if (fe_isneg(&x) != (s[31] >> 7)) mont_neg(&FP, &x, &x);
  h->X = x;
  h->Y = y;
  h->Z = FE_ONE;
  fmul(&h->T, &x, &y);
  return 0;
}

static void ge_tobytes(uint8_t s[32], const u256* X, const u256* Y, const u256* Z) {
  u256 recip, x, y;
  fe_invert(&recip, Z);
  fmul(&x, X, &recip);
  fmul(&y, Y, &recip);
  fe_tobytes(s, &y);
  s[31] |= (uint8_t)(fe_isneg(&x) << 7);
}

/* GroupElement.slide restated literally */
static void slide(signed char r[256], const uint8_t a[32]) {
  for (int i = 0; i < 256; ++i) r[i] = 1 & (a[i >> 3] >> (i & 7));
  for (int i = 0; i < 256; ++i) {
    if (!r[i]) continue;
    for (int b = 1; b <= 6 && i + b < 256; ++b) {
      if (!r[i + b]) continue;
      if (r[i] + (r[i + b] << b) <= 15) {
        r[i] += r[i + b] << b;
        r[i + b] = 0;
      } else if (r[i] - (r[i + b] << b) >= -15) {
        r[i] -= r[i + b] << b;
        for (int k = i + b; k < 256; ++k) {
          if (!r[k]) { r[k] = 1; break; }
          r[k] = 0;
        }
      } else {
        break;
      }
    }
  }
}

int or_ed_slide_escapes(const uint8_t s[32]) {
  /* the carry escaped iff sum r_i 2^i (signed) is negative, i.e. the top nonzero digit < 0 */
  signed char r[256];
  slide(r, s);
  for (int i = 255; i >= 0; --i)
    if (r[i]) return r[i] < 0;
  return 0;
}

static void ed_init(void) {
  if (g_init) return;
  u256 p = {{0xFFFFFFFFFFFFFFEDULL, ~0ULL, ~0ULL, 0x7FFFFFFFFFFFFFFFULL}};
  u256 l = {{0x5812631A5CF5D3EDULL, 0x14DEF9DEA2F79CD6ULL, 0ULL, 0x1000000000000000ULL}};
  mont_init(&FP, &p);
  mont_init(&SL, &l);
  u256 one = {{1, 0, 0, 0}}, t;
  mont_to(&FP, &FE_ONE, &one);
  memset(&FE_ZERO, 0, sizeof FE_ZERO);
  /* d = -121665/121666 */
  u256 a, b;
  u256_set_u64(&t, 121665); mont_to(&FP, &a, &t);
  u256_set_u64(&t, 121666); mont_to(&FP, &b, &t);
  mont_inv(&FP, &b, &b);
  mont_mul(&FP, &FE_D, &a, &b);
  mont_neg(&FP, &FE_D, &FE_D);
  mont_add(&FP, &FE_D2, &FE_D, &FE_D);
  /* sqrt(-1) = 2^((p-1)/4) */
  u256 e = {{0xFFFFFFFFFFFFFFFBULL, ~0ULL, ~0ULL, 0x1FFFFFFFFFFFFFFFULL}};
  u256_set_u64(&t, 2); mont_to(&FP, &a, &t);
  mont_pow(&FP, &FE_SQRTM1, &a, &e);
  /* base point: y = 4/5, x even */
  uint8_t by[32];
  u256_set_u64(&t, 4); mont_to(&FP, &a, &t);
  u256_set_u64(&t, 5); mont_to(&FP, &b, &t);
  mont_inv(&FP, &b, &b);
  mont_mul(&FP, &a, &a, &b);
  fe_tobytes(by, &a);
  ge_p3 B;
  ge_frombytes(&B, by);
  precompute_dbl(B_TAB, &B);
  g_init = 1;
}

static pthread_once_t g_once = PTHREAD_ONCE_INIT;
static void ensure_init(void) { pthread_once(&g_once, ed_init); }

int or_ed_key_decode(or_ed_key* k, const uint8_t a[32]) {
  ensure_init();
  if (ge_frombytes(&k->A, a)) return CG_KEY_INVALID;
  ge_tobytes(k->abyte, &k->A.X, &k->A.Y, &k->A.Z);
  /* Aneg = A.negate() = zero.sub(A.toCached()).toP3() ; Aneg.precompute(false) */
  ge_p3 zero = {FE_ZERO, FE_ONE, FE_ONE, FE_ZERO};
  ge_cached c;
  ge_p1p1 t;
  ge_p3 neg;
  p3_to_cached(&c, &k->A);
  ge_sub(&t, &zero, &c);
  p1p1_to_p3(&neg, &t);
  precompute_dbl(k->negA_tab, &neg);
  return 0;
}

int or_ed_verify(const or_ed_key* k, const uint8_t* msg, size_t msg_len, const uint8_t* sig, size_t sig_len) {
  ensure_init();
  if (sig_len != 64) return CG_SIG_MALFORMED;
  uint8_t hbuf[64];
  or_sha512_ctx sc;
  or_sha512_init(&sc);
  or_sha512_update(&sc, sig, 32);
  or_sha512_update(&sc, k->abyte, 32);
  or_sha512_update(&sc, msg, msg_len);
  or_sha512_final(&sc, hbuf);
  u256 h;
  u512_mod(&SL, &h, hbuf); /* Ed25519ScalarOps.reduce */
  uint8_t hb[32];
  u256_to_le(hb, &h);
  signed char aslide[256], bslide[256];
  slide(aslide, hb);
  slide(bslide, sig + 32);
  int i;
  for (i = 255; i >= 0; --i)
    if (aslide[i] || bslide[i]) break;
  ge_p2 r = {FE_ZERO, FE_ONE, FE_ONE};
  ge_p1p1 t;
  ge_p3 u;
  for (; i >= 0; --i) {
    p2_dbl(&t, &r);
    if (aslide[i] > 0) {
      p1p1_to_p3(&u, &t);
      ge_madd(&t, &u, &k->negA_tab[aslide[i] / 2]);
    } else if (aslide[i] < 0) {
      p1p1_to_p3(&u, &t);
      ge_msub(&t, &u, &k->negA_tab[(-aslide[i]) / 2]);
    }
    if (bslide[i] > 0) {
      p1p1_to_p3(&u, &t);
      ge_madd(&t, &u, &B_TAB[bslide[i] / 2]);
    } else if (bslide[i] < 0) {
      p1p1_to_p3(&u, &t);
      ge_msub(&t, &u, &B_TAB[(-bslide[i]) / 2]);
    }
    p1p1_to_p2(&r, &t);
  }
  uint8_t rcalc[32];
  ge_tobytes(rcalc, &r.X, &r.Y, &r.Z);
  return memcmp(rcalc, sig, 32) == 0 ? CG_VALID : CG_INVALID;
}
