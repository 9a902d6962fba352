/* C restatement of SHA256withECDSA verification as BouncyCastle 1.57 performs it.
 * TEST INFRASTRUCTURE ONLY (oracle / CPU "port" baseline).
 *
 * Called by the reference at core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559
 * for ECDSA_SECP256K1_SHA256 (Crypto.kt:92-103) and ECDSA_SECP256R1_SHA256 (Crypto.kt:106-117).
 *   DSABase.engineVerify      hash = SHA-256(M); decode (strict DER) else SignatureException
 *   ECDSASigner.verifySignature  r,s in [1,n-1]; c = s^-1; u1 = e c; u2 = r c;
 *                             R = ECAlgorithms.sumOfTwoMultiplies(G, u1, Q, u2)
 *                             (implShamirsTrickWNaf, WNafUtil window 5 for 256-bit scalars,
 *                              affine-normalised odd-multiple tables, Jacobian accumulator);
 *                             R = infinity -> false; accept iff r*Z^2 == X or (r+n)*Z^2 == X
 *                             while r+n < p (BC's inversion-free x == r mod n test).
 *   Q decode                  coordinates < p and on the curve, else KEY_INVALID.
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "bn.h"
#include "oracle.h"

typedef struct {
  mont_ctx fp, fn;
  u256 a, b;       /* Montgomery form */
  int a_is_m3;     /* a == -3 */
  u256 gx, gy;     /* Montgomery form */
  u256 n_plain, p_plain;
} curve_t;

typedef struct { u256 x, y; } aff_t;               /* Montgomery form */
typedef struct { u256 X, Y, Z; int inf; } jac_t;

struct or_ec_key {
  int scheme;
  aff_t Q;
  aff_t tab[8]; /* odd multiples 1..15 of Q (affine) — BC WNafPreCompInfo for the key's point */
};

static curve_t C_K1, C_R1;
static aff_t G_TAB_K1[8], G_TAB_R1[8];
static pthread_once_t g_once = PTHREAD_ONCE_INIT;

size_t or_ec_key_size(void) { return sizeof(or_ec_key); }

static void hex_to_u256(u256* r, const char* hex) {
  uint8_t b[32];
  for (int i = 0; i < 32; ++i) {
    unsigned v;
    char t[3] = {hex[2 * i], hex[2 * i + 1], 0};
    v = (unsigned)strtoul(t, 0, 16);
    b[i] = (uint8_t)v;
  }
  u256_from_be(r, b);
}

static void jac_dbl(const curve_t* c, jac_t* r, const jac_t* p) {
  if (p->inf || u256_is_zero(&p->Y)) { r->inf = 1; return; }
  const mont_ctx* f = &c->fp;
  u256 t1, t2, t3, t4, X3, Y3, Z3;
  if (c->a_is_m3) {
    u256 delta, gamma, beta, alpha;
    mont_sq(f, &delta, &p->Z);
    mont_sq(f, &gamma, &p->Y);
    mont_mul(f, &beta, &p->X, &gamma);
    mont_sub(f, &t1, &p->X, &delta);
    mont_add(f, &t2, &p->X, &delta);
    mont_mul(f, &alpha, &t1, &t2);
    mont_add(f, &t1, &alpha, &alpha);
    mont_add(f, &alpha, &alpha, &t1);              /* alpha = 3 (X - d)(X + d) */
    mont_sq(f, &X3, &alpha);
    mont_add(f, &t1, &beta, &beta);
    mont_add(f, &t1, &t1, &t1);                    /* 4 beta */
    mont_add(f, &t2, &t1, &t1);                    /* 8 beta */
    mont_sub(f, &X3, &X3, &t2);
    mont_add(f, &t3, &p->Y, &p->Z);
    mont_sq(f, &Z3, &t3);
    mont_sub(f, &Z3, &Z3, &gamma);
    mont_sub(f, &Z3, &Z3, &delta);
    mont_sub(f, &t1, &t1, &X3);
    mont_mul(f, &Y3, &alpha, &t1);
    mont_sq(f, &t4, &gamma);
    mont_add(f, &t4, &t4, &t4);
    mont_add(f, &t4, &t4, &t4);
    mont_add(f, &t4, &t4, &t4);                    /* 8 gamma^2 */
    mont_sub(f, &Y3, &Y3, &t4);
  } else { /* a = 0 */
    u256 A, B, Cc, D, E, F;
    mont_sq(f, &A, &p->X);
    mont_sq(f, &B, &p->Y);
    mont_sq(f, &Cc, &B);
    mont_add(f, &t1, &p->X, &B);
    mont_sq(f, &t1, &t1);
    mont_sub(f, &t1, &t1, &A);
    mont_sub(f, &t1, &t1, &Cc);
    mont_add(f, &D, &t1, &t1);
    mont_add(f, &E, &A, &A);
    mont_add(f, &E, &E, &A);
    mont_sq(f, &F, &E);
    mont_add(f, &t2, &D, &D);
    mont_sub(f, &X3, &F, &t2);
    mont_sub(f, &t3, &D, &X3);
    mont_mul(f, &Y3, &E, &t3);
    mont_add(f, &t4, &Cc, &Cc);
    mont_add(f, &t4, &t4, &t4);
    mont_add(f, &t4, &t4, &t4);
    mont_sub(f, &Y3, &Y3, &t4);
    mont_mul(f, &Z3, &p->Y, &p->Z);
    mont_add(f, &Z3, &Z3, &Z3);
  }
  r->X = X3; r->Y = Y3; r->Z = Z3; r->inf = 0;
}

/* r = p + (x2, y2) (affine), exception-complete */
static void jac_add_aff(const curve_t* c, jac_t* r, const jac_t* p, const aff_t* q, int negate) {
  const mont_ctx* f = &c->fp;
  u256 qy = q->y;
  if (negate) mont_neg(f, &qy, &qy);
  if (p->inf) {
    r->X = q->x; r->Y = qy; r->Z = f->one; r->inf = 0;
    return;
  }
  u256 Z1Z1, U2, S2, H, R, HH, HHH, V, t;
  mont_sq(f, &Z1Z1, &p->Z);
  mont_mul(f, &U2, &q->x, &Z1Z1);
  mont_mul(f, &S2, &qy, &p->Z);
  mont_mul(f, &S2, &S2, &Z1Z1);
  mont_sub(f, &H, &U2, &p->X);
  mont_sub(f, &R, &S2, &p->Y);
  if (u256_is_zero(&H)) {
    if (u256_is_zero(&R)) { jac_dbl(c, r, p); return; }
    r->inf = 1;
    return;
  }
  mont_sq(f, &HH, &H);
  mont_mul(f, &HHH, &H, &HH);
  mont_mul(f, &V, &p->X, &HH);
  jac_t o;
  mont_sq(f, &o.X, &R);
  mont_sub(f, &o.X, &o.X, &HHH);
  mont_add(f, &t, &V, &V);
  mont_sub(f, &o.X, &o.X, &t);
  mont_sub(f, &t, &V, &o.X);
  mont_mul(f, &o.Y, &R, &t);
  mont_mul(f, &t, &p->Y, &HHH);
  mont_sub(f, &o.Y, &o.Y, &t);
  mont_mul(f, &o.Z, &p->Z, &H);
  o.inf = 0;
  *r = o;
}

/* odd multiples P, 3P, .., 15P normalised to affine (BC WNafUtil.precompute + normalizeAll) */
static void precomp_odd(const curve_t* c, aff_t tab[8], const aff_t* P) {
  const mont_ctx* f = &c->fp;
  jac_t j[8], twoP, Pj = {P->x, P->y, f->one, 0};
  jac_dbl(c, &twoP, &Pj);
  j[0] = Pj;
  for (int i = 1; i < 8; ++i) {
    /* j[i] = j[i-1] + 2P  (general Jacobian add via normalising 2P would change counts; use
       affine 2P when finite) */
    if (twoP.inf) { j[i] = j[i - 1]; continue; }
    u256 zi, zi2, zi3;
    aff_t t2;
    mont_inv(f, &zi, &twoP.Z);
    mont_sq(f, &zi2, &zi);
    mont_mul(f, &zi3, &zi2, &zi);
    mont_mul(f, &t2.x, &twoP.X, &zi2);
    mont_mul(f, &t2.y, &twoP.Y, &zi3);
    jac_add_aff(c, &j[i], &j[i - 1], &t2, 0);
  }
  for (int i = 0; i < 8; ++i) {
    if (j[i].inf) { memset(&tab[i], 0, sizeof tab[i]); continue; }
    u256 zi, zi2, zi3;
    mont_inv(f, &zi, &j[i].Z);
    mont_sq(f, &zi2, &zi);
    mont_mul(f, &zi3, &zi2, &zi);
    mont_mul(f, &tab[i].x, &j[i].X, &zi2);
    mont_mul(f, &tab[i].y, &j[i].Y, &zi3);
  }
}

static void curve_setup(curve_t* c, const char* p, const char* a, const char* b, const char* gx, const char* gy,
                        const char* n, int a_is_m3, aff_t gtab[8]) {
  u256 t;
  hex_to_u256(&c->p_plain, p);
  hex_to_u256(&c->n_plain, n);
  mont_init(&c->fp, &c->p_plain);
  mont_init(&c->fn, &c->n_plain);
  hex_to_u256(&t, a); mont_to(&c->fp, &c->a, &t);
  hex_to_u256(&t, b); mont_to(&c->fp, &c->b, &t);
  hex_to_u256(&t, gx); mont_to(&c->fp, &c->gx, &t);
  hex_to_u256(&t, gy); mont_to(&c->fp, &c->gy, &t);
  c->a_is_m3 = a_is_m3;
  aff_t G = {c->gx, c->gy};
  precomp_odd(c, gtab, &G);
}

static void ec_init(void) {
  curve_setup(&C_R1, "ffffffff00000001000000000000000000000000ffffffffffffffffffffffff",
              "ffffffff00000001000000000000000000000000fffffffffffffffffffffffc",
              "5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b",
              "6b17d1f2e12c4247f8bce6e563a440f277037d812deb33a0f4a13945d898c296",
              "4fe342e2fe1a7f9b8ee7eb4a7c0f9e162bce33576b315ececbb6406837bf51f5",
              "ffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551", 1, G_TAB_R1);
  curve_setup(&C_K1, "fffffffffffffffffffffffffffffffffffffffffffffffffffffffefffffc2f",
              "0000000000000000000000000000000000000000000000000000000000000000",
              "0000000000000000000000000000000000000000000000000000000000000007",
              "79be667ef9dcbbac55a06295ce870b07029bfcdb2dce28d959f2815b16f81798",
              "483ada7726a3c4655da4fbfc0e1108a8fd17b448a68554199c47d08ffb10d4b8",
              "fffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141", 0, G_TAB_K1);
}

static const curve_t* curve_of(int scheme) { return scheme == CG_ECDSA_SECP256K1_SHA256 ? &C_K1 : &C_R1; }

static int on_curve(const curve_t* c, const aff_t* q) {
  const mont_ctx* f = &c->fp;
  u256 l, r, t;
  mont_sq(f, &l, &q->y);
  mont_sq(f, &r, &q->x);
  mont_add(f, &r, &r, &c->a);
  mont_mul(f, &r, &r, &q->x);
  mont_add(f, &r, &r, &c->b);
  mont_sub(f, &t, &l, &r);
  return u256_is_zero(&t);
}

static const uint8_t SPKI_R1[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                                    0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
static const uint8_t SPKI_K1[23] = {0x30, 0x56, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02,
                                    0x01, 0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a, 0x03, 0x42, 0x00};

int or_ec_key_decode(or_ec_key* k, int scheme, int fmt, const uint8_t* key, size_t len) {
  pthread_once(&g_once, ec_init);
  const curve_t* c = curve_of(scheme);
  const mont_ctx* f = &c->fp;
  uint8_t pt[65];
  size_t plen;
  if (fmt == CG_KEY_SPKI) {
    /* Crypto.decodePublicKey (Crypto.kt:321-325): this scheme's id-ecPublicKey + named-curve
       algorithm identifier, then any point ECCurve.decodePoint accepts. The DER header of a
       33-byte (compressed) point differs in the two length bytes only. */
    const uint8_t* pre = scheme == CG_ECDSA_SECP256K1_SHA256 ? SPKI_K1 : SPKI_R1;
    size_t pl = scheme == CG_ECDSA_SECP256K1_SHA256 ? sizeof SPKI_K1 : sizeof SPKI_R1;
    if (len == pl + 65) plen = 65;
    else if (len == pl + 33) plen = 33;
    else return CG_KEY_INVALID;
    for (size_t i = 0; i < pl; ++i) {
      uint8_t want = pre[i];
      if (i == 1 || i == pl - 2) want = (uint8_t)(want - (65 - plen));
      if (key[i] != want) return CG_KEY_INVALID;
    }
    memcpy(pt, key + pl, plen);
  } else if (fmt == CG_KEY_RAW) {
    if (len != 64) return CG_KEY_INVALID;
    pt[0] = 4;
    memcpy(pt + 1, key, 64);
    plen = 65;
  } else if (fmt == CG_KEY_SEC1) {
    if (len != 65 && len != 33) return CG_KEY_INVALID;
    memcpy(pt, key, len);
    plen = len;
  } else {
    return CG_KEY_INVALID;
  }
  u256 x, y;
  if (plen == 65) {
    /* 04 uncompressed; 06/07 hybrid, whose tag must carry y's parity (ECCurve.decodePoint) */
    if (pt[0] != 4 && pt[0] != 6 && pt[0] != 7) return CG_KEY_INVALID;
    u256_from_be(&x, pt + 1);
    u256_from_be(&y, pt + 33);
    if (u256_cmp(&x, &c->p_plain) >= 0 || u256_cmp(&y, &c->p_plain) >= 0) return CG_KEY_INVALID;
    if (pt[0] != 4 && (int)(y.v[0] & 1) != (pt[0] & 1)) return CG_KEY_INVALID;
    mont_to(f, &k->Q.x, &x);
    mont_to(f, &k->Q.y, &y);
    if (!on_curve(c, &k->Q)) return CG_KEY_INVALID;
  } else {
    if (pt[0] != 2 && pt[0] != 3) return CG_KEY_INVALID;
    u256_from_be(&x, pt + 1);
    if (u256_cmp(&x, &c->p_plain) >= 0) return CG_KEY_INVALID;
    mont_to(f, &k->Q.x, &x);
    u256 rhs, yy, e, one = {{1, 0, 0, 0}}, t;
    mont_sq(f, &rhs, &k->Q.x);
    mont_add(f, &rhs, &rhs, &c->a);
    mont_mul(f, &rhs, &rhs, &k->Q.x);
    mont_add(f, &rhs, &rhs, &c->b);
    u256_add(&e, &c->p_plain, &one); /* (p+1)/4 */
    for (int i = 0; i < 2; ++i) {
      for (int w = 0; w < 3; ++w) e.v[w] = (e.v[w] >> 1) | (e.v[w + 1] << 63);
      e.v[3] >>= 1;
    }
    mont_pow(f, &yy, &rhs, &e);
    mont_sq(f, &t, &yy);
    mont_sub(f, &t, &t, &rhs);
    if (!u256_is_zero(&t)) return CG_KEY_INVALID;
    u256 yplain;
    mont_from(f, &yplain, &yy);
    if ((int)(yplain.v[0] & 1) != (pt[0] & 1)) mont_neg(f, &yy, &yy);
    k->Q.y = yy;
  }
  k->scheme = scheme;
  precomp_odd(c, k->tab, &k->Q);
  return 0;
}

/* StdDSAEncoder.decode restated (strict DER). r/s out as 32-byte big-endian when they fit. */
static int der_len(const uint8_t* b, size_t n, size_t* i, size_t* out) {
  if (*i >= n) return -1;
  uint8_t l0 = b[(*i)++];
  if (l0 < 0x80) { *out = l0; return 0; }
  size_t nb = l0 & 0x7f;
  if (nb == 0 || nb > 4 || *i + nb > n) return -1;
  size_t v = 0;
  for (size_t k = 0; k < nb; ++k) v = (v << 8) | b[(*i)++];
  /* DER: minimal long form */
  if (v < 0x80) return -1;
  if (nb > 1 && (v >> (8 * (nb - 1))) == 0) return -1;
  *out = v;
  return 0;
}

/* returns 0 (ok), CG_SIG_MALFORMED. *range_ok: 1 if value in [1, 2^256), else 0 */
static int der_int(const uint8_t* b, size_t n, size_t* i, uint8_t out[32], int* range_ok) {
  if (*i >= n || b[*i] != 0x02) return CG_SIG_MALFORMED;
  (*i)++;
  size_t ln;
  if (der_len(b, n, i, &ln)) return CG_SIG_MALFORMED;
  if (ln == 0 || *i + ln > n) return CG_SIG_MALFORMED;
  const uint8_t* c = b + *i;
  if (ln > 1 && ((c[0] == 0 && c[1] < 0x80) || (c[0] == 0xff && c[1] >= 0x80))) return CG_SIG_MALFORMED;
  *i += ln;
  memset(out, 0, 32);
  if (c[0] & 0x80) { *range_ok = 0; return 0; } /* negative */
  /* strip the single sign pad */
  if (c[0] == 0 && ln > 1) { c++; ln--; }
  if (ln > 32) { *range_ok = 0; return 0; }
  memcpy(out + 32 - ln, c, ln);
  int nz = 0;
  for (int k = 0; k < 32; ++k) nz |= out[k];
  *range_ok = nz != 0;
  return 0;
}

int or_der_parse(const uint8_t* sig, size_t len, uint8_t r[32], uint8_t s[32], int* range_ok) {
  size_t i = 0, sl;
  if (len < 2 || sig[0] != 0x30) return CG_SIG_MALFORMED;
  i = 1;
  if (der_len(sig, len, &i, &sl)) return CG_SIG_MALFORMED;
  if (i + sl != len) return CG_SIG_MALFORMED;
  int ok1 = 0, ok2 = 0;
  if (der_int(sig, len, &i, r, &ok1)) return CG_SIG_MALFORMED;
  if (i >= len) return CG_SIG_MALFORMED; /* one element */
  if (der_int(sig, len, &i, s, &ok2)) return CG_SIG_MALFORMED;
  if (i != len) return CG_SIG_MALFORMED; /* three or more elements / junk inside */
  *range_ok = ok1 && ok2;
  return 0;
}

/* WNafUtil.generateWindowNaf(5, k) */
static int wnaf5(signed char* naf, const u256* k) {
  u256 x = *k;
  int len = 0;
  memset(naf, 0, 258);
  int pos = 0;
  while (!u256_is_zero(&x)) {
    if (x.v[0] & 1) {
      int d = (int)(x.v[0] & 31);
      if (d >= 16) d -= 32;
      naf[pos] = (signed char)d;
      u256 dd = {{0, 0, 0, 0}};
      if (d > 0) { dd.v[0] = (uint64_t)d; u256_sub(&x, &x, &dd); }
      else { dd.v[0] = (uint64_t)(-d); u256_add(&x, &x, &dd); }
    }
    /* x >>= 1 */
    for (int w = 0; w < 3; ++w) x.v[w] = (x.v[w] >> 1) | (x.v[w + 1] << 63);
    x.v[3] >>= 1;
    ++pos;
    len = pos;
  }
  return len;
}

int or_ec_verify(const or_ec_key* k, const uint8_t* msg, size_t msg_len, const uint8_t* sig, size_t sig_len) {
  pthread_once(&g_once, ec_init);
  const curve_t* c = curve_of(k->scheme);
  const mont_ctx* fn = &c->fn;
  const mont_ctx* fp = &c->fp;
  uint8_t hash[32], rb[32], sb[32];
  or_sha256(msg, msg_len, hash);
  int range_ok;
  if (or_der_parse(sig, sig_len, rb, sb, &range_ok)) return CG_SIG_MALFORMED;
  if (!range_ok) return CG_INVALID;
  u256 r, s, e;
  u256_from_be(&r, rb);
  u256_from_be(&s, sb);
  u256_from_be(&e, hash);
  if (u256_cmp(&r, &c->n_plain) >= 0 || u256_cmp(&s, &c->n_plain) >= 0) return CG_INVALID;
  /* c = s^-1 mod n ; u1 = e c ; u2 = r c   (scalar arithmetic mod n in Montgomery form) */
  u256 em, rm, sm, ci, u1m, u2m, u1, u2;
  u256_mod(fn, &em, &e);
  mont_to(fn, &em, &em);
  mont_to(fn, &rm, &r);
  mont_to(fn, &sm, &s);
  mont_inv(fn, &ci, &sm);
  mont_mul(fn, &u1m, &em, &ci);
  mont_mul(fn, &u2m, &rm, &ci);
  mont_from(fn, &u1, &u1m);
  mont_from(fn, &u2, &u2m);
  signed char n1[258], n2[258];
  int l1 = wnaf5(n1, &u1), l2 = wnaf5(n2, &u2);
  int top = (l1 > l2 ? l1 : l2) - 1;
  const aff_t* gt = k->scheme == CG_ECDSA_SECP256K1_SHA256 ? G_TAB_K1 : G_TAB_R1;
  jac_t R = {{{0}}, {{0}}, {{0}}, 1};
  for (int i = top; i >= 0; --i) {
    jac_dbl(c, &R, &R);
    if (n1[i]) jac_add_aff(c, &R, &R, &gt[(n1[i] < 0 ? -n1[i] : n1[i]) / 2], n1[i] < 0);
    if (n2[i]) jac_add_aff(c, &R, &R, &k->tab[(n2[i] < 0 ? -n2[i] : n2[i]) / 2], n2[i] < 0);
  }
  if (R.inf) return CG_INVALID;
  /* BC: D = Z^2 (Jacobian); while r < p: if r*D == X return true; r += n */
  u256 D, X, rr = r, t;
  mont_sq(fp, &D, &R.Z);
  X = R.X;
  for (int pass = 0; pass < 2; ++pass) {
    if (u256_cmp(&rr, &c->p_plain) >= 0) break;
    u256 rmp;
    mont_to(fp, &rmp, &rr);
    mont_mul(fp, &t, &rmp, &D);
    if (u256_cmp(&t, &X) == 0) return CG_VALID;
    if (u256_add(&rr, &rr, &c->n_plain)) break; /* overflow past 2^256 */
  }
  return CG_INVALID;
}
