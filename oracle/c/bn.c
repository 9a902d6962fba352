/* Generic 256-bit Montgomery arithmetic for the C oracle. TEST INFRASTRUCTURE ONLY. */
#include "bn.h"

#include "oracle.h"

extern __thread or_counters g_or_counters;
typedef unsigned __int128 u128;

int u256_cmp(const u256* a, const u256* b) {
  for (int i = 3; i >= 0; --i) {
    if (a->v[i] < b->v[i]) return -1;
    if (a->v[i] > b->v[i]) return 1;
  }
  return 0;
}
int u256_is_zero(const u256* a) { return (a->v[0] | a->v[1] | a->v[2] | a->v[3]) == 0; }

uint64_t u256_add(u256* r, const u256* a, const u256* b) {
  u128 c = 0;
  for (int i = 0; i < 4; ++i) {
    c += (u128)a->v[i] + b->v[i];
    r->v[i] = (uint64_t)c;
    c >>= 64;
  }
  return (uint64_t)c;
}
uint64_t u256_sub(u256* r, const u256* a, const u256* b) {
  uint64_t br = 0;
  for (int i = 0; i < 4; ++i) {
    u128 t = (u128)a->v[i] - b->v[i] - br;
    r->v[i] = (uint64_t)t;
    br = (uint64_t)(t >> 64) & 1;
  }
  return br;
}
void u256_from_be(u256* r, const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 0; j < 8; ++j) v = (v << 8) | b[(3 - i) * 8 + j];
    r->v[i] = v;
  }
}
void u256_from_le(u256* r, const uint8_t b[32]) {
  for (int i = 0; i < 4; ++i) {
    uint64_t v = 0;
    for (int j = 7; j >= 0; --j) v = (v << 8) | b[i * 8 + j];
    r->v[i] = v;
  }
}
void u256_to_be(uint8_t b[32], const u256* a) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[(3 - i) * 8 + j] = (uint8_t)(a->v[i] >> (56 - 8 * j));
}
void u256_to_le(uint8_t b[32], const u256* a) {
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) b[i * 8 + j] = (uint8_t)(a->v[i] >> (8 * j));
}
void u256_set_u64(u256* r, uint64_t x) {
  memset(r, 0, sizeof *r);
  r->v[0] = x;
}

static void mont_mul_raw(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
  uint64_t t[6] = {0, 0, 0, 0, 0, 0};
  for (int i = 0; i < 4; ++i) {
    u128 carry = 0;
    for (int j = 0; j < 4; ++j) {
      carry += (u128)a->v[j] * b->v[i] + t[j];
      t[j] = (uint64_t)carry;
      carry >>= 64;
    }
    carry += t[4];
    t[4] = (uint64_t)carry;
    t[5] = (uint64_t)(carry >> 64);
    uint64_t m = t[0] * c->mp;
    carry = ((u128)m * c->m.v[0] + t[0]) >> 64;
    for (int j = 1; j < 4; ++j) {
      carry += (u128)m * c->m.v[j] + t[j];
      t[j - 1] = (uint64_t)carry;
      carry >>= 64;
    }
    carry += t[4];
    t[3] = (uint64_t)carry;
    t[4] = t[5] + (uint64_t)(carry >> 64);
  }
  u256 res = {{t[0], t[1], t[2], t[3]}};
  u256 sub;
  uint64_t br = u256_sub(&sub, &res, &c->m);
  if (t[4] || !br) res = sub;
  *r = res;
}

void mont_mul(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
  g_or_counters.fe_mul++;
  mont_mul_raw(c, r, a, b);
}
void mont_sq(const mont_ctx* c, u256* r, const u256* a) {
  g_or_counters.fe_sq++;
  mont_mul_raw(c, r, a, a);
}

void mont_add(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
  u256 t, s;
  uint64_t cy = u256_add(&t, a, b);
  uint64_t br = u256_sub(&s, &t, &c->m);
  *r = (cy || !br) ? s : t;
}
void mont_sub(const mont_ctx* c, u256* r, const u256* a, const u256* b) {
  u256 t;
  if (u256_sub(&t, a, b)) u256_add(&t, &t, &c->m);
  *r = t;
}
void mont_neg(const mont_ctx* c, u256* r, const u256* a) {
  u256 z = {{0, 0, 0, 0}};
  mont_sub(c, r, &z, a);
}

/* a mod m for arbitrary a < 2^256 (m > 2^255 or small multiples handled by loop) */
void u256_mod(const mont_ctx* c, u256* r, const u256* a) {
  /* shift-subtract */
  u256 x = *a;
  while (u256_cmp(&x, &c->m) >= 0) {
    /* find largest shift */
    u256 mm = c->m;
    int sh = 0;
    while (!(mm.v[3] >> 63)) {
      u256 t = mm;
      /* t <<= 1 */
      for (int i = 3; i > 0; --i) t.v[i] = (t.v[i] << 1) | (t.v[i - 1] >> 63);
      t.v[0] <<= 1;
      if (u256_cmp(&t, &x) > 0) break;
      mm = t;
      ++sh;
    }
    u256_sub(&x, &x, &mm);
  }
  *r = x;
}

void mont_init(mont_ctx* c, const u256* m) {
  c->m = *m;
  uint64_t inv = 1;
  for (int i = 0; i < 7; ++i) inv *= 2 - m->v[0] * inv;  /* Newton: inv = m^-1 mod 2^64 */
  c->mp = (uint64_t)0 - inv;
  /* one = 2^256 mod m = (2^256 - m) mod m */
  u256 z = {{0, 0, 0, 0}}, t;
  u256_sub(&t, &z, m);
  u256_mod(c, &c->one, &t);
  /* r2 = 2^512 mod m: double `one` 256 times mod m */
  u256 x = c->one;
  for (int i = 0; i < 256; ++i) mont_add(c, &x, &x, &x);
  c->r2 = x;
}

void mont_to(const mont_ctx* c, u256* r, const u256* a) { mont_mul_raw(c, r, a, &c->r2); }
void mont_from(const mont_ctx* c, u256* r, const u256* a) {
  u256 one = {{1, 0, 0, 0}};
  mont_mul_raw(c, r, a, &one);
}

void mont_pow(const mont_ctx* c, u256* r, const u256* a, const u256* e) {
  u256 acc = c->one;
  int started = 0;
  for (int i = 255; i >= 0; --i) {
    if (started) mont_sq(c, &acc, &acc);
    if ((e->v[i >> 6] >> (i & 63)) & 1) {
      if (started) mont_mul(c, &acc, &acc, a);
      else { acc = *a; started = 1; }
    }
  }
  *r = acc;
}

void mont_inv(const mont_ctx* c, u256* r, const u256* a) {
  u256 e, two = {{2, 0, 0, 0}};
  u256_sub(&e, &c->m, &two);
  mont_pow(c, r, a, &e);
}

void u512_mod(const mont_ctx* c, u256* r, const uint8_t x_le[64]) {
  /* x = lo + hi * 2^256 ; result = lo mod m + (hi mod m) * (2^256 mod m) mod m, via Montgomery:
     mont_mul(hi_mod, r2) = hi * 2^256 mod m. */
  u256 lo, hi, lom, him, t;
  u256_from_le(&lo, x_le);
  u256_from_le(&hi, x_le + 32);
  u256_mod(c, &lom, &lo);
  u256_mod(c, &him, &hi);
  mont_mul_raw(c, &t, &him, &c->r2); /* him * 2^512 / 2^256 = him * 2^256 mod m */
  mont_add(c, r, &t, &lom);
}
