/* 256-bit modular arithmetic for the C oracle (TEST INFRASTRUCTURE ONLY).
 * Generic Montgomery (CIOS, 4 x 64-bit limbs) over any odd modulus < 2^256. Deliberately
 * plain: it is the checker and the CPU "port" baseline, not a fast implementation. */
#ifndef CORDA_ORACLE_BN_H
#define CORDA_ORACLE_BN_H
#include <stdint.h>
#include <string.h>

typedef struct { uint64_t v[4]; } u256;
typedef struct {
  u256 m;       /* modulus */
  uint64_t mp;  /* -m^-1 mod 2^64 */
  u256 r2;      /* 2^512 mod m */
  u256 one;     /* 2^256 mod m  (Montgomery 1) */
} mont_ctx;

void mont_init(mont_ctx* c, const u256* m);
void mont_mul(const mont_ctx* c, u256* r, const u256* a, const u256* b); /* counts fe_mul */
void mont_sq(const mont_ctx* c, u256* r, const u256* a);                 /* counts fe_sq */
void mont_add(const mont_ctx* c, u256* r, const u256* a, const u256* b);
void mont_sub(const mont_ctx* c, u256* r, const u256* a, const u256* b);
void mont_neg(const mont_ctx* c, u256* r, const u256* a);
void mont_to(const mont_ctx* c, u256* r, const u256* a);   /* a < m  -> aR mod m */
void mont_from(const mont_ctx* c, u256* r, const u256* a); /* aR -> a */
void mont_pow(const mont_ctx* c, u256* r, const u256* a, const u256* e);
void mont_inv(const mont_ctx* c, u256* r, const u256* a);  /* Fermat, m prime */

int u256_cmp(const u256* a, const u256* b);
int u256_is_zero(const u256* a);
uint64_t u256_add(u256* r, const u256* a, const u256* b); /* returns carry */
uint64_t u256_sub(u256* r, const u256* a, const u256* b); /* returns borrow */
void u256_from_be(u256* r, const uint8_t b[32]);
void u256_from_le(u256* r, const uint8_t b[32]);
void u256_to_be(uint8_t b[32], const u256* a);
void u256_to_le(uint8_t b[32], const u256* a);
void u256_set_u64(u256* r, uint64_t x);
/* r = (x mod m) for a 512-bit little-endian integer x (used by sc_reduce / hash reduction) */
void u512_mod(const mont_ctx* c, u256* r, const uint8_t x_le[64]);
void u256_mod(const mont_ctx* c, u256* r, const u256* a); /* a mod m for a < 2^256 */
#endif
