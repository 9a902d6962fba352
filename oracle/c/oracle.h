/* C restatement of the reference's signature-verification and tx-id hashing semantics.
 *
 * TEST INFRASTRUCTURE ONLY: the on-box oracle for large batches and the CPU baseline
 * ("kind": "port") of bench.py. The product (libcordagpu.so) never links this.
 *
 * Restated algorithms (the reference's arithmetic lives in un-vendored jars; see
 * oracle/__init__.py for how parity is pinned):
 *   ed25519_i2p.c  net.i2p.crypto:eddsa:0.2.0 EdDSAEngine.engineVerify, GroupElement
 *                  decode / slide / doubleScalarMultiplyVariableTime / toByteArray
 *                  (called at core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559)
 *   ecdsa_bc.c     bcprov-jdk15on:1.57 SHA256withECDSA: StdDSAEncoder.decode (strict DER),
 *                  ECDSASigner.verifySignature, ECAlgorithms.implShamirsTrickWNaf (w = 5)
 *   sha2.c         FIPS 180-4 SHA-256 / SHA-512 (JDK SUN MessageDigest, SecureHash.kt:37)
 *   oracle.c       Crypto.doVerify / isValid status mapping (Crypto.kt:474-484,553-559),
 *                  MerkleTree.getMerkleTree (MerkleTree.kt:27-66), computeNonce /
 *                  serializedHash (MerkleTransaction.kt:16-33), batch driver over threads.
 *
 * Item layout is include/cordagpu.h's, so one arena can be checked by both.
 */
#ifndef CORDA_ORACLE_H
#define CORDA_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#include "../../include/cordagpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* --- SHA-2 --- */
void or_sha256(const uint8_t* msg, size_t len, uint8_t out[32]);
void or_sha512(const uint8_t* msg, size_t len, uint8_t out[64]);
typedef struct { uint64_t h[8]; uint8_t buf[128]; uint64_t len; } or_sha512_ctx;
void or_sha512_init(or_sha512_ctx* c);
void or_sha512_update(or_sha512_ctx* c, const uint8_t* d, size_t n);
void or_sha512_final(or_sha512_ctx* c, uint8_t out[64]);

/* --- operation counters (thread-local): field multiplies/squarings, SHA compressions --- */
typedef struct {
  uint64_t fe_mul, fe_sq, sc_mul, sha256_blocks, sha512_blocks;
} or_counters;
void or_counters_reset(void);
or_counters or_counters_get(void);

/* --- Ed25519 (i2p 0.2.0) --- */
typedef struct or_ed_key or_ed_key; /* opaque decoded key: A, Abyte, -A precomputed table */
size_t or_ed_key_size(void);
/* returns 0 on success, CG_KEY_INVALID if A does not decode */
int or_ed_key_decode(or_ed_key* k, const uint8_t a[32]);
const uint8_t* or_ed_key_abyte(const or_ed_key* k);
/* returns CG_VALID / CG_INVALID / CG_SIG_MALFORMED */
int or_ed_verify(const or_ed_key* k, const uint8_t* msg, size_t msg_len, const uint8_t* sig, size_t sig_len);
/* slide() value helpers for tests: returns 1 if the carry escaped past bit 255 */
int or_ed_slide_escapes(const uint8_t s[32]);

/* --- ECDSA (BC 1.57) --- */
typedef struct or_ec_key or_ec_key;
size_t or_ec_key_size(void);
int or_ec_key_decode(or_ec_key* k, int scheme, int fmt, const uint8_t* key, size_t len);
int or_ec_verify(const or_ec_key* k, const uint8_t* msg, size_t msg_len, const uint8_t* sig, size_t sig_len);
/* strict DER parse; returns 0 if OK (r,s big-endian 32-byte + flags), CG_SIG_MALFORMED otherwise.
 * *range_ok = 1 iff 1 <= r,s < 2^256 after sign check (range vs n is checked by the caller) */
int or_der_parse(const uint8_t* sig, size_t len, uint8_t r[32], uint8_t s[32], int* range_ok);

/* --- Corda-level --- */
int or_verify_item(const cg_key* key, const cg_item* it, const uint8_t* arena, uint64_t arena_len, uint32_t mode);
/* Batch over nthreads threads (0 = all cores); keys are decoded once each (as the JVM decodes
 * a PublicKey object once). Returns 0. */
int or_verify_batch(const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items,
                    const uint8_t* arena, uint64_t arena_len, uint32_t mode, uint8_t* status_out, int nthreads);
/* checkSignaturesAreValid over n_tx transactions (tx t = items[tx_first[t] .. tx_first[t+1])):
 * first_fail[t] = index within the tx of the first signature that does not verify, or -1.
 * Returns the number of signatures verified (fail-fast stops early). */
uint64_t or_check_txs(const cg_key* keys, uint32_t n_keys, const cg_item* items, const uint64_t* tx_first,
                      uint64_t n_tx, const uint8_t* arena, uint64_t arena_len, int64_t* first_fail, int nthreads);
/* MerkleTree.getMerkleTree(leaves).hash; returns -1 on empty. */
int or_merkle_root(const uint8_t* leaves, size_t n, uint8_t out[32]);
/* WireTransaction.id for one tx; comp_offs/comp_lens index `arena`; salt leaf last. */
int or_tx_id(const uint8_t* arena, const uint64_t* comp_offs, const uint32_t* comp_lens, uint32_t n_comp,
             const uint8_t salt[32], const uint8_t* salt_blob, uint32_t salt_blob_len, uint8_t out[32]);
int or_tx_ids_batch(const cg_tx* txs, uint64_t n_tx, const cg_component* comps, const uint8_t* arena,
                    uint8_t* ids_out, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
