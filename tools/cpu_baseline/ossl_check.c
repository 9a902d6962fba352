/* CPU reference points with OpenSSL (bench.py cpu_baseline.openssl and cpu_baseline.configs0.openssl).
 * BASELINE configs[0]:
 * the same checkSignaturesAreValid loop as oracle/c or_check_txs (fail-fast per transaction,
 * workers pulling the next transaction from a shared counter), each Ed25519 signature verified
 * with EVP_DigestVerify on a fresh EVP_PKEY (the JVM builds a fresh PublicKey per deserialised
 * transaction). An industrial point of comparison, NOT the oracle: OpenSSL rejects S >= L, which
 * i2p 0.2.0 accepts. libcrypto is loaded with dlopen; without it the entry
 * point returns -1 and bench.py records it as absent. Not product code. */
#include <dlfcn.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <unistd.h>

#include "../../include/cordagpu.h"

#define NID_ED25519_ 1087
typedef void* (*pkey_new_raw_fn)(int, void*, const unsigned char*, size_t);
typedef void* (*md_ctx_new_fn)(void);
typedef void (*md_ctx_free_fn)(void*);
typedef void (*pkey_free_fn)(void*);
typedef int (*dv_init_fn)(void*, void**, const void*, void*, void*);
typedef int (*dv_fn)(void*, const unsigned char*, size_t, const unsigned char*, size_t);
typedef void* (*d2i_pubkey_fn)(void**, const unsigned char**, long);
typedef const void* (*md_fn)(void);

static struct {
  pkey_new_raw_fn pkey_new_raw;
  md_ctx_new_fn md_ctx_new;
  md_ctx_free_fn md_ctx_free;
  pkey_free_fn pkey_free;
  dv_init_fn dv_init;
  dv_fn dv;
  d2i_pubkey_fn d2i_pubkey;
  md_fn sha256;
  void* (*md_fetch)(void*, const char*, const char*);
  void (*md_free)(void*);
  int (*md_ctx_reset)(void*);
  int ok;
} F;

static int load(void) {
  if (F.ok) return 1;
  void* h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
  if (!h) return 0;
  F.pkey_new_raw = (pkey_new_raw_fn)dlsym(h, "EVP_PKEY_new_raw_public_key");
  F.md_ctx_new = (md_ctx_new_fn)dlsym(h, "EVP_MD_CTX_new");
  F.md_ctx_free = (md_ctx_free_fn)dlsym(h, "EVP_MD_CTX_free");
  F.pkey_free = (pkey_free_fn)dlsym(h, "EVP_PKEY_free");
  F.dv_init = (dv_init_fn)dlsym(h, "EVP_DigestVerifyInit");
  F.dv = (dv_fn)dlsym(h, "EVP_DigestVerify");
  F.d2i_pubkey = (d2i_pubkey_fn)dlsym(h, "d2i_PUBKEY");
  F.sha256 = (md_fn)dlsym(h, "EVP_sha256");
  F.md_fetch = (void* (*)(void*, const char*, const char*))dlsym(h, "EVP_MD_fetch");
  F.md_free = (void (*)(void*))dlsym(h, "EVP_MD_free");
  F.md_ctx_reset = (int (*)(void*))dlsym(h, "EVP_MD_CTX_reset");
  F.ok = F.pkey_new_raw && F.md_ctx_new && F.md_ctx_free && F.pkey_free && F.dv_init && F.dv && F.d2i_pubkey &&
         F.sha256 && F.md_fetch && F.md_free && F.md_ctx_reset;
  return F.ok;
}

/* 1 valid, 0 not (any failure: OpenSSL has no exception split) */
static int verify_one(const cg_key* k, const cg_item* it, const uint8_t* arena, uint64_t arena_len) {
  if (k->scheme != CG_EDDSA_ED25519_SHA512 || k->fmt != CG_KEY_RAW || k->len != 32) return 0;
  if (k->off + 32 > arena_len || it->sig_off + it->sig_len > arena_len || it->msg_off + it->msg_len > arena_len)
    return 0;
  void* pk = F.pkey_new_raw(NID_ED25519_, NULL, arena + k->off, 32);
  if (!pk) return 0;
  void* ctx = F.md_ctx_new();
  int ok = ctx && F.dv_init(ctx, NULL, NULL, NULL, pk) == 1 &&
           F.dv(ctx, arena + it->sig_off, it->sig_len, arena + it->msg_off, it->msg_len) == 1;
  if (ctx) F.md_ctx_free(ctx);
  F.pkey_free(pk);
  return ok;
}

typedef struct {
  const cg_key* keys;
  uint32_t n_keys;
  const cg_item* items;
  const uint64_t* tx_first;
  uint64_t n_tx;
  const uint8_t* arena;
  uint64_t arena_len;
  int64_t* first_fail;
  uint64_t next, verified;
} job_t;

static void* worker(void* p) {
  job_t* j = (job_t*)p;
  uint64_t done = 0;
  for (;;) {
    const uint64_t t = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
    if (t >= j->n_tx) break;
    int64_t ff = -1;
    for (uint64_t i = j->tx_first[t]; i < j->tx_first[t + 1]; ++i) {
      const cg_item* it = &j->items[i];
      ++done;
      if (it->key_idx >= j->n_keys || !verify_one(&j->keys[it->key_idx], it, j->arena, j->arena_len)) {
        ff = (int64_t)(i - j->tx_first[t]);
        break;
      }
    }
    j->first_fail[t] = ff;
  }
  __atomic_fetch_add(&j->verified, done, __ATOMIC_RELAXED);
  return NULL;
}

int64_t ob_check_txs(const cg_key* keys, uint32_t n_keys, const cg_item* items, const uint64_t* tx_first,
                     uint64_t n_tx, const uint8_t* arena, uint64_t arena_len, int64_t* first_fail, int nthreads) {
  if (!load()) return -1;
  if (nthreads <= 0) nthreads = 1;
  job_t j = {keys, n_keys, items, tx_first, n_tx, arena, arena_len, first_fail, 0, 0};
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, worker, &j);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  return (int64_t)j.verified;
}

/* ---- the headline mix (bench.py cpu_baseline.openssl): every item verified independently --------
 * Ed25519 keys through EVP_PKEY_new_raw_public_key; ECDSA keys (secp256r1 / secp256k1, raw 64-byte
 * X||Y wrapped in the curve's SubjectPublicKeyInfo header, or SPKI as given) through d2i_PUBKEY;
 * each key decoded ONCE per call (inside the timed call) and shared read-only by the workers, as
 * Crypto.doVerify receives an already-decoded PublicKey. A per-item decode serialises on OpenSSL
 * 3.0's decoder locks (16 threads ran slower than one: profiles/r03/v8/bench_full.json). Then
 * EVP_DigestVerify, SHA-256 fetched once for ECDSA. Status: 0 valid, 1 anything else. */
static const uint8_t SPKI_R1[26] = {0x30, 0x59, 0x30, 0x13, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02, 0x01,
                                    0x06, 0x08, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x03, 0x01, 0x07, 0x03, 0x42, 0x00};
static const uint8_t SPKI_K1[23] = {0x30, 0x56, 0x30, 0x10, 0x06, 0x07, 0x2a, 0x86, 0x48, 0xce, 0x3d, 0x02,
                                    0x01, 0x06, 0x05, 0x2b, 0x81, 0x04, 0x00, 0x0a, 0x03, 0x42, 0x00};

static void* decode_key(const cg_key* k, const uint8_t* arena, uint64_t arena_len) {
  if (k->off + k->len > arena_len) return NULL;
  if (k->scheme == CG_EDDSA_ED25519_SHA512) {
    if (k->fmt != CG_KEY_RAW || k->len != 32) return NULL;
    return F.pkey_new_raw(NID_ED25519_, NULL, arena + k->off, 32);
  }
  if (k->scheme != CG_ECDSA_SECP256R1_SHA256 && k->scheme != CG_ECDSA_SECP256K1_SHA256) return NULL;
  uint8_t der[128];
  const uint8_t* p = der;
  long n = 0;
  if (k->fmt == CG_KEY_RAW && k->len == 64) {
    const uint8_t* hdr = k->scheme == CG_ECDSA_SECP256R1_SHA256 ? SPKI_R1 : SPKI_K1;
    const int hl = k->scheme == CG_ECDSA_SECP256R1_SHA256 ? 26 : 23;
    for (int i = 0; i < hl; ++i) der[i] = hdr[i];
    der[hl] = 0x04;
    for (int i = 0; i < 64; ++i) der[hl + 1 + i] = arena[k->off + i];
    n = hl + 65;
  } else if (k->fmt == CG_KEY_SPKI && k->len <= sizeof der) {
    for (int i = 0; i < k->len; ++i) der[i] = arena[k->off + i];
    n = k->len;
  } else {
    return NULL;
  }
  return F.d2i_pubkey(NULL, &p, n);
}

typedef struct {
  const cg_key* keys;
  uint32_t n_keys;
  void** pkeys;
  const void* sha256;
  const cg_item* items;
  uint64_t n;
  const uint8_t* arena;
  uint64_t arena_len;
  uint8_t* status;
  uint64_t next;
} items_job_t;

static void* keys_worker(void* p) {
  items_job_t* j = (items_job_t*)p;
  for (;;) {
    const uint64_t k = __atomic_fetch_add(&j->next, 1, __ATOMIC_RELAXED);
    if (k >= j->n_keys) break;
    j->pkeys[k] = decode_key(&j->keys[k], j->arena, j->arena_len);
  }
  return NULL;
}

static void* items_worker(void* p) {
  items_job_t* j = (items_job_t*)p;
  void* ctx = F.md_ctx_new();
  for (;;) {
    const uint64_t b = __atomic_fetch_add(&j->next, 256, __ATOMIC_RELAXED);
    if (b >= j->n) break;
    const uint64_t e = b + 256 < j->n ? b + 256 : j->n;
    for (uint64_t i = b; i < e; ++i) {
      const cg_item* it = &j->items[i];
      void* pk = it->key_idx < j->n_keys ? j->pkeys[it->key_idx] : NULL;
      int ok = 0;
      if (pk && ctx && it->sig_off + it->sig_len <= j->arena_len && it->msg_off + it->msg_len <= j->arena_len) {
        const void* md = j->keys[it->key_idx].scheme == CG_EDDSA_ED25519_SHA512 ? NULL : j->sha256;
        ok = F.dv_init(ctx, NULL, md, NULL, pk) == 1 &&
             F.dv(ctx, j->arena + it->sig_off, it->sig_len, j->arena + it->msg_off, it->msg_len) == 1;
        F.md_ctx_reset(ctx);
      }
      j->status[i] = ok ? 0 : 1;
    }
  }
  if (ctx) F.md_ctx_free(ctx);
  return NULL;
}

static void run_workers(void* (*fn)(void*), items_job_t* j, int nthreads) {
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  j->next = 0;
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, fn, j);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
}

/* Returns n, or -1 when libcrypto.so.3 cannot be loaded. */
int64_t ob_verify_items(const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n, const uint8_t* arena,
                        uint64_t arena_len, uint8_t* status, int nthreads) {
  if (!load()) return -1;
  if (nthreads <= 0) nthreads = 1;
  void* sha256 = F.md_fetch(NULL, "SHA256", NULL);
  void** pkeys = (void**)calloc(n_keys ? n_keys : 1, sizeof(void*));
  items_job_t j = {keys, n_keys, pkeys, sha256, items, n, arena, arena_len, status, 0};
  run_workers(keys_worker, &j, nthreads);
  run_workers(items_worker, &j, nthreads);
  for (uint32_t k = 0; k < n_keys; ++k)
    if (pkeys[k]) F.pkey_free(pkeys[k]);
  free(pkeys);
  if (sha256) F.md_free(sha256);
  return (int64_t)n;
}
