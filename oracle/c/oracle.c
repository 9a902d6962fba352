/* Corda-level control flow of the C oracle. TEST INFRASTRUCTURE ONLY.
 *   or_verify_item  Crypto.doVerify (Crypto.kt:474-484) / Crypto.isValid (Crypto.kt:553-559)
 *                   mapped onto include/cordagpu.h status codes.
 *   or_merkle_root  MerkleTree.getMerkleTree (MerkleTree.kt:27-66)
 *   or_tx_id        WireTransaction.id (WireTransaction.kt:39,104; MerkleTransaction.kt:16-33,93)
 *   or_verify_batch / or_tx_ids_batch  the same over a std pthread pool (CPU baseline).
 */
#include <pthread.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include "oracle.h"

__thread or_counters g_or_counters;
static or_counters g_total;
static pthread_mutex_t g_total_mu = PTHREAD_MUTEX_INITIALIZER;
void or_counters_reset(void) {
  pthread_mutex_lock(&g_total_mu);
  memset(&g_total, 0, sizeof g_total);
  pthread_mutex_unlock(&g_total_mu);
  memset(&g_or_counters, 0, sizeof g_or_counters);
}
/* totals of finished pool workers plus this thread's own */
or_counters or_counters_get(void) {
  pthread_mutex_lock(&g_total_mu);
  or_counters r = g_total;
  pthread_mutex_unlock(&g_total_mu);
  r.fe_mul += g_or_counters.fe_mul; r.fe_sq += g_or_counters.fe_sq; r.sc_mul += g_or_counters.sc_mul;
  r.sha256_blocks += g_or_counters.sha256_blocks; r.sha512_blocks += g_or_counters.sha512_blocks;
  return r;
}
static void counters_flush(void) {
  pthread_mutex_lock(&g_total_mu);
  g_total.fe_mul += g_or_counters.fe_mul; g_total.fe_sq += g_or_counters.fe_sq; g_total.sc_mul += g_or_counters.sc_mul;
  g_total.sha256_blocks += g_or_counters.sha256_blocks; g_total.sha512_blocks += g_or_counters.sha512_blocks;
  pthread_mutex_unlock(&g_total_mu);
  memset(&g_or_counters, 0, sizeof g_or_counters);
}

static const uint8_t ED_SPKI[12] = {0x30, 0x2a, 0x30, 0x05, 0x06, 0x03, 0x2b, 0x65, 0x70, 0x03, 0x21, 0x00};
/* explicit NULL parameter: normalised away by Crypto.findSignatureScheme (Crypto.kt:219-228),
   accepted by i2p 0.2.0 EdDSAPublicKey.decode */
static const uint8_t ED_SPKI_NULL[14] = {0x30, 0x2c, 0x30, 0x07, 0x06, 0x03, 0x2b, 0x65,
                                         0x70, 0x05, 0x00, 0x03, 0x21, 0x00};

static int scheme_supported(int s) {
  return s == CG_ECDSA_SECP256K1_SHA256 || s == CG_ECDSA_SECP256R1_SHA256 || s == CG_EDDSA_ED25519_SHA512;
}

/* decoded key slot */
typedef struct {
  int status; /* 0 ok, CG_KEY_INVALID, CG_UNSUPPORTED */
  int scheme;
  void* k;
} keyslot;

static void decode_key(keyslot* ks, const cg_key* key, const uint8_t* arena, uint64_t arena_len) {
  ks->scheme = key->scheme;
  ks->k = NULL;
  if (!scheme_supported(key->scheme)) { ks->status = CG_UNSUPPORTED; return; }
  if (key->off + key->len > arena_len) { ks->status = CG_KEY_INVALID; return; }
  const uint8_t* kb = arena + key->off;
  if (key->scheme == CG_EDDSA_ED25519_SHA512) {
    const uint8_t* a = NULL;
    if (key->fmt == CG_KEY_RAW && key->len == 32) a = kb;
    else if (key->fmt == CG_KEY_SPKI && key->len == 44 && memcmp(kb, ED_SPKI, 12) == 0) a = kb + 12;
    else if (key->fmt == CG_KEY_SPKI && key->len == 46 && memcmp(kb, ED_SPKI_NULL, 14) == 0) a = kb + 14;
    if (!a) { ks->status = CG_KEY_INVALID; return; }
    ks->k = malloc(or_ed_key_size());
    ks->status = or_ed_key_decode((or_ed_key*)ks->k, a);
  } else {
    ks->k = malloc(or_ec_key_size());
    ks->status = or_ec_key_decode((or_ec_key*)ks->k, key->scheme, key->fmt, kb, key->len);
  }
}

static int verify_with(const keyslot* ks, const cg_item* it, const uint8_t* arena, uint64_t arena_len, uint32_t mode) {
  if (ks->status == CG_UNSUPPORTED) return CG_UNSUPPORTED;
  if (ks->status) return CG_KEY_INVALID;
  if (it->sig_off + it->sig_len > arena_len || it->msg_off + it->msg_len > arena_len) return CG_NOT_RUN;
  if (mode == CG_MODE_DOVERIFY && (it->sig_len == 0 || it->msg_len == 0)) return CG_EMPTY;
  const uint8_t* sig = arena + it->sig_off;
  const uint8_t* msg = arena + it->msg_off;
  if (ks->scheme == CG_EDDSA_ED25519_SHA512) return or_ed_verify((const or_ed_key*)ks->k, msg, it->msg_len, sig, it->sig_len);
  return or_ec_verify((const or_ec_key*)ks->k, msg, it->msg_len, sig, it->sig_len);
}

int or_verify_item(const cg_key* key, const cg_item* it, const uint8_t* arena, uint64_t arena_len, uint32_t mode) {
  keyslot ks;
  decode_key(&ks, key, arena, arena_len);
  int st = verify_with(&ks, it, arena, arena_len, mode);
  free(ks.k);
  return st;
}

typedef struct {
  const cg_key* keys;
  uint32_t n_keys;
  keyslot* slots;
  const cg_item* items;
  uint64_t n_items;
  const uint8_t* arena;
  uint64_t arena_len;
  uint32_t mode;
  uint8_t* status;
  int nthreads;
  int tid;
} job_t;

static void* key_worker(void* p) {
  job_t* j = (job_t*)p;
  memset(&g_or_counters, 0, sizeof g_or_counters);
  for (uint64_t i = (uint64_t)j->tid; i < j->n_keys; i += (uint64_t)j->nthreads)
    decode_key(&j->slots[i], &j->keys[i], j->arena, j->arena_len);
  counters_flush();
  return NULL;
}

static void* item_worker(void* p) {
  job_t* j = (job_t*)p;
  uint64_t chunk = (j->n_items + j->nthreads - 1) / j->nthreads;
  uint64_t b = chunk * j->tid, e = b + chunk < j->n_items ? b + chunk : j->n_items;
  memset(&g_or_counters, 0, sizeof g_or_counters);
  for (uint64_t i = b; i < e; ++i) {
    const cg_item* it = &j->items[i];
    j->status[i] = it->key_idx < j->n_keys
                       ? (uint8_t)verify_with(&j->slots[it->key_idx], it, j->arena, j->arena_len, j->mode)
                       : (uint8_t)CG_NOT_RUN;
  }
  counters_flush();
  return NULL;
}

static int resolve_threads(int n) {
  if (n > 0) return n;
  long c = sysconf(_SC_NPROCESSORS_ONLN);
  return c > 0 ? (int)c : 1;
}

static void run_pool(void* (*fn)(void*), job_t* base, int nthreads) {
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  job_t* jobs = (job_t*)malloc(sizeof(job_t) * nthreads);
  for (int t = 0; t < nthreads; ++t) {
    jobs[t] = *base;
    jobs[t].tid = t;
    pthread_create(&th[t], NULL, fn, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

int or_verify_batch(const cg_key* keys, uint32_t n_keys, const cg_item* items, uint64_t n_items, const uint8_t* arena,
                    uint64_t arena_len, uint32_t mode, uint8_t* status_out, int nthreads) {
  nthreads = resolve_threads(nthreads);
  keyslot* slots = (keyslot*)calloc(n_keys ? n_keys : 1, sizeof(keyslot));
  job_t j = {keys, n_keys, slots, items, n_items, arena, arena_len, mode, status_out, nthreads, 0};
  run_pool(key_worker, &j, nthreads < (int)n_keys ? nthreads : (n_keys ? (int)n_keys : 1));
  j.nthreads = nthreads;
  run_pool(item_worker, &j, nthreads);
  for (uint32_t i = 0; i < n_keys; ++i) free(slots[i].k);
  free(slots);
  return 0;
}

/* ---- TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-61) over a
 * batch of transactions, the BASELINE configs[0] CPU shape: workers take the next transaction from
 * a shared counter (test-utils Injectors.kt:18-55 startTightLoopInjector style); a transaction's
 * signatures are verified in list order through Crypto.doVerify semantics and the loop stops at
 * the first failure (its exception escapes). Each signature's key is decoded with it: the JVM
 * builds a fresh PublicKey object for TransactionSignature.by when it deserialises the
 * SignedTransaction (Kryo.kt:330-339), so nothing is cached across transactions. */
typedef struct {
  const cg_key* keys;
  uint32_t n_keys;
  const cg_item* items;
  const uint64_t* tx_first;
  uint64_t n_tx;
  const uint8_t* arena;
  uint64_t arena_len;
  int64_t* first_fail;
  uint64_t* next;
  uint64_t verified;
} ckjob_t;

static void* ck_worker(void* p) {
  ckjob_t* j = (ckjob_t*)p;
  uint64_t done = 0;
  for (;;) {
    const uint64_t t = __atomic_fetch_add(j->next, 1, __ATOMIC_RELAXED);
    if (t >= j->n_tx) break;
    int64_t ff = -1;
    for (uint64_t i = j->tx_first[t]; i < j->tx_first[t + 1]; ++i) {
      const cg_item* it = &j->items[i];
      const int st = it->key_idx < j->n_keys
                         ? or_verify_item(&j->keys[it->key_idx], it, j->arena, j->arena_len, CG_MODE_DOVERIFY)
                         : CG_NOT_RUN;
      ++done;
      if (st != CG_VALID) {
        ff = (int64_t)(i - j->tx_first[t]);
        break;
      }
    }
    j->first_fail[t] = ff;
  }
  __atomic_fetch_add(&((ckjob_t*)p)->verified, done, __ATOMIC_RELAXED);
  return NULL;
}

uint64_t or_check_txs(const cg_key* keys, uint32_t n_keys, const cg_item* items, const uint64_t* tx_first,
                      uint64_t n_tx, const uint8_t* arena, uint64_t arena_len, int64_t* first_fail, int nthreads) {
  nthreads = resolve_threads(nthreads);
  uint64_t next = 0;
  ckjob_t j = {keys, n_keys, items, tx_first, n_tx, arena, arena_len, first_fail, &next, 0};
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  for (int t = 0; t < nthreads; ++t) pthread_create(&th[t], NULL, ck_worker, &j);
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  return j.verified;
}

/* ---- Merkle ---- */
int or_merkle_root(const uint8_t* leaves, size_t n, uint8_t out[32]) {
  if (n == 0) return -1;
  size_t m = 1;
  while (m < n) m <<= 1;
  uint8_t* lv = (uint8_t*)calloc(m, 32);
  memcpy(lv, leaves, 32 * n);
  while (m > 1) {
    for (size_t i = 0; i < m / 2; ++i) or_sha256(lv + 64 * i, 64, lv + 32 * i);
    m /= 2;
  }
  memcpy(out, lv, 32);
  free(lv);
  return 0;
}

static void nonce(const uint8_t salt[32], uint32_t idx, uint8_t out[32]) {
  uint8_t b[36];
  memcpy(b, salt, 32);
  b[32] = (uint8_t)(idx >> 24); b[33] = (uint8_t)(idx >> 16); b[34] = (uint8_t)(idx >> 8); b[35] = (uint8_t)idx;
  or_sha256(b, 36, out);
}

static void component_hash(const uint8_t* blob, uint32_t len, int is_salt, const uint8_t salt[32], uint32_t idx,
                           uint8_t out[32]) {
  if (is_salt) { or_sha256(blob, len, out); return; }
  uint8_t* buf = (uint8_t*)malloc((size_t)len + 32);
  memcpy(buf, blob, len);
  nonce(salt, idx, buf + len);
  or_sha256(buf, (size_t)len + 32, out);
  free(buf);
}

int or_tx_id(const uint8_t* arena, const uint64_t* comp_offs, const uint32_t* comp_lens, uint32_t n_comp,
             const uint8_t salt[32], const uint8_t* salt_blob, uint32_t salt_blob_len, uint8_t out[32]) {
  uint32_t n = n_comp + 1;
  uint8_t* leaves = (uint8_t*)malloc(32 * (size_t)n);
  for (uint32_t i = 0; i < n_comp; ++i) component_hash(arena + comp_offs[i], comp_lens[i], 0, salt, i, leaves + 32 * i);
  component_hash(salt_blob, salt_blob_len, 1, salt, n_comp, leaves + 32 * n_comp);
  int r = or_merkle_root(leaves, n, out);
  free(leaves);
  return r;
}

typedef struct {
  const cg_tx* txs;
  uint64_t n_tx;
  const cg_component* comps;
  const uint8_t* arena;
  uint8_t* ids;
  int nthreads, tid;
} txjob_t;

static void* tx_worker(void* p) {
  txjob_t* j = (txjob_t*)p;
  memset(&g_or_counters, 0, sizeof g_or_counters);
  for (uint64_t t = (uint64_t)j->tid; t < j->n_tx; t += (uint64_t)j->nthreads) {
    const cg_tx* tx = &j->txs[t];
    if (tx->n == 0) { memset(j->ids + 32 * t, 0, 32); continue; }
    uint8_t* leaves = (uint8_t*)malloc(32 * (size_t)tx->n);
    const uint8_t* salt = j->arena + tx->salt_off;
    for (uint32_t i = 0; i < tx->n; ++i) {
      const cg_component* c = &j->comps[tx->first + i];
      component_hash(j->arena + c->off, c->len, c->flags & 1, salt, i, leaves + 32 * i);
    }
    or_merkle_root(leaves, tx->n, j->ids + 32 * t);
    free(leaves);
  }
  counters_flush();
  return NULL;
}

int or_tx_ids_batch(const cg_tx* txs, uint64_t n_tx, const cg_component* comps, const uint8_t* arena, uint8_t* ids_out,
                    int nthreads) {
  nthreads = resolve_threads(nthreads);
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * nthreads);
  txjob_t* jobs = (txjob_t*)malloc(sizeof(txjob_t) * nthreads);
  for (int t = 0; t < nthreads; ++t) {
    txjob_t j = {txs, n_tx, comps, arena, ids_out, nthreads, t};
    jobs[t] = j;
    pthread_create(&th[t], NULL, tx_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
  return 0;
}
