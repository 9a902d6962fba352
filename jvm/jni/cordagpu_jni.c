/* cordagpu_jni.c -- JNI shim between net.corda.core.crypto.CryptoBatch (jvm/src/main/kotlin) and
 * libcordagpu.so (include/cordagpu.h). Plain C, direct ByteBuffers only: the JVM hands over the
 * addresses of its off-heap buffers, the engine copies what it needs and keeps no pointer after a
 * call returns (a buffer passed to cg_host_register stays pinned until cg_host_unregister).
 *
 * Build (on a node with a JDK; this repository's image has none, so it is not compiled here):
 *   gcc -O2 -shared -fPIC -I$JAVA_HOME/include -I$JAVA_HOME/include/linux -Iinclude \
 *       jvm/jni/cordagpu_jni.c -Lcorda_amd -lcordagpu -o libcordagpu_jni.so
 */
#include <jni.h>
#include <stdint.h>
#include <stdio.h>

#include "cordagpu.h"

#define ADDR(b) ((b) ? (*env)->GetDirectBufferAddress(env, (b)) : NULL)

static void throw_state(JNIEnv* env, const char* fn, int rc) {
  char msg[768];
  const char* why = cg_last_error();
  snprintf(msg, sizeof msg, "%s failed (%d): %s", fn, rc, why ? why : "");
  jclass ex = (*env)->FindClass(env, "java/lang/IllegalStateException");
  if (ex) (*env)->ThrowNew(env, ex, msg);
}

static cg_config make_config(jlong chunk_items, jint host_threads, jlong table_bytes_max) {
  cg_config cfg = {0}; /* ABI v2: reserved words must be 0 */
  cfg.chunk_items = (uint64_t)chunk_items;
  cfg.host_threads = (uint32_t)host_threads;
  cfg.table_bytes_max = (uint64_t)table_bytes_max; /* 0: automatic (include/cordagpu.h) */
  return cfg;
}

JNIEXPORT jlong JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeOpen(JNIEnv* env, jobject self, jint dev,
                                                                         jlong chunk_items, jint host_threads,
                                                                         jlong table_bytes_max) {
  cg_config cfg = make_config(chunk_items, host_threads, table_bytes_max);
  cfg.device = dev;
  cg_ctx* ctx = 0;
  int rc = cg_open(&ctx, &cfg);
  if (rc != CG_OK) {
    throw_state(env, "cg_open", rc);
    return 0;
  }
  return (jlong)(intptr_t)ctx;
}

/* Exactly one of ctx / pool is non-zero (CryptoBatch.handles). */
JNIEXPORT void JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeClose(JNIEnv* env, jobject self, jlong ctx,
                                                                          jlong pool) {
  if (ctx) cg_close((cg_ctx*)(intptr_t)ctx);
  if (pool) cg_pool_close((cg_pool*)(intptr_t)pool);
}

/* One JVM process, every GPU of the node: a pool over the device list. */
JNIEXPORT jlong JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeOpenPool(JNIEnv* env, jobject self,
                                                                             jintArray devs, jlong chunk_items,
                                                                             jint host_threads, jlong table_bytes_max) {
  jsize n = (*env)->GetArrayLength(env, devs);
  jint* d = (*env)->GetIntArrayElements(env, devs, 0);
  cg_config cfg = make_config(chunk_items, host_threads, table_bytes_max);
  cg_pool* pool = 0;
  int rc = cg_pool_open(&pool, (const int32_t*)d, (uint32_t)n, &cfg);
  (*env)->ReleaseIntArrayElements(env, devs, d, JNI_ABORT);
  if (rc != CG_OK) {
    throw_state(env, "cg_pool_open", rc);
    return 0;
  }
  return (jlong)(intptr_t)pool;
}

/* Crypto.doVerify / isValid over (key, sig, clear) items: cg_verify_batch; stats: a 56-byte cg_stats.
 * pool != 0: cg_pool_verify_batch, the items sharded over every healthy device of the pool (no
 * per-stage stats then: the stats buffer is left untouched and the binding skips its device timers). */
JNIEXPORT jint JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeVerify(
    JNIEnv* env, jobject self, jlong ctx, jlong pool, jobject keys, jint n_keys, jobject items, jlong n_items,
    jobject arena, jlong arena_len, jint mode, jobject status, jobject stats) {
  if (pool)
    return cg_pool_verify_batch((cg_pool*)(intptr_t)pool, (const cg_key*)ADDR(keys), (uint32_t)n_keys,
                                (const cg_item*)ADDR(items), (uint64_t)n_items, (const uint8_t*)ADDR(arena),
                                (uint64_t)arena_len, (uint32_t)mode, (uint8_t*)ADDR(status), 0);
  return cg_verify_batch((cg_ctx*)(intptr_t)ctx, (const cg_key*)ADDR(keys), (uint32_t)n_keys,
                         (const cg_item*)ADDR(items), (uint64_t)n_items, (const uint8_t*)ADDR(arena),
                         (uint64_t)arena_len, (uint32_t)mode, (uint8_t*)ADDR(status), (cg_stats*)ADDR(stats));
}

/* Crypto.doVerify(txId, TransactionSignature) over many transactions, over the 12-byte signature
 * table and the dense signature stream: cg_verify_tx_signatures_packed (pool != 0:
 * cg_pool_verify_tx_signatures_packed over every device of the pool; no per-stage stats then). */
JNIEXPORT jint JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeVerifyTxSignaturesPacked(
    JNIEnv* env, jobject self, jlong ctx, jlong pool, jobject keys, jint n_keys, jobject ids, jlong n_ids,
    jobject sigs, jlong n_sigs, jobject sig_bytes, jlong sig_bytes_len, jobject tmpls, jint n_tmpls, jobject arena,
    jlong arena_len, jint mode, jobject status, jobject stats) {
  if (pool)
    return cg_pool_verify_tx_signatures_packed((cg_pool*)(intptr_t)pool, (const cg_key*)ADDR(keys), (uint32_t)n_keys,
                                               (const uint8_t*)ADDR(ids), (uint64_t)n_ids,
                                               (const cg_txsig_packed*)ADDR(sigs), (uint64_t)n_sigs,
                                               (const uint8_t*)ADDR(sig_bytes), (uint64_t)sig_bytes_len,
                                               (const cg_signable_tmpl*)ADDR(tmpls), (uint32_t)n_tmpls,
                                               (const uint8_t*)ADDR(arena), (uint64_t)arena_len, (uint32_t)mode,
                                               (uint8_t*)ADDR(status), 0);
  return cg_verify_tx_signatures_packed((cg_ctx*)(intptr_t)ctx, (const cg_key*)ADDR(keys), (uint32_t)n_keys,
                                        (const uint8_t*)ADDR(ids), (uint64_t)n_ids, (const cg_txsig_packed*)ADDR(sigs),
                                        (uint64_t)n_sigs, (const uint8_t*)ADDR(sig_bytes), (uint64_t)sig_bytes_len,
                                        (const cg_signable_tmpl*)ADDR(tmpls), (uint32_t)n_tmpls,
                                        (const uint8_t*)ADDR(arena), (uint64_t)arena_len, (uint32_t)mode,
                                        (uint8_t*)ADDR(status), (cg_stats*)ADDR(stats));
}

/* WireTransaction ids + every signature (cg_verify_transactions; pool != 0: cg_pool_verify_transactions,
 * the whole call on one healthy device, the next one on a device fault). */
JNIEXPORT jint JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeVerifyTransactions(
    JNIEnv* env, jobject self, jlong ctx, jlong pool, jobject txs, jlong n_tx, jobject comps, jlong n_comps,
    jobject keys, jint n_keys, jobject sigs, jlong n_sigs, jobject tmpls, jint n_tmpls, jobject arena, jlong arena_len,
    jint mode, jobject ids_out, jobject tx_status_out, jobject sig_status_out) {
  if (pool)
    return cg_pool_verify_transactions((cg_pool*)(intptr_t)pool, (const cg_tx*)ADDR(txs), (uint64_t)n_tx,
                                       (const cg_component*)ADDR(comps), (uint64_t)n_comps, (const cg_key*)ADDR(keys),
                                       (uint32_t)n_keys, (const cg_txsig*)ADDR(sigs), (uint64_t)n_sigs,
                                       (const cg_signable_tmpl*)ADDR(tmpls), (uint32_t)n_tmpls,
                                       (const uint8_t*)ADDR(arena), (uint64_t)arena_len, (uint32_t)mode,
                                       (uint8_t*)ADDR(ids_out), (uint8_t*)ADDR(tx_status_out),
                                       (uint8_t*)ADDR(sig_status_out), 0);
  return cg_verify_transactions((cg_ctx*)(intptr_t)ctx, (const cg_tx*)ADDR(txs), (uint64_t)n_tx,
                                (const cg_component*)ADDR(comps), (uint64_t)n_comps, (const cg_key*)ADDR(keys),
                                (uint32_t)n_keys, (const cg_txsig*)ADDR(sigs), (uint64_t)n_sigs,
                                (const cg_signable_tmpl*)ADDR(tmpls), (uint32_t)n_tmpls, (const uint8_t*)ADDR(arena),
                                (uint64_t)arena_len, (uint32_t)mode, (uint8_t*)ADDR(ids_out),
                                (uint8_t*)ADDR(tx_status_out), (uint8_t*)ADDR(sig_status_out));
}

/* A direct buffer the node keeps across calls: pinned once (cg_host_register), so its bytes reach
 * every device by DMA without the runtime's CPU staging copy. */
JNIEXPORT jint JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeHostRegister(JNIEnv* env, jobject self,
                                                                               jobject buf, jlong len) {
  return cg_host_register(ADDR(buf), (uint64_t)len);
}

JNIEXPORT jint JNICALL Java_net_corda_core_crypto_CryptoBatch_nativeHostUnregister(JNIEnv* env, jobject self,
                                                                                 jobject buf) {
  return cg_host_unregister(ADDR(buf));
}
