// core/src/main/kotlin/net/corda/core/crypto/CryptoBatch.kt (new file in the Corda tree).
// The JVM side of libcordagpu.so (include/cordagpu.h) through jvm/jni/cordagpu_jni.c. Not compiled
// in this repository (no JDK / Kotlin compiler in its image); corda_amd/ is the Python mirror of the
// same calls, and the GPU tests drive that mirror.
package net.corda.core.crypto

import net.corda.core.serialization.serialize
import net.corda.core.transactions.SignedTransaction
import java.nio.ByteBuffer
import java.nio.ByteOrder
import java.security.PublicKey
import java.security.SignatureException

data class BatchItem(val publicKey: PublicKey, val signatureData: ByteArray, val clearData: ByteArray)

object CryptoBatch {
    init { System.loadLibrary("cordagpu_jni") }           // links libcordagpu.so

    private external fun nativeOpen(device: Int): Long
    private external fun nativeOpenPool(devices: IntArray): Long
    private external fun nativeVerify(ctx: Long, keys: ByteBuffer, nKeys: Int, items: ByteBuffer, nItems: Long,
                                      arena: ByteBuffer, arenaLen: Long, mode: Int, status: ByteBuffer): Int
    private external fun nativeClose(ctx: Long)
    private external fun nativeVerifyTransactions(ctx: Long, txs: ByteBuffer, nTx: Long, comps: ByteBuffer, nComps: Long,
                                                  keys: ByteBuffer, nKeys: Int, sigs: ByteBuffer, nSigs: Long,
                                                  tmpls: ByteBuffer, nTmpls: Int, arena: ByteBuffer, arenaLen: Long,
                                                  mode: Int, idsOut: ByteBuffer, txStatusOut: ByteBuffer,
                                                  sigStatusOut: ByteBuffer): Int
    private external fun nativeVerifyTxSignatures(ctx: Long, pool: Long, keys: ByteBuffer, nKeys: Int, ids: ByteBuffer,
                                                  nIds: Long, sigs: ByteBuffer, nSigs: Long, tmpls: ByteBuffer,
                                                  nTmpls: Int, arena: ByteBuffer, arenaLen: Long, mode: Int,
                                                  status: ByteBuffer): Int

    const val MODE_DOVERIFY = 0
    const val MODE_ISVALID = 1
    private const val KEY_SPKI = 1

    private val ctxDelegate = lazy { nativeOpen(0) }
    private val ctx: Long by ctxDelegate

    /** Releases the device context (cg_close); a later call opens a new one only in a new process. */
    fun close() { if (ctxDelegate.isInitialized()) nativeClose(ctx) }
    /** Set by a node that drives every GPU from one process: the tx-signature calls then shard over the pool. */
    @Volatile var pool: Long = 0
    fun usePool(devices: IntArray) { pool = nativeOpenPool(devices) }

    private fun direct(n: Int): ByteBuffer = ByteBuffer.allocateDirect(maxOf(n, 1)).order(ByteOrder.LITTLE_ENDIAN)
    private fun ByteBuffer.align4() { while (position() % 4 != 0) put(0) }

    /** cg_key table + arena prefix for the distinct keys, in first-use order. */
    private class Keys(keys: Collection<PublicKey>, arena: ByteBuffer) {
        val index = LinkedHashMap<PublicKey, Int>()
        val table: ByteBuffer
        init {
            keys.forEach { index.getOrPut(it) { index.size } }
            table = ByteBuffer.allocateDirect(16 * maxOf(index.size, 1)).order(ByteOrder.LITTLE_ENDIAN)
            for (k in index.keys) {
                val enc = k.encoded                                   // X.509 SubjectPublicKeyInfo
                arena.align4()
                table.putLong(arena.position().toLong()).putShort(enc.size.toShort())
                    .put(Crypto.findSignatureScheme(k).schemeNumberID.toByte()).put(KEY_SPKI.toByte()).putInt(0)
                arena.put(enc)
            }
        }
    }

    /** Batch overload of Crypto.doVerify / isValid: one status byte per item (include/cordagpu.h). */
    fun verifyBatch(items: List<BatchItem>, mode: Int = MODE_DOVERIFY): ByteArray {
        val arena = direct(items.sumOf { it.signatureData.size + it.clearData.size + 8 } +
                           items.map { it.publicKey }.distinct().sumOf { it.encoded.size + 4 } + 16)
        val keys = Keys(items.map { it.publicKey }, arena)
        val rec = direct(32 * items.size)
        for (it in items) {
            arena.align4()
            val sigOff = arena.position().toLong(); arena.put(it.signatureData)
            arena.align4()
            val msgOff = arena.position().toLong(); arena.put(it.clearData)
            rec.putLong(sigOff).putLong(msgOff).putInt(it.clearData.size).putInt(keys.index[it.publicKey]!!)
               .putShort(it.signatureData.size.toShort()).putShort(0).putInt(0)
        }
        val status = direct(items.size)
        val rc = nativeVerify(ctx, keys.table, keys.index.size, rec, items.size.toLong(), arena,
                              arena.position().toLong(), mode, status)
        check(rc == 0) { "cg_verify_batch failed: $rc" }
        return ByteArray(items.size).also { status.get(it) }
    }

    /** SignableData(id, metadata) = prefix || id || suffix: found by serialising with two ids that
     *  differ in every byte (0^32 and 0xFF^32) and taking the first differing offset, then checking
     *  that the bytes around the id agree (a prefix that happens to end in 0x00, or an earlier run of
     *  zero bytes, cannot shift the split). Mirrors corda_amd/signable.py:template. */
    fun signableTemplate(m: SignatureMetadata): Pair<ByteArray, ByteArray> {
        val a = SignableData(SecureHash.zeroHash, m).serialize().bytes
        val b = SignableData(SecureHash.SHA256(ByteArray(32) { 0xFF.toByte() }), m).serialize().bytes
        check(a.size == b.size) { "SignableData serialisation depends on the id's value" }
        val at = a.indices.first { a[it] != b[it] }
        check(at + 32 <= a.size && (at until at + 32).all { a[it] == 0.toByte() && b[it] == 0xFF.toByte() } &&
              (at + 32 until a.size).all { a[it] == b[it] }) { "id not found as 32 contiguous bytes" }
        return a.copyOfRange(0, at) to a.copyOfRange(at + 32, a.size)
    }

    /** Batch Crypto.doVerify(txId, TransactionSignature) (Crypto.kt:499-502) for every signature of
     *  every transaction, SignableData spliced on the device: one status byte per signature, in order. */
    fun verifyTxSignatures(txs: List<Pair<SecureHash, List<TransactionSignature>>>, mode: Int = MODE_DOVERIFY): ByteArray {
        val all = txs.flatMap { it.second }
        val metas = LinkedHashMap<SignatureMetadata, Int>()
        all.forEach { metas.getOrPut(it.signatureMetadata) { metas.size } }
        val split = metas.keys.map { signableTemplate(it) }
        val arena = direct(all.sumOf { it.bytes.size + 4 } + split.sumOf { it.first.size + it.second.size + 8 } +
                           all.map { it.by }.distinct().sumOf { it.encoded.size + 4 } + 16)
        val keys = Keys(all.map { it.by }, arena)
        val tmpls = direct(24 * split.size)
        for ((pre, suf) in split) {
            arena.align4(); val p = arena.position().toLong(); arena.put(pre)
            arena.align4(); val s = arena.position().toLong(); arena.put(suf)
            tmpls.putLong(p).putLong(s).putInt(pre.size).putInt(suf.size)
        }
        val ids = direct(32 * txs.size)
        val sigs = direct(24 * all.size)
        txs.forEachIndexed { t, (id, list) ->
            ids.put(id.bytes)
            for (sig in list) {
                arena.align4()
                val off = arena.position().toLong(); arena.put(sig.bytes)
                sigs.putLong(off).putInt(t).putInt(keys.index[sig.by]!!).putShort(sig.bytes.size.toShort())
                    .putShort(metas[sig.signatureMetadata]!!.toShort()).putInt(0)
            }
        }
        val status = direct(all.size)
        val rc = nativeVerifyTxSignatures(ctx, pool, keys.table, keys.index.size, ids, txs.size.toLong(), sigs,
                                          all.size.toLong(), tmpls, split.size, arena, arena.position().toLong(),
                                          mode, status)
        check(rc == 0) { "cg_verify_tx_signatures failed: $rc" }
        return ByteArray(all.size).also { status.get(it) }
    }

    /** cg_verify_batch over tables already in the C ABI's layout (the out-of-process verifier's batch
     *  request body, VerifierBatchApi.kt): no re-encoding. One status byte per item. */
    fun verifyPacked(keys: ByteBuffer, nKeys: Int, items: ByteBuffer, nItems: Int, arena: ByteBuffer, arenaLen: Long,
                     mode: Int = MODE_DOVERIFY): ByteArray {
        val status = direct(nItems)
        val rc = nativeVerify(ctx, keys, nKeys, items, nItems.toLong(), arena, arenaLen, mode, status)
        check(rc == 0) { "cg_verify_batch failed: $rc" }
        return ByteArray(nItems).also { status.get(it) }
    }

    /** WireTransaction ids + every signature in one call (cg_verify_transactions, include/cordagpu.h):
     *  the tables are the C ABI's own (cg_tx / cg_component / cg_txsig / cg_signable_tmpl, built by the
     *  out-of-process verifier from the request body it already holds). Fills the 32-byte ids, one
     *  status per transaction (Merkle) and one per signature. */
    fun verifyTransactionsPacked(txs: ByteBuffer, nTx: Long, comps: ByteBuffer, nComps: Long, keys: ByteBuffer,
                                 nKeys: Int, sigs: ByteBuffer, nSigs: Long, tmpls: ByteBuffer, nTmpls: Int,
                                 arena: ByteBuffer, arenaLen: Long, idsOut: ByteBuffer, txStatusOut: ByteBuffer,
                                 sigStatusOut: ByteBuffer, mode: Int = MODE_DOVERIFY) {
        val rc = nativeVerifyTransactions(ctx, txs, nTx, comps, nComps, keys, nKeys, sigs, nSigs, tmpls, nTmpls, arena,
                                          arenaLen, mode, idsOut, txStatusOut, sigStatusOut)
        check(rc == 0) { "cg_verify_transactions failed: $rc" }
    }

    /** Re-raise what the serial Crypto.doVerify would have done for an item; a scheme the GPU does not
     *  run (status 4: RSA / SPHINCS / COMPOSITE) is verified here by the JVM itself. */
    fun raiseForStatus(status: Byte, item: BatchItem) {
        val scheme = Crypto.findSignatureScheme(item.publicKey)
        when (status.toInt() and 0xff) {
            0 -> return
            1 -> throw SignatureException("Signature Verification failed!")
            2 -> throw SignatureException(if (scheme == Crypto.EDDSA_ED25519_SHA512) "signature length is wrong"
                                          else "error decoding signature bytes.")
            3 -> Crypto.decodePublicKey(scheme, item.publicKey.encoded)   // throws the JVM's own key exception
            4 -> { Crypto.doVerify(item.publicKey, item.signatureData, item.clearData); return }  // host fallback
            5 -> throw IllegalArgumentException(if (item.signatureData.isEmpty()) "Signature data is empty!"
                                                else "Clear data is empty, nothing to verify!")
            else -> throw IllegalStateException("signature not verified: re-queue")   // CG_NOT_RUN
        }
    }

    /** TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-61) for many
     *  transactions in one call; the first failure in list order throws what the serial loop threw. */
    fun checkSignaturesAreValidBatch(stxs: List<SignedTransaction>) {
        val st = verifyTxSignatures(stxs.map { it.id to it.sigs })
        var k = 0
        for (stx in stxs) for (sig in stx.sigs) {
            val s = st[k++]
            if (s.toInt() != 0) raiseForStatus(s, BatchItem(sig.by, sig.bytes,
                                               SignableData(stx.id, sig.signatureMetadata).serialize().bytes))
        }
    }
}
