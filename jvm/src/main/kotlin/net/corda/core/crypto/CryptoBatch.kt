// core/src/main/kotlin/net/corda/core/crypto/CryptoBatch.kt (new file in the Corda tree).
// The JVM side of libcordagpu.so (include/cordagpu.h) through jvm/jni/cordagpu_jni.c. Not compiled
// in this repository (no JDK / Kotlin compiler in its image); corda_amd/ is the Python mirror of the
// same calls, and the GPU tests drive that mirror. tests/test_jvm_binding.py checks this file's
// status mapping, packing constants and config keys against the Python mirror and the C header.
package net.corda.core.crypto

import com.codahale.metrics.Gauge
import com.codahale.metrics.MetricRegistry
import com.typesafe.config.Config
import net.corda.core.serialization.serialize
import net.corda.core.transactions.SignedTransaction
import java.nio.ByteBuffer
import java.nio.ByteOrder
import java.security.InvalidKeyException
import java.security.PublicKey
import java.security.SignatureException
import java.util.concurrent.TimeUnit
import java.util.concurrent.atomic.AtomicInteger
import java.util.concurrent.locks.ReentrantReadWriteLock
import kotlin.concurrent.read
import kotlin.concurrent.write

data class BatchItem(val publicKey: PublicKey, val signatureData: ByteArray, val clearData: ByteArray)

/**
 * The engine's node.conf block (INTEGRATION.md §5), beside the reference's verifierType
 * (NodeConfiguration.kt:33,98-101):
 *
 *   gpuVerifier { devices = [0, 1, 2, 3, 4, 5, 6, 7], minBatch = 4096, chunkItems = 0, hostThreads = 0,
 *                 tableBytesMax = 0 }
 *
 * devices: HIP ordinals this process drives (one: a cg_ctx; several: a cg_pool sharding every batch:
 *   every entry point works with either, see CryptoBatch.withHandles).
 * minBatch: batches with fewer signatures than this never leave the JVM (Crypto.doVerify per
 *   signature, the reference's own serial path): a GPU call has a fixed cost of a few ms.
 * chunkItems: cg_config.chunk_items (0: the library's default).
 * hostThreads: cg_config.host_threads, host threads of this process's scans (0: the cgroup CPU quota
 *   divided by the contexts the process opens).
 * tableBytesMax: cg_config.table_bytes_max, HBM per device for the constant fixed-base tables (0:
 *   automatic: ~91 GB when the device has room, ~25 / ~6.9 GB when other processes share it; a node
 *   that runs several verifier processes per GPU sets e.g. 26000000000).
 */
data class GpuVerifierConfig(val devices: IntArray = intArrayOf(0), val minBatch: Int = 4096,
                             val chunkItems: Long = 0, val hostThreads: Int = 0, val tableBytesMax: Long = 0) {
    init {
        require(devices.isNotEmpty() && devices.all { it >= 0 }) { "gpuVerifier.devices: at least one ordinal >= 0" }
        require(minBatch >= 0 && chunkItems >= 0 && hostThreads >= 0 && tableBytesMax >= 0) { "gpuVerifier: negative setting" }
    }

    companion object {
        fun fromConfig(c: Config): GpuVerifierConfig {
            val g = c.getConfig("gpuVerifier")
            fun <T> opt(key: String, get: (String) -> T, def: T) = if (g.hasPath(key)) get(key) else def
            return GpuVerifierConfig(
                devices = opt("devices", { g.getIntList(it).toIntArray() }, intArrayOf(0)),
                minBatch = opt("minBatch", g::getInt, 4096),
                chunkItems = opt("chunkItems", g::getLong, 0L),
                hostThreads = opt("hostThreads", g::getInt, 0),
                tableBytesMax = opt("tableBytesMax", g::getLong, 0L))
        }
    }
}

object CryptoBatch {
    init { System.loadLibrary("cordagpu_jni") }           // links libcordagpu.so

    private external fun nativeOpen(device: Int, chunkItems: Long, hostThreads: Int, tableBytesMax: Long): Long
    private external fun nativeOpenPool(devices: IntArray, chunkItems: Long, hostThreads: Int, tableBytesMax: Long): Long
    private external fun nativeClose(ctx: Long, pool: Long)
    private external fun nativeVerify(ctx: Long, pool: Long, keys: ByteBuffer, nKeys: Int, items: ByteBuffer, nItems: Long,
                                      arena: ByteBuffer, arenaLen: Long, mode: Int, status: ByteBuffer,
                                      stats: ByteBuffer): Int
    private external fun nativeVerifyTransactions(ctx: Long, pool: Long, txs: ByteBuffer, nTx: Long, comps: ByteBuffer, nComps: Long,
                                                  keys: ByteBuffer, nKeys: Int, sigs: ByteBuffer, nSigs: Long,
                                                  tmpls: ByteBuffer, nTmpls: Int, arena: ByteBuffer, arenaLen: Long,
                                                  mode: Int, idsOut: ByteBuffer, txStatusOut: ByteBuffer,
                                                  sigStatusOut: ByteBuffer): Int
    /** cg_(pool_)verify_tx_signatures_packed: the 12-byte table (cg_txsig_packed: tx_idx, key_idx,
     *  sig_len, tmpl) and the signatures back to back, each at a 4-byte boundary, in their own buffer
     *  (round 6; the 24-byte cg_txsig form shipped ~12 B more per signature). */
    private external fun nativeVerifyTxSignaturesPacked(ctx: Long, pool: Long, keys: ByteBuffer, nKeys: Int,
                                                        ids: ByteBuffer, nIds: Long, sigs: ByteBuffer, nSigs: Long,
                                                        sigBytes: ByteBuffer, sigBytesLen: Long, tmpls: ByteBuffer,
                                                        nTmpls: Int, arena: ByteBuffer, arenaLen: Long, mode: Int,
                                                        status: ByteBuffer, stats: ByteBuffer): Int
    /** cg_host_register / cg_host_unregister: a direct buffer the node keeps for many calls, pinned
     *  once so that its bytes reach the device by DMA without the runtime's CPU staging copy. */
    private external fun nativeHostRegister(buf: ByteBuffer, len: Long): Int
    private external fun nativeHostUnregister(buf: ByteBuffer): Int

    const val MODE_DOVERIFY = 0
    const val MODE_ISVALID = 1
    private const val KEY_SPKI = 1

    // include/cordagpu.h per-item verdicts
    const val CG_VALID = 0
    const val CG_INVALID = 1
    const val CG_SIG_MALFORMED = 2
    const val CG_KEY_INVALID = 3
    const val CG_UNSUPPORTED = 4
    const val CG_EMPTY = 5
    const val CG_NOT_RUN = 255
    // include/cordagpu.h return codes
    private const val CG_OK = 0
    private const val CG_ERR_DEVICE = -2

    // cg_item.sig_len / cg_txsig.sig_len are 16-bit. A longer JVM signature is packed as a short
    // surrogate with the verdict the JVM gives the real bytes (corda_amd/batch.py sig_field):
    // Ed25519: length != 64 -> SIG_MALFORMED; ECDSA: a canonical SEQUENCE{INTEGER, INTEGER} has an
    // INTEGER of 32k+ content bytes, out of [1, n-1] -> INVALID; anything else fails BC's decode.
    const val SIG_LEN_MAX = 0xFFFF
    private val SIG_SURROGATE_MALFORMED = byteArrayOf(0x00)
    private val SIG_SURROGATE_INVALID = byteArrayOf(0x30, 0x06, 0x02, 0x01, 0x00, 0x02, 0x01, 0x01)

    // cg_stats: n_items, n_keys (u64), ms_h2d, ms_key_prep, ms_verify, ms_d2h, ms_total (f64)
    private const val STATS_BYTES = 56

    @Volatile private var config = GpuVerifierConfig()
    // the native handles (exactly one non-zero while open: ctx for one device, pool for several). Every
    // native call holds the read lock from reading them until it returns; open and close() take the
    // write lock, so close() waits for the calls in flight and never frees a handle under one (ADVICE r5)
    private val rw = ReentrantReadWriteLock()
    private var ctx: Long = 0
    private var pool: Long = 0

    // Metrics named like the reference's verifier service (OutOfProcessTransactionVerifierService.kt:35-46)
    private fun metric(name: String) = "CryptoBatch.$name"
    @Volatile private var metrics: MetricRegistry? = null
    private val inFlight = AtomicInteger(0)

    /** Applies node.conf's gpuVerifier block; takes effect at the next open (close() first to re-open). */
    fun configure(c: GpuVerifierConfig) { config = c }

    /** Feeds a node's MetricRegistry: a timer per batch, success / failure meters per signature, the
     *  batches in flight, and the device's stage times from cg_stats. */
    fun registerMetrics(registry: MetricRegistry) {
        registry.register(metric("VerificationsInFlight"), Gauge { inFlight.get() })
        metrics = registry
    }

    /** Runs one native call with the open handles (ctx, pool), opening them on first use, under the
     *  read lock: close() cannot free them until the call has returned. Every entry point calls the
     *  engine through here, whichever of ctx (one device) / pool (several) is open. */
    private inline fun <T> withHandles(call: (Long, Long) -> T): T {
        while (true) {
            rw.read { if (ctx != 0L || pool != 0L) return call(ctx, pool) }
            rw.write {
                if (ctx == 0L && pool == 0L) {
                    val c = config
                    if (c.devices.size == 1) ctx = nativeOpen(c.devices[0], c.chunkItems, c.hostThreads, c.tableBytesMax)
                    else pool = nativeOpenPool(c.devices, c.chunkItems, c.hostThreads, c.tableBytesMax)
                }
            }
        }
    }

    /** Releases the device context / pool (cg_close / cg_pool_close) once the calls in flight have
     *  returned (write lock). A later call opens a new one. */
    fun close() {
        rw.write {
            if (ctx != 0L || pool != 0L) nativeClose(ctx, pool)
            ctx = 0
            pool = 0
        }
    }

    /** The C ABI's failure contract (include/cordagpu.h): CG_ERR_DEVICE leaves exactly the items no
     *  device could run as CG_NOT_RUN (a pool has already re-run a failed device's shard on the healthy
     *  ones). Those items, and only those, go to the engine once more through `rerun` (given their
     *  indices, it returns their new statuses); what is still NOT_RUN after that stays NOT_RUN, and
     *  raiseForStatus verifies it with the JVM's own Crypto.doVerify. Any other non-zero code is the
     *  caller's input, not the device: thrown. Never throws for the whole batch on a device fault. */
    private fun requeueNotRun(rc: Int, what: String, status: ByteArray, rerun: ((IntArray) -> ByteArray)?) {
        if (rc == CG_OK) return
        check(rc == CG_ERR_DEVICE) { "$what failed: $rc" }
        val todo = status.indices.filter { (status[it].toInt() and 0xff) == CG_NOT_RUN }.toIntArray()
        if (todo.isEmpty() || rerun == null) return
        val again = try { rerun(todo) } catch (e: IllegalStateException) { return }   // still no device: stay NOT_RUN
        for ((k, i) in todo.withIndex()) status[i] = again[k]
    }

    private inline fun <T> timed(n: Int, body: () -> T): T {
        val m = metrics
        val t = m?.timer(metric("Verification.Duration"))?.time()
        inFlight.incrementAndGet()
        try {
            return body()
        } finally {
            inFlight.decrementAndGet()
            t?.stop()
            m?.meter(metric("Verification.Signatures"))?.mark(n.toLong())
        }
    }

    private fun record(stats: ByteBuffer, status: ByteArray) {
        val m = metrics ?: return
        val ok = status.count { it.toInt() == CG_VALID }
        m.meter(metric("Verification.Success")).mark(ok.toLong())
        m.meter(metric("Verification.Failure")).mark((status.size - ok).toLong())
        // a pool call fills no cg_stats (n_items stays 0): no device stage times to report (ADVICE r5)
        if (stats.getLong(0) == 0L) return
        val names = arrayOf("Device.H2D", "Device.KeyPrep", "Device.Verify", "Device.D2H", "Device.Total")
        for ((i, n) in names.withIndex())
            m.timer(metric(n)).update((stats.getDouble(16 + 8 * i) * 1e6).toLong(), TimeUnit.NANOSECONDS)
    }

    private fun direct(n: Int): ByteBuffer = ByteBuffer.allocateDirect(maxOf(n, 1)).order(ByteOrder.LITTLE_ENDIAN)
    private fun ByteBuffer.align4() { while (position() % 4 != 0) put(0) }

    /** The bytes to pack for a signature: itself, or its surrogate past the 16-bit length field. */
    fun sigField(scheme: SignatureScheme, sig: ByteArray): ByteArray = when {
        sig.size <= SIG_LEN_MAX -> sig
        (scheme == Crypto.ECDSA_SECP256K1_SHA256 || scheme == Crypto.ECDSA_SECP256R1_SHA256) && derIsTwoIntegers(sig) ->
            SIG_SURROGATE_INVALID
        else -> SIG_SURROGATE_MALFORMED
    }

    /** (length, next index) of a minimal definite DER length at b[i], or null (batch.py _der_len_at). */
    private fun derLenAt(b: ByteArray, i: Int): Pair<Int, Int>? {
        if (i >= b.size) return null
        val l0 = b[i].toInt() and 0xff
        if (l0 < 0x80) return l0 to i + 1
        val nb = l0 and 0x7f
        if (nb == 0 || nb > 4 || i + 1 + nb > b.size || b[i + 1].toInt() == 0) return null
        var v = 0L
        for (k in 0 until nb) v = (v shl 8) or (b[i + 1 + k].toLong() and 0xff)
        if (v < 0x80 || v > Int.MAX_VALUE) return null
        return v.toInt() to i + 1 + nb
    }

    /** Exactly the canonical DER of SEQUENCE{INTEGER, INTEGER} (batch.py der_is_two_integers). */
    fun derIsTwoIntegers(b: ByteArray): Boolean {
        if (b.size < 2 || b[0].toInt() != 0x30) return false
        val r = derLenAt(b, 1) ?: return false
        if (r.second.toLong() + r.first != b.size.toLong()) return false
        var i = r.second
        var n = 0
        while (i < b.size) {
            if (b[i].toInt() != 0x02) return false
            val (ln, j) = derLenAt(b, i + 1) ?: return false
            if (ln == 0 || j.toLong() + ln > b.size) return false
            if (ln > 1) {
                val b0 = b[j].toInt() and 0xff
                val b1 = b[j + 1].toInt() and 0xff
                if ((b0 == 0 && b1 < 0x80) || (b0 == 0xff && b1 >= 0x80)) return false
            }
            i = j + ln
            n++
        }
        return n == 2
    }

    /** cg_key table + arena prefix for the distinct keys, in first-use order. */
    private class Keys(keys: Collection<PublicKey>, arena: ByteBuffer) {
        val index = LinkedHashMap<PublicKey, Int>()
        val schemes = ArrayList<SignatureScheme>()
        val table: ByteBuffer
        init {
            keys.forEach { index.getOrPut(it) { index.size } }
            table = ByteBuffer.allocateDirect(16 * maxOf(index.size, 1)).order(ByteOrder.LITTLE_ENDIAN)
            for (k in index.keys) {
                val scheme = Crypto.findSignatureScheme(k)
                schemes.add(scheme)
                // cg_key.len is 16-bit; no key of a GPU scheme is that long, so one byte (which fails
                // to decode, as the real key would) stands in (batch.py Builder.key)
                val enc = k.encoded.let { if (it.size > SIG_LEN_MAX) byteArrayOf(0) else it }
                arena.align4()
                table.putLong(arena.position().toLong()).putShort(enc.size.toShort())
                    .put(scheme.schemeNumberID.toByte()).put(KEY_SPKI.toByte()).putInt(0)
                arena.put(enc)
            }
        }
    }

    /** Batch overload of Crypto.doVerify / isValid: one status byte per item (include/cordagpu.h).
     *  One device or several (the pool shards the items); on a device fault the items left NOT_RUN are
     *  re-queued once (requeueNotRun), and any still NOT_RUN reach the caller as NOT_RUN. */
    fun verifyBatch(items: List<BatchItem>, mode: Int = MODE_DOVERIFY): ByteArray = timed(items.size) {
        verifyItems(items, mode, requeue = true)
    }

    private fun verifyItems(items: List<BatchItem>, mode: Int, requeue: Boolean): ByteArray {
        val arena = direct(items.sumOf { minOf(it.signatureData.size, SIG_LEN_MAX) + it.clearData.size + 8 } +
                           items.map { it.publicKey }.distinct().sumOf { it.encoded.size + 4 } + 16)
        val keys = Keys(items.map { it.publicKey }, arena)
        val rec = direct(32 * items.size)
        for (it in items) {
            val ki = keys.index[it.publicKey]!!
            val sig = sigField(keys.schemes[ki], it.signatureData)
            arena.align4()
            val sigOff = arena.position().toLong(); arena.put(sig)
            arena.align4()
            val msgOff = arena.position().toLong(); arena.put(it.clearData)
            rec.putLong(sigOff).putLong(msgOff).putInt(it.clearData.size).putInt(ki)
               .putShort(sig.size.toShort()).putShort(0).putInt(0)
        }
        val status = direct(items.size)
        val stats = direct(STATS_BYTES)
        val rc = withHandles { c, p ->
            nativeVerify(c, p, keys.table, keys.index.size, rec, items.size.toLong(), arena, arena.position().toLong(),
                         mode, status, stats)
        }
        val st = ByteArray(items.size).also { status.get(it) }
        requeueNotRun(rc, "cg_verify_batch", st,
                      if (requeue) { todo -> verifyItems(todo.map { items[it] }, mode, requeue = false) } else null)
        record(stats, st)
        return st
    }

    /** Crypto.doVerify for every item, throwing what the first failing item's serial call throws.
     *  Below gpuVerifier.minBatch the items never leave the JVM. */
    fun doVerifyAll(items: List<BatchItem>) {
        if (items.size < config.minBatch) {
            for (it in items) Crypto.doVerify(it.publicKey, it.signatureData, it.clearData)
            return
        }
        val st = verifyBatch(items, MODE_DOVERIFY)
        for ((i, it) in items.withIndex()) if (st[i].toInt() != CG_VALID) raiseForStatus(st[i], it)
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
     *  every transaction, SignableData spliced on the device: one status byte per signature, in order.
     *  With several devices configured the call shards over the pool (cg_pool_verify_tx_signatures). On
     *  a device fault only the signatures left NOT_RUN are re-queued (requeueNotRun). */
    fun verifyTxSignatures(txs: List<Pair<SecureHash, List<TransactionSignature>>>, mode: Int = MODE_DOVERIFY): ByteArray {
        val all = txs.flatMap { it.second }
        return timed(all.size) { verifySigs(txs, mode, requeue = true) }
    }

    private fun verifySigs(txs: List<Pair<SecureHash, List<TransactionSignature>>>, mode: Int, requeue: Boolean): ByteArray {
        val all = txs.flatMap { it.second }
        val metas = LinkedHashMap<SignatureMetadata, Int>()
        all.forEach { metas.getOrPut(it.signatureMetadata) { metas.size } }
        val split = metas.keys.map { signableTemplate(it) }
        // arena: key and template bytes; the signatures go to their own stream (cg_txsig_packed, round 6:
        // 12 bytes of table per signature instead of the 24-byte cg_txsig, no offsets)
        val arena = direct(split.sumOf { it.first.size + it.second.size + 8 } +
                           all.map { it.by }.distinct().sumOf { it.encoded.size + 4 } + 16)
        val keys = Keys(all.map { it.by }, arena)
        val tmpls = direct(24 * split.size)
        for ((pre, suf) in split) {
            arena.align4(); val p = arena.position().toLong(); arena.put(pre)
            arena.align4(); val s = arena.position().toLong(); arena.put(suf)
            tmpls.putLong(p).putLong(s).putInt(pre.size).putInt(suf.size)
        }
        val ids = direct(32 * txs.size)
        val sigs = direct(12 * all.size)
        val stream = direct(all.sumOf { minOf(it.bytes.size, SIG_LEN_MAX) + 4 })
        txs.forEachIndexed { t, (id, list) ->
            ids.put(id.bytes)
            for (sig in list) {
                val ki = keys.index[sig.by]!!
                val bytes = sigField(keys.schemes[ki], sig.bytes)
                stream.put(bytes).align4()          // signature i at the 4-byte-aligned end of signature i - 1
                sigs.putInt(t).putInt(ki).putShort(bytes.size.toShort())
                    .putShort(metas[sig.signatureMetadata]!!.toShort())
            }
        }
        val status = direct(all.size)
        val stats = direct(STATS_BYTES)
        val rc = withHandles { c, p ->
            nativeVerifyTxSignaturesPacked(c, p, keys.table, keys.index.size, ids, txs.size.toLong(), sigs,
                                           all.size.toLong(), stream, stream.position().toLong(), tmpls, split.size,
                                           arena, arena.position().toLong(), mode, status, stats)
        }
        val st = ByteArray(all.size).also { status.get(it) }
        // the re-queue: the NOT_RUN signatures, each as a one-signature transaction of its own id
        val owner = txs.flatMap { (id, list) -> list.map { id to it } }
        requeueNotRun(rc, "cg_verify_tx_signatures_packed", st,
                      if (requeue) { todo -> verifySigs(todo.map { owner[it].first to listOf(owner[it].second) }, mode, false) }
                      else null)
        record(stats, st)
        return st
    }

    /** cg_verify_batch over tables already in the C ABI's layout (the out-of-process verifier's batch
     *  request body, VerifierBatchApi.kt): no re-encoding. One status byte per item; one device or a
     *  pool. On a device fault the NOT_RUN items' records are re-queued once as a table of their own
     *  (same keys and arena); any still NOT_RUN go back to the node as NOT_RUN. */
    fun verifyPacked(keys: ByteBuffer, nKeys: Int, items: ByteBuffer, nItems: Int, arena: ByteBuffer, arenaLen: Long,
                     mode: Int = MODE_DOVERIFY): ByteArray = timed(nItems) {
        require(nKeys >= 0 && nItems >= 0 && arenaLen >= 0) { "negative table size" }
        require(keys.capacity().toLong() >= 16L * nKeys && items.capacity().toLong() >= 32L * nItems &&
                arena.capacity().toLong() >= arenaLen) { "a table is shorter than its count" }
        verifyPackedItems(keys, nKeys, items, nItems, arena, arenaLen, mode, requeue = true)
    }

    private fun verifyPackedItems(keys: ByteBuffer, nKeys: Int, items: ByteBuffer, nItems: Int, arena: ByteBuffer,
                                  arenaLen: Long, mode: Int, requeue: Boolean): ByteArray {
        val status = direct(nItems)
        val stats = direct(STATS_BYTES)
        val rc = withHandles { c, p -> nativeVerify(c, p, keys, nKeys, items, nItems.toLong(), arena, arenaLen, mode, status, stats) }
        val st = ByteArray(nItems).also { status.get(it) }
        requeueNotRun(rc, "cg_verify_batch", st, if (!requeue) null else { todo ->
            val sub = direct(32 * todo.size)
            val rec = ByteArray(32)
            for (i in todo) { items.duplicate().apply { position(32 * i) }.get(rec); sub.put(rec) }
            verifyPackedItems(keys, nKeys, sub, todo.size, arena, arenaLen, mode, requeue = false)
        })
        record(stats, st)
        return st
    }

    /** WireTransaction ids + every signature in one call (cg_verify_transactions, include/cordagpu.h):
     *  the tables are the C ABI's own (cg_tx / cg_component / cg_txsig / cg_signable_tmpl, built by the
     *  out-of-process verifier from the request body it already holds). Fills the 32-byte ids, one
     *  status per transaction (Merkle) and one per signature. With a pool the call runs whole on one
     *  healthy device and fails over to the next (cg_pool_verify_transactions: a signature may reference
     *  any transaction's id, so it is not sharded). When no device could run it the signatures stay
     *  NOT_RUN and the ids are not computed: IllegalStateException, the request is redelivered whole. */
    fun verifyTransactionsPacked(txs: ByteBuffer, nTx: Long, comps: ByteBuffer, nComps: Long, keys: ByteBuffer,
                                 nKeys: Int, sigs: ByteBuffer, nSigs: Long, tmpls: ByteBuffer, nTmpls: Int,
                                 arena: ByteBuffer, arenaLen: Long, idsOut: ByteBuffer, txStatusOut: ByteBuffer,
                                 sigStatusOut: ByteBuffer, mode: Int = MODE_DOVERIFY) {
        val rc = withHandles { c, p ->
            nativeVerifyTransactions(c, p, txs, nTx, comps, nComps, keys, nKeys, sigs, nSigs, tmpls, nTmpls, arena,
                                     arenaLen, mode, idsOut, txStatusOut, sigStatusOut)
        }
        check(rc == CG_OK) { "cg_verify_transactions failed: $rc (no device could run it: redeliver the request)" }
    }

    /** Pins a direct buffer the caller keeps across calls (cg_host_register); unregister before freeing it. */
    fun registerHostBuffer(buf: ByteBuffer) {
        require(buf.isDirect) { "only a direct buffer can be registered" }
        check(nativeHostRegister(buf, buf.capacity().toLong()) == 0) { "cg_host_register failed" }
    }
    fun unregisterHostBuffer(buf: ByteBuffer) { check(nativeHostUnregister(buf) == 0) { "cg_host_unregister failed" } }

    /** Re-raise what the serial Crypto.doVerify would have done for an item. Fails closed: every
     *  status but CG_VALID ends in a throw, or in the JVM's own doVerify (which throws or returns as the
     *  serial call does) for a scheme the GPU does not run. Mapping (INTEGRATION.md §2):
     *    1 INVALID       SignatureException("Signature Verification failed!")      Crypto.kt:478-483
     *    2 SIG_MALFORMED SignatureException (the engine's decode message)
     *    3 KEY_INVALID   the JVM decoder's own exception, else InvalidKeyException
     *    4 UNSUPPORTED   Crypto.doVerify on the host (RSA / SPHINCS / COMPOSITE)
     *    5 EMPTY         IllegalArgumentException (Crypto.kt:476-477)
     *  255 NOT_RUN       no device ran it (after the re-queue): Crypto.doVerify on the host, as UNSUPPORTED
     *    other           IllegalStateException (not a status the engine writes) */
    fun raiseForStatus(status: Byte, item: BatchItem) {
        val scheme = Crypto.findSignatureScheme(item.publicKey)
        when (status.toInt() and 0xff) {
            CG_VALID -> return
            CG_INVALID -> throw SignatureException("Signature Verification failed!")
            CG_SIG_MALFORMED -> throw SignatureException(if (scheme == Crypto.EDDSA_ED25519_SHA512) "signature length is wrong"
                                                         else "error decoding signature bytes.")
            CG_KEY_INVALID -> {
                Crypto.decodePublicKey(scheme, item.publicKey.encoded)   // throws the JVM's own key exception
                throw InvalidKeyException("public key rejected by the batch engine: ${scheme.schemeCodeName}")
            }
            CG_UNSUPPORTED -> { Crypto.doVerify(item.publicKey, item.signatureData, item.clearData); return }
            CG_NOT_RUN -> { Crypto.doVerify(item.publicKey, item.signatureData, item.clearData); return }
            CG_EMPTY -> throw IllegalArgumentException(if (item.signatureData.isEmpty()) "Signature data is empty!"
                                                      else "Clear data is empty, nothing to verify!")
            else -> throw IllegalStateException("unknown engine status $status")
        }
    }

    /** TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-61) for many
     *  transactions in one call; the first failure in list order throws what the serial loop threw.
     *  Below gpuVerifier.minBatch signatures the reference's serial loop runs unchanged. */
    fun checkSignaturesAreValidBatch(stxs: List<SignedTransaction>) {
        if (stxs.sumOf { it.sigs.size } < config.minBatch) {
            for (stx in stxs) for (sig in stx.sigs) sig.verify(stx.id)
            return
        }
        val st = verifyTxSignatures(stxs.map { it.id to it.sigs })
        var k = 0
        for (stx in stxs) for (sig in stx.sigs) {
            val s = st[k++]
            if (s.toInt() != CG_VALID) raiseForStatus(s, BatchItem(sig.by, sig.bytes,
                                                      SignableData(stx.id, sig.signatureMetadata).serialize().bytes))
        }
    }
}
