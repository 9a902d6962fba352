// node-api/src/main/kotlin/net/corda/nodeapi/VerifierBatchApi.kt (new file in the Corda tree), beside
// VerifierApi (VerifierApi.kt:10-58): the batch-signature request / response pair of the out-of-process
// verifier. The body is the C ABI's own tables (include/cordagpu.h cg_key / cg_item / arena) behind a
// fixed little-endian header, so the verifier hands slices of it to cg_verify_batch without
// re-encoding. The wire format is the one corda_amd/verifier.py implements and tests/test_verifier.py
// checks (INTEGRATION.md §4). Not compiled in this repository (no JDK / Kotlin compiler in its image).
package net.corda.nodeapi

import org.apache.activemq.artemis.api.core.SimpleString
import org.apache.activemq.artemis.api.core.client.ClientMessage
import org.apache.activemq.artemis.reader.MessageUtil
import java.nio.ByteBuffer
import java.nio.ByteOrder

object VerifierBatchApi {
    /** Message property that marks a batch-signature request on VERIFICATION_REQUESTS_QUEUE_NAME. */
    const val BATCH_SIGNATURES_FIELD_NAME = "batch-signatures"
    private const val VERIFICATION_ID_FIELD_NAME = "id"          // the property VerifierApi uses
    private const val REQ_MAGIC = 0x51424743                       // "CGBQ" little-endian
    private const val RSP_MAGIC = 0x52424743                       // "CGBR"
    private const val VERSION: Short = 1
    const val REQ_HEADER = 40                                      // <4sHHqIIQQ
    const val RSP_HEADER = 28                                      // <4sHHqQI
    const val KEY_BYTES = 16                                       // sizeof(cg_key)
    const val ITEM_BYTES = 32                                      // sizeof(cg_item)

    class MalformedMessage(msg: String) : IllegalArgumentException(msg)

    /** keys / items / arena are the cg_key / cg_item tables and the byte arena they index. */
    class BatchSignatureRequest(val verificationId: Long, val mode: Int, val nKeys: Int, val nItems: Int,
                                val body: ByteBuffer, val responseAddress: SimpleString?) {
        /** Direct-buffer slices of the body in the C ABI layout (for CryptoBatch.verifyPacked). Offsets
         *  and lengths in Long, each checked to fit the body (parse() has checked that they add up). */
        fun keys(): ByteBuffer = slice(REQ_HEADER.toLong(), nKeys.toLong() * KEY_BYTES)
        fun items(): ByteBuffer = slice(REQ_HEADER + nKeys.toLong() * KEY_BYTES, nItems.toLong() * ITEM_BYTES)
        fun arena(): ByteBuffer = slice(REQ_HEADER + nKeys.toLong() * KEY_BYTES + nItems.toLong() * ITEM_BYTES, arenaLen())
        fun arenaLen(): Long = body.getLong(32)

        private fun slice(off: Long, len: Long): ByteBuffer {
            if (off < 0 || len < 0 || off + len > body.limit()) throw MalformedMessage("slice outside the body")
            val d = body.duplicate()
            d.position(Math.toIntExact(off)).limit(Math.toIntExact(off + len))
            return d.slice().order(ByteOrder.LITTLE_ENDIAN)
        }

        fun writeToClientMessage(message: ClientMessage) {
            message.putLongProperty(VERIFICATION_ID_FIELD_NAME, verificationId)
            message.putBooleanProperty(BATCH_SIGNATURES_FIELD_NAME, true)
            val bytes = ByteArray(body.limit())
            body.duplicate().apply { position(0) }.get(bytes)
            message.writeBodyBufferBytes(bytes)
            if (responseAddress != null) MessageUtil.setJMSReplyTo(message, responseAddress)
        }

        companion object {
            fun isBatch(message: ClientMessage): Boolean =
                message.containsProperty(BATCH_SIGNATURES_FIELD_NAME)

            /** Parses and checks the header against the body length (a request that does not add up
             *  is answered with an error, never with statuses). The body lands in a direct buffer. */
            fun fromClientMessage(message: ClientMessage): BatchSignatureRequest {
                val raw = ByteArray(message.bodySize).apply { message.bodyBuffer.readBytes(this) }
                val body = ByteBuffer.allocateDirect(raw.size).order(ByteOrder.LITTLE_ENDIAN).put(raw)
                body.flip()
                return parse(body, MessageUtil.getJMSReplyTo(message))
            }

            fun parse(body: ByteBuffer, replyTo: SimpleString?): BatchSignatureRequest {
                if (body.limit() < REQ_HEADER) throw MalformedMessage("short request header")
                if (body.getInt(0) != REQ_MAGIC || body.getShort(4) != VERSION)
                    throw MalformedMessage("not a batch-signature request")
                val mode = body.getShort(6).toInt()
                if (mode != 0 && mode != 1) throw MalformedMessage("unknown mode $mode")
                val id = body.getLong(8)
                // the header's counts are unsigned (verifier.py <4sHHqIIQQ): n_keys u32, n_items and
                // arena_len u64. A u64 with the top bit set reads as a negative Long here: rejected,
                // as is any count whose table could not fit a body (a ByteBuffer holds < 2^31 bytes),
                // so the sum below cannot wrap and every slice lies inside the body
                val nKeys = body.getInt(16).toLong() and 0xffffffffL
                val nItems = body.getLong(24)
                val arenaLen = body.getLong(32)
                if (nItems < 0 || arenaLen < 0 || nKeys > Int.MAX_VALUE / KEY_BYTES ||
                    nItems > Int.MAX_VALUE / ITEM_BYTES || arenaLen > Int.MAX_VALUE)
                    throw MalformedMessage("a header count is out of range")
                if (body.limit().toLong() != REQ_HEADER + nKeys * KEY_BYTES + nItems * ITEM_BYTES + arenaLen)
                    throw MalformedMessage("body length does not match the header")
                return BatchSignatureRequest(id, mode, nKeys.toInt(), nItems.toInt(), body, replyTo)
            }
        }
    }

    /** status: one byte per item (CG_VALID ... CG_NOT_RUN); error: request-level failure, no statuses. */
    class BatchSignatureResponse(val verificationId: Long, val status: ByteArray, val error: String?) {
        fun writeToClientMessage(message: ClientMessage) {
            val err = error?.toByteArray(Charsets.UTF_8) ?: ByteArray(0)
            val b = ByteBuffer.allocate(RSP_HEADER + status.size + err.size).order(ByteOrder.LITTLE_ENDIAN)
            b.putInt(RSP_MAGIC).putShort(VERSION).putShort(0).putLong(verificationId).putLong(status.size.toLong())
                .putInt(err.size).put(status).put(err)
            message.putLongProperty(VERIFICATION_ID_FIELD_NAME, verificationId)
            message.putBooleanProperty(BATCH_SIGNATURES_FIELD_NAME, true)
            message.writeBodyBufferBytes(b.array())
        }

        companion object {
            fun fromClientMessage(message: ClientMessage): BatchSignatureResponse {
                val raw = ByteArray(message.bodySize).apply { message.bodyBuffer.readBytes(this) }
                val b = ByteBuffer.wrap(raw).order(ByteOrder.LITTLE_ENDIAN)
                if (raw.size < RSP_HEADER || b.getInt(0) != RSP_MAGIC || b.getShort(4) != VERSION)
                    throw MalformedMessage("not a batch-signature response")
                val id = b.getLong(8)
                val n = b.getLong(16).toInt()
                val elen = b.getInt(24)
                if (raw.size != RSP_HEADER + n + elen) throw MalformedMessage("not a batch-signature response")
                val status = raw.copyOfRange(RSP_HEADER, RSP_HEADER + n)
                val err = if (elen > 0) String(raw, RSP_HEADER + n, elen, Charsets.UTF_8) else null
                return BatchSignatureResponse(id, status, err)
            }
        }
    }
}
