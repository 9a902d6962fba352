// verifier/src/main/kotlin/net/corda/verifier/BatchVerifierHandler.kt (new file in the Corda tree): the
// branch Verifier.kt's message handler (Verifier.kt:69-84) gains for a batch-signature request. One
// verifier process owns one GPU and one cg_ctx (CryptoBatch); Artemis keeps load-balancing requests
// across verifier processes exactly as it does today. Python mirror: corda_amd/verifier.py
// VerifierWorker.handle. Not compiled in this repository (no JDK / Kotlin compiler in its image).
//
// The patch to Verifier.kt's handler is one branch in front of the existing body:
//
//     consumer.setMessageHandler {
//         if (VerifierBatchApi.BatchSignatureRequest.isBatch(it)) {          // <- new
//             BatchVerifierHandler.handle(session, replyProducer, it)       // <- new
//             return@setMessageHandler                                     // <- new
//         }                                                                // <- new
//         val request = VerifierApi.VerificationRequest.fromClientMessage(it)
//         ...                                                              // unchanged
//     }
package net.corda.verifier

import net.corda.core.crypto.CryptoBatch
import net.corda.core.utilities.loggerFor
import net.corda.nodeapi.VerifierBatchApi.BatchSignatureRequest
import net.corda.nodeapi.VerifierBatchApi.BatchSignatureResponse
import net.corda.nodeapi.VerifierBatchApi.MalformedMessage
import org.apache.activemq.artemis.api.core.client.ClientMessage
import org.apache.activemq.artemis.api.core.client.ClientProducer
import org.apache.activemq.artemis.api.core.client.ClientSession
import org.apache.activemq.artemis.reader.MessageUtil

object BatchVerifierHandler {
    private val log = loggerFor<BatchVerifierHandler>()

    /** Decode, verify on this process's GPU (one cg_verify_batch call), reply to JMSReplyTo,
     *  acknowledge: the same life cycle as a VerificationRequest (Verifier.kt:69-84). A request that
     *  cannot be decoded or run is answered with an error and no statuses, never with statuses that
     *  read as valid. */
    fun handle(session: ClientSession, replyProducer: ClientProducer, message: ClientMessage) {
        val reply = session.createMessage(false)
        val response = try {
            val req = BatchSignatureRequest.fromClientMessage(message)
            try {
                val status = CryptoBatch.verifyPacked(req.keys(), req.nKeys, req.items(), req.nItems, req.arena(),
                                                      req.arenaLen(), req.mode)
                BatchSignatureResponse(req.verificationId, status, null)
            } catch (t: Throwable) {
                log.debug("Batch verification failed:", t)
                BatchSignatureResponse(req.verificationId, ByteArray(0), "${t.javaClass.simpleName}: ${t.message}")
            }
        } catch (e: MalformedMessage) {
            BatchSignatureResponse(if (message.containsProperty("id")) message.getLongProperty("id") else -1L,
                                   ByteArray(0), "MalformedMessage: ${e.message}")
        }
        response.writeToClientMessage(reply)
        replyProducer.send(MessageUtil.getJMSReplyTo(message), reply)
        message.acknowledge()
    }
}
