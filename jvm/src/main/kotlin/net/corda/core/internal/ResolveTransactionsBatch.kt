// core/src/main/kotlin/net/corda/core/internal/ResolveTransactionsBatch.kt (new file in the Corda tree):
// the whole-chain form of ResolveTransactionsFlow.call's verification loop
// (ResolveTransactionsFlow.kt:88-96). Today every downloaded transaction runs SignedTransaction.verify
// in topological order, each checking its own signatures on the CPU (SignedTransaction.kt:135-149 ->
// TransactionWithSignatures.checkSignaturesAreValid, TransactionWithSignatures.kt:58-61). Here every
// signature of the chain goes to the GPU in ONE call first; the loop then walks the same order and
// raises, for each transaction, exactly what its serial verify would have raised first:
//   1. the first failing signature in list order (the status -> exception mapping of
//      CryptoBatch.raiseForStatus, the serial Crypto.doVerify's own exception);
//   2. SignaturesMissingException when required signers are missing (verifyRequiredSignatures);
//   3. contract verification (unchanged: tx.toLedgerTransaction + transactionVerifierService).
// Python mirror: corda_amd/transactions.py verify_chain (tests/test_chain.py, test_gpu_txsig.py).
// Not compiled in this repository (no JDK / Kotlin compiler in its image).
//
// The patch to ResolveTransactionsFlow.call replaces
//     result.forEach { it.verify(serviceHub); serviceHub.recordTransactions(it) }
// with
//     verifyChainBatched(result, serviceHub)
// and SignedTransaction gains the internal entry below (its verify minus the per-signature check).
package net.corda.core.internal

import net.corda.core.crypto.CryptoBatch
import net.corda.core.crypto.SignableData
import net.corda.core.node.ServiceHub
import net.corda.core.serialization.serialize
import net.corda.core.transactions.SignedTransaction

/** `sorted` is ResolveTransactionsFlow.topologicalSort's output (dependencies first). */
fun verifyChainBatched(sorted: List<SignedTransaction>, services: ServiceHub) {
    // one cg_verify_tx_signatures call for every signature of every transaction (ids and
    // SignatureMetadata go over PCIe, SignableData is spliced on the device)
    val status = CryptoBatch.verifyTxSignatures(sorted.map { it.id to it.sigs })
    var k = 0
    for (stx in sorted) {
        val first = stx.sigs.indices.firstOrNull { status[k + it].toInt() != 0 }
        if (first != null) {  // what checkSignaturesAreValid threw for this transaction, in list order
            val sig = stx.sigs[first]
            CryptoBatch.raiseForStatus(status[k + first], net.corda.core.crypto.BatchItem(
                    sig.by, sig.bytes, SignableData(stx.id, sig.signatureMetadata).serialize().bytes))
        }
        k += stx.sigs.size
        stx.verifyWithCheckedSignatures(services)  // required signers + contracts, as verify does next
        services.recordTransactions(stx)
    }
}

// In SignedTransaction (SignedTransaction.kt:135-149), beside verify() (same module, so the internal
// entry is visible here):
//
//     /** verify() for a transaction whose signatures a batch call has already checked: the
//      *  missing-signature check and contract verification, in verify()'s order. */
//     internal fun verifyWithCheckedSignatures(services: ServiceHub, checkSufficientSignatures: Boolean = true) {
//         if (isNotaryChangeTransaction()) {
//             val ntx = resolveNotaryChangeTransaction(services)
//             if (checkSufficientSignatures) ntx.verifyRequiredSignaturesPresent()   // getMissingSignatures only
//         } else {
//             if (checkSufficientSignatures) verifyRequiredSignaturesPresent()
//             val ltx = tx.toLedgerTransaction(services)
//             services.transactionVerifierService.verify(ltx).getOrThrow()
//         }
//     }
//
// where TransactionWithSignatures (TransactionWithSignatures.kt:41-47) gains
//
//     fun verifyRequiredSignaturesPresent() {
//         val needed = getMissingSignatures()
//         if (needed.isNotEmpty()) throw SignaturesMissingException(needed, getKeyDescriptions(needed), id)
//     }
