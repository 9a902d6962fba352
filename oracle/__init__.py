"""CPU oracle for the corda_amd batch signature-verification path.

TEST INFRASTRUCTURE ONLY. Nothing in the product path (``corda_amd``,
``libcordagpu.so``) imports, links or calls anything under ``oracle/``. Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
use it, and only as the checker / the timed CPU port.

Contents
--------
``ed25519_i2p``   Python big-int restatement of net.i2p.crypto:eddsa:0.2.0
                  ``EdDSAEngine.engineVerify`` (called from
                  core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559).
``ecdsa_bc``      Python restatement of org.bouncycastle:bcprov-jdk15on:1.57
                  ``SHA256withECDSA`` (DSABase.engineVerify -> StdDSAEncoder.decode ->
                  ECDSASigner.verifySignature), schemes at Crypto.kt:92-117.
``corda``         Crypto.doVerify / isValid / TransactionWithSignatures control flow
                  and the Merkle tx-id rules (MerkleTree.kt:27-66,
                  MerkleTransaction.kt:16-33, SecureHash.kt:25,37,42).
``c/``            C restatement of the same (liboracle.so): the on-box oracle for
                  large batches and the CPU baseline ("kind": "port").

Parity pinning: the reference is JVM code whose arithmetic
lives in un-vendored jars (i2p eddsa 0.2.0, BouncyCastle 1.57) and no JVM exists in
this image, so the reference cannot be run.  The reference's own tests pin only
behaviour (valid => true, corruption => exception, empty => IAE), and those
behaviours are reproduced in tests/.  Bit-level parity of the restatement is pinned
against RFC 8032 §7.1 vectors, FIPS 180-4 vectors and an independent implementation
(OpenSSL 3.0.2) for every valid signature in the golden fixtures.  Edge-case
verdicts that OpenSSL does not share (S >= L malleability, slide() carry drop,
non-canonical A re-encoding, BC DER strictness) follow the published upstream
algorithms and are marked "[ext] unpinned by a JVM run" in DESIGN.md.
"""
