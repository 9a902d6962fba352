"""GPU form of the composite-key and host-fallback cases (tests/composite_cases.py): composite
leaves verified by the HIP kernels through the C ABI, the threshold logic on the host; RSA items
verified through the host fallback without IllegalArgumentException, alone, mixed into a GPU
batch, and inside the transaction pipeline (cg_verify_transactions ids spliced into
SignableData for the fallback)."""
import hashlib
import json
import os

import numpy as np
import pytest

import composite_cases as CC
from corda_amd import batch as B
from corda_amd import signable
from corda_amd import transactions as T
from corda_amd.crypto import PublicKey, SignatureException, TransactionSignature

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def crypto(engine):
    return CC.crypto_with(engine)


def test_two_of_three_truth_table_gpu(crypto):
    CC.two_of_three_truth_table(crypto)


def test_composite_edges_gpu(crypto):
    CC.composite_clear_data_must_be_a_hash(crypto)
    CC.composite_leaf_exception_propagates(crypto)


def test_rsa_fallback_gpu(crypto):
    CC.rsa_fallback(crypto)


def test_composite_notary_gpu(crypto):
    CC.composite_notary_satisfied_by_one_leaf(crypto)


def _rsa_sign(msg):
    """SHA256WITHRSAANDMGF1 (PSS) with the fixture's test key and a salt derived from the message."""
    from corda_amd.hostverify import rsa_pss_sign
    k = json.load(open(os.path.join(CC.GOLDEN, "rsa.json")))["test_private_key"]
    n, d = int(k["n"], 16), int(k["d"], 16)
    salt = hashlib.sha256(b"salt" + bytes(msg)).digest()
    return PublicKey(1, bytes.fromhex(k["spki"]), B.KEY_SPKI), rsa_pss_sign(n, d, msg, salt)


def test_wire_transactions_with_rsa_signers_gpu(crypto):
    """A transaction signed by an RSA key next to Ed25519 keys: ids on the GPU, the RSA signature
    verified by the host fallback over SignableData(id) -- valid passes, corrupted fails with the
    serial loop's first-failure semantics."""
    from oracle import corda as ocorda, ed25519_i2p as ed
    rng = np.random.default_rng(4)
    seed = ed.entropy_seed(20)
    ek = PublicKey(4, ed.public_from_seed(seed))
    stxs, bad = [], []
    for t in range(6):
        comps = [rng.integers(0, 256, int(rng.integers(1, 200)), dtype=np.uint8).tobytes() for _ in range(4)]
        salt = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        tid = ocorda.tx_id(comps, salt, b"\x01" + salt)
        rk, rsig = _rsa_sign(signable.serialize(tid, 1, 1))
        if t % 2:
            rsig = rsig[:-1] + bytes([rsig[-1] ^ 1])
        sigs = [TransactionSignature(ed.sign(seed, signable.serialize(tid, 1, 4)), ek, 1, 4),
                TransactionSignature(rsig, rk, 1, 1)]
        stxs.append(T.SignedWireTransaction(T.WireTransactionData(comps, salt, b"\x01" + salt), sigs))
        bad.append(t % 2 == 1)
    ids, results = T.verify_wire_transactions(stxs, crypto)
    for b_, res in zip(bad, results):
        if b_:
            assert res is not None and res[0] == 1 and isinstance(res[1], SignatureException), res
        else:
            assert res is None, res
