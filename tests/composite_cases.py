"""Composite-key / host-fallback cases shared by the CPU suite (an oracle-backed engine stand-in)
and the GPU suite (the real engine): restated from CompositeKeyTests.kt:46-177 and the
TransactionWithSignatures / SignedTransaction rules (TransactionWithSignatures.kt:41-78)."""
import hashlib
import json
import os

import numpy as np
import pytest

from corda_amd import batch as B
from corda_amd import signable
from corda_amd import transactions as T
from corda_amd.composite import CompositeKey, CompositeSignaturesWithKeys
from corda_amd.crypto import (BatchItem, HOST_EXCEPTION, IllegalArgumentException, PublicKey, SignatureException,
                              TransactionSignature, _Crypto)
from oracle import ed25519_i2p as ed

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class OracleEngine:
    """CPU stand-in for corda_amd.engine.Engine in the host-logic tests (test infrastructure)."""

    def verify(self, batch, mode=0):
        from oracle import c_oracle
        return c_oracle.verify_batch(batch, mode, 4)


def crypto_with(engine):
    c = _Crypto()
    c.use_engine(engine)
    return c


def party(n):
    seed = ed.entropy_seed(n)
    return seed, PublicKey(4, ed.public_from_seed(seed), B.KEY_RAW)


SECURE_HASH = hashlib.sha256(b"Transaction").digest()  # CompositeKeyTests.kt:38-39


def tx_sig(seed, key, tx_id=SECURE_HASH, meta=(1, 4)):
    pre, suf = signable.template(*meta)
    return TransactionSignature(ed.sign(seed, pre + tx_id + suf), key, *meta)


def two_of_three_truth_table(crypto):
    (sa, a), (sb, b), (sc, c) = party(20), party(70), party(80)
    asig, bsig, csig = tx_sig(sa, a), tx_sig(sb, b), tx_sig(sc, c)
    k = CompositeKey.Builder().add_keys(a, b, c).build(threshold=2)
    cases = [([asig], False), ([bsig], False), ([csig], False), ([asig, bsig], True), ([asig, csig], True),
             ([bsig, csig], True), ([asig, bsig, csig], True)]
    broken_bob = TransactionSignature(asig.bytes, b, 1, 4)  # Alice's bytes claimed by Bob (:175-176)
    cases.append(([asig, broken_bob], False))
    items = [BatchItem(k, CompositeSignaturesWithKeys(s), SECURE_HASH) for s, _ in cases]
    st, err = crypto.verify_batch_ex(items, B.MODE_ISVALID)
    assert [bool(x == B.VALID) for x in st] == [e for _, e in cases], st
    assert not err
    # one-at-a-time API, both modes, and the serialized stand-in form
    for s, want in cases:
        assert crypto.is_valid(k, CompositeSignaturesWithKeys(s), SECURE_HASH) is want
        assert crypto.is_valid(k, CompositeSignaturesWithKeys(s).serialize(), SECURE_HASH) is want
        if want:
            assert crypto.do_verify(k, CompositeSignaturesWithKeys(s), SECURE_HASH) is True
        else:
            with pytest.raises(SignatureException, match="Signature Verification failed!"):
                crypto.do_verify(k, CompositeSignaturesWithKeys(s), SECURE_HASH)


def composite_clear_data_must_be_a_hash(crypto):
    """CompositeSignature.State.engineVerify wraps the buffer as SecureHash.SHA256: not 32 bytes ->
    IllegalArgumentException -- so a composite TransactionSignature checked through
    doVerify(txId, sig) over the ~270-byte SignableData throws (Corda 0.15 behaviour)."""
    (sa, a), (sb, b) = party(20), party(70)
    k = CompositeKey.Builder().add_keys(a, b).build(threshold=1)
    sig = CompositeSignaturesWithKeys([tx_sig(sa, a)])
    with pytest.raises(IllegalArgumentException, match="Failed requirement"):
        crypto.is_valid(k, sig, SECURE_HASH + b"x")
    st, err = crypto.verify_batch_ex([BatchItem(k, sig, SECURE_HASH[:31])], B.MODE_DOVERIFY)
    assert st[0] == HOST_EXCEPTION and isinstance(err[0], IllegalArgumentException)
    # not fulfilled -> false before the clear data is looked at
    k2 = CompositeKey.Builder().add_keys(a, b).build()
    assert crypto.is_valid(k2, sig, b"short") is False


def composite_leaf_exception_propagates(crypto):
    (sa, a), (sb, b) = party(20), party(70)
    k = CompositeKey.Builder().add_keys(a, b).build()
    good_a, good_b = tx_sig(sa, a), tx_sig(sb, b)
    bad_len = TransactionSignature(good_b.bytes[:63], b, 1, 4)  # i2p: "signature length is wrong"
    with pytest.raises(SignatureException, match="signature length is wrong"):
        crypto.is_valid(k, CompositeSignaturesWithKeys([good_a, bad_len]), SECURE_HASH)
    # `all` stops at the first false: a bad leaf after a false one is never reached
    wrong = TransactionSignature(good_b.bytes, a, 1, 4)
    assert crypto.is_valid(k, CompositeSignaturesWithKeys([wrong, bad_len]), SECURE_HASH) is False


def rsa_fallback(crypto):
    """RSA keys are supported by Corda: the GPU says CG_UNSUPPORTED and the host verifies them --
    never IllegalArgumentException. Verdicts vs OpenSSL on the committed fixtures."""
    items = json.load(open(os.path.join(GOLDEN, "rsa.json")))["items"]
    batch_items = [BatchItem(PublicKey(1, bytes.fromhex(i["key"]), B.KEY_SPKI), bytes.fromhex(i["sig"]),
                             bytes.fromhex(i["msg"])) for i in items]
    st, err = crypto.verify_batch_ex(batch_items, B.MODE_ISVALID)
    for j, it in enumerate(items):
        want = it["expect"]
        if want == "SignatureException":
            assert st[j] == HOST_EXCEPTION and isinstance(err[j], SignatureException), (j, it["note"])
        else:
            assert st[j] == B.STATUS_BY_NAME[want], (j, it["note"], st[j])
        assert (st[j] == B.VALID) == (it["openssl"] == "accept"), (j, it["note"])
    ok = next(i for i in items if i["expect"] == "VALID")
    pk = PublicKey(1, bytes.fromhex(ok["key"]), B.KEY_SPKI)
    assert crypto.do_verify(pk, bytes.fromhex(ok["sig"]), bytes.fromhex(ok["msg"])) is True
    bad = next(i for i in items if i["expect"] == "INVALID")
    with pytest.raises(SignatureException, match="Signature Verification failed!"):
        crypto.do_verify(PublicKey(1, bytes.fromhex(bad["key"]), B.KEY_SPKI), bytes.fromhex(bad["sig"]),
                         bytes.fromhex(bad["msg"]))
    # mixed with GPU items in one batch: each keeps its own verdict
    (sa, a) = party(20)
    msg = b"mixed batch"
    mixed = [BatchItem(a, ed.sign(sa, msg), msg), batch_items[0], BatchItem(a, ed.sign(sa, msg), msg + b"!")]
    st, _ = crypto.verify_batch_ex(mixed, B.MODE_DOVERIFY)
    assert list(st) == [B.VALID, B.VALID, B.INVALID]


def composite_notary_satisfied_by_one_leaf(crypto):
    """A distributed notary whose identity is a 1-of-2 CompositeKey: its required signature is
    fulfilled by one member's ordinary signature (getMissingSignatures is composite-aware,
    TransactionWithSignatures.kt:72-78); without it, SignaturesMissingException names "notary"."""
    (s1, n1), (s2, n2), (sa, alice) = party(301), party(302), party(20)
    notary = CompositeKey.Builder().add_keys(n1, n2).build(threshold=1)
    tx_id = hashlib.sha256(b"notarised tx").digest()
    signable_data = lambda tid, s: signable.template(s.platform_version, s.scheme_number_id)[0] + bytes(tid) + \
        signable.template(s.platform_version, s.scheme_number_id)[1]  # noqa: E731
    cmd = T.Command("Move(amount=5)", (alice,))
    stx = T.SignedTransaction(tx_id, [tx_sig(sa, alice, tx_id), tx_sig(s2, n2, tx_id)], {alice, notary}, [cmd], notary)
    T.verify_signatures_except(stx, signable_data, crypto=crypto)   # passes: n2 fulfils the notary key
    stx2 = T.SignedTransaction(tx_id, [tx_sig(sa, alice, tx_id)], {alice, notary}, [cmd], notary)
    with pytest.raises(T.SignaturesMissingException) as ei:
        T.verify_signatures_except(stx2, signable_data, crypto=crypto)
    assert ei.value.missing == {notary} and ei.value.descriptions == ["notary"]
    assert bytes(tx_id).hex().upper()[:6] in str(ei.value)
    T.verify_signatures_except(stx2, signable_data, allowed_to_be_missing=(notary,), crypto=crypto)
    stx3 = T.SignedTransaction(tx_id, [tx_sig(s2, n2, tx_id)], {alice, notary}, [cmd], notary)
    with pytest.raises(T.SignaturesMissingException) as ei:
        T.verify_signatures_except(stx3, signable_data, crypto=crypto)
    assert ei.value.missing == {alice} and ei.value.descriptions == ["Move(amount=5)"]


def all_cases(crypto):
    two_of_three_truth_table(crypto)
    composite_clear_data_must_be_a_hash(crypto)
    composite_leaf_exception_propagates(crypto)
    rsa_fallback(crypto)
    composite_notary_satisfied_by_one_leaf(crypto)
    return np.zeros(0)
