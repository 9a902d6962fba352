"""CompositeKey structure (CompositeKeyTests.kt), composite signature verification and the host
fallback for the schemes the GPU does not run, on the CPU: the host logic of corda_amd/composite.py,
corda_amd/hostverify.py and corda_amd/crypto.py with the C oracle standing in for the GPU engine
(the same cases run against the real engine in tests/test_gpu_composite.py)."""
import hashlib

import pytest

import composite_cases as CC
from corda_amd import batch as B
from corda_amd.composite import ArithmeticException, CompositeKey, NodeAndWeight, expanded, is_fulfilled_by
from corda_amd.crypto import IllegalArgumentException, PublicKey


@pytest.fixture(scope="module")
def crypto():
    return CC.crypto_with(CC.OracleEngine())


@pytest.fixture(scope="module")
def abc():
    return CC.party(20)[1], CC.party(70)[1], CC.party(80)[1]


def test_single_key_fulfilment(abc):
    a, b, c = abc
    assert is_fulfilled_by(a, a) and not is_fulfilled_by(a, c)


def test_or_and_trees(abc):
    a, b, c = abc
    a_or_b = CompositeKey.Builder().add_keys(a, b).build(threshold=1)
    assert a_or_b.is_fulfilled_by(a) and a_or_b.is_fulfilled_by(b) and a_or_b.is_fulfilled_by([a, b])
    assert not a_or_b.is_fulfilled_by(c)
    a_and_b = CompositeKey.Builder().add_keys(a, b).build()
    assert not a_and_b.is_fulfilled_by([a]) and not a_and_b.is_fulfilled_by([b]) and a_and_b.is_fulfilled_by([a, b])
    ab_or_c = CompositeKey.Builder().add_keys(a_and_b, c).build(threshold=1)
    assert ab_or_c.is_fulfilled_by([a, b]) and ab_or_c.is_fulfilled_by([c]) and not ab_or_c.is_fulfilled_by([a])
    # a composite key among the keys to check fulfils nothing (CompositeKey.kt:187)
    assert not ab_or_c.is_fulfilled_by([c, a_and_b])
    assert expanded([ab_or_c, a]) == {a, b, c}


def test_der_round_trip_with_weighting(abc):
    a, b, c = abc
    ab = CompositeKey.Builder().add_keys(a, b).build()
    tree = CompositeKey.Builder().add_keys(ab, c).build(threshold=1)
    assert CompositeKey.get_instance(tree.encoded) == tree
    ab = CompositeKey.Builder().add_key(a, 2).add_key(b, 1).build(threshold=2)
    tree = CompositeKey.Builder().add_key(ab, 3).add_key(c, 2).build(threshold=3)
    back = CompositeKey.get_instance(tree.encoded)
    assert back == tree and back.encoded == tree.encoded
    assert tree.encoded[:2] == b"\x30\x81" or tree.encoded[0] == 0x30


def test_tree_canonical_form(abc):
    a, b, _ = abc
    assert CompositeKey.Builder().add_keys(a).build() == a
    node1 = CompositeKey.Builder().add_keys(a, b).build(1)
    node2 = CompositeKey.Builder().add_keys(a, b).build(2)
    assert not node2.is_fulfilled_by(a)
    t1 = CompositeKey.Builder().add_key(node1, 13).add_key(node2, 27).build()
    t2 = CompositeKey.Builder().add_key(node2, 27).add_key(node1, 13).build()
    assert t1 == t2 and hash(t1) == hash(t2)
    t3 = CompositeKey.Builder().add_keys(node1, node2).build()
    t4 = CompositeKey.Builder().add_keys(node2, node1).build()
    assert t3 == t4 and hash(t3) == hash(t4) and t3.encoded == t4.encoded
    t5 = CompositeKey.Builder().add_key(node1, 3).add_key(node1, 14).build()
    t6 = CompositeKey.Builder().add_key(node1, 14).add_key(node1, 3).build()
    assert t5 == t6
    assert CompositeKey.Builder().add_keys(t1).build() == t1


def test_key_equality_is_by_encoding():
    seed, a = CC.party(20)
    a_spki = PublicKey(4, bytes.fromhex("302a300506032b6570032100") + a.encoded, B.KEY_SPKI)
    assert a == a_spki and hash(a) == hash(a_spki)
    k = CompositeKey.Builder().add_keys(a, CC.party(70)[1]).build(threshold=1)
    assert k.is_fulfilled_by([a_spki])


def test_composite_key_constraints(abc):
    a, b, _ = abc
    with pytest.raises(IllegalArgumentException):
        CompositeKey.Builder().add_key(a, 0)
    with pytest.raises(IllegalArgumentException):
        CompositeKey.Builder().add_key(a, -1)
    with pytest.raises(IllegalArgumentException):
        CompositeKey.Builder().add_key(a).build(0)
    with pytest.raises(IllegalArgumentException):
        CompositeKey.Builder().add_key(a).build(-1)
    with pytest.raises(IllegalArgumentException, match="cannot be bigger"):
        CompositeKey.Builder().add_key(a, 2).add_key(b, 2).build(5)
    with pytest.raises(IllegalArgumentException, match="single child"):
        CompositeKey.Builder().add_key(a, 3).build(2)
    # Int.MAX_VALUE + Int.MAX_VALUE: the default threshold's Int sum wraps negative
    with pytest.raises(IllegalArgumentException, match="positive integer"):
        CompositeKey.Builder().add_key(a, 2**31 - 1).add_key(b, 2**31 - 1).build()
    # an explicit threshold reaches Math.addExact
    with pytest.raises(ArithmeticException):
        CompositeKey.Builder().add_key(a, 2**31 - 1).add_key(b, 2**31 - 1).build(1)
    with pytest.raises(IllegalArgumentException, match="duplicated"):
        CompositeKey.Builder().add_keys(a, b, a).build()
    with pytest.raises(IllegalArgumentException, match="duplicated"):
        k1 = CompositeKey.Builder().add_keys(a, b).build()
        k2 = CompositeKey.Builder().add_keys(b, a).build()
        CompositeKey.Builder().add_keys(k1, k2).build()
    with pytest.raises(IllegalArgumentException, match="without child"):
        CompositeKey.Builder().build()


def test_cycle_detection(abc):
    a, b, _ = abc
    k1 = CompositeKey.Builder().add_keys(a, b).build()
    k2 = CompositeKey.Builder().add_keys(a, k1).build()
    k3 = CompositeKey.Builder().add_keys(a, k2).build()
    k4 = CompositeKey.Builder().add_keys(a, k3).build()
    k5 = CompositeKey.Builder().add_keys(a, k4).build()
    k6 = CompositeKey.Builder().add_keys(a, k5, k2).build()
    for k in (k1, k2, k3, k4, k5, k6):
        k.check_validity()
    k3.children = k3.children + [NodeAndWeight(k5, 1)]  # the reflection trick of CompositeKeyTests.kt:243
    for k in (k3, k4, k5, k6):
        with pytest.raises(IllegalArgumentException, match="Cycle"):
            k.check_validity()
    k1.check_validity()
    k2.check_validity()


def test_two_of_three_truth_table(crypto):
    CC.two_of_three_truth_table(crypto)


def test_composite_clear_data_must_be_a_hash(crypto):
    CC.composite_clear_data_must_be_a_hash(crypto)


def test_composite_leaf_exception_propagates(crypto):
    CC.composite_leaf_exception_propagates(crypto)


def test_rsa_fallback_vs_openssl_fixtures(crypto):
    CC.rsa_fallback(crypto)


def test_composite_notary_and_missing_signatures(crypto):
    CC.composite_notary_satisfied_by_one_leaf(crypto)


def test_sphincs_has_no_host_verifier(crypto):
    from corda_amd.crypto import BatchItem, HOST_EXCEPTION, UnsupportedOperationException
    st, err = crypto.verify_batch_ex([BatchItem(PublicKey(5, b"\x00" * 64, B.KEY_SPKI), b"s", b"m")])
    assert st[0] == HOST_EXCEPTION and isinstance(err[0], UnsupportedOperationException)


def test_rsa_is_pss_not_pkcs1v15():
    """RSA_SHA256 is BC "SHA256WITHRSAANDMGF1" (Crypto.kt:85): a PSS signature made here verifies,
    OpenSSL accepts it with the PSS options, and the PKCS#1 v1.5 signature of the same message is
    false."""
    import json
    import os
    import subprocess
    import tempfile
    from corda_amd import hostverify as H
    k = json.load(open(os.path.join(CC.GOLDEN, "rsa.json")))["test_private_key"]
    n, d = int(k["n"], 16), int(k["d"], 16)
    msg = b"a transaction id signed by an RSA key"
    sig = H.rsa_pss_sign(n, d, msg, bytes(range(32)))
    key = H.rsa_decode_key(bytes.fromhex(k["spki"]))
    assert H.rsa_verify(key, sig, msg) is True
    assert H.rsa_verify(key, sig, msg + b"!") is False
    kk = (n.bit_length() + 7) // 8
    di = bytes.fromhex("3031300d060960864801650304020105000420") + hashlib.sha256(msg).digest()
    em = b"\x00\x01" + b"\xff" * (kk - 3 - len(di)) + b"\x00" + di
    v15 = pow(int.from_bytes(em, "big"), d, n).to_bytes(kk, "big")
    assert H.rsa_verify(key, v15, msg) is False
    with tempfile.TemporaryDirectory() as t:
        for name, data in (("k.der", bytes.fromhex(k["spki"])), ("s", sig), ("m", msg)):
            open(os.path.join(t, name), "wb").write(data)
        r = subprocess.run(["openssl", "dgst", "-sha256", "-keyform", "DER", "-verify", os.path.join(t, "k.der"),
                            "-sigopt", "rsa_padding_mode:pss", "-sigopt", "rsa_pss_saltlen:32",
                            "-sigopt", "rsa_mgf1_md:sha256", "-signature", os.path.join(t, "s"), os.path.join(t, "m")],
                           capture_output=True)
        assert r.returncode == 0, r.stdout + r.stderr


def test_composite_empty_clear_data_checked_before_deserialising(crypto):
    """doVerify's empty checks run before the composite engine deserialises the signature: a
    malformed non-empty signature with empty clear data is IllegalArgumentException("Clear data
    is empty, nothing to verify!"), as on the JVM (Crypto.kt:476-477)."""
    from corda_amd.composite import CompositeKey
    (_, a), (_, b) = CC.party(20), CC.party(21)
    k = CompositeKey.Builder().add_keys(a, b).build(threshold=1)
    with pytest.raises(IllegalArgumentException, match="Clear data is empty, nothing to verify!"):
        crypto.do_verify(k, b"\x01not a CompositeSignaturesWithKeys", b"")
    with pytest.raises(IllegalArgumentException, match="Signature data is empty!"):
        crypto.do_verify(k, b"", b"")
