"""The oracle pinned by data the reference itself holds (CPU only).

tests/golden/ref_certs.json is made by tools/gen/ref_vectors.py from the X.509 certificates inside
the reference's JKS keystores and config/dev/corda_dev_ca.cer. Their ECDSA-SHA256 signatures were
produced by the reference's own certificate code over BouncyCastle (Crypto.kt:833-850,
X509Utilities.kt:30), so each genuine item is a BC-made (issuer key, signature, TBSCertificate)
triple that Crypto.doVerify must accept. The builder-made corruptions around them carry the BC 1.57
restatement's verdicts.
"""
import numpy as np

import golden_io
from oracle import c_oracle, corda


def _items():
    return golden_io.load("ref_certs.json")


def test_reference_certificates_present():
    items = _items()
    genuine = [i for i in items if i["origin"] == "reference"]
    # 6 certificates: secp256k1 dev root CA / client CA chain and the secp256r1 intermediate CA
    assert len(genuine) >= 6
    assert {i["scheme"] for i in genuine} == {2, 3}
    assert all(i["expect"] == "VALID" and i["openssl"] == "VALID" for i in genuine)


def test_python_oracle_accepts_every_reference_signature():
    for it in _items():
        st = corda.verify_item(it["scheme"], it["key_fmt"], bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]),
                               bytes.fromhex(it["msg"]))
        assert corda.STATUS_NAMES[st] == it["expect"], (it["class"], it["note"])
        st = corda.verify_item(it["scheme"], it["key_fmt"], bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]),
                               bytes.fromhex(it["msg"]), corda.MODE_ISVALID)
        assert corda.STATUS_NAMES[st] == it["expect_isvalid"], (it["class"], it["note"])


def test_c_oracle_matches_reference_vectors():
    items = _items()
    b, exp, exp_iv = golden_io.sig_batch(items)
    assert np.array_equal(c_oracle.verify_batch(b, 0, 4), exp)
    assert np.array_equal(c_oracle.verify_batch(b, 1, 4), exp_iv)


def test_openssl_agrees_where_semantics_agree():
    """OpenSSL (recorded by the generator) agrees with the BC restatement on every item except
    the one known lenient case: OpenSSL 3 may accept trailing bytes after the DER SEQUENCE on some
    signatures, BC 1.57 never does (StdDSAEncoder re-encodes and compares)."""
    for it in _items():
        if it["openssl"] is None:
            continue
        if it["class"] == "E6":
            assert it["expect"] == "SIG_MALFORMED"
            continue
        assert (it["openssl"] == "VALID") == (it["expect"] == "VALID"), (it["class"], it["note"])


def test_reference_ed25519_vectors():
    """tests/golden/ref_ed25519.json (tools/gen/kryo_captures.py): the two i2p-made signatures the
    tutorial prints (over the 32-byte id) and corruptions of them; both oracles agree."""
    items = golden_io.load("ref_ed25519.json")
    genuine = [i for i in items if i["origin"] == "reference"]
    assert len(genuine) == 2 and all(i["expect"] == "VALID" for i in genuine)
    b, exp, exp_iv = golden_io.sig_batch(items)
    assert np.array_equal(c_oracle.verify_batch(b, 0, 4), exp)
    assert np.array_equal(c_oracle.verify_batch(b, 1, 4), exp_iv)
    for it in items:
        st = corda.verify_item(4, 0, bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"]))
        assert corda.STATUS_NAMES[st] == it["expect"], it["note"]
