"""Host packing at the ABI's field widths (corda_amd/batch.py): a signature longer than the
16-bit cg_item.sig_len is packed as a surrogate whose verdict equals the reference's verdict on
the real bytes (checked against the oracle on the real bytes), never truncated."""
import numpy as np

from corda_amd import batch as B
from oracle import c_oracle, corda, ecdsa_bc, ed25519_i2p


def _ed_key_sig(msg):
    seed = ed25519_i2p.entropy_seed(70)
    return ed25519_i2p.public_from_seed(seed), ed25519_i2p.sign(seed, msg)


def _packed_status(scheme, key, sig, msg, mode=B.MODE_DOVERIFY):
    b = B.BatchBuilder()
    b.add_with_key(scheme, B.KEY_RAW, key, sig, msg)
    batch = b.build()
    assert int(batch.items["sig_len"][0]) <= B.SIG_LEN_MAX
    return batch, int(c_oracle.verify_batch(batch, mode, 1)[0])


def test_ed25519_signature_with_64k_trailing_junk_is_malformed_not_valid():
    msg = b"transaction id bytes" * 10
    pub, sig = _ed_key_sig(msg)
    long_sig = sig + bytes(65536)            # a valid signature followed by 64 KiB of junk
    assert corda.verify_item(corda.EDDSA_ED25519_SHA512, corda.KEY_RAW, pub, sig, msg) == corda.VALID
    expect = corda.verify_item(corda.EDDSA_ED25519_SHA512, corda.KEY_RAW, pub, long_sig, msg)
    assert expect == corda.SIG_MALFORMED     # i2p: "signature length is wrong"
    batch, st = _packed_status(B.EDDSA_ED25519_SHA512, pub, long_sig, msg)
    assert st == expect
    assert int(batch.items["sig_len"][0]) == len(B.SIG_SURROGATE_MALFORMED)


def test_oversize_signature_keeps_key_precedence():
    msg = b"m" * 40
    _, sig = _ed_key_sig(msg)
    bad_key = bytes([0xff] * 31 + [0x7f])    # y >= p with no square root: key decode fails first
    long_sig = sig + bytes(70000)
    expect = corda.verify_item(corda.EDDSA_ED25519_SHA512, corda.KEY_RAW, bad_key, long_sig, msg)
    _, st = _packed_status(B.EDDSA_ED25519_SHA512, bad_key, long_sig, msg)
    assert st == expect


def _der_len(n):
    return bytes([n]) if n < 0x80 else bytes([0x80 | ((n.bit_length() + 7) // 8)]) + n.to_bytes(
        (n.bit_length() + 7) // 8, "big")


def test_ecdsa_oversize_signatures_follow_bc_decode():
    scheme = corda.ECDSA_SECP256R1_SHA256
    c = ecdsa_bc.CURVES[scheme]
    d = 0x1234567
    Q = ecdsa_bc.public_point(scheme, d)
    key = ecdsa_bc.raw_key(Q)
    msg = b"clear data" * 8
    r, s = ecdsa_bc.sign(scheme, d, msg, 0xabcdef123)
    good = ecdsa_bc.der_encode_sig(r, s)
    cases = {
        "valid DER + 64 KiB trailing": good + bytes(65536),
        # canonical SEQUENCE{INTEGER huge, INTEGER s}: decodes, r >= n -> false
        "huge r": (lambda body: b"\x30" + _der_len(len(body)) + body)(
            b"\x02" + _der_len(70000) + b"\x01" + bytes(69999) + ecdsa_bc.der_encode_int(s)),
        "huge non-minimal INTEGER": (lambda body: b"\x30" + _der_len(len(body)) + body)(
            b"\x02" + _der_len(70000) + bytes(70000) + ecdsa_bc.der_encode_int(s)),
    }
    assert c.n > 0
    for name, sig in cases.items():
        assert len(sig) > B.SIG_LEN_MAX
        assert B.der_is_two_integers(sig) == (name == "huge r"), name
        expect = corda.verify_item(scheme, corda.KEY_RAW, key, sig, msg)
        _, st = _packed_status(scheme, key, sig, msg)
        assert st == expect, (name, st, expect)
        for mode in (B.MODE_DOVERIFY, B.MODE_ISVALID):
            assert _packed_status(scheme, key, sig, msg, mode)[1] == corda.verify_item(
                scheme, corda.KEY_RAW, key, sig, msg, mode), name


def test_der_shape_matches_oracle_on_fixtures():
    import golden_io
    for it in golden_io.load("ecdsa.json"):
        sig = bytes.fromhex(it["sig"])
        try:
            ecdsa_bc.der_decode_sig(sig)
            ok = True
        except ecdsa_bc.MalformedSignature:
            ok = False
        assert B.der_is_two_integers(sig) == ok, it.get("class")


def test_short_inputs_pack_unchanged():
    msg = b"x" * 300
    pub, sig = _ed_key_sig(msg)
    b = B.BatchBuilder()
    b.add_with_key(B.EDDSA_ED25519_SHA512, B.KEY_RAW, pub, sig, msg)
    batch = b.build()
    it = batch.items[0]
    assert int(it["sig_len"]) == 64 and int(it["msg_len"]) == 300
    assert bytes(batch.arena[int(it["sig_off"]):int(it["sig_off"]) + 64]) == sig
    assert np.array_equal(c_oracle.verify_batch(batch, 0, 1), np.zeros(1, np.uint8))
