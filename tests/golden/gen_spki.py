#!/usr/bin/env python3
"""Generates tests/golden/spki.json: the X.509 SubjectPublicKeyInfo forms a JVM caller can hand
the engine (CG_KEY_SPKI), valid and malformed, for all three GPU schemes.

The Kotlin binding sends ``PublicKey.getEncoded()``, which Corda decodes with
``Crypto.decodePublicKey(encoded)`` (Crypto.kt:321-325, via Kryo's PublicKeySerializer,
Kryo.kt:388-398): BC parses the SubjectPublicKeyInfo, ``findSignatureScheme`` maps the
normalised AlgorithmIdentifier to a scheme (DERNull parameters count as absent, Crypto.kt:219-228;
only the identifiers of Crypto.kt:92-133 are known), and the scheme's KeyFactory decodes the key:
i2p 0.2.0 EdDSAPublicKey (44-byte form, or 46 bytes with NULL parameters), BC's BCECPublicKey
(named curve; the point as ECCurve.decodePoint reads it: uncompressed, compressed or hybrid).

Classes:  K0 accepted forms (then verified: VALID / INVALID);  K1 malformed (KEY_INVALID).
Expected verdicts come from the oracle restatement (oracle/corda.py, oracle/ecdsa_bc.py); every
item is also run through the ``openssl`` CLI with the same SPKI bytes, and the agreement recorded
("agree", or "disagree-expected" with the reason in ``openssl_reason``: OpenSSL follows RFC 8410,
which forbids the NULL parameter i2p accepts; its PEM reader ignores trailing bytes and the
BIT STRING's unused-bits byte, which BC / i2p reject). OpenSSL agrees on every compressed and
hybrid point form. Runs in the build container only; separate RNG so the other fixtures do not
move.

Usage:  python tests/golden/gen_spki.py
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)

from oracle import corda, ecdsa_bc, ed25519_i2p as ed  # noqa: E402
import gen_golden as G  # noqa: E402  (helpers only; its main() is not run)

RNG = random.Random(0x5B41)
ITEMS = []
WHY_TRAILING = ("OpenSSL's PEM reader ignores bytes after the DER object; BC 1.57 ASN1Primitive.fromByteArray "
                "(SubjectPublicKeyInfo.getInstance) rejects extra data")


def _why(note):
    if "trailing" in note:
        return WHY_TRAILING
    if "unused bit" in note:
        return "OpenSSL ignores the BIT STRING's unused-bits byte; i2p 0.2.0 EdDSAPublicKey.decode requires 0"
    return None


def rbytes(n):
    return bytes(RNG.getrandbits(8) for _ in range(n))


def add(scheme, spki, sig, msg, cls, note, disagree_reason=None):
    st = corda.verify_item(scheme, corda.KEY_SPKI, spki, sig, msg)
    st_iv = corda.verify_item(scheme, corda.KEY_SPKI, spki, sig, msg, mode=corda.MODE_ISVALID)
    item = {"scheme": scheme, "key_fmt": corda.KEY_SPKI, "key": spki.hex(), "sig": sig.hex(), "msg": msg.hex(),
            "expect": corda.STATUS_NAMES[st], "expect_isvalid": corda.STATUS_NAMES[st_iv],
            "class": cls, "note": note}
    ok = G.openssl_verify(scheme, spki, sig, msg)
    ours = st == corda.VALID
    if ok == ours:
        item["openssl"] = "agree"
    elif disagree_reason:
        item["openssl"] = "disagree-expected"
        item["openssl_reason"] = disagree_reason
    else:
        raise SystemExit(f"OpenSSL disagrees on {cls} {note}: oracle={corda.STATUS_NAMES[st]} openssl={ok}")
    ITEMS.append(item)
    return st


def der_tlv(tag, body):
    return bytes([tag]) + ecdsa_bc._der_len(len(body)) + body


def gen_ed25519():
    S4 = corda.EDDSA_ED25519_SHA512
    null_pre = corda.ED25519_SPKI_PREFIX_NULL
    why_null = "RFC 8410: parameters MUST be absent; i2p 0.2.0 accepts NULL (Java keystore form)"
    for t in range(4):
        seed = rbytes(32)
        A = ed.public_from_seed(seed)
        m = rbytes(RNG.choice([32, 270]))
        sig = ed.sign(seed, m)
        canon = corda.ED25519_SPKI_PREFIX + A
        assert add(S4, canon, sig, m, "K0", "canonical 44-byte SPKI") == corda.VALID
        add(S4, canon, G.flip(sig, RNG.randrange(512)), m, "K0", "canonical SPKI, corrupted signature")
        assert add(S4, null_pre + A, sig, m, "K0", "46-byte SPKI with NULL parameters",
                   disagree_reason=why_null) == corda.VALID
        add(S4, null_pre + A, sig, G.flip(m, 3), "K0", "NULL parameters, corrupted message")
        # malformed: every one is KEY_INVALID on the JVM (decodePublicKey throws) and here
        bad = [
            (canon[:-1], "length 43 (truncated)"),
            (canon + b"\x00", "length 45 (trailing byte)"),
            (null_pre + A + b"\x00", "NULL-parameter form with a trailing byte"),
            (bytes.fromhex("302d300806032b65640a0101032100") + A,
             "old draft OID 1.3.101.100 (not in Crypto's algorithmMap)"),
            (bytes.fromhex("302a300506032b6571032100") + A, "OID 1.3.101.113 (Ed448) around a 32-byte key"),
            (bytes.fromhex("302a300506032b656e032100") + A, "OID 1.3.101.110 (X25519)"),
            (bytes.fromhex("302a300506032b6570032101") + A, "BIT STRING with 1 unused bit (i2p checks the byte is 0)"),
            (bytes.fromhex("302b300506032b6570032100") + A, "outer SEQUENCE length off by one"),
            (bytes.fromhex("302a300506032b6570042100") + A, "OCTET STRING instead of BIT STRING"),
            (bytes.fromhex("302c300706032b65700500032100")[:-3] + bytes.fromhex("032100") + A[:30],
             "NULL-parameter header, key cut short"),
            (G.ec_spki(corda.ECDSA_SECP256R1_SHA256, ecdsa_bc.raw_key(ecdsa_bc.public_point(3, 7))),
             "secp256r1 SPKI given as an Ed25519 key"),
        ]
        if t == 0:
            for spki, note in bad:
                add(S4, spki, sig, m, "K1", note, disagree_reason=_why(note))
    # a 44-byte SPKI whose A does not decode, and one with y >= p (non-canonical, decodes)
    seed = ed.entropy_seed(120)
    m = b"spki decode"
    sig = ed.sign(seed, m)
    while True:
        kb = rbytes(32)
        try:
            ed.decode_point(kb)
        except ed.KeyDecodeError:
            break
    add(S4, corda.ED25519_SPKI_PREFIX + kb, sig, m, "K1", "A has no square root")
    add(S4, null_pre + kb, sig, m, "K1", "NULL parameters, A has no square root")


def gen_ecdsa():
    oids = {3: bytes.fromhex("06082a8648ce3d030107"), 2: bytes.fromhex("06052b8104000a")}
    ecpk = bytes.fromhex("06072a8648ce3d0201")
    for scheme in (corda.ECDSA_SECP256R1_SHA256, corda.ECDSA_SECP256K1_SHA256):
        other = 2 if scheme == 3 else 3
        c = ecdsa_bc.CURVES[scheme]
        for t in range(4):
            d = RNG.randrange(1, c.n)
            Q = ecdsa_bc.public_point(scheme, d)
            x, y = Q
            X, Y = x.to_bytes(32, "big"), y.to_bytes(32, "big")
            m = rbytes(RNG.choice([32, 270]))
            r, s = ecdsa_bc.sign(scheme, d, m, RNG.randrange(1, c.n))
            sig = ecdsa_bc.der_encode_sig(r, s)
            unc = ecdsa_bc.spki_prefix(scheme, 65) + b"\x04" + X + Y
            cmp_ = ecdsa_bc.spki_prefix(scheme, 33) + bytes([2 | (y & 1)]) + X
            hyb = ecdsa_bc.spki_prefix(scheme, 65) + bytes([6 | (y & 1)]) + X + Y
            assert add(scheme, unc, sig, m, "K0", "canonical SPKI (uncompressed point)") == corda.VALID
            add(scheme, unc, ecdsa_bc.der_encode_sig(r, (s + 1) % c.n or 1), m, "K0", "canonical SPKI, wrong s")
            assert add(scheme, cmp_, sig, m, "K0", "SPKI around a compressed point") == corda.VALID
            add(scheme, cmp_, sig, G.flip(m, 5), "K0", "compressed point, corrupted message")
            assert add(scheme, hyb, sig, m, "K0", "SPKI around a hybrid (06/07) point") == corda.VALID
            if t >= 2:
                continue
            wrong_par = ecdsa_bc.spki_prefix(scheme, 33) + bytes([3 - (y & 1)]) + X
            add(scheme, wrong_par, sig, m, "K0", "compressed point with the other parity: -Q (verifies as INVALID)")
            alg_other = der_tlv(0x30, ecpk + oids[other])
            bad = [
                (unc[:-1], f"length {len(unc) - 1} (truncated)"),
                (unc + b"\x00", f"length {len(unc) + 1} (trailing byte)"),
                (cmp_ + b"\x00", "compressed form with a trailing byte"),
                (ecdsa_bc.spki_prefix(scheme, 65) + bytes([7 - (y & 1)]) + X + Y, "hybrid tag with the wrong parity"),
                (ecdsa_bc.spki_prefix(scheme, 65) + b"\x05" + X + Y, "point tag 05"),
                (ecdsa_bc.spki_prefix(scheme, 33) + b"\x04" + X, "tag 04 on a 33-byte point"),
                (der_tlv(0x30, alg_other + der_tlv(0x03, b"\x00\x04" + X + Y)),
                 "the other curve's OID around this curve's point"),
                (der_tlv(0x30, der_tlv(0x30, bytes.fromhex("06072a8648ce3d0401") + oids[scheme])
                         + der_tlv(0x03, b"\x00\x04" + X + Y)), "ecdsa-with-SHA1 OID as the key algorithm"),
                (der_tlv(0x30, der_tlv(0x30, ecpk) + der_tlv(0x03, b"\x00\x04" + X + Y)), "no curve parameters"),
                (der_tlv(0x30, der_tlv(0x30, ecpk + oids[scheme]) + der_tlv(0x03, b"\x00\x00")), "point at infinity (00)"),
            ]
            xo = bytearray(Y)
            xo[31] ^= 1
            bad.append((ecdsa_bc.spki_prefix(scheme, 65) + b"\x04" + X + bytes(xo), "point not on the curve"))
            bad.append((ecdsa_bc.spki_prefix(scheme, 65) + b"\x04" + (c.p + 1).to_bytes(32, "big") + Y, "x >= p"))
            xs = x
            while True:  # an x with no point on the curve, compressed
                xs = (xs + 1) % c.p
                rhs = (xs ** 3 + c.a * xs + c.b) % c.p
                if pow(rhs, (c.p - 1) // 2, c.p) == c.p - 1:
                    break
            bad.append((ecdsa_bc.spki_prefix(scheme, 33) + b"\x02" + xs.to_bytes(32, "big"), "compressed x not on the curve"))
            bad.append((corda.ED25519_SPKI_PREFIX + X, "Ed25519 SPKI given as an EC key"))
            for spki, note in bad:
                add(scheme, spki, sig, m, "K1", note, disagree_reason=_why(note))


def main():
    gen_ed25519()
    gen_ecdsa()
    meta = {"generator": "tests/golden/gen_spki.py", "rng_seed": "0x5B41",
            "oracle": "oracle/corda.py (decode_key), oracle/ecdsa_bc.py (decode_spki, decode_point)",
            "cross_check": "openssl 3.0.2 CLI on every item, the SPKI bytes as the PEM public key"}
    with open(os.path.join(HERE, "spki.json"), "w") as f:
        json.dump({"meta": meta, "items": ITEMS}, f, indent=0)
    from collections import Counter
    print("spki.json", len(ITEMS), "items;", dict(Counter((i["class"], i["expect"]) for i in ITEMS)),
          "openssl", dict(Counter(i["openssl"] for i in ITEMS)))


if __name__ == "__main__":
    main()
