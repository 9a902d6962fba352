"""Extracts reference-produced ECDSA vectors from the certificates the reference itself holds.

Runs in the build container only (it reads /root/reference as plain data; nothing under
/root/reference is executed or imported). Writes tests/golden/ref_certs.json, which the CPU and GPU
tests load; the GPU box never needs /root/reference.

Source of the signatures. Corda's dev CA / node certificates were made by the reference's own
certificate code (X509Utilities.createCertificate -> ContentSignerBuilder over BouncyCastle
"SHA256withECDSA", core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:833-850,
X509Utilities.kt:30) and checked into the tree inside Java KeyStores (JKS) and one PEM file:

    node/src/main/resources/net/corda/node/internal/certificates/cordadevcakeys.jks
    node/src/main/resources/net/corda/node/internal/certificates/cordatruststore.jks
    samples/{trader,attachment}-demo/src/main/resources/certificates/{sslkeystore,truststore}.jks
    config/dev/corda_dev_ca.cer

JKS stores certificates in the clear (only private keys are protected), so each X.509 certificate
gives one reference-made signature item: (issuer SubjectPublicKeyInfo, DER ECDSA signature,
TBSCertificate bytes as the clear data). That is exactly what Crypto.doVerify(issuerKey, sig,
tbs) checks (Crypto.kt:457,474-484) and what BC's certificate verification runs.

Besides the genuine items the script derives corruption variants (each labelled "builder-made")
whose expected verdicts come from the BC 1.57 restatement (oracle/ecdsa_bc.py) and, where the
semantics agree, OpenSSL.

JKS layout (Sun's JavaKeyStore engine): magic FEEDFEED, version 2, entry count; per entry a tag
(1 private key: alias, date, protected key, chain of certificates; 2 trusted certificate: alias,
date, certificate), every certificate as (type UTF, u32 length, DER); a trailing SHA-1 keyed by
the store password (not checked here: it only authenticates the store).
"""
import glob
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from corda_amd import der  # noqa: E402
from oracle import corda as ocorda, ecdsa_bc  # noqa: E402

REF = "/root/reference"
SOURCES = [
    "node/src/main/resources/net/corda/node/internal/certificates/cordadevcakeys.jks",
    "node/src/main/resources/net/corda/node/internal/certificates/cordatruststore.jks",
    "samples/trader-demo/src/main/resources/certificates/sslkeystore.jks",
    "samples/trader-demo/src/main/resources/certificates/truststore.jks",
    "samples/attachment-demo/src/main/resources/certificates/sslkeystore.jks",
    "samples/attachment-demo/src/main/resources/certificates/truststore.jks",
    "config/dev/corda_dev_ca.cer",
]

OID_ECDSA_SHA256 = der.oid("1.2.840.10045.4.3.2")
OID_EC_PUBLIC_KEY = der.oid("1.2.840.10045.2.1")
CURVE_BY_OID = {der.oid("1.2.840.10045.3.1.7"): 3,  # secp256r1 -> ECDSA_SECP256R1_SHA256
                der.oid("1.3.132.0.10"): 2}         # secp256k1 -> ECDSA_SECP256K1_SHA256


def _utf(b, i):
    (n,) = struct.unpack_from(">H", b, i)
    return b[i + 2:i + 2 + n].decode("utf-8", "replace"), i + 2 + n


def _cert(b, i):
    ctype, i = _utf(b, i)
    (n,) = struct.unpack_from(">I", b, i)
    return ctype, b[i + 4:i + 4 + n], i + 4 + n


def jks_certificates(data):
    """[(alias, entry kind, chain position, DER certificate)] of a JKS byte string."""
    magic, version, count = struct.unpack_from(">III", data, 0)
    if magic != 0xFEEDFEED or version not in (1, 2):
        raise ValueError("not a JKS keystore")
    out, i = [], 12
    for _ in range(count):
        (tag,) = struct.unpack_from(">I", data, i)
        alias, i = _utf(data, i + 4)
        i += 8  # creation date
        if tag == 1:
            (klen,) = struct.unpack_from(">I", data, i)
            i += 4 + klen
            (nchain,) = struct.unpack_from(">I", data, i)
            i += 4
            for pos in range(nchain):
                ctype, c, i = _cert(data, i)
                out.append((alias, "private-key-chain", pos, ctype, c))
        elif tag == 2:
            ctype, c, i = _cert(data, i)
            out.append((alias, "trusted-cert", 0, ctype, c))
        else:
            raise ValueError(f"unknown JKS entry tag {tag}")
    if len(data) - i != 20:
        raise ValueError("JKS trailer is not a 20-byte SHA-1")
    return out


def pem_certificates(text):
    import base64
    out, cur = [], None
    for line in text.splitlines():
        if line.startswith("-----BEGIN CERTIFICATE"):
            cur = []
        elif line.startswith("-----END CERTIFICATE"):
            out.append(base64.b64decode("".join(cur)))
            cur = None
        elif cur is not None:
            cur.append(line.strip())
    return out


def parse_cert(c):
    """Raw TBSCertificate, signature algorithm OID, signature bytes, issuer / subject Name DER,
    SubjectPublicKeyInfo DER."""
    tag, body, end = der.read_tlv(c)
    assert tag == 0x30 and end == len(c)
    # TBSCertificate keeps its own tag + length: the signed bytes.
    t_tag, _, t_end = der.read_tlv(body, 0)
    tbs = body[:t_end]
    a_tag, alg, a_end = der.read_tlv(body, t_end)
    s_tag, sigbits, s_end = der.read_tlv(body, a_end)
    assert t_tag == 0x30 and a_tag == 0x30 and s_tag == 0x03 and s_end == len(body)
    alg_oid = der.read_tlv(alg, 0)
    sig = der.read_bit_string(s_tag, sigbits)
    # TBSCertificate fields: [0] version?, serial, sigalg, issuer, validity, subject, spki, ...
    fields, i = [], 0
    _, tbody, _ = der.read_tlv(tbs)
    while i < len(tbody):
        s = i
        t, v, i = der.read_tlv(tbody, i)
        fields.append((t, tbody[s:i]))
    k = 1 if fields[0][0] == 0xA0 else 0
    issuer, subject, spki = fields[k + 2][1], fields[k + 4][1], fields[k + 5][1]
    return {"tbs": tbs, "alg": bytes([alg_oid[0]]) + der._len_bytes(len(alg_oid[1])) + alg_oid[1],
            "sig": sig, "issuer": issuer, "subject": subject, "spki": spki}


def spki_scheme(spki):
    seq = der.read_seq(spki)
    alg = der.read_seq(der.tlv(seq[0][0], seq[0][1]))
    alg_oid = der.tlv(alg[0][0], alg[0][1])
    if alg_oid != OID_EC_PUBLIC_KEY or len(alg) < 2:
        return None
    return CURVE_BY_OID.get(der.tlv(alg[1][0], alg[1][1]))


def openssl_verify(spki, sig, msg):
    with tempfile.TemporaryDirectory() as d:
        open(os.path.join(d, "k.der"), "wb").write(spki)
        open(os.path.join(d, "s"), "wb").write(sig)
        open(os.path.join(d, "m"), "wb").write(msg)
        subprocess.check_call(["openssl", "pkey", "-pubin", "-inform", "DER", "-in", os.path.join(d, "k.der"),
                               "-out", os.path.join(d, "k.pem")], stderr=subprocess.DEVNULL)
        r = subprocess.run(["openssl", "dgst", "-sha256", "-verify", os.path.join(d, "k.pem"), "-signature",
                            os.path.join(d, "s"), os.path.join(d, "m")], capture_output=True)
        return r.returncode == 0


def oracle_status(scheme, spki, sig, msg, mode=ocorda.MODE_DOVERIFY):
    return ocorda.STATUS_NAMES[ocorda.verify_item(scheme, 1, spki, sig, msg, mode)]


def variants(c, scheme):
    """Builder-made corruptions of one genuine item: (class, note, spki, sig, msg)."""
    curve = ecdsa_bc.CURVES[scheme]
    r, s = ecdsa_bc.der_decode_sig(c["sig"])
    msg = bytearray(c["tbs"])
    msg[len(msg) // 2] ^= 0x01
    out = [("E1", "one bit of the TBSCertificate flipped", c["spki"], c["sig"], bytes(msg)),
           ("E2", "high-S twin (n - s): BC 1.57 has no low-S rule", c["spki"],
            ecdsa_bc.der_encode_sig(r, curve.n - s), c["tbs"]),
           ("E3", "s = n", c["spki"], ecdsa_bc.der_encode_sig(r, curve.n), c["tbs"]),
           ("E3", "r = 0", c["spki"], ecdsa_bc.der_encode_sig(0, s), c["tbs"]),
           ("E6", "one trailing byte after the SEQUENCE", c["spki"], c["sig"] + b"\x00", c["tbs"]),
           ("E5", "r INTEGER with a redundant leading 0x00",
            c["spki"], _nonminimal(r, s), c["tbs"]),
           ("E5", "BER long-form SEQUENCE length", c["spki"], _longform(c["sig"]), c["tbs"]),
           ("A7", "empty clear data (Crypto.doVerify IllegalArgumentException)", c["spki"], c["sig"], b""),
           ("A7", "empty signature (Crypto.doVerify IllegalArgumentException)", c["spki"], b"", c["tbs"])]
    return out


def _nonminimal(r, s):
    rb = ecdsa_bc.der_encode_int(r)
    rb = b"\x02" + bytes([rb[1] + 1]) + b"\x00" + rb[2:]
    sb = ecdsa_bc.der_encode_int(s)
    body = rb + sb
    return b"\x30" + bytes([len(body)]) + body


def _longform(sig):
    body = sig[2:]
    return b"\x30\x81" + bytes([len(body)]) + body


def main():
    certs, provenance = {}, {}
    for rel in SOURCES:
        path = os.path.join(REF, rel)
        data = open(path, "rb").read()
        if rel.endswith(".jks"):
            found = [(a, kind, pos, c) for a, kind, pos, _t, c in jks_certificates(data)]
        else:
            found = [("pem", "pem", 0, c) for c in pem_certificates(data.decode())]
        for alias, kind, pos, c in found:
            h = hashlib.sha256(c).hexdigest()
            certs[h] = c
            provenance.setdefault(h, []).append(f"{rel}:{alias}:{kind}[{pos}]")
    parsed = {h: parse_cert(c) for h, c in certs.items()}
    by_subject = {}
    for h, p in parsed.items():
        by_subject.setdefault(p["subject"], []).append(h)

    items, skipped = [], []
    for h in sorted(parsed):
        p = parsed[h]
        issuers = by_subject.get(p["issuer"], [])
        if p["alg"] != OID_ECDSA_SHA256:
            skipped.append({"cert_sha256": h, "why": "signature algorithm is not ecdsa-with-SHA256",
                            "alg": p["alg"].hex()})
            continue
        if not issuers:
            skipped.append({"cert_sha256": h, "why": "issuer certificate not in the reference tree"})
            continue
        # Pick the issuer whose key verifies (a subject name could repeat across stores).
        chosen = None
        for ih in issuers:
            ispki = parsed[ih]["spki"]
            scheme = spki_scheme(ispki)
            if scheme is not None and openssl_verify(ispki, p["sig"], p["tbs"]):
                chosen = (ih, ispki, scheme)
                break
        if chosen is None:
            skipped.append({"cert_sha256": h, "why": "no issuer key in the tree verifies it (openssl)"})
            continue
        ih, ispki, scheme = chosen
        st = oracle_status(scheme, ispki, p["sig"], p["tbs"])
        st_iv = oracle_status(scheme, ispki, p["sig"], p["tbs"], ocorda.MODE_ISVALID)
        items.append({"scheme": scheme, "key_fmt": 1, "key": ispki.hex(), "sig": p["sig"].hex(),
                      "msg": p["tbs"].hex(), "expect": "VALID", "expect_isvalid": "VALID",
                      "class": "E0", "origin": "reference", "oracle": st, "oracle_isvalid": st_iv,
                      "openssl": "VALID", "cert_sha256": h, "issuer_sha256": ih,
                      "note": "; ".join(provenance[h])})
        for cls, note, k2, s2, m2 in variants({"spki": ispki, "sig": p["sig"], "tbs": p["tbs"]}, scheme):
            exp = oracle_status(scheme, k2, s2, m2)
            exp_iv = oracle_status(scheme, k2, s2, m2, ocorda.MODE_ISVALID)
            ossl = None
            if s2 and m2:
                ossl = "VALID" if openssl_verify(k2, s2, m2) else "not VALID"
            items.append({"scheme": scheme, "key_fmt": 1, "key": k2.hex(), "sig": s2.hex(), "msg": m2.hex(),
                          "expect": exp, "expect_isvalid": exp_iv, "class": cls, "origin": "builder-made",
                          "openssl": ossl, "cert_sha256": h, "note": note})
    # Cross-pair: each genuine signature against a different issuer key of the same curve.
    genuine = [it for it in items if it["origin"] == "reference"]
    for a in genuine:
        for b in genuine:
            if b["scheme"] == a["scheme"] and b["key"] != a["key"]:
                k2, s2, m2 = bytes.fromhex(b["key"]), bytes.fromhex(a["sig"]), bytes.fromhex(a["msg"])
                items.append({"scheme": a["scheme"], "key_fmt": 1, "key": b["key"], "sig": a["sig"],
                              "msg": a["msg"], "expect": oracle_status(a["scheme"], k2, s2, m2),
                              "expect_isvalid": oracle_status(a["scheme"], k2, s2, m2, ocorda.MODE_ISVALID),
                              "class": "E9", "origin": "builder-made",
                              "openssl": "VALID" if openssl_verify(k2, s2, m2) else "not VALID",
                              "cert_sha256": a["cert_sha256"], "note": "signature checked under another issuer's key"})
                break
    out = {"meta": {"generator": "tools/gen/ref_vectors.py",
                    "sources": SOURCES,
                    "certificates": len(certs),
                    "genuine_items": len(genuine),
                    "skipped": skipped,
                    "expect": "genuine items: VALID by construction (BC signed them; openssl verifies them); "
                              "builder-made items: oracle/ecdsa_bc.py verdicts, openssl recorded beside them"},
           "items": items}
    dst = os.path.join(ROOT, "tests", "golden", "ref_certs.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(f"{len(certs)} certificates, {len(genuine)} genuine items, {len(items)} items -> {dst}")
    for s in skipped:
        print("skipped:", s)


if __name__ == "__main__":
    main()
