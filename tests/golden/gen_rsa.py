"""Generates tests/golden/rsa.json: SHA256WITHRSAANDMGF1 (Corda RSA_SHA256, scheme 1,
Crypto.kt:78-89) fixtures for the host fallback (corda_amd/hostverify.py): RSASSA-PSS with
SHA-256, MGF1(SHA-256), 32-byte salt. Signatures and keys come from the OpenSSL 3 CLI (run here
once; the fixture is committed); every item records OpenSSL's own accept / reject as the pin.
`expect` is the BC 1.57 PSSSigner restatement's outcome: VALID or INVALID (verifySignature
returns false for every failure, including PKCS#1 v1.5 signatures, inputs >= n and inputs
longer than the modulus).

usage: python tests/golden/gen_rsa.py  (needs the openssl CLI)
"""
import json
import os
import random
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
PSS = ["-sigopt", "rsa_padding_mode:pss", "-sigopt", "rsa_pss_saltlen:32", "-sigopt", "rsa_mgf1_md:sha256"]


def sh(*args, data=None):
    return subprocess.run(args, input=data, capture_output=True, check=True).stdout


def ossl_verify(pub_der, msg, sig, d):
    kp, mp, sp = (os.path.join(d, n) for n in ("k.der", "m.bin", "s.bin"))
    open(kp, "wb").write(pub_der)
    open(mp, "wb").write(msg)
    open(sp, "wb").write(sig)
    r = subprocess.run(["openssl", "dgst", "-sha256", "-keyform", "DER", "-verify", kp] + PSS +
                       ["-signature", sp, mp], capture_output=True)
    return "accept" if r.returncode == 0 else "reject"


def main():
    rng = random.Random(0x45A)
    items = []
    private = None
    with tempfile.TemporaryDirectory() as d:
        for bits in (2048, 1024, 3072):
            key = os.path.join(d, f"k{bits}.pem")
            sh("openssl", "genrsa", "-out", key, str(bits))
            pub = sh("openssl", "rsa", "-in", key, "-pubout", "-outform", "DER")
            if private is None:  # one TEST key's private exponent, so tests can sign new messages
                txt = sh("openssl", "rsa", "-in", key, "-text", "-noout").decode()

                def field(name, nxt):
                    body = txt.split(name + ":")[1].split(nxt)[0]
                    return int("".join(body.split()).replace(":", ""), 16)
                private = {"spki": pub.hex(), "n": hex(field("modulus", "publicExponent")),
                           "d": hex(field("privateExponent", "prime1")), "e": 65537,
                           "note": "test-only key, generated for this fixture"}
            for k in range(4):
                msg = bytes(rng.randrange(256) for _ in range(rng.choice([1, 32, 270, 700])))
                mp = os.path.join(d, "m.bin")
                open(mp, "wb").write(msg)
                sig = sh("openssl", "dgst", "-sha256", "-sign", key, *PSS, mp)
                v15 = sh("openssl", "dgst", "-sha256", "-sign", key, mp)
                cases = [("valid", msg, sig, "VALID"),
                         ("PKCS#1 v1.5 signature of the same message (not Corda's scheme)", msg, v15, "INVALID")]
                m2 = bytearray(msg)
                m2[rng.randrange(len(m2))] ^= 1 << rng.randrange(8)
                cases.append(("flip message bit", bytes(m2), sig, "INVALID"))
                s2 = bytearray(sig)
                s2[rng.randrange(len(s2))] ^= 1 << rng.randrange(8)
                cases.append(("flip signature bit", msg, bytes(s2), "INVALID"))
                if k == 0:
                    cases.append(("signature longer than the modulus", msg, b"\x00" + sig, "INVALID"))
                    cases.append(("signature >= n", msg, b"\xff" * len(sig), "INVALID"))
                    cases.append(("empty signature", msg, b"", "INVALID"))
                for note, m, s, exp in cases:
                    items.append({"scheme": 1, "key_fmt": 1, "key": pub.hex(), "sig": s.hex(), "msg": m.hex(),
                                  "bits": bits, "note": note, "expect": exp,
                                  "openssl": ossl_verify(pub, m, s, d)})
        # the same valid signature against another modulus: decodes to garbage padding
        a, b = items[0], items[len(items) // 2]
        items.append({"scheme": 1, "key_fmt": 1, "key": b["key"], "sig": a["sig"], "msg": a["msg"], "bits": b["bits"],
                      "note": "signature of another key", "expect": "INVALID",
                      "openssl": ossl_verify(bytes.fromhex(b["key"]), bytes.fromhex(a["msg"]), bytes.fromhex(a["sig"]),
                                             d)})
    meta = {"generator": "tests/golden/gen_rsa.py", "openssl": sh("openssl", "version").decode().strip(),
            "note": "expect = BC 1.57 PSSSigner restatement (hostverify.py); openssl = OpenSSL's PSS verdict"}
    with open(os.path.join(HERE, "rsa.json"), "w") as f:
        json.dump({"meta": meta, "test_private_key": private, "items": items}, f, indent=0)
    print(len(items), "items")


if __name__ == "__main__":
    main()
