"""Host-side verification for the schemes the GPU engine does not run (status CG_UNSUPPORTED):
the mirror of the JVM falling back to ``Crypto.isValid`` for them ("RSA (id 1),
SPHINCS (id 5) and COMPOSITE (id 6) return CG_UNSUPPORTED, and the Kotlin side falls back to
Crypto.isValid"). Corda accepts all three (Crypto.kt:177-184, isSupportedSignatureScheme :891).

* RSA_SHA256 (scheme 1, BouncyCastle "SHA256WITHRSAANDMGF1", Crypto.kt:78-89): RSASSA-PSS with
  SHA-256, MGF1(SHA-256), a 32-byte salt and trailer 0xBC, restated from BC 1.57
  ``PSSSignatureSpi.SHA256withRSA`` -> ``PSSSigner.verifySignature`` over ``RSABlindedEngine``
  [ext, recalled]: every failure, including an input longer than the modulus or >= n (the
  engine's DataLengthException is caught inside verifySignature), is ``false``, never an
  exception; the top bits of the encoded message beyond emBits are masked, not checked. A
  PKCS#1 v1.5 signature is ``false``. Pinned by OpenSSL PSS fixtures (tests/golden/rsa.json,
  tests/golden/gen_rsa.py) with OpenSSL's own verdict per item.
* COMPOSITE (scheme 6): corda_amd/composite.py (threshold logic on the host, leaves on the GPU).
* SPHINCS-256 (scheme 5): no host verifier in this mirror (BC's PQC provider is not restated);
  ``verify`` raises UnsupportedOperationException. A JVM caller still falls back to its own
  ``Crypto.isValid`` for it.
"""
import hashlib

from . import der

RSA_OID = der.oid("1.2.840.113549.1.1.1")
PSS_SALT_LEN = 32   # PSSSignatureSpi.SHA256withRSA: new PSSParameterSpec("SHA-256", "MGF1", SHA256, 32, 1)
PSS_TRAILER = 0xBC


class UnsupportedOperationException(Exception):
    """java.lang.UnsupportedOperationException"""


class InvalidKeySpecException(Exception):
    """java.security.spec.InvalidKeySpecException (Crypto.decodePublicKey, Crypto.kt:349-356)"""


def rsa_decode_key(encoded):
    """SPKI -> (n, e); InvalidKeySpecException for anything else."""
    try:
        alg, params, bits = der.read_spki(encoded)
        if alg != RSA_OID or params not in (b"", der.tlv(0x05, b"")):
            raise der.DerError("not an rsaEncryption key")
        seq = der.read_seq(bits)
        if len(seq) != 2:
            raise der.DerError("RSAPublicKey is not 2 INTEGERs")
        n, e = der.read_integer(*seq[0]), der.read_integer(*seq[1])
        if n <= 0 or e <= 0:
            raise der.DerError("non-positive modulus or exponent")
        return n, e
    except der.DerError as x:
        raise InvalidKeySpecException(f"This public key cannot be decoded, please ensure it is X509 encoded and "
                                      f"that it corresponds to the input scheme's code name. ({x})") from None


def mgf1_sha256(seed, length):
    out = bytearray()
    counter = 0
    while len(out) < length:
        out += hashlib.sha256(bytes(seed) + counter.to_bytes(4, "big")).digest()
        counter += 1
    return bytes(out[:length])


def rsa_verify(key, sig, msg):
    """SHA256WITHRSAANDMGF1 (BC PSSSigner.verifySignature) -> bool."""
    n, e = key
    h_len = s_len = 32
    k = (n.bit_length() + 7) // 8
    em_bits = n.bit_length() - 1
    block_len = (em_bits + 7) // 8
    sig = bytes(sig)
    if len(sig) > k:                       # RSACoreEngine.convertInput: DataLengthException, caught
        return False
    s = int.from_bytes(sig, "big")
    if s >= n:
        return False
    m = pow(s, e, n)
    mb = m.to_bytes((m.bit_length() + 7) // 8, "big")
    if len(mb) > block_len:                # does not fit the emBits block: caught, false
        return False
    block = bytearray(block_len - len(mb)) + mb
    if block[-1] != PSS_TRAILER:
        return False
    db_len = block_len - h_len - 1
    if db_len < s_len + 1:
        return False
    h = bytes(block[db_len:db_len + h_len])
    db = bytearray(a ^ b for a, b in zip(block[:db_len], mgf1_sha256(h, db_len)))
    db[0] &= 0xFF >> (8 * block_len - em_bits)
    if any(db[:block_len - h_len - s_len - 2]) or db[block_len - h_len - s_len - 2] != 0x01:
        return False
    salt = bytes(db[db_len - s_len:db_len])
    return hashlib.sha256(bytes(8) + hashlib.sha256(bytes(msg)).digest() + salt).digest() == h


def rsa_pss_sign(n, d, msg, salt):
    """EMSA-PSS encode + RSA (test helper for fixtures; the reference's signer is BC PSSSigner)."""
    h_len = 32
    em_bits = n.bit_length() - 1
    block_len = (em_bits + 7) // 8
    mh = hashlib.sha256(bytes(8) + hashlib.sha256(bytes(msg)).digest() + bytes(salt)).digest()
    db = bytes(block_len - len(salt) - h_len - 2) + b"\x01" + bytes(salt)
    masked = bytearray(a ^ b for a, b in zip(db, mgf1_sha256(mh, len(db))))
    masked[0] &= 0xFF >> (8 * block_len - em_bits)
    em = bytes(masked) + mh + bytes([PSS_TRAILER])
    return pow(int.from_bytes(em, "big"), d, n).to_bytes((n.bit_length() + 7) // 8, "big")


def verify(scheme, public_key, sig, msg):
    """Crypto.isValid for a host-verified scheme -> bool, or raises the reference's exception."""
    if scheme == 1:
        return rsa_verify(rsa_decode_key(public_key.encoded), sig, msg)
    raise UnsupportedOperationException(
        f"no host verifier for scheme {scheme} in this mirror; the JVM caller falls back to its own Crypto.isValid")
