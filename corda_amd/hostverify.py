"""Host-side verification for the schemes the GPU engine does not run (status CG_UNSUPPORTED):
the mirror of the JVM falling back to ``Crypto.isValid`` for them ("RSA (id 1),
SPHINCS (id 5) and COMPOSITE (id 6) return CG_UNSUPPORTED, and the Kotlin side falls back to
Crypto.isValid"). Corda accepts all three (Crypto.kt:177-184, isSupportedSignatureScheme :891).

* RSA_SHA256 (scheme 1, "SHA256WITHRSA" on BouncyCastle, Crypto.kt:78-91): PKCS#1 v1.5 signature
  verification, restated from BC 1.57 ``DigestSignatureSpi.engineVerify`` over
  ``PKCS1Encoding(RSABlindedEngine)`` [ext, recalled]: an input of k+1 or more bytes, or >= n, and
  a block whose type-1 padding is wrong (not 00 01, fewer than 8 FF bytes, a non-FF pad byte)
  throw SignatureException; a well-padded block whose DigestInfo differs from SHA-256(msg) is
  ``false``; the DigestInfo is accepted with or without the NULL parameters. Pinned by the
  OpenSSL-generated fixtures in tests/golden/rsa.json (valid, wrong message, wrong key, corrupt
  signature); the exception-vs-false split and the NULL-less form are unpinned.
* COMPOSITE (scheme 6): corda_amd/composite.py (threshold logic on the host, leaves on the GPU).
* SPHINCS-256 (scheme 5): no host verifier in this mirror (BC's PQC provider is not restated);
  ``verify`` raises UnsupportedOperationException. A JVM caller still falls back to its own
  ``Crypto.isValid`` for it.
"""
import hashlib

from . import der

RSA_OID = der.oid("1.2.840.113549.1.1.1")
_SHA256_DIGESTINFO = bytes.fromhex("3031300d060960864801650304020105000420")
_SHA256_DIGESTINFO_NO_NULL = bytes.fromhex("302f300b0609608648016503040201" "0420")


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


def rsa_verify(key, sig, msg):
    """SHA256withRSA; returns bool or raises SignatureException (crypto.SignatureException)."""
    from .crypto import SignatureException
    n, e = key
    k = (n.bit_length() + 7) // 8
    sig = bytes(sig)
    if len(sig) > k:
        raise SignatureException("org.bouncycastle.crypto.DataLengthException: input too large for RSA cipher.")
    s = int.from_bytes(sig, "big")
    if s >= n:
        raise SignatureException("org.bouncycastle.crypto.DataLengthException: input too large for RSA cipher.")
    em = pow(s, e, n).to_bytes(k, "big")
    if em[0] != 0 or em[1] != 1:
        raise SignatureException("org.bouncycastle.crypto.InvalidCipherTextException: block incorrect")
    i = 2
    while i < len(em) and em[i] == 0xFF:
        i += 1
    if i >= len(em) or em[i] != 0 or i - 2 < 8:
        raise SignatureException("org.bouncycastle.crypto.InvalidCipherTextException: block incorrect")
    t = em[i + 1:]
    h = hashlib.sha256(bytes(msg)).digest()
    return t == _SHA256_DIGESTINFO + h or t == _SHA256_DIGESTINFO_NO_NULL + h


def verify(scheme, public_key, sig, msg):
    """Crypto.isValid for a host-verified scheme -> bool, or raises the reference's exception."""
    if scheme == 1:
        return rsa_verify(rsa_decode_key(public_key.encoded), sig, msg)
    raise UnsupportedOperationException(
        f"no host verifier for scheme {scheme} in this mirror; the JVM caller falls back to its own Crypto.isValid")
