"""Host mirror of Corda's ``Crypto`` verification API over the MI355X engine.

Mirrors core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:
  * ``Crypto.do_verify(scheme, public_key, signature_data, clear_data)`` — Crypto.kt:474-484:
    unsupported scheme -> IllegalArgumentException; empty signature / clear data ->
    IllegalArgumentException; verification false -> SignatureException("Signature
    Verification failed!"); returns True.
  * ``Crypto.is_valid(...)`` — Crypto.kt:553-559: returns a boolean; engine-level failures
    (malformed signature encoding) raise SignatureException, bad keys InvalidKeyException.
  * ``Crypto.verify_batch(items, mode)`` — the batch overload this engine adds: one status
    byte per item (include/cordagpu.h), computed on the GPU.
  * ``Crypto.raise_for_status`` maps a status byte back onto the exception the serial JVM
    call would have thrown, so a batch caller can reproduce fail-fast semantics
    (TransactionWithSignatures.kt:58-62) exactly.

Public keys are passed as ``PublicKey(scheme, encoded, fmt)`` (fmt: raw / SPKI / SEC1), the
byte forms a JVM caller would hand over JNI.
"""
import threading
from dataclasses import dataclass

from . import batch as B
from .engine import Engine

RSA_SHA256 = 1
ECDSA_SECP256K1_SHA256 = B.ECDSA_SECP256K1_SHA256
ECDSA_SECP256R1_SHA256 = B.ECDSA_SECP256R1_SHA256
EDDSA_ED25519_SHA512 = B.EDDSA_ED25519_SHA512
SPHINCS256_SHA256 = 5
COMPOSITE_KEY = 6

SCHEME_CODE_NAMES = {
    RSA_SHA256: "RSA_SHA256",
    ECDSA_SECP256K1_SHA256: "ECDSA_SECP256K1_SHA256",
    ECDSA_SECP256R1_SHA256: "ECDSA_SECP256R1_SHA256",
    EDDSA_ED25519_SHA512: "EDDSA_ED25519_SHA512",
    SPHINCS256_SHA256: "SPHINCS-256_SHA512",
    COMPOSITE_KEY: "COMPOSITE",
}
GPU_SCHEMES = (ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256, EDDSA_ED25519_SHA512)


class SignatureException(Exception):
    """java.security.SignatureException"""


class InvalidKeyException(Exception):
    """java.security.InvalidKeyException"""


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException"""


@dataclass(frozen=True)
class PublicKey:
    scheme: int
    encoded: bytes
    fmt: int = B.KEY_RAW


@dataclass(frozen=True)
class BatchItem:
    public_key: PublicKey
    signature_data: bytes
    clear_data: bytes


class _Crypto:
    def __init__(self):
        self._engine = None
        self._lock = threading.Lock()

    def engine(self):
        with self._lock:
            if self._engine is None:
                self._engine = Engine(0)
            return self._engine

    def use_engine(self, engine):
        with self._lock:
            self._engine = engine

    @staticmethod
    def find_signature_scheme(public_key):
        if public_key.scheme not in SCHEME_CODE_NAMES:
            raise IllegalArgumentException(f"Unsupported key/algorithm for schemeCodeName: {public_key.scheme}")
        return public_key.scheme

    @staticmethod
    def pack(items):
        b = B.BatchBuilder()
        for it in items:
            b.add_with_key(it.public_key.scheme, it.public_key.fmt, it.public_key.encoded, it.signature_data,
                           it.clear_data)
        return b.build()

    def verify_batch(self, items, mode=B.MODE_DOVERIFY):
        """Batch overload: list[BatchItem] -> numpy uint8 status per item (GPU)."""
        if not items:
            import numpy as np
            return np.zeros(0, dtype=np.uint8)
        return self.engine().verify(self.pack(items), mode)

    @staticmethod
    def raise_for_status(status, scheme_name="", do_verify=True):
        """The exception Crypto.doVerify (do_verify=True) / isValid would raise for `status`,
        or the return value (True / False)."""
        if status == B.VALID:
            return True
        if status == B.INVALID:
            if do_verify:
                raise SignatureException("Signature Verification failed!")
            return False
        if status == B.SIG_MALFORMED:
            raise SignatureException("signature length is wrong" if scheme_name == "EDDSA_ED25519_SHA512"
                                     else "error decoding signature bytes.")
        if status == B.KEY_INVALID:
            raise InvalidKeyException("public key could not be decoded")
        if status == B.UNSUPPORTED:
            raise IllegalArgumentException(f"Unsupported key/algorithm for schemeCodeName: {scheme_name}")
        if status == B.EMPTY:
            raise IllegalArgumentException("Signature data is empty!")
        raise RuntimeError(f"item not verified (status {status})")

    def do_verify(self, public_key, signature_data, clear_data):
        """Crypto.doVerify(publicKey, signatureData, clearData) (Crypto.kt:457 -> :474-484)."""
        scheme = self.find_signature_scheme(public_key)
        if scheme not in GPU_SCHEMES:
            raise IllegalArgumentException(
                f"Unsupported key/algorithm for schemeCodeName: {SCHEME_CODE_NAMES[scheme]}")
        if len(signature_data) == 0:
            raise IllegalArgumentException("Signature data is empty!")
        if len(clear_data) == 0:
            raise IllegalArgumentException("Clear data is empty, nothing to verify!")
        st = int(self.verify_batch([BatchItem(public_key, signature_data, clear_data)], B.MODE_DOVERIFY)[0])
        return self.raise_for_status(st, SCHEME_CODE_NAMES[scheme], do_verify=True)

    def is_valid(self, public_key, signature_data, clear_data):
        """Crypto.isValid(publicKey, signatureData, clearData) (Crypto.kt:536 -> :553-559)."""
        scheme = self.find_signature_scheme(public_key)
        if scheme not in GPU_SCHEMES:
            raise IllegalArgumentException(
                f"Unsupported key/algorithm for schemeCodeName: {SCHEME_CODE_NAMES[scheme]}")
        st = int(self.verify_batch([BatchItem(public_key, signature_data, clear_data)], B.MODE_ISVALID)[0])
        return self.raise_for_status(st, SCHEME_CODE_NAMES[scheme], do_verify=False)


Crypto = _Crypto()
