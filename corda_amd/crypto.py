"""Host mirror of Corda's ``Crypto`` verification API over the MI355X engine.

Mirrors core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:
  * ``Crypto.do_verify(public_key, signature_data, clear_data)`` -- Crypto.kt:457 -> :474-484:
    unsupported scheme -> IllegalArgumentException; empty signature / clear data ->
    IllegalArgumentException; verification false -> SignatureException("Signature Verification
    failed!"); returns True.
  * ``Crypto.is_valid(...)`` -- Crypto.kt:536 -> :553-559: returns a boolean; engine exceptions
    propagate.
  * ``Crypto.do_verify_tx(tx_id, transaction_signature)`` / ``is_valid_tx`` -- Crypto.kt:499-502,
    :516-519: the clear data is SignableData(txId, metadata) (corda_amd/signable.py).
  * ``Crypto.verify_batch(items, mode)`` -- the batch overload this engine adds: one status byte
    per item (include/cordagpu.h). Ed25519 / ECDSA items run on the GPU. The schemes the GPU
    returns CG_UNSUPPORTED for are NOT errors -- Corda supports them (Crypto.kt:177-184, :891) --
    and are routed to the host, as the Kotlin binding falls back to ``Crypto.isValid``:
      - RSA_SHA256: corda_amd/hostverify.py;
      - COMPOSITE: corda_amd/composite.py -- the threshold walk on the host, every leaf signature
        expanded into the same GPU batch (isValid semantics over SignableData(txId, leaf meta));
      - SPHINCS-256: no host verifier in this mirror -> UnsupportedOperationException.
    Items decided on the host with an exception the C status bytes cannot express get the
    mirror-only status HOST_EXCEPTION and their exception in ``verify_batch_ex``'s error map.
  * ``Crypto.raise_for_status`` maps a status byte back onto the exception the serial JVM call
    would have thrown, so a batch caller reproduces fail-fast semantics
    (TransactionWithSignatures.kt:58-62) exactly.

Key-decode failures (status KEY_INVALID) are the exceptions the JVM raises when it builds the key
object, before any verification [ext, recalled]: a raw Ed25519 key (Kryo.kt:330-339 ->
i2p GroupElement) -> IllegalArgumentException("not a valid point"); an X.509 key through
Crypto.decodePublicKey (Crypto.kt:349-356, the ECDSA Kryo path Kryo.kt:388-398) ->
InvalidKeySpecException("This public key cannot be decoded, ...").

Public keys are ``PublicKey(scheme, encoded, fmt)`` (fmt: raw / SPKI / SEC1), the byte forms a JVM
caller hands over JNI; two PublicKeys are equal when their X.509 encodings are (as JVM keys are),
and ``CompositeKey`` (corda_amd/composite.py) is a PublicKey too.
"""
import threading
from dataclasses import dataclass

import numpy as np

from . import batch as B
from . import keys as K
from .engine import Engine
from .hostverify import InvalidKeySpecException, UnsupportedOperationException

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
HOST_EXCEPTION = 240  # mirror-only status: decided on the host with an exception (see verify_batch_ex)

__all__ = ["Crypto", "PublicKey", "BatchItem", "TransactionSignature", "SignatureException", "InvalidKeyException",
           "IllegalArgumentException", "InvalidKeySpecException", "UnsupportedOperationException", "HOST_EXCEPTION"]


class SignatureException(Exception):
    """java.security.SignatureException"""


class InvalidKeyException(Exception):
    """java.security.InvalidKeyException"""


class IllegalArgumentException(ValueError):
    """java.lang.IllegalArgumentException"""


@dataclass(frozen=True, eq=False)
class PublicKey:
    scheme: int
    encoded: bytes
    fmt: int = B.KEY_RAW

    def spki(self):
        return K.canonical_spki(self.scheme, self.fmt, self.encoded)

    def __eq__(self, other):
        return isinstance(other, PublicKey) and self.scheme == other.scheme and self.spki() == other.spki()

    def __hash__(self):
        return hash((self.scheme, self.spki()))

    def __repr__(self):
        return f"PublicKey({SCHEME_CODE_NAMES.get(self.scheme, self.scheme)}, {self.spki().hex()[-16:]})"


@dataclass(frozen=True)
class TransactionSignature:
    """TransactionSignature(bytes, by, SignatureMetadata(platformVersion, schemeNumberID))
    (TransactionSignature.kt:14, SignatureMetadata.kt:15)."""
    bytes: bytes
    by: object                 # PublicKey or composite.CompositeKey
    platform_version: int = 1
    scheme_number_id: int = 4


@dataclass(frozen=True)
class BatchItem:
    public_key: object         # PublicKey or composite.CompositeKey
    signature_data: object     # bytes; composite.CompositeSignaturesWithKeys for a CompositeKey
    clear_data: bytes


def key_exception(public_key):
    """The exception the JVM raises building a key object from undecodable bytes [ext, recalled]."""
    if public_key is not None and public_key.scheme == EDDSA_ED25519_SHA512 and public_key.fmt == B.KEY_RAW:
        return IllegalArgumentException("not a valid point")
    return InvalidKeySpecException("This public key cannot be decoded, please ensure it is X509 encoded and that it "
                                   "corresponds to the input scheme's code name.")


class _Crypto:
    def __init__(self):
        self._engine = None
        self._lock = threading.Lock()
        self.last_errors = {}

    def engine(self):
        with self._lock:
            if self._engine is None:
                self._engine = Engine(0)
            return self._engine

    def use_engine(self, engine):
        """Any object with ``verify(batch, mode)``: an Engine (one GPU) or an EnginePool."""
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

    # ------------------------------------------------------------------ batch
    def verify_batch_ex(self, items, mode=B.MODE_DOVERIFY):
        """(status per item, {index: exception}) -- the exception map holds the items whose status
        is HOST_EXCEPTION (host-decided with an exception no C status expresses)."""
        from . import composite as C
        from . import hostverify
        n = len(items)
        st = np.full(n, B.NOT_RUN, dtype=np.uint8)
        errors = {}
        gpu = {B.MODE_DOVERIFY: [], B.MODE_ISVALID: []}   # (ref, BatchItem); ref = item index or (i, j) leaf
        leaves = {}                                        # composite item -> [leaf refs in order]
        host_leaf = {}                                     # (i, j) -> status / exception

        def host_scheme(scheme, pk, sig, msg, m):
            """(status, exception) of a host-verified scheme, isValid / doVerify semantics."""
            try:
                if scheme == RSA_SHA256:
                    key = hostverify.rsa_decode_key(pk.encoded)
                    if m == B.MODE_DOVERIFY and (len(sig) == 0 or len(msg) == 0):
                        return B.EMPTY, None
                    return (B.VALID if hostverify.rsa_verify(key, sig, msg) else B.INVALID), None
                if m == B.MODE_DOVERIFY and (len(sig) == 0 or len(msg) == 0):
                    return B.EMPTY, None
                hostverify.verify(scheme, pk, sig, msg)
            except Exception as e:  # noqa: BLE001 - the reference's exception, kept for the caller
                return HOST_EXCEPTION, e
            return B.NOT_RUN, None

        for i, it in enumerate(items):
            pk = it.public_key
            if pk.scheme not in SCHEME_CODE_NAMES:
                st[i] = B.UNSUPPORTED
                continue
            if pk.scheme in GPU_SCHEMES:
                gpu[mode].append((i, it))
                continue
            if pk.scheme != COMPOSITE_KEY:
                s, e = host_scheme(pk.scheme, pk, it.signature_data, it.clear_data, mode)
                st[i] = s
                if e is not None:
                    errors[i] = e
                continue
            # CompositeSignature engine (CompositeSignature.kt:75-84) behind doVerify / isValid
            try:
                key = pk if isinstance(pk, C.CompositeKey) else C.CompositeKey.get_instance(pk.encoded)
                sig = it.signature_data
                # doVerify's empty checks come first, signature then clear data (Crypto.kt:476-477),
                # before the engine deserialises anything
                if mode == B.MODE_DOVERIFY and not isinstance(sig, C.CompositeSignaturesWithKeys) and len(sig) == 0:
                    st[i] = B.EMPTY
                    continue
                if mode == B.MODE_DOVERIFY and len(it.clear_data) == 0:
                    st[i] = B.EMPTY
                    continue
                if not isinstance(sig, C.CompositeSignaturesWithKeys):
                    sig = C.CompositeSignaturesWithKeys.deserialize(sig)
                if not key.is_fulfilled_by([s.by for s in sig.sigs]):
                    st[i] = B.INVALID
                    continue
                if len(it.clear_data) != 32:
                    raise IllegalArgumentException("Failed requirement.")  # SecureHash.SHA256(buffer)
                refs = []
                for j, (s, msg) in enumerate(C.leaf_messages(sig, it.clear_data)):
                    ref = (i, j)
                    refs.append(ref)
                    if s.by.scheme in GPU_SCHEMES:
                        gpu[B.MODE_ISVALID].append((ref, BatchItem(s.by, s.bytes, msg)))
                    else:  # RSA / SPHINCS leaves on the host; a composite leaf cannot be fulfilled
                        host_leaf[ref] = host_scheme(s.by.scheme, s.by, s.bytes, msg, B.MODE_ISVALID)
                leaves[i] = (refs, sig)
            except Exception as e:  # noqa: BLE001
                st[i] = HOST_EXCEPTION
                errors[i] = e

        leaf_st = {}
        for m, lst in gpu.items():
            if not lst:
                continue
            out = self.engine().verify(self.pack([b for _, b in lst]), m)
            for (ref, _), s in zip(lst, out):
                if isinstance(ref, tuple):
                    leaf_st[ref] = (int(s), None)
                else:
                    st[ref] = s
        for ref, v in host_leaf.items():
            leaf_st[ref] = v
        # the `all { it.isValid(clearData) }` reduction: the first false or exception decides
        for i, (refs, sig) in leaves.items():
            verdict = B.VALID
            for j, ref in enumerate(refs):
                s, e = leaf_st[ref]
                if s == B.VALID:
                    continue
                if s == B.INVALID:
                    verdict = B.INVALID
                    break
                if e is None:
                    leaf = sig.sigs[j]
                    try:
                        self.raise_for_status(s, SCHEME_CODE_NAMES.get(leaf.by.scheme, ""), do_verify=False,
                                              key=leaf.by)
                    except Exception as x:  # noqa: BLE001
                        e = x
                errors[i] = e
                verdict = HOST_EXCEPTION
                break
            st[i] = verdict
        self.last_errors = errors
        return st, errors

    def verify_batch(self, items, mode=B.MODE_DOVERIFY):
        """Batch overload: list[BatchItem] -> numpy uint8 status per item (exceptions of host-decided
        items in ``last_errors``)."""
        if not items:
            self.last_errors = {}
            return np.zeros(0, dtype=np.uint8)
        return self.verify_batch_ex(items, mode)[0]

    # ------------------------------------------------------------------ status -> JVM outcome
    @staticmethod
    def raise_for_status(status, scheme_name="", do_verify=True, error=None, key=None):
        """The exception Crypto.doVerify (do_verify=True) / isValid would raise for `status`,
        or the return value (True / False)."""
        if status == B.VALID:
            return True
        if status == B.INVALID:
            if do_verify:
                raise SignatureException("Signature Verification failed!")
            return False
        if status == HOST_EXCEPTION:
            raise error if error is not None else RuntimeError("host-decided item without its exception")
        if status == B.SIG_MALFORMED:
            raise SignatureException("signature length is wrong" if scheme_name == "EDDSA_ED25519_SHA512"
                                     else "error decoding signature bytes.")
        if status == B.KEY_INVALID:
            raise key_exception(key)
        if status == B.UNSUPPORTED:
            raise IllegalArgumentException(f"Unsupported key/algorithm for schemeCodeName: {scheme_name}")
        if status == B.EMPTY:
            raise IllegalArgumentException("Signature data is empty!")
        raise RuntimeError(f"item not verified (status {status})")

    def _one(self, public_key, signature_data, clear_data, mode):
        scheme = self.find_signature_scheme(public_key)
        st, err = self.verify_batch_ex([BatchItem(public_key, signature_data, clear_data)], mode)
        s = int(st[0])
        if s == B.EMPTY:  # doVerify's own messages, signature first (Crypto.kt:476-477)
            sig_empty = isinstance(signature_data, (bytes, bytearray)) and len(signature_data) == 0
            raise IllegalArgumentException("Signature data is empty!" if sig_empty
                                           else "Clear data is empty, nothing to verify!")
        return self.raise_for_status(s, SCHEME_CODE_NAMES[scheme], do_verify=mode == B.MODE_DOVERIFY,
                                     error=err.get(0), key=public_key)

    def do_verify(self, public_key, signature_data, clear_data):
        """Crypto.doVerify(publicKey, signatureData, clearData) (Crypto.kt:457 -> :474-484)."""
        return self._one(public_key, signature_data, clear_data, B.MODE_DOVERIFY)

    def is_valid(self, public_key, signature_data, clear_data):
        """Crypto.isValid(publicKey, signatureData, clearData) (Crypto.kt:536 -> :553-559)."""
        return self._one(public_key, signature_data, clear_data, B.MODE_ISVALID)

    def do_verify_tx(self, tx_id, ts):
        """Crypto.doVerify(txId, transactionSignature) (Crypto.kt:499-502)."""
        from . import signable
        pre, suf = signable.template(ts.platform_version, ts.scheme_number_id)
        return self.do_verify(ts.by, ts.bytes, pre + bytes(tx_id) + suf)

    def is_valid_tx(self, tx_id, ts):
        """Crypto.isValid(txId, transactionSignature) (Crypto.kt:516-519)."""
        from . import signable
        pre, suf = signable.template(ts.platform_version, ts.scheme_number_id)
        return self.is_valid(ts.by, ts.bytes, pre + bytes(tx_id) + suf)


Crypto = _Crypto()
