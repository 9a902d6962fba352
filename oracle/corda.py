"""Corda-level control flow restated on top of the arithmetic oracles.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* ``verify_item``  = Crypto.doVerify(scheme, pub, sig, clear) / Crypto.isValid(...)
  (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:474-484 and :553-559), mapped
  onto the batch status codes of include/cordagpu.h.
* ``merkle_root``  = MerkleTree.getMerkleTree (MerkleTree.kt:27-66).
* ``compute_nonce`` / ``component_hash`` / ``tx_id`` = MerkleTransaction.kt:16-33,93 and
  WireTransaction.id (WireTransaction.kt:39,104).
* ``check_signatures_are_valid`` = TransactionWithSignatures.checkSignaturesAreValid
  (TransactionWithSignatures.kt:58-62): serial, fail-fast on the first bad signature.
"""
import hashlib
import struct

from . import ecdsa_bc, ed25519_i2p

# ---- status codes (must match include/cordagpu.h) ----
VALID = 0          # isValid == true
INVALID = 1        # isValid == false  (doVerify: SignatureException("Signature Verification failed!"))
SIG_MALFORMED = 2  # engine SignatureException (length / DER decode)
KEY_INVALID = 3    # key decode IllegalArgumentException / InvalidKeyException
UNSUPPORTED = 4    # IllegalArgumentException("Unsupported key/algorithm ...")
EMPTY = 5          # doVerify IllegalArgumentException("Signature data is empty!" / "Clear data is empty ...")
NOT_RUN = 255

STATUS_NAMES = {VALID: "VALID", INVALID: "INVALID", SIG_MALFORMED: "SIG_MALFORMED",
                KEY_INVALID: "KEY_INVALID", UNSUPPORTED: "UNSUPPORTED", EMPTY: "EMPTY", NOT_RUN: "NOT_RUN"}

ECDSA_SECP256K1_SHA256 = 2
ECDSA_SECP256R1_SHA256 = 3
EDDSA_ED25519_SHA512 = 4

KEY_RAW = 0    # Ed25519: 32-byte A (as Kryo writes it, Kryo.kt:333); ECDSA: 64-byte X||Y big-endian
KEY_SPKI = 1   # X.509 SubjectPublicKeyInfo DER (PublicKey.encoded)
KEY_SEC1 = 2   # ECDSA only: 04||X||Y or 02/03||X

MODE_DOVERIFY = 0   # Crypto.doVerify semantics: empty sig / clear -> EMPTY
MODE_ISVALID = 1    # Crypto.isValid semantics: no empty checks

ED25519_SPKI_PREFIX = bytes.fromhex("302a300506032b6570032100")


def decode_key(scheme, key_fmt, key):
    """Returns a decoded key object or raises KeyDecodeError / ValueError."""
    key = bytes(key)
    if scheme == EDDSA_ED25519_SHA512:
        if key_fmt == KEY_SPKI:
            if len(key) != 44 or key[:12] != ED25519_SPKI_PREFIX:
                raise ed25519_i2p.KeyDecodeError("bad SubjectPublicKeyInfo")
            key = key[12:]
        elif key_fmt != KEY_RAW:
            raise ed25519_i2p.KeyDecodeError("bad key format")
        return ed25519_i2p.PublicKey(key)
    if key_fmt == KEY_SPKI:
        return ecdsa_bc.decode_spki(scheme, key)
    if key_fmt == KEY_RAW and len(key) != 64:
        raise ecdsa_bc.KeyDecodeError("bad raw key length")
    if key_fmt not in (KEY_RAW, KEY_SEC1):
        raise ecdsa_bc.KeyDecodeError("bad key format")
    return ecdsa_bc.decode_point(ecdsa_bc.CURVES[scheme], key)


def verify_item(scheme, key_fmt, key, sig, msg, mode=MODE_DOVERIFY, decoded=None):
    """One batch item -> status byte. Precedence: UNSUPPORTED, KEY_INVALID, EMPTY,
    SIG_MALFORMED, INVALID/VALID (key decode happens before doVerify on the JVM)."""
    if scheme not in (ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256, EDDSA_ED25519_SHA512):
        return UNSUPPORTED
    try:
        k = decoded if decoded is not None else decode_key(scheme, key_fmt, key)
    except (ed25519_i2p.KeyDecodeError, ecdsa_bc.KeyDecodeError):
        return KEY_INVALID
    if mode == MODE_DOVERIFY and (len(sig) == 0 or len(msg) == 0):
        return EMPTY
    try:
        if scheme == EDDSA_ED25519_SHA512:
            ok = ed25519_i2p.verify(k, msg, sig)
        else:
            ok = ecdsa_bc.verify(scheme, k, msg, sig)
    except (ed25519_i2p.SignatureLengthError, ecdsa_bc.MalformedSignature):
        return SIG_MALFORMED
    return VALID if ok else INVALID


# ---------------- hashing / Merkle ----------------
ZERO_HASH = bytes(32)


def sha256(b):
    return hashlib.sha256(bytes(b)).digest()


def hash_concat(a, b):
    """SecureHash.hashConcat (SecureHash.kt:25)."""
    return sha256(bytes(a) + bytes(b))


class MerkleTreeException(ValueError):
    pass


def merkle_root(leaves):
    """MerkleTree.getMerkleTree(...).hash (MerkleTree.kt:27-66): empty -> exception,
    zero-hash padding to the next power of two, pairwise SHA256(L||R) per level,
    a single leaf is its own root."""
    if len(leaves) == 0:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    lv = [bytes(x) for x in leaves]
    n = len(lv)
    while n & (n - 1):
        lv.append(ZERO_HASH)
        n += 1
    while len(lv) > 1:
        lv = [hash_concat(lv[i], lv[i + 1]) for i in range(0, len(lv), 2)]
    return lv[0]


def compute_nonce(salt32, index):
    """computeNonce (MerkleTransaction.kt:33): SHA256(salt || BE32(index))."""
    return sha256(bytes(salt32) + struct.pack(">i", index))


def component_hash(blob, salt32, index, is_salt=False):
    """serializedHash(x, privacySalt, index) (MerkleTransaction.kt:16-25)."""
    if is_salt:
        return sha256(blob)
    return sha256(bytes(blob) + compute_nonce(salt32, index))


def tx_id(component_blobs, salt32, salt_blob):
    """WireTransaction.id: Merkle root over availableComponentHashes, the salt's own
    serialised blob appended last (MerkleTransaction.kt:74-93)."""
    hashes = [component_hash(b, salt32, i) for i, b in enumerate(component_blobs)]
    hashes.append(component_hash(salt_blob, salt32, len(component_blobs), is_salt=True))
    return merkle_root(hashes)


class SignatureException(Exception):
    pass


def check_signatures_are_valid(tx_id_bytes, sigs, message_of):
    """TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-62)
    restated over status codes: returns the index of the first non-VALID signature and its
    status (fail-fast order), or (None, VALID)."""
    for i, (scheme, key_fmt, key, sig, meta) in enumerate(sigs):
        st = verify_item(scheme, key_fmt, key, sig, message_of(tx_id_bytes, meta))
        if st != VALID:
            return i, st
    return None, VALID
