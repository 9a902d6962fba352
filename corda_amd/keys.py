"""Canonical X.509 SubjectPublicKeyInfo of a public key: what ``PublicKey.getEncoded()`` returns
on the JVM for every scheme, whatever byte form the caller handed over (raw, SPKI, SEC1). Used
for key equality (a JVM key equals another of the same point: i2p compares Abyte, BC compares Q)
and for CompositeKey child ordering (NodeAndWeight.compareTo over node.encoded,
CompositeKey.kt:146-151). Host-side only."""
from . import der

ED25519_SPKI_PREFIX = bytes.fromhex("302a300506032b6570032100")
EC_SPKI_PREFIX = {  # id-ecPublicKey + named curve, uncompressed point (BC's default encoding)
    3: bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200"),   # secp256r1
    2: bytes.fromhex("3056301006072a8648ce3d020106052b8104000a034200"),         # secp256k1
}
_P = {3: 2**256 - 2**224 + 2**192 + 2**96 - 1, 2: 2**256 - 2**32 - 977}
_B = {3: 0x5ac635d8aa3a93e7b3ebbd55769886bc651d06b0cc53b0f63bce3c3e27d2604b, 2: 7}
_A = {3: -3, 2: 0}
KEY_RAW, KEY_SPKI, KEY_SEC1 = 0, 1, 2


ED25519_SPKI_PREFIX_NULL = bytes.fromhex("302c300706032b65700500032100")  # NULL parameters


def _ec_spki_header(scheme, point_len):
    pre = bytearray(EC_SPKI_PREFIX[scheme])
    pre[1] -= 65 - point_len   # outer SEQUENCE length
    pre[-2] -= 65 - point_len  # BIT STRING length
    return bytes(pre)


def _ec_uncompressed(scheme, b):
    """04 || X || Y from a raw 64-byte X||Y or a SEC1 point (uncompressed, hybrid, compressed);
    None if it cannot be formed."""
    p = _P[scheme]
    if len(b) == 64:
        return b"\x04" + b
    if len(b) == 65 and b[0] == 4:
        return b
    if len(b) == 65 and b[0] in (6, 7):
        return b"\x04" + b[1:] if (b[64] & 1) == (b[0] & 1) else None
    if len(b) == 33 and b[0] in (2, 3):
        x = int.from_bytes(b[1:], "big")
        if x >= p:
            return None
        y2 = (pow(x, 3, p) + _A[scheme] * x + _B[scheme]) % p
        y = pow(y2, (p + 1) // 4, p)  # p = 3 mod 4 for both curves
        if y * y % p != y2:
            return None
        if (y & 1) != (b[0] & 1):
            y = p - y
        return b"\x04" + x.to_bytes(32, "big") + y.to_bytes(32, "big")
    return None


def canonical_spki(scheme, fmt, encoded):
    """SPKI bytes the JVM key object would report, or the input bytes when they cannot be put in
    that form (such a key fails to decode on the JVM and on the GPU alike)."""
    b = bytes(encoded)
    if fmt == KEY_SPKI:
        # the JVM key object re-encodes the forms Crypto.decodePublicKey accepts canonically
        # (i2p: absent parameters; BC: uncompressed point)
        if scheme == 4 and len(b) == 46 and b[:14] == ED25519_SPKI_PREFIX_NULL:
            return ED25519_SPKI_PREFIX + b[14:]
        if scheme in EC_SPKI_PREFIX:
            for plen in (65, 33):
                h = _ec_spki_header(scheme, plen)
                if len(b) == len(h) + plen and b[:len(h)] == h:
                    u = _ec_uncompressed(scheme, b[len(h):])
                    return EC_SPKI_PREFIX[scheme] + u if u is not None else b
        return b
    if scheme == 4 and fmt == KEY_RAW and len(b) == 32:
        return ED25519_SPKI_PREFIX + b
    if scheme in EC_SPKI_PREFIX and fmt in (KEY_RAW, KEY_SEC1):
        u = _ec_uncompressed(scheme, b)
        if u is not None:  # the prefix ends with the BIT STRING header 03 42 00; 04 || X || Y follows
            return EC_SPKI_PREFIX[scheme] + u
    return b


def compare_encoded(a, b):
    """ByteSequence.compareTo (utilities/ByteArrays.kt:73-85): unsigned lexicographic, then size."""
    for x, y in zip(a, b):
        if x != y:
            return -1 if x < y else 1
    return (len(a) > len(b)) - (len(a) < len(b))


def decode_spki_key(encoded):
    """Crypto.decodePublicKey(encodedKey) (Crypto.kt:321-325) for the mirror: the scheme from the
    algorithm identifier, the key kept in SPKI form. CompositeKey SPKIs are returned by
    corda_amd.composite (it calls this for its children)."""
    from .composite import COMPOSITE_OID, CompositeKey
    from .crypto import IllegalArgumentException, PublicKey
    alg, params, _ = der.read_spki(encoded)
    if alg == COMPOSITE_OID:
        return CompositeKey.get_instance(encoded)
    if alg == der.oid("1.3.101.112"):
        return PublicKey(4, bytes(encoded), KEY_SPKI)
    if alg == der.oid("1.2.840.10045.2.1"):
        if params == der.oid("1.2.840.10045.3.1.7"):
            return PublicKey(3, bytes(encoded), KEY_SPKI)
        if params == der.oid("1.3.132.0.10"):
            return PublicKey(2, bytes(encoded), KEY_SPKI)
    if alg == der.oid("1.2.840.113549.1.1.1"):
        return PublicKey(1, bytes(encoded), KEY_SPKI)
    raise IllegalArgumentException(f"Unrecognised algorithm: {alg.hex()}")
