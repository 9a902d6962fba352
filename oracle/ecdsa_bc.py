"""Python restatement of SHA256withECDSA verification as BouncyCastle 1.57 does it.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Never imported by the product path.

BouncyCastle (org.bouncycastle:bcprov-jdk15on:1.57, ``constants.properties``
bouncycastleVersion, core/build.gradle:70) is an un-vendored dependency; Corda calls it
through JCA at core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559 for schemes
ECDSA_SECP256K1_SHA256 (id 2, Crypto.kt:92-103) and ECDSA_SECP256R1_SHA256 (id 3,
Crypto.kt:106-117). Published algorithm restated:

DSABase.engineVerify(sigBytes):
  hash = SHA-256(M)
  try { (r, s) = StdDSAEncoder.decode(sigBytes) } catch (Exception) {
      throw SignatureException("error decoding signature bytes.") }
  return ECDSASigner.verifySignature(hash, r, s)

StdDSAEncoder.decode: ASN1Primitive.fromByteArray (one object, no trailing data),
  must be a SEQUENCE of exactly 2 elements, its DER re-encoding must equal the input
  (CVE-2016-1000338/-1000342 fix, 1.56+), both elements ASN1Integer (non-minimal
  INTEGER contents rejected as malformed), values are signed two's complement.

ECDSASigner.verifySignature: e = hash as unsigned integer (256-bit n => no
  truncation); r, s must be in [1, n-1] else false; c = s^-1 mod n; u1 = e c mod n;
  u2 = r c mod n; R = u1 G + u2 Q; R = infinity -> false; accept iff x(R) == r (mod n).
  High-S is accepted (no low-S rule).

Public key (BCECPublicKey from SPKI / ECCurve.decodePoint): coordinates must be field
elements (< p) and the point must be on the curve, else IllegalArgumentException at
key decode (=> KEY_INVALID here).
"""
import hashlib


class Curve:
    def __init__(self, name, p, a, b, gx, gy, n):
        self.name, self.p, self.a, self.b, self.n = name, p, a, b, n
        self.G = (gx, gy)

    def on_curve(self, pt):
        x, y = pt
        return (y * y - (x * x * x + self.a * x + self.b)) % self.p == 0


P256 = Curve(
    "secp256r1",
    0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFF,
    0xFFFFFFFF00000001000000000000000000000000FFFFFFFFFFFFFFFFFFFFFFFC,
    0x5AC635D8AA3A93E7B3EBBD55769886BC651D06B0CC53B0F63BCE3C3E27D2604B,
    0x6B17D1F2E12C4247F8BCE6E563A440F277037D812DEB33A0F4A13945D898C296,
    0x4FE342E2FE1A7F9B8EE7EB4A7C0F9E162BCE33576B315ECECBB6406837BF51F5,
    0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
)
K256 = Curve(
    "secp256k1",
    0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEFFFFFC2F,
    0,
    7,
    0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
    0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8,
    0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141,
)
CURVES = {2: K256, 3: P256}   # Corda schemeNumberID -> curve


class KeyDecodeError(ValueError):
    """IllegalArgumentException from BC point decoding (=> InvalidKeyException)."""


class MalformedSignature(ValueError):
    """SignatureException("error decoding signature bytes.")."""


# ---------------- affine group law with infinity (None) ----------------
def ec_add(c, P1, P2):
    if P1 is None:
        return P2
    if P2 is None:
        return P1
    p = c.p
    x1, y1 = P1
    x2, y2 = P2
    if x1 == x2:
        if (y1 + y2) % p == 0:
            return None
        lam = (3 * x1 * x1 + c.a) * pow(2 * y1, p - 2, p) % p
    else:
        lam = (y2 - y1) * pow(x2 - x1, p - 2, p) % p
    x3 = (lam * lam - x1 - x2) % p
    return (x3, (lam * (x1 - x3) - y1) % p)


def ec_mul(c, k, P1):
    R = None
    Q = P1
    while k > 0:
        if k & 1:
            R = ec_add(c, R, Q)
        Q = ec_add(c, Q, Q)
        k >>= 1
    return R


# ---------------- key decode ----------------
SPKI_PREFIX = {
    3: bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200"),
    2: bytes.fromhex("3056301006072a8648ce3d020106052b8104000a034200"),
}


def decode_point(c, data):
    """SEC1 point (04||X||Y, 06/07||X||Y hybrid, 02/03||X) or raw 64-byte X||Y -> affine point.
    Mirrors ECCurve.decodePoint + validation (coordinates < p, on curve; a hybrid encoding's
    tag must carry y's parity; the point at infinity (00) is rejected by ECPublicKeyParameters)."""
    p = c.p
    if len(data) == 64:
        data = b"\x04" + bytes(data)
    if len(data) == 65 and data[0] in (4, 6, 7):
        x = int.from_bytes(data[1:33], "big")
        y = int.from_bytes(data[33:65], "big")
        if x >= p or y >= p:
            raise KeyDecodeError("x value invalid in Fp field element")
        if data[0] != 4 and (y & 1) != (data[0] & 1):
            raise KeyDecodeError("Inconsistent Y coordinate in hybrid encoding")
        if not c.on_curve((x, y)):
            raise KeyDecodeError("Invalid point coordinates")
        return (x, y)
    if len(data) == 33 and data[0] in (2, 3):
        x = int.from_bytes(data[1:33], "big")
        if x >= p:
            raise KeyDecodeError("x value invalid in Fp field element")
        rhs = (x * x * x + c.a * x + c.b) % p
        y = pow(rhs, (p + 1) // 4, p)          # p = 3 mod 4 for both curves
        if y * y % p != rhs:
            raise KeyDecodeError("Invalid point compression")
        if (y & 1) != (data[0] & 1):
            y = p - y if y else y
        return (x, y)
    raise KeyDecodeError("Invalid point encoding")


def spki_prefix(scheme, point_len):
    """DER header of SEQUENCE{AlgorithmIdentifier{id-ecPublicKey, namedCurve}, BIT STRING} for a
    point of point_len bytes (65: uncompressed / hybrid, 33: compressed)."""
    pre = bytearray(SPKI_PREFIX[scheme])
    pre[1] -= 65 - point_len          # outer SEQUENCE length
    pre[-2] -= 65 - point_len         # BIT STRING length (unused-bits byte + point)
    return bytes(pre)


def decode_spki(scheme, data):
    """Crypto.decodePublicKey (Crypto.kt:321-325) for an EC key: the algorithm identifier must be
    this scheme's (id-ecPublicKey + its named curve, Crypto.kt:96/110), DER with no trailing data;
    the point is whatever ECCurve.decodePoint accepts (uncompressed, compressed, hybrid)."""
    data = bytes(data)
    for plen in (65, 33):
        pre = spki_prefix(scheme, plen)
        if len(data) == len(pre) + plen and data[: len(pre)] == pre:
            return decode_point(CURVES[scheme], data[len(pre):])
    raise KeyDecodeError("bad SubjectPublicKeyInfo")


# ---------------- DER (StdDSAEncoder.decode, BC 1.57) ----------------
def _read_len(b, i):
    if i >= len(b):
        raise MalformedSignature("truncated")
    l0 = b[i]
    i += 1
    if l0 < 0x80:
        return l0, i
    nb = l0 & 0x7F
    if nb == 0 or nb > 4 or i + nb > len(b):
        raise MalformedSignature("bad length")      # indefinite/huge: not DER
    v = int.from_bytes(b[i:i + nb], "big")
    return v, i + nb


def _der_len(n):
    if n < 0x80:
        return bytes([n])
    nb = (n.bit_length() + 7) // 8
    return bytes([0x80 | nb]) + n.to_bytes(nb, "big")


def der_decode_sig(sig):
    """Returns (r, s) as signed ints, or raises MalformedSignature.

    Accepted iff the input is exactly the DER encoding SEQUENCE{INTEGER r, INTEGER s}:
    tag 0x30, minimal definite length, no trailing bytes, exactly two elements, each
    tag 0x02 with minimal length and minimal non-empty two's complement contents."""
    b = bytes(sig)
    if len(b) < 2 or b[0] != 0x30:
        raise MalformedSignature("not a SEQUENCE")
    seqlen, i = _read_len(b, 1)
    if i + seqlen != len(b):
        raise MalformedSignature("length mismatch / trailing data")
    if _der_len(seqlen) != b[1:i]:
        raise MalformedSignature("non-minimal length")
    vals = []
    while i < len(b):
        if b[i] != 0x02:
            raise MalformedSignature("element is not an INTEGER")
        ln, j = _read_len(b, i + 1)
        if _der_len(ln) != b[i + 1:j]:
            raise MalformedSignature("non-minimal length")
        if j + ln > len(b):
            raise MalformedSignature("truncated INTEGER")
        content = b[j:j + ln]
        if ln == 0:
            raise MalformedSignature("zero length INTEGER")
        if ln > 1 and ((content[0] == 0 and content[1] < 0x80) or (content[0] == 0xFF and content[1] >= 0x80)):
            raise MalformedSignature("malformed integer")
        vals.append(int.from_bytes(content, "big", signed=True))
        i = j + ln
    if len(vals) != 2:
        raise MalformedSignature("malformed signature")
    return vals[0], vals[1]


def der_encode_int(v):
    ln = max(1, (v.bit_length() + 8) // 8) if v >= 0 else ((-v - 1).bit_length() + 8) // 8
    c = v.to_bytes(ln, "big", signed=True)
    return b"\x02" + _der_len(len(c)) + c


def der_encode_sig(r, s):
    body = der_encode_int(r) + der_encode_int(s)
    return b"\x30" + _der_len(len(body)) + body


# ---------------- verify / sign ----------------
def verify(scheme, Q, msg, sig):
    """DSABase.engineVerify + ECDSASigner.verifySignature restated.
    Q: decoded affine public point. Raises MalformedSignature; returns bool."""
    c = CURVES[scheme]
    n = c.n
    e = int.from_bytes(hashlib.sha256(bytes(msg)).digest(), "big")
    r, s = der_decode_sig(sig)
    if r < 1 or r >= n or s < 1 or s >= n:
        return False
    w = pow(s, n - 2, n)
    u1 = e * w % n
    u2 = r * w % n
    R = ec_add(c, ec_mul(c, u1, c.G), ec_mul(c, u2, Q))
    if R is None:
        return False
    return R[0] % n == r


def sign(scheme, d, msg, k):
    """Plain ECDSA sign with a caller-chosen nonce k (fixture generation only)."""
    c = CURVES[scheme]
    n = c.n
    e = int.from_bytes(hashlib.sha256(bytes(msg)).digest(), "big")
    R = ec_mul(c, k, c.G)
    r = R[0] % n
    s = pow(k, n - 2, n) * (e + r * d) % n
    assert r != 0 and s != 0
    return r, s


def public_point(scheme, d):
    c = CURVES[scheme]
    return ec_mul(c, d, c.G)


def raw_key(Q):
    return Q[0].to_bytes(32, "big") + Q[1].to_bytes(32, "big")
