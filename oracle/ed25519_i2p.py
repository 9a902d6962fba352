"""Python big-int restatement of Ed25519 verification as net.i2p.crypto:eddsa:0.2.0 does it.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py). Never imported by the product path.

The i2p library is an un-vendored dependency of the reference
(build.gradle:48 ``eddsa_version``, core/build.gradle:67); it is called through JCA at
core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:553-559 for scheme
EDDSA_ED25519_SHA512 (Crypto.kt:120-133). Its published algorithm, restated here:

EdDSAEngine.engineVerify(sig):
  1. ``sig.length != 64``  -> SignatureException("signature length is wrong")
  2. h = SHA-512(sig[0:32] || Abyte || M)          (Abyte = canonical re-encoding of A)
  3. h = Ed25519ScalarOps.reduce(h)                 (h mod L, canonical)
  4. R = B.doubleScalarMultiplyVariableTime(-A, h, sig[32:64])
         = h*(-A) + S*B, with S recoded by ``slide()`` over 256 bits, NO S < L check
  5. return R.toByteArray() == sig[0:32]            (byte compare, canonical encoding)

GroupElement(curve, bytes) (public-key decode, EdDSAPublicKeySpec):
  y = bytes with bit 255 masked (y >= p accepted and reduced), x = sqrt((y^2-1)/(dy^2+1))
  via x = u v^3 (u v^7)^((p-5)/8); no root -> IllegalArgumentException; then the sign
  fix-up ``if isNegative(x) != bit255: x = -x`` (x = 0 with sign 1 is accepted).
"""
import hashlib

P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
D2 = (2 * D) % P
SQRT_M1 = pow(2, (P - 1) // 4, P)


class KeyDecodeError(ValueError):
    """IllegalArgumentException at EdDSAPublicKeySpec / GroupElement decode."""


class SignatureLengthError(ValueError):
    """SignatureException("signature length is wrong") from EdDSAEngine.engineVerify."""


def _inv(x):
    return pow(x, P - 2, P)


def _is_negative(x):
    # Ed25519FieldElement.isNegative(): low bit of the canonical encoding.
    return (x % P) & 1


def decode_point(s):
    """GroupElement(curve, byte[] s) restated; returns affine (x, y) reduced mod p."""
    if len(s) != 32:
        raise KeyDecodeError("public-key length is wrong")
    yraw = int.from_bytes(s, "little") & ((1 << 255) - 1)
    y = yraw % P
    yy = y * y % P
    u = (yy - 1) % P
    v = (yy * D + 1) % P
    v3 = v * v % P * v % P
    x = v3 * v3 % P * v % P * u % P            # u v^7
    x = pow(x, (P - 5) // 8, P)                # (u v^7)^((p-5)/8)
    x = v3 * u % P * x % P                     # u v^3 (u v^7)^((p-5)/8)
    vxx = x * x % P * v % P
    if (vxx - u) % P != 0:
        if (vxx + u) % P != 0:
            raise KeyDecodeError("not a valid GroupElement")
        x = x * SQRT_M1 % P
    if _is_negative(x) != (s[31] >> 7):
        x = (-x) % P
    return (x, y)


def encode_point(pt):
    x, y = pt
    b = bytearray((y % P).to_bytes(32, "little"))
    b[31] |= _is_negative(x) << 7
    return bytes(b)


# --- group law, extended twisted Edwards coordinates (a = -1); complete formulas ---
def _to_ext(pt):
    x, y = pt
    return (x, y, 1, x * y % P)


def _add(p1, p2):
    X1, Y1, Z1, T1 = p1
    X2, Y2, Z2, T2 = p2
    a = (Y1 - X1) * (Y2 - X2) % P
    b = (Y1 + X1) * (Y2 + X2) % P
    c = T1 * D2 % P * T2 % P
    d = Z1 * 2 * Z2 % P
    e, f, g, h = b - a, d - c, d + c, b + a
    return (e * f % P, g * h % P, f * g % P, e * h % P)


def _neg(p1):
    X, Y, Z, T = p1
    return ((-X) % P, Y, Z, (-T) % P)


def _dbl(p1):
    return _add(p1, p1)


def _to_affine(p1):
    X, Y, Z, _ = p1
    zi = _inv(Z)
    return (X * zi % P, Y * zi % P)


IDENT = (0, 1, 1, 0)
_BY = 4 * _inv(5) % P
B_AFFINE = decode_point(_BY.to_bytes(32, "little"))
B = _to_ext(B_AFFINE)


def scalarmult(k, pt_ext):
    r = IDENT
    q = pt_ext
    while k > 0:
        if k & 1:
            r = _add(r, q)
        q = _dbl(q)
        k >>= 1
    return r


def slide(a):
    """GroupElement.slide(byte[] a) restated literally (i2p 0.2.0 / ref10 ge_double_scalarmult).

    Returns 256 signed digits r[i] in [-15, 15]; a carry that would run past bit 255 is
    dropped (the ``for k in i+b..255`` loop simply ends)."""
    r = [(a[i >> 3] >> (i & 7)) & 1 for i in range(256)]
    for i in range(256):
        if r[i] == 0:
            continue
        for b in range(1, 7):
            if i + b >= 256:
                break
            if r[i + b] == 0:
                continue
            if r[i] + (r[i + b] << b) <= 15:
                r[i] += r[i + b] << b
                r[i + b] = 0
            elif r[i] - (r[i + b] << b) >= -15:
                r[i] -= r[i + b] << b
                for k in range(i + b, 256):
                    if r[k] == 0:
                        r[k] = 1
                        break
                    r[k] = 0
            else:
                break
    return r


def slide_value(a):
    """Integer value sum(r[i] 2^i) of slide(a): S, or S - 2^256 when the carry escaped."""
    return sum(d << i for i, d in enumerate(slide(a)))


def double_scalar_mult_vartime(negA_ext, h, s_bytes):
    """B.doubleScalarMultiplyVariableTime(-A, h, S) with i2p's loop structure:
    digits from slide(), odd-multiple tables {1,3,..,15} of -A and of B."""
    aslide = slide(h.to_bytes(32, "little"))
    bslide = slide(s_bytes)
    tabA = [negA_ext]
    tabB = [B]
    a2 = _dbl(negA_ext)
    b2 = _dbl(B)
    for _ in range(7):
        tabA.append(_add(tabA[-1], a2))
        tabB.append(_add(tabB[-1], b2))
    i = 255
    while i >= 0 and aslide[i] == 0 and bslide[i] == 0:
        i -= 1
    r = IDENT
    while i >= 0:
        r = _dbl(r)
        if aslide[i] > 0:
            r = _add(r, tabA[aslide[i] // 2])
        elif aslide[i] < 0:
            r = _add(r, _neg(tabA[(-aslide[i]) // 2]))
        if bslide[i] > 0:
            r = _add(r, tabB[bslide[i] // 2])
        elif bslide[i] < 0:
            r = _add(r, _neg(tabB[(-bslide[i]) // 2]))
        i -= 1
    return r


class PublicKey:
    """EdDSAPublicKey: decoded A, canonical Abyte, and -A (i2p precomputes it per key)."""

    def __init__(self, abytes):
        self.raw = bytes(abytes)
        self.A = decode_point(self.raw)            # may raise KeyDecodeError
        self.Abyte = encode_point(self.A)
        self.negA = _neg(_to_ext(self.A))


def verify(pub, msg, sig):
    """EdDSAEngine.engineVerify restated. ``pub`` is a PublicKey (already decoded)."""
    if len(sig) != 64:
        raise SignatureLengthError("signature length is wrong")
    h = hashlib.sha512(bytes(sig[:32]) + pub.Abyte + bytes(msg)).digest()
    h = int.from_bytes(h, "little") % L
    R = double_scalar_mult_vartime(pub.negA, h, bytes(sig[32:64]))
    return encode_point(_to_affine(R)) == bytes(sig[:32])


def verify_fast(pub, msg, sig):
    """Same verdict as ``verify`` computed as h*(-A) + (slide_value(S) mod L)*B with
    plain double-and-add; used to cross-check the literal loop."""
    if len(sig) != 64:
        raise SignatureLengthError("signature length is wrong")
    h = int.from_bytes(hashlib.sha512(bytes(sig[:32]) + pub.Abyte + bytes(msg)).digest(), "little") % L
    s_eff = slide_value(bytes(sig[32:64])) % L
    R = _add(scalarmult(h, pub.negA), scalarmult(s_eff, B))
    return encode_point(_to_affine(R)) == bytes(sig[:32])


# ---------------- signing side (fixture generation only) ----------------
def secret_expand(seed):
    h = hashlib.sha512(seed).digest()
    a = bytearray(h[:32])
    a[0] &= 248
    a[31] &= 63
    a[31] |= 64
    return int.from_bytes(a, "little"), h[32:]


def public_from_seed(seed):
    a, _ = secret_expand(seed)
    return encode_point(_to_affine(scalarmult(a, B)))


def sign(seed, msg):
    """RFC 8032 Ed25519 sign (what i2p EdDSAEngine.engineSign computes)."""
    a, prefix = secret_expand(seed)
    A = encode_point(_to_affine(scalarmult(a, B)))
    r = int.from_bytes(hashlib.sha512(prefix + bytes(msg)).digest(), "little") % L
    R = encode_point(_to_affine(scalarmult(r, B)))
    k = int.from_bytes(hashlib.sha512(R + A + bytes(msg)).digest(), "little") % L
    S = (r + k * a) % L
    return R + S.to_bytes(32, "little")


def entropy_seed(n):
    """Crypto.deriveEdDSAKeyPairFromEntropy (Crypto.kt:751-757): seed =
    BigInteger(n).toByteArray() (two's complement, big-endian, minimal) right-padded
    with zeros to 32 bytes."""
    if n == 0:
        tb = b"\x00"
    else:
        nbytes = (n.bit_length() + 8) // 8 if n > 0 else ((-n - 1).bit_length() + 8) // 8
        tb = n.to_bytes(nbytes, "big", signed=True)
    return (tb + bytes(32))[:32]


def small_order_points():
    """The 8 points of order dividing 8 (torsion subgroup), affine."""
    pts = []
    # L * (any curve point) lies in the torsion subgroup; pick one of full order 8.
    T = None
    for yv in range(2, 200):
        try:
            cand = _to_ext(decode_point(yv.to_bytes(32, "little")))
        except KeyDecodeError:
            continue
        t = scalarmult(L, cand)
        if _to_affine(scalarmult(4, t)) != (0, 1):
            T = t
            break
    acc = IDENT
    for _ in range(8):
        pts.append(_to_affine(acc))
        acc = _add(acc, T)
    return pts
