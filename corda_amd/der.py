"""Minimal strict DER reader / writer for the host mirror: SubjectPublicKeyInfo (PublicKey.encoded)
of the schemes the GPU does not run (RSA, CompositeKey) and the canonical SPKI forms of the GPU
schemes (equality and ordering of keys, CompositeKey.NodeAndWeight.compareTo,
CompositeKey.kt:146-151). BouncyCastle is the reference's parser (SubjectPublicKeyInfo.getInstance,
Crypto.kt:251-254); only definite, minimal encodings are accepted here."""


class DerError(ValueError):
    pass


def _len_bytes(n):
    if n < 0x80:
        return bytes([n])
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return bytes([0x80 | len(b)]) + b


def tlv(tag, content):
    return bytes([tag]) + _len_bytes(len(content)) + bytes(content)


def read_tlv(b, i=0):
    """(tag, content, next index) of the TLV at b[i]."""
    if i + 2 > len(b):
        raise DerError("truncated")
    tag, l0, j = b[i], b[i + 1], i + 2
    if l0 & 0x80:
        nb = l0 & 0x7F
        if nb == 0 or nb > 4 or j + nb > len(b) or b[j] == 0:
            raise DerError("bad length")
        ln = int.from_bytes(b[j:j + nb], "big")
        if ln < 0x80:
            raise DerError("non-minimal length")
        j += nb
    else:
        ln = l0
    if j + ln > len(b):
        raise DerError("truncated")
    return tag, bytes(b[j:j + ln]), j + ln


def read_seq(b):
    """Elements (tag, content) of a SEQUENCE that spans all of b."""
    tag, body, end = read_tlv(b)
    if tag != 0x30 or end != len(b):
        raise DerError("not a SEQUENCE")
    out, i = [], 0
    while i < len(body):
        t, c, i = read_tlv(body, i)
        out.append((t, c))
    return out


def integer(v):
    ln = max(1, (v.bit_length() + 8) // 8) if v >= 0 else ((-v - 1).bit_length() + 8) // 8
    return tlv(0x02, v.to_bytes(ln, "big", signed=True))


def read_integer(tag, content):
    if tag != 0x02 or not content:
        raise DerError("not an INTEGER")
    if len(content) > 1 and ((content[0] == 0 and content[1] < 0x80) or (content[0] == 0xFF and content[1] >= 0x80)):
        raise DerError("malformed integer")
    return int.from_bytes(content, "big", signed=True)


def oid(dotted):
    arcs = [int(x) for x in dotted.split(".")]
    out = bytearray()
    for v in [40 * arcs[0] + arcs[1]] + arcs[2:]:
        enc = [v & 0x7F]
        v >>= 7
        while v:
            enc.append(0x80 | (v & 0x7F))
            v >>= 7
        out += bytes(reversed(enc))
    return tlv(0x06, bytes(out))


def bit_string(data):
    return tlv(0x03, b"\x00" + bytes(data))


def read_bit_string(tag, content):
    if tag != 0x03 or not content or content[0] != 0:
        raise DerError("not a BIT STRING with 0 unused bits")
    return content[1:]


def spki(alg_oid_der, params_der, key_bits):
    alg = tlv(0x30, alg_oid_der + (params_der or b""))
    return tlv(0x30, alg + bit_string(key_bits))


def read_spki(b):
    """(algorithm OID TLV bytes, parameters TLV bytes or b'', subjectPublicKey bytes)."""
    top = read_seq(b)
    if len(top) != 2:
        raise DerError("SubjectPublicKeyInfo is not a 2-element SEQUENCE")
    (t0, alg), (t1, bits) = top
    if t0 != 0x30:
        raise DerError("bad AlgorithmIdentifier")
    items = read_seq(tlv(0x30, alg))
    if not items or items[0][0] != 0x06 or len(items) > 2:
        raise DerError("bad AlgorithmIdentifier")
    oid_der = tlv(0x06, items[0][1])
    params = tlv(items[1][0], items[1][1]) if len(items) == 2 else b""
    return oid_der, params, read_bit_string(t1, bits)
