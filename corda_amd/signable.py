"""SignableData message templates: the clear data a TransactionSignature signs.

Reference: ``Crypto.doVerify(txId, transactionSignature)`` verifies the signature over
``SignableData(txId, transactionSignature.signatureMetadata).serialize().bytes``
(core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:499-502; SignableData.kt:13,
SignatureMetadata.kt:15). The node serialises with the Kryo P2P context
(node-api/.../serialization/SerializationScheme.kt:191,216: header ``corda\\0\\0\\1``,
references on) and DefaultKryoCustomizer (core/.../serialization/DefaultKryoCustomizer.kt:52-58:
CompatibleFieldSerializer, EXTENDED cached field names).

For a fixed (platformVersion, schemeNumberID) those bytes are ``prefix || txId || suffix``: the
txId is the only per-transaction part. The engine therefore takes one template per metadata
value and splices the device-computed ids into it (``cg_verify_transactions*``), instead of the
host serialising one object per signature.

PARITY UNPINNED. No JDK, Kotlin or Kryo jar exists in this image, so
the bytes below are a restatement of Kryo 4.0's documented wire format, not a capture:
  * writeClassAndObject: varint(NAME + 2 = 1), varint(nameId), class name as Kryo ASCII
    (last char | 0x80); then the reference marker varint(NOT_NULL = 1);
  * CompatibleFieldSerializer, first use of a class in the graph: varint(#fields) and the
    EXTENDED field names ``DeclaringClass.field`` sorted by field name; each field value in
    its own OutputChunked chunk: varint(len) data varint(0);
  * int fields: zig-zag varints; byte[]: reference marker, varint(len + 1), bytes.
Only the template bytes depend on this; the splicing, hashing and verification do not. One JVM
capture of ``SignableData(id, SignatureMetadata(v, s)).serialize()`` replaces ``template()``.
"""

KRYO_HEADER_V0_1 = b"corda\x00\x00\x01"  # SerializationScheme.kt:191


def _varint(v):
    out = bytearray()
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _zigzag(v):
    return _varint(((v << 1) ^ (v >> 31)) & 0xFFFFFFFF)


def _ascii(s):
    b = bytearray(s.encode("ascii"))
    b[-1] |= 0x80
    return bytes(b)


def _chunk(data):
    return _varint(len(data)) + data + _varint(0)


class _Graph:
    """Per-serialisation Kryo state: class-name ids and the classes whose field schema was
    already written."""

    def __init__(self):
        self.names = {}
        self.schemas = set()

    def class_ref(self, name):
        if name in self.names:
            return _varint(1) + _varint(self.names[name])
        nid = len(self.names)
        self.names[name] = nid
        return _varint(1) + _varint(nid) + _ascii(name)

    def schema(self, cls, fields):
        if cls in self.schemas:
            return b""
        self.schemas.add(cls)
        return _varint(len(fields)) + b"".join(_ascii(f"{cls}.{f}") for f in sorted(fields))


TXID_MARK = b"\x00" * 32


def serialize(tx_id, platform_version=1, scheme_number_id=4):
    """SignableData(txId, SignatureMetadata(platformVersion, schemeNumberID)) bytes."""
    assert len(tx_id) == 32
    g = _Graph()
    out = bytearray(KRYO_HEADER_V0_1)
    out += g.class_ref("net.corda.core.crypto.SignableData") + _varint(1)
    out += g.schema("SignableData", ["signatureMetadata", "txId"])
    # field "signatureMetadata" (final class: writeObjectOrNull, no class id)
    md = _varint(1) + g.schema("SignatureMetadata", ["platformVersion", "schemeNumberID"])
    md += _chunk(_zigzag(platform_version)) + _chunk(_zigzag(scheme_number_id))
    out += _chunk(md)
    # field "txId" (declared SecureHash, runtime SecureHash$SHA256: writeClassAndObject)
    h = g.class_ref("net.corda.core.crypto.SecureHash$SHA256") + _varint(1)
    h += g.schema("OpaqueBytes", ["bytes"])
    h += _chunk(_varint(1) + _varint(len(tx_id) + 1) + bytes(tx_id))
    out += _chunk(h)
    return bytes(out)


def template(platform_version=1, scheme_number_id=4):
    """(prefix, suffix) with serialize(id, ...) == prefix + id + suffix for every 32-byte id."""
    a = serialize(TXID_MARK, platform_version, scheme_number_id)
    b = serialize(b"\xff" * 32, platform_version, scheme_number_id)
    pos = next(i for i in range(len(a)) if a[i] != b[i])
    prefix, suffix = a[:pos], a[pos + 32:]
    assert a[pos:pos + 32] == TXID_MARK and b[:pos] == prefix and b[pos + 32:] == suffix
    return prefix, suffix
