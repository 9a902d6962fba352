"""Kryo 4.0 P2P encoding of Corda 0.15 objects, on the host.

What it produces:
  * the leaf bytes of the transaction Merkle tree: every component of ``availableComponents``
    (inputs, attachments, outputs, commands, notary?, timeWindow?, privacySalt) is hashed as
    ``SHA256(x.serialize(P2P_CONTEXT.withoutReferences()).bytes || nonce)``
    (core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:16-33, 74-93);
  * the clear data of a transaction signature, ``SignableData(txId, metadata).serialize()``
    with the default P2P context, references on (Crypto.kt:499-502; corda_amd/signable.py);
  * ``PublicKey.toBase58String()`` = Base58(key.serialize()) (EncodingUtils.kt:66-67).

The serializer (node-api/.../serialization/SerializationScheme.kt:183-203) writes the header
``corda\\0\\0\\1`` and ``kryo.writeClassAndObject(obj)`` into an ``Output`` over a stream, with the
Kryo set up by DefaultKryoCustomizer (core/.../serialization/DefaultKryoCustomizer.kt:52-127):
CompatibleFieldSerializer by default, EXTENDED cached field names, the registrations listed
there, the custom serializers of core/.../serialization/Kryo.kt, and CordaClassResolver
(CordaClassResolver.kt:74-105: unregistered classes are written by name).

The writer below restates Kryo 4.0.0's wire mechanics as they bear on the bytes:
  * ``Output`` buffers; ``OutputChunked`` (1024-byte buffer) emits ``varint(len) data`` on every
    flush and ``0`` at ``endChunks``; a flush also flushes the stream underneath, so the chunks of
    nested CompatibleFieldSerializer fields cascade into their parents' chunk streams;
  * CompatibleFieldSerializer: on a class's first use in the graph, varint(#fields) and the
    EXTENDED names ``DeclaringSimpleName.field`` sorted by that full name; then one
    ``OutputChunked`` per object, ``endChunks()`` after each field;
  * classes: registered -> varint(id + 2); else varint(1), varint(nameId) and, on the name's
    first use, the name as a Kryo string (ASCII with the last byte | 0x80 when 1 < len < 64,
    else UTF-8 with a varint char-count + 1 prefix);
  * references (MapReferenceResolver): with references on, ``writeClassAndObject`` writes
    varint(NOT_NULL = 1) after the class of a first-seen object (varint(id + 2) for a repeat) and
    ``writeObjectOrNull`` the same before the object; with references off, a final-typed field is
    one NULL / NOT_NULL byte unless its serializer accepts null (byte[], String);
  * ints / longs: zig-zag varints (9-byte varlong form); ``writeInt`` without the flag is 4
    bytes big-endian.

PINNED by two captures the reference holds (tests/golden/kryo_captures.json, tools/gen/kryo_captures.py):
  * ``docs/source/tutorial-cordapp.rst:472`` — a whole ``SignedTransaction.txBits`` (1 310 bytes,
    an earlier Corda version's WireTransaction serializer, registrations WireTransaction = 12,
    EdDSAPublicKey = 44, X500Name = 55) plus two ``toBase58String`` keys: the writer reproduces
    every byte from the values the tutorial prints (tests/test_kryo.py). That settles the chunk
    cascade, the field order across the class hierarchy (``AbstractParty.owningKey`` before
    ``Party.name``), the X500Name framing (raw DER, no length), the reference markers and
    the key framing;
  * ``samples/irs-demo/src/main/resources/net/corda/irs/simulation/trade.json:3,25`` — two keys
    this snapshot's IRS simulation parses at run time (IRSSimulation.kt:116 ->
    JacksonSupport.PartyDeserializer -> parsePublicKeyBase58): EdDSAPublicKey is registration
    45 in 0.15. The other 0.15 ids follow from DefaultKryoCustomizer's order after it
    (EdDSAPrivateKey 46, CompositeKey 47, ..., X500Name 55, BCECPublicKey 58).
Still unpinned: java.time.Instant's serializer (TimeWindow) and the library registrations'
exact count between SerializedBytes (13) and BufferedInputStream (only the EdDSA id is used).
"""
from dataclasses import dataclass, field

HEADER = b"corda\x00\x00\x01"  # SerializationScheme.kt:191,216
NULL, NOT_NULL = 0, 1


# ------------------------------------------------------------------ byte-level primitives
def varint(v):
    """Kryo writeVarInt(v, true): little-endian base-128, at most 5 bytes for an int."""
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def zigzag32(v):
    """Kryo writeVarInt(v, false)."""
    return varint(((v << 1) ^ (v >> 31)) & 0xFFFFFFFF)


def varlong(v, optimize_positive):
    """Kryo 4 writeVarLong: 1-8 bytes of 7 bits, the 9th byte carries the top 8 bits whole."""
    if not optimize_positive:
        v = ((v << 1) ^ (v >> 63))
    v &= (1 << 64) - 1
    out = bytearray()
    for _ in range(8):
        if v >> 7 == 0:
            out.append(v)
            return bytes(out)
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v & 0xFF)
    return bytes(out)


def kryo_string(s):
    """Output.writeString bytes (null -> 0x80; ASCII form for 1 < len < 64; else UTF-8)."""
    if s is None:
        return b"\x80"
    n = len(s)
    if n == 0:
        return b"\x81"
    if 1 < n < 64 and all(ord(c) <= 127 for c in s):
        b = bytearray(s.encode("ascii"))
        b[-1] |= 0x80
        return bytes(b)
    return _utf8_length(n + 1) + _utf8_chars(s)


def _utf8_length(v):
    if v >> 6 == 0:
        return bytes([v | 0x80])
    if v >> 13 == 0:
        return bytes([(v | 0x40 | 0x80) & 0xFF, (v >> 6) & 0xFF])
    if v >> 20 == 0:
        return bytes([(v | 0x40 | 0x80) & 0xFF, ((v >> 6) | 0x80) & 0xFF, (v >> 13) & 0xFF])
    if v >> 27 == 0:
        return bytes([(v | 0x40 | 0x80) & 0xFF, ((v >> 6) | 0x80) & 0xFF, ((v >> 13) | 0x80) & 0xFF,
                      (v >> 20) & 0xFF])
    return bytes([(v | 0x40 | 0x80) & 0xFF, ((v >> 6) | 0x80) & 0xFF, ((v >> 13) | 0x80) & 0xFF,
                  ((v >> 20) | 0x80) & 0xFF, (v >> 27) & 0xFF])


def _utf8_chars(s):
    out = bytearray()
    for ch in s:
        c = ord(ch)
        if c <= 0x7F:
            out.append(c)
        elif c > 0x07FF:
            out += bytes([0xE0 | ((c >> 12) & 0x0F), 0x80 | ((c >> 6) & 0x3F), 0x80 | (c & 0x3F)])
        else:
            out += bytes([0xC0 | ((c >> 6) & 0x1F), 0x80 | (c & 0x3F)])
    return bytes(out)


# ------------------------------------------------------------------ Output / OutputChunked
class Output:
    """com.esotericsoftware.kryo.io.Output, byte content only. A root output (parent None) is
    unbounded: its flushes only move bytes to its stream and cannot change them."""

    def __init__(self, parent=None, capacity=None):
        self.parent, self.cap, self.buf = parent, capacity, bytearray()

    def _require(self, n):
        if self.cap is None or self.cap - len(self.buf) >= n:
            return
        if n > self.cap:
            raise ValueError("Kryo buffer overflow")
        self.flush()

    def write_byte(self, b):                 # Output.write(int) / writeByte
        self._require(1)
        self.buf.append(b & 0xFF)

    def write_atomic(self, bs):              # writeVarInt / writeInt / writeLong: require(n) first
        self._require(len(bs))
        self.buf += bs

    def write_bytes(self, bs):               # Output.writeBytes: fills, flushes, continues
        bs = bytes(bs)
        if self.cap is None:
            self.buf += bs
            return
        i = 0
        take = min(self.cap - len(self.buf), len(bs))
        while True:
            self.buf += bs[i:i + take]
            i += take
            if i == len(bs):
                return
            take = min(self.cap, len(bs) - i)
            self._require(take)

    def write_string(self, s):
        enc = kryo_string(s)
        if self.cap is None or s is None or len(s) == 0:
            self.write_atomic(enc) if self.cap is not None else self.buf.extend(enc)
            return
        if 1 < len(s) < 64 and all(ord(c) <= 127 for c in s):
            # ASCII: copied as far as it fits (writeAscii_slow), then the last byte gets | 0x80
            raw = s.encode("ascii")
            self.write_bytes(raw)
            self.buf[-1] |= 0x80
            return
        self.write_atomic(_utf8_length(len(s) + 1))
        self.write_bytes(_utf8_chars(s))

    def flush(self):                         # Output.flush: write buffer to the stream, flush it
        if self.parent is None:
            return
        data = bytes(self.buf)
        self.buf.clear()
        self.parent.write_bytes(data)
        self.parent.flush()

    def getvalue(self):
        assert self.parent is None
        return bytes(self.buf)


class OutputChunked(Output):
    """com.esotericsoftware.kryo.io.OutputChunked (buffer 1024 as CompatibleFieldSerializer
    creates it): every non-empty flush is varint(len) || data into the stream underneath."""

    def __init__(self, parent, capacity=1024):
        super().__init__(parent, capacity)

    def flush(self):
        if len(self.buf) > 0:
            for b in varint(len(self.buf)):   # writeChunkSize: byte by byte into the stream
                self.parent.write_byte(b)
        super().flush()

    def end_chunks(self):
        self.flush()
        self.parent.write_byte(0)


# ------------------------------------------------------------------ classes and serializers
@dataclass(frozen=True)
class JField:
    declaring: str   # simple name of the declaring class (EXTENDED cached field names)
    name: str
    kind: str        # int | long | bytes | string | boxed_int | final | any
    jclass: object = None  # for kind "final": the field's (final) JClass

    @property
    def extended(self):
        return f"{self.declaring}.{self.name}"


class JClass:
    """A Java class as this Kryo sees it: its name, registration id (None: written by name) and
    serializer ("cfs" = CompatibleFieldSerializer over ``fields``, or a callable
    ``write(kryo, out, value)``)."""

    def __init__(self, name, reg=None, fields=(), write=None, accepts_null=False, use_references=True):
        self.name, self.reg = name, reg
        self.fields = sorted(fields, key=lambda f: f.extended)  # FieldSerializer.compare (Kryo 4)
        self.custom = write
        self.accepts_null = accepts_null
        self.use_references = use_references

    def __repr__(self):
        return f"JClass({self.name})"

    def write(self, kryo, out, value):
        if self.custom is not None:
            self.custom(kryo, out, value)
            return
        # CompatibleFieldSerializer.write (Kryo 4.0.0)
        if self not in kryo.schemas:
            kryo.schemas.add(self)
            out.write_atomic(varint(len(self.fields)))
            for f in self.fields:
                out.write_string(f.extended)
        ch = OutputChunked(out)
        for f in self.fields:
            kryo.write_field(ch, f, value.get(f.name) if isinstance(value, JObj) else value[f.name])
            ch.end_chunks()


@dataclass
class JObj:
    """An instance: its class and field values by field name."""
    jclass: JClass
    values: dict = field(default_factory=dict)

    def get(self, name):
        return self.values.get(name)

    def __hash__(self):
        return id(self)

    def __eq__(self, other):
        return self is other


class Kryo:
    """One serialisation graph: reference table, class-name ids, written CFS schemas."""

    def __init__(self, references):
        self.references = references
        self.name_ids = {}
        self.written = {}
        self.schemas = set()

    def write_class(self, out, jc):
        if jc is None:
            out.write_atomic(varint(NULL))
            return
        if jc.reg is not None:
            out.write_atomic(varint(jc.reg + 2))
            return
        out.write_atomic(varint(1))
        if jc.name in self.name_ids:
            out.write_atomic(varint(self.name_ids[jc.name]))
            return
        nid = len(self.name_ids)
        self.name_ids[jc.name] = nid
        out.write_atomic(varint(nid))
        out.write_string(jc.name)

    def _reference_or_null(self, out, jc, value, may_be_null):
        """Kryo.writeReferenceOrNull (MapReferenceResolver): True when nothing more is written."""
        if value is None:
            out.write_atomic(varint(NULL))
            return True
        if not jc.use_references:
            if may_be_null:
                out.write_atomic(varint(NOT_NULL))
            return False
        key = id(value)
        if key in self.written:
            out.write_atomic(varint(self.written[key][0] + 2))
            return True
        self.written[key] = (len(self.written), value)  # keep value alive: ids stay unique
        out.write_atomic(varint(NOT_NULL))
        return False

    def write_class_and_object(self, out, jc, value):
        if value is None:
            self.write_class(out, None)
            return
        self.write_class(out, jc)
        if self.references and self._reference_or_null(out, jc, value, False):
            return
        jc.write(self, out, value)

    def write_object_or_null(self, out, jc, value):
        if self.references:
            if self._reference_or_null(out, jc, value, True):
                return
        elif not jc.accepts_null:
            if value is None:
                out.write_byte(NULL)
                return
            out.write_byte(NOT_NULL)
        jc.write(self, out, value)

    def write_field(self, out, f, value):
        if f.kind == "int":
            out.write_atomic(zigzag32(value))
        elif f.kind == "long":
            out.write_atomic(varlong(value, False))
        elif f.kind == "bytes":
            self.write_object_or_null(out, BYTE_ARRAY, value)
        elif f.kind == "string":
            self.write_object_or_null(out, STRING, value)
        elif f.kind == "boxed_int":
            self.write_object_or_null(out, INTEGER, value)
        elif f.kind == "final":
            self.write_object_or_null(out, f.jclass, value)
        elif f.kind == "any":
            jc, v = (None, None) if value is None else value
            self.write_class_and_object(out, jc, v)
        else:
            raise ValueError(f.kind)


def _write_byte_array(kryo, out, b):         # DefaultArraySerializers.ByteArraySerializer
    if b is None:
        out.write_atomic(varint(NULL))
        return
    out.write_atomic(varint(len(b) + 1))
    out.write_bytes(b)


BYTE_ARRAY = JClass("[B", write=_write_byte_array, accepts_null=True)
STRING = JClass("java.lang.String", write=lambda k, o, s: o.write_string(s), accepts_null=True)
INTEGER = JClass("java.lang.Integer", write=lambda k, o, v: o.write_atomic(zigzag32(v)), use_references=False)


def _with_length(kryo, out, b):              # Kryo.kt:220-223 writeBytesWithLength
    out.write_atomic(varint(len(b)))
    out.write_bytes(b)


def _write_collection(kryo, out, items):     # CollectionSerializer, no generic element type
    out.write_atomic(varint(len(items)))
    for jc, v in items:
        kryo.write_class_and_object(out, jc, v)


def _write_nothing(kryo, out, value):        # CordaClassResolver KotlinObjectSerializer
    pass


# ------------------------------------------------------------------ the class table (0.15)
class Registry:
    """Registration ids of one Corda version (Kryo's 10 primitive defaults are 0-9)."""

    def __init__(self, eddsa_public_key, x500_name, bcec_public_key, wire_transaction=12):
        self.ed_key = JClass("net.i2p.crypto.eddsa.EdDSAPublicKey", eddsa_public_key, write=_with_length)
        self.ec_key = JClass("org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPublicKey", bcec_public_key,
                             write=_with_length)
        self.x500 = JClass("org.bouncycastle.asn1.x500.X500Name", x500_name,
                           write=lambda k, o, der: o.write_bytes(der))   # Kryo.kt:525-533
        self.wire_transaction = wire_transaction
        self.array_list = JClass("java.util.ArrayList", write=_write_collection)
        self.party = JClass("net.corda.core.identity.Party", fields=[
            JField("AbstractParty", "owningKey", "any"), JField("Party", "name", "any")])
        self.secure_hash = JClass("net.corda.core.crypto.SecureHash$SHA256",
                                  fields=[JField("OpaqueBytes", "bytes", "bytes")])
        self.state_ref = JClass("net.corda.core.contracts.StateRef", fields=[
            JField("StateRef", "txhash", "any"), JField("StateRef", "index", "int")])
        self.transaction_state = JClass("net.corda.core.contracts.TransactionState", fields=[
            JField("TransactionState", "data", "any"), JField("TransactionState", "notary", "final", self.party),
            JField("TransactionState", "encumbrance", "boxed_int")])
        self.command = JClass("net.corda.core.contracts.Command", fields=[
            JField("Command", "value", "any"), JField("Command", "signers", "any")])
        self.privacy_salt = JClass("net.corda.core.contracts.PrivacySalt",
                                   fields=[JField("OpaqueBytes", "bytes", "bytes")])
        self.signature_metadata = JClass("net.corda.core.crypto.SignatureMetadata", fields=[
            JField("SignatureMetadata", "platformVersion", "int"), JField("SignatureMetadata", "schemeNumberID", "int")])
        self.signable_data = JClass("net.corda.core.crypto.SignableData", fields=[
            JField("SignableData", "txId", "any"),
            JField("SignableData", "signatureMetadata", "final", self.signature_metadata)])
        # java.time.Instant (Kryo 4 TimeSerializers: writeLong(epochSecond, true), writeInt(nano, true)): UNPINNED
        self.instant = JClass("java.time.Instant",
                              write=lambda k, o, t: (o.write_atomic(varlong(t[0], True)), o.write_atomic(varint(t[1]))))
        self.time_windows = {kind: JClass(f"net.corda.core.contracts.TimeWindow${kind}", fields=fl) for kind, fl in (
            ("Between", [JField("Between", "fromTime", "final", self.instant),
                         JField("Between", "untilTime", "final", self.instant)]),
            ("From", [JField("From", "fromTime", "final", self.instant)]),
            ("Until", [JField("Until", "untilTime", "final", self.instant)]))}
        self._cfs = {}

    def cfs(self, name, fields):
        """A caller-defined CompatibleFieldSerializer class (ContractState / CommandData types)."""
        key = (name, tuple(fields))
        if key not in self._cfs:
            self._cfs[key] = JClass(name, fields=fields)
        return self._cfs[key]

    def kotlin_object(self, name):
        key = (name, "object")
        if key not in self._cfs:
            self._cfs[key] = JClass(name, write=_write_nothing)
        return self._cfs[key]


# Corda 0.15-SNAPSHOT (this reference): EdDSAPublicKey = 45 (pinned by trade.json), then the
# DefaultKryoCustomizer order: EdDSAPrivateKey 46, CompositeKey 47, StackTraceElement[] 48,
# NonEmptySet 49, BitSet 50, Class 51, FileInputStream 52, CertPath 53, X509CertPath 54,
# X500Name 55, X509CertificateHolder 56, BCECPrivateKey 57, BCECPublicKey 58.
V015 = Registry(eddsa_public_key=45, x500_name=55, bcec_public_key=58)
# The Corda version that wrote docs/source/tutorial-cordapp.rst's capture (ids read off the capture).
TUTORIAL = Registry(eddsa_public_key=44, x500_name=55, bcec_public_key=None)


# ------------------------------------------------------------------ component model
@dataclass(frozen=True)
class SecureHash:
    bytes_: bytes

    def __post_init__(self):
        if len(self.bytes_) != 32:
            raise ValueError("SHA-256 hash must be 32 bytes")


@dataclass(frozen=True)
class StateRef:
    txhash: SecureHash
    index: int


@dataclass(frozen=True)
class PublicKeyRef:
    """A PublicKey as Kryo writes it: Ed25519 (scheme 4) as its 32-byte A
    (Ed25519PublicKeySerializer, Kryo.kt:330-339), EC keys as SPKI (PublicKeySerializer, :388-398)."""
    scheme: int
    encoded: bytes


@dataclass(frozen=True)
class Party:
    name_der: bytes          # BC X500Name.getEncoded()
    owning_key: PublicKeyRef


@dataclass(frozen=True)
class TimeWindow:
    from_time: tuple = None  # (epochSecond, nano) or None
    until_time: tuple = None


@dataclass(frozen=True)
class CordaObject:
    """A CommandData / ContractState value: class name and (field, kind, value) triples, kinds as
    JField ("int", "long", "bytes", "string", "boxed_int", "party", "object" = nested CordaObject
    of a final class, "any" = nested CordaObject written with its class); a class with no fields
    may be a Kotlin ``object`` (kotlin_object=True: nothing written)."""
    class_name: str
    fields: tuple = ()
    kotlin_object: bool = False


@dataclass(frozen=True)
class Command:
    value: CordaObject
    signers: tuple           # PublicKeyRef, ... (java.util.ArrayList, as the tutorial capture shows)


@dataclass(frozen=True)
class TransactionState:
    data: CordaObject
    notary: Party
    encumbrance: int = None


@dataclass(frozen=True)
class PrivacySalt:
    bytes_: bytes


# ------------------------------------------------------------------ object -> (JClass, value)
def _simple(name):
    return name.rsplit(".", 1)[-1].rsplit("$", 1)[-1]


def to_java(reg, obj):
    """(JClass, value) for the writer."""
    if isinstance(obj, SecureHash):
        return reg.secure_hash, JObj(reg.secure_hash, {"bytes": obj.bytes_})
    if isinstance(obj, PublicKeyRef):
        return (reg.ed_key if obj.scheme == 4 else reg.ec_key), obj.encoded
    if isinstance(obj, Party):
        return reg.party, JObj(reg.party, {"owningKey": to_java(reg, obj.owning_key),
                                           "name": (reg.x500, obj.name_der)})
    if isinstance(obj, StateRef):
        return reg.state_ref, JObj(reg.state_ref, {"txhash": to_java(reg, obj.txhash), "index": obj.index})
    if isinstance(obj, PrivacySalt):
        return reg.privacy_salt, JObj(reg.privacy_salt, {"bytes": obj.bytes_})
    if isinstance(obj, TimeWindow):
        kind = "Between" if obj.from_time and obj.until_time else ("From" if obj.from_time else "Until")
        jc = reg.time_windows[kind]
        return jc, JObj(jc, {"fromTime": obj.from_time, "untilTime": obj.until_time})
    if isinstance(obj, Command):
        jc = reg.command
        signers = (reg.array_list, [to_java(reg, k) for k in obj.signers])
        return jc, JObj(jc, {"value": to_java(reg, obj.value), "signers": signers})
    if isinstance(obj, TransactionState):
        jc = reg.transaction_state
        return jc, JObj(jc, {"data": to_java(reg, obj.data), "notary": to_java(reg, obj.notary)[1],
                             "encumbrance": obj.encumbrance})
    if isinstance(obj, CordaObject):
        if obj.kotlin_object:
            return reg.kotlin_object(obj.class_name), obj
        simple = _simple(obj.class_name)
        jfields, values = [], {}
        for fname, kind, v in obj.fields:
            if kind == "party":
                jfields.append(JField(simple, fname, "final", reg.party))
                values[fname] = None if v is None else to_java(reg, v)[1]
            elif kind == "object":
                jc, jv = to_java(reg, v)
                jfields.append(JField(simple, fname, "final", jc))
                values[fname] = jv
            elif kind == "any":
                jfields.append(JField(simple, fname, "any"))
                values[fname] = None if v is None else to_java(reg, v)
            else:
                jfields.append(JField(simple, fname, kind))
                values[fname] = v
        jc = reg.cfs(obj.class_name, tuple(jfields))
        return jc, JObj(jc, values)
    raise TypeError(type(obj))


def serialize(obj, references=False, reg=V015):
    """x.serialize(context).bytes: references=False is P2P_CONTEXT.withoutReferences() (the Merkle
    leaf form, MerkleTransaction.kt:25,30); references=True the default P2P context."""
    k = Kryo(references)
    out = Output()
    out.write_bytes(HEADER)
    jc, v = to_java(reg, obj)
    k.write_class_and_object(out, jc, v)
    return out.getvalue()


def public_key_base58_bytes(key, reg=V015):
    """PublicKey.serialize().bytes, the payload of toBase58String() (EncodingUtils.kt:67)."""
    return serialize(key, references=True, reg=reg)


def signable_data(tx_id, platform_version, scheme_number_id, reg=V015):
    """SignableData(txId, SignatureMetadata(v, s)).serialize().bytes (Crypto.kt:499-502, default
    P2P context: references on)."""
    k = Kryo(True)
    out = Output()
    out.write_bytes(HEADER)
    md = JObj(reg.signature_metadata, {"platformVersion": platform_version, "schemeNumberID": scheme_number_id})
    sd = JObj(reg.signable_data, {"txId": to_java(reg, SecureHash(bytes(tx_id))), "signatureMetadata": md})
    k.write_class_and_object(out, reg.signable_data, sd)
    return out.getvalue()


@dataclass
class WireTransaction:
    """The components of a WireTransaction (WireTransaction.kt:20-31), in availableComponents order."""
    inputs: list = field(default_factory=list)
    attachments: list = field(default_factory=list)
    outputs: list = field(default_factory=list)
    commands: list = field(default_factory=list)
    notary: Party = None
    time_window: TimeWindow = None
    privacy_salt: PrivacySalt = None

    def available_components(self):
        """MerkleTransaction.kt:77-86 (the salt is appended by data())."""
        out = list(self.inputs) + list(self.attachments) + list(self.outputs) + list(self.commands)
        if self.notary is not None:
            out.append(self.notary)
        if self.time_window is not None:
            out.append(self.time_window)
        return out

    def data(self):
        """WireTransactionData for the GPU id pipeline (corda_amd/transactions.py)."""
        from .transactions import WireTransactionData
        return WireTransactionData(components=[serialize(c) for c in self.available_components()],
                                   salt=self.privacy_salt.bytes_, salt_blob=serialize(self.privacy_salt))


# ------------------------------------------------------------------ X.500 names (BC X500Name)
_X500_OIDS = {"CN": "2.5.4.3", "O": "2.5.4.10", "OU": "2.5.4.11", "L": "2.5.4.7", "C": "2.5.4.6", "ST": "2.5.4.8"}


def x500_der(dn):
    """BC ``X500Name(dn).encoded`` for a simple comma-separated DN, RDNs in the written order;
    BCStyle value types: C as PrintableString, the others UTF8String."""
    from .der import oid, tlv
    rdns = []
    for part in dn.split(","):
        k, v = part.split("=", 1)
        k = k.strip()
        val = tlv(0x13 if k == "C" else 0x0C, v.encode("utf-8"))
        rdns.append(tlv(0x31, tlv(0x30, oid(_X500_OIDS[k]) + val)))
    return tlv(0x30, b"".join(rdns))


# ------------------------------------------------------------------ reader (tests)
class Reader:
    """Reads the format back: chunked fields are the concatenation of their chunks, which is the
    nested field's own byte stream (so the reader recurses on the payload)."""

    def __init__(self, b, i=0):
        self.b, self.i = bytes(b), i

    def varint(self):
        v = s = 0
        while True:
            c = self.b[self.i]
            self.i += 1
            v |= (c & 0x7F) << s
            s += 7
            if not c & 0x80:
                return v

    def string(self):
        c = self.b[self.i]
        if c & 0x80 == 0:                      # ASCII form
            j = self.i
            while not self.b[j] & 0x80:
                j += 1
            s = self.b[self.i:j] + bytes([self.b[j] & 0x7F])
            self.i = j + 1
            return s.decode("ascii")
        n = (c & 0x3F)
        self.i += 1
        if c & 0x40:
            sh = 6
            while True:
                c = self.b[self.i]
                self.i += 1
                n |= (c & 0x7F) << sh
                sh += 7
                if not c & 0x80:
                    break
        if n == 0:
            return None
        s = self.b[self.i:self.i + n - 1].decode("utf-8")
        self.i += n - 1
        return s

    def chunks(self):
        """One chunked field's payload (concatenated chunks up to the 0 chunk)."""
        out = bytearray()
        while True:
            n = self.varint()
            if n == 0:
                return bytes(out)
            out += self.b[self.i:self.i + n]
            self.i += n


def decode(blob):
    """(class name or registration id, [field names], {field: payload}) of a serialised CFS
    object written without references (structure tests)."""
    if bytes(blob[:8]) != HEADER:
        raise ValueError("not a Kryo P2P blob (header)")
    r = Reader(blob, 8)
    t = r.varint()
    if t == 1:
        r.varint()
        name = r.string()
    else:
        name = t - 2
    names = [r.string() for _ in range(r.varint())]
    out = {}
    for n in names:
        out[n] = r.chunks()
    if r.i != len(r.b):
        raise ValueError("trailing bytes")
    return name, names, out
