"""Kryo encoding of WireTransaction components: the leaf bytes of the
transaction Merkle tree, on the host.

Reference: each component of ``availableComponents`` (inputs, attachments, outputs, commands,
notary?, timeWindow?, privacySalt) is hashed as
``SHA256(x.serialize(P2P_CONTEXT.withoutReferences()).bytes || nonce)``
(core/src/main/kotlin/net/corda/core/transactions/MerkleTransaction.kt:16-33, 74-93). The bytes
are the Kryo P2P scheme: header ``corda\\0\\0\\1`` then ``kryo.writeClassAndObject(x)``
(node-api/.../serialization/SerializationScheme.kt:183-216), with DefaultKryoCustomizer's setup
(core/.../serialization/DefaultKryoCustomizer.kt:52-127): CompatibleFieldSerializer by default,
EXTENDED cached field names, the registrations listed there, and the custom serializers of
core/.../serialization/Kryo.kt (Ed25519PublicKeySerializer :330-339, PublicKeySerializer
:388-398, CompositeKeySerializer :358-372, X500NameSerializer :525-533).

PARITY UNPINNED. No JDK, Kotlin, Kryo 4.0.0 or kryo-serializers 0.41 jar exists in this image
(SURVEY.md §8(c)): this is a restatement of Kryo 4.0's documented wire format, not a capture.
The assumptions a single JVM capture of one component of each type would settle:
  * Kryo.writeClass: registered class -> varint(id + 2); unregistered -> varint(1) (NAME), then
    varint(name id) and, on the name's first use in the graph, the class name as Kryo ASCII
    (last char | 0x80). Registration ids: Kryo's ten primitive defaults (0-9), then
    DefaultKryoCustomizer's register() calls in order; the library helpers
    (UnmodifiableCollectionsSerializer ... ImmutableMultimapSerializer) are taken to register
    LIB_REGISTRATIONS classes between them (REG below);
  * no references (withoutReferences()): objects carry no reference ids; a nullable non-final
    field is writeClassAndObject (varint(0) for null), a final-typed one writeObjectOrNull
    (one byte 0 / 1 before the object);
  * CompatibleFieldSerializer: on a class's first use in the graph, varint(#fields) then the
    EXTENDED names ``DeclaringSimpleName.field`` in field-name order; every field value in its
    own OutputChunked chunk (varint(len) data ... varint(0));
  * int fields are zig-zag varints; java.time.Instant (Kryo 4 TimeSerializers) is
    writeLong(epochSecond) (8 bytes, big-endian) + varint(nano); byte[] is varint(len + 1) bytes.
Only the leaf bytes depend on these; the nonce / leaf / Merkle hashing (GPU) and the signature
verification do not. The component types restated: StateRef, SecureHash (attachment ids),
TransactionState with a caller-supplied state encoder, Command, Party (X500Name + owning key),
TimeWindow, PrivacySalt. A decoder (``decode``) reads the same format back for the tests.
"""
from dataclasses import dataclass, field

HEADER = b"corda\x00\x00\x01"  # SerializationScheme.kt:191

# Registration ids (assumption, see the module docstring): primitives 0-9, then the customizer.
LIB_REGISTRATIONS = 33
_REG_ORDER = ["java.util.Arrays$ArrayList", "net.corda.core.transactions.SignedTransaction",
              "net.corda.core.transactions.WireTransaction", "net.corda.core.serialization.SerializedBytes"]
REG = {name: 10 + i for i, name in enumerate(_REG_ORDER)}
_after_lib = 10 + len(_REG_ORDER) + LIB_REGISTRATIONS
for i, name in enumerate(["java.io.BufferedInputStream", "sun.net.www.protocol.jar.JarURLConnection$JarURLInputStream",
                          "sun.security.ec.ECPublicKeyImpl", "net.i2p.crypto.eddsa.EdDSAPublicKey",
                          "net.i2p.crypto.eddsa.EdDSAPrivateKey", "net.corda.core.crypto.composite.CompositeKey"]):
    REG[name] = _after_lib + i
REG["org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPublicKey"] = _after_lib + 20  # after the later registrations


# ------------------------------------------------------------------ primitives
def varint(v):
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
    return varint(((v << 1) ^ (v >> 31)) & 0xFFFFFFFF)


def ascii_(s):
    b = bytearray(s.encode("ascii"))
    b[-1] |= 0x80
    return bytes(b)


def chunk(data):
    return varint(len(data)) + data + varint(0)


def byte_array(b):
    return varint(len(b) + 1) + bytes(b)


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
    """A PublicKey as Kryo writes it: Ed25519 (scheme 4) as its 32-byte A, others as SPKI."""
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
class Command:
    value_class: str         # the CommandData's class name
    value_fields: tuple      # ((name, int), ...) of a CommandData data class
    signers: tuple           # PublicKeyRef, ...


@dataclass(frozen=True)
class TransactionState:
    data_class: str
    data_fields: tuple       # ((name, bytes or int), ...)
    contract: str
    notary: Party
    encumbrance: int = None


@dataclass(frozen=True)
class PrivacySalt:
    bytes_: bytes


# ------------------------------------------------------------------ writer
class _Writer:
    def __init__(self):
        self.out = bytearray(HEADER)
        self.names = {}
        self.schemas = set()

    def cls(self, name):
        if name in REG:
            return varint(REG[name] + 2)
        if name in self.names:
            return varint(1) + varint(self.names[name])
        self.names[name] = len(self.names)
        return varint(1) + varint(self.names[name]) + ascii_(name)

    def schema(self, simple, fields):
        if simple in self.schemas:
            return b""
        self.schemas.add(simple)
        return varint(len(fields)) + b"".join(ascii_(f"{d}.{f}") for f, d in sorted(fields))

    def compat(self, simple, fields_with_values):
        """CompatibleFieldSerializer body: fields_with_values = [(name, declaring, bytes)]."""
        fv = sorted(fields_with_values)
        return self.schema(simple, [(f, d) for f, d, _ in fv]) + b"".join(chunk(v) for _, _, v in fv)

    # objects ------------------------------------------------------
    def secure_hash(self, h):
        return self.cls("net.corda.core.crypto.SecureHash$SHA256") + \
            self.compat("SHA256", [("bytes", "OpaqueBytes", b"\x01" + byte_array(h.bytes_))])

    def public_key(self, k):
        if k.scheme == 4:  # Ed25519PublicKeySerializer: writeBytesWithLength(abyte)
            return self.cls("net.i2p.crypto.eddsa.EdDSAPublicKey") + varint(len(k.encoded)) + k.encoded
        return self.cls("org.bouncycastle.jcajce.provider.asymmetric.ec.BCECPublicKey") + \
            varint(len(k.encoded)) + k.encoded  # PublicKeySerializer: writeBytesWithLength(encoded)

    def party_body(self, p):
        return self.compat("Party", [
            ("name", "Party", self.cls("org.bouncycastle.asn1.x500.X500Name") + bytes(p.name_der)),
            ("owningKey", "AbstractParty", self.public_key(p.owning_key))])

    def party(self, p):
        return self.cls("net.corda.core.identity.Party") + self.party_body(p)

    def state_ref(self, r):
        return self.cls("net.corda.core.contracts.StateRef") + self.compat("StateRef", [
            ("index", "StateRef", zigzag32(r.index)), ("txhash", "StateRef", self.secure_hash(r.txhash))])

    def instant(self, t):
        if t is None:
            return b"\x00"
        return b"\x01" + int(t[0]).to_bytes(8, "big", signed=True) + varint(int(t[1]))

    def time_window(self, tw):
        kind = "Between" if tw.from_time and tw.until_time else ("From" if tw.from_time else "Until")
        fields = []
        if tw.from_time:
            fields.append(("fromTime", kind, self.instant(tw.from_time)))
        if tw.until_time:
            fields.append(("untilTime", kind, self.instant(tw.until_time)))
        return self.cls(f"net.corda.core.contracts.TimeWindow${kind}") + self.compat(kind, fields)

    def _value(self, v):
        return zigzag32(v) if isinstance(v, int) else b"\x01" + byte_array(v)

    # Class-name ids are assigned in stream order: the outer class first, then the fields in the
    # order they are written (field-name order).
    def command(self, c):
        head = self.cls("net.corda.core.contracts.Command")
        simple = c.value_class.rsplit(".", 1)[-1].rsplit("$", 1)[-1]
        signers = self.cls("java.util.Arrays$ArrayList") + varint(len(c.signers)) + \
            b"".join(self.public_key(k) for k in c.signers)  # ArraysAsListSerializer: length, elements
        value = self.cls(c.value_class) + self.compat(simple, [(f, simple, self._value(v)) for f, v in c.value_fields])
        return head + self.compat("Command", [("signers", "Command", signers), ("value", "Command", value)])

    def transaction_state(self, s):
        head = self.cls("net.corda.core.contracts.TransactionState")
        simple = s.data_class.rsplit(".", 1)[-1].rsplit("$", 1)[-1]
        data = self.cls(s.data_class) + self.compat(simple, [(f, simple, self._value(v)) for f, v in s.data_fields])
        # Int? and Party are final types: writeObjectOrNull (a 0 / 1 byte, no class)
        enc = b"\x00" if s.encumbrance is None else b"\x01" + zigzag32(s.encumbrance)
        return head + self.compat("TransactionState", [
            ("contract", "TransactionState", b"\x01" + ascii_(s.contract)),
            ("data", "TransactionState", data), ("encumbrance", "TransactionState", enc),
            ("notary", "TransactionState", b"\x01" + self.party_body(s.notary))])

    def privacy_salt(self, s):
        return self.cls("net.corda.core.contracts.PrivacySalt") + \
            self.compat("PrivacySalt", [("bytes", "OpaqueBytes", b"\x01" + byte_array(s.bytes_))])


def serialize(obj):
    """x.serialize(P2P_CONTEXT.withoutReferences()).bytes for one component."""
    w = _Writer()
    fn = {SecureHash: w.secure_hash, StateRef: w.state_ref, Party: w.party, TimeWindow: w.time_window,
          Command: w.command, TransactionState: w.transaction_state, PrivacySalt: w.privacy_salt}[type(obj)]
    w.out += fn(obj)
    return bytes(w.out)


@dataclass
class WireTransaction:
    """The components of a WireTransaction (WireTransaction.kt:39-104), in availableComponents order."""
    inputs: list = field(default_factory=list)
    attachments: list = field(default_factory=list)
    outputs: list = field(default_factory=list)
    commands: list = field(default_factory=list)
    notary: Party = None
    time_window: TimeWindow = None
    privacy_salt: PrivacySalt = None

    def available_components(self):
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


# ------------------------------------------------------------------ reader (tests)
class _Reader:
    def __init__(self, b):
        if bytes(b[:8]) != HEADER:
            raise ValueError("not a Kryo P2P blob (header)")
        self.b, self.i, self.names, self.schemas = bytes(b), 8, [], {}
        self.by_id = {v: k for k, v in REG.items()}

    def varint(self):
        v = s = 0
        while True:
            c = self.b[self.i]
            self.i += 1
            v |= (c & 0x7F) << s
            s += 7
            if not c & 0x80:
                return v

    def ascii_(self):
        j = self.i
        while not self.b[j] & 0x80:
            j += 1
        s = self.b[self.i:j] + bytes([self.b[j] & 0x7F])
        self.i = j + 1
        return s.decode("ascii")

    def cls(self):
        t = self.varint()
        if t == 0:
            return None
        if t >= 2:
            return self.by_id[t - 2]
        nid = self.varint()
        if nid == len(self.names):
            self.names.append(self.ascii_())
        return self.names[nid]

    def fields(self, simple):
        if simple not in self.schemas:
            self.schemas[simple] = [self.ascii_() for _ in range(self.varint())]
        out = {}
        for name in self.schemas[simple]:
            n = self.varint()
            out[name.split(".", 1)[1]] = self.b[self.i:self.i + n]
            self.i += n
            if self.varint() != 0:
                raise ValueError("multi-chunk field")
        return out


def decode(blob):
    """(class name, {field: raw chunk bytes}) of a serialised component (structure tests)."""
    r = _Reader(blob)
    name = r.cls()
    simple = name.rsplit(".", 1)[-1].rsplit("$", 1)[-1]
    f = r.fields(simple)
    if r.i != len(r.b):
        raise ValueError("trailing bytes")
    return name, f
