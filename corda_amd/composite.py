"""Composite keys and composite signatures, host logic over the GPU batch.

Restates core/src/main/kotlin/net/corda/core/crypto/composite/:
  * ``CompositeKey`` (CompositeKey.kt:35-269): a weighted threshold tree of public keys. Children
    are kept sorted (NodeAndWeight.compareTo: weight, then node.encoded, :146-151); construction
    checks the constraints of checkConstraints (:73-85: no duplicate child, >= 2 children,
    threshold > 0, threshold <= total weight with overflow-checked addition); checkValidity
    (:110-122) adds cycle detection and runs on first use of isFulfilledBy. ``Builder.build``
    (:258-267) collapses a single child. ``encoded`` / ``get_instance`` are the DER form of
    getEncoded / getInstance (:41-59, :172-181) under CordaObjectIdentifier.compositeKey.
  * ``is_fulfilled_by`` (CompositeKey.kt:186-209, CryptoUtils.kt:88-92): a composite key among
    the keys to check fulfils nothing; otherwise each child contributes its weight when it is
    fulfilled (a leaf: is in the set), and the node is fulfilled when the sum reaches threshold.
  * ``CompositeSignaturesWithKeys`` (CompositeSignaturesWithKeys.kt:11) and
    ``composite_engine_verify`` = CompositeSignature.State.engineVerify (CompositeSignature.kt:75-84):
    if the key is fulfilled by the signatures' keys, the clear data must be a 32-byte SecureHash
    (SecureHash.SHA256(bytes) requires 32 bytes, SecureHash.kt:16-20; anything else is
    IllegalArgumentException), and then ``all`` leaf signatures must verify as
    ``Crypto.isValid(txId, leaf)`` -- over SignableData(txId, leaf.metadata) -- stopping at the
    first false; a leaf's exception propagates.
The leaves are what the GPU verifies (crypto.py expands them into the batch); only the threshold
walk and the all-verify reduction stay on the host. Kotlin Int arithmetic is kept: the default
threshold is a wrapping sum (so Int.MAX_VALUE + Int.MAX_VALUE fails as "threshold ... should be a
positive integer", CompositeKeyTests.kt:205-208), the constraint sum uses Math.addExact.

The Kryo bytes of CompositeSignaturesWithKeys are not reproduced (no JVM here, parity unpinned);
the mirror passes the object itself, or ``serialize()``'s documented stand-in encoding.
"""
import struct

from . import der, keys as K

COMPOSITE_OID = der.oid("2.25.30086077608615255153862931087626791002")  # CordaObjectIdentifier.kt:35


def _int32(v):
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


class ArithmeticException(ArithmeticError):
    """java.lang.ArithmeticException (Math.addExact overflow)"""


def _exact_add(a, b):
    r = a + b
    if r != _int32(r):
        raise ArithmeticException("integer overflow")
    return r


def _iae(msg):
    from .crypto import IllegalArgumentException
    return IllegalArgumentException(msg)


def encoded_of(key):
    """node.encoded of a PublicKey or CompositeKey (X.509 SPKI)."""
    if isinstance(key, CompositeKey):
        return key.encoded
    return K.canonical_spki(key.scheme, key.fmt, key.encoded)


class NodeAndWeight:
    """CompositeKey.NodeAndWeight (CompositeKey.kt:140-163)."""
    __slots__ = ("node", "weight")

    def __init__(self, node, weight):
        if weight <= 0:
            raise _iae(f"A non-positive weight was detected. Node info: {node!r}, weight: {weight}")
        self.node = node
        self.weight = weight

    def _cmp(self, other):
        if self.weight != other.weight:
            return -1 if self.weight < other.weight else 1
        return K.compare_encoded(encoded_of(self.node), encoded_of(other.node))

    def __lt__(self, other):
        return self._cmp(other) < 0

    def __eq__(self, other):
        return isinstance(other, NodeAndWeight) and self.node == other.node and self.weight == other.weight

    def __hash__(self):
        return hash((self.node, self.weight))

    def __repr__(self):
        return f"NodeAndWeight({self.node!r}, {self.weight})"

    def to_der(self):
        return der.tlv(0x30, der.bit_string(encoded_of(self.node)) + der.integer(self.weight))


class CompositeKey:
    """A CompositeKey; build with ``CompositeKey.Builder``."""
    scheme = 6          # Crypto.COMPOSITE_KEY.schemeNumberID
    fmt = K.KEY_SPKI

    def __init__(self, threshold, children, _check=True):
        self.threshold = threshold
        self.children = sorted(children)
        self._validated = False
        if _check:
            self._check_constraints()

    # ---- constraints (CompositeKey.kt:73-133)
    def _total_weight(self):
        s = 0
        for c in self.children:
            if c.weight <= 0:
                raise _iae(f"Non-positive weight: {c.weight} detected.")
            s = _exact_add(s, c.weight)
        return s

    def _check_constraints(self):
        if len(self.children) != len(set(self.children)):
            raise _iae("CompositeKey with duplicated child nodes detected.")
        if len(self.children) <= 1:
            raise _iae("CompositeKey must consist of two or more child nodes.")
        if self.threshold <= 0:
            raise _iae(f"CompositeKey threshold is set to {self.threshold}, but it should be a positive integer.")
        total = self._total_weight()
        if self.threshold > total:
            raise _iae(f"CompositeKey threshold: {self.threshold} cannot be bigger than aggregated weight of child "
                       f"nodes: {total}")

    def _cycle_detection(self, visited):
        for c in self.children:
            if isinstance(c.node, CompositeKey):
                cur = dict(visited)
                if id(c.node) in cur:
                    # the JVM message embeds node.toString(), which itself recurses round the cycle
                    # (a StackOverflowError there); the mirror names the node by its threshold
                    raise _iae(f"Cycle detected for CompositeKey: (threshold {c.node.threshold}, "
                               f"{len(c.node.children)} children)")
                cur[id(c.node)] = True
                c.node._cycle_detection(cur)

    def check_validity(self):
        self._cycle_detection({id(self): True})
        self._check_constraints()
        for c in self.children:
            if isinstance(c.node, CompositeKey):
                c.node._check_constraints()
        self._validated = True

    # ---- fulfilment (CompositeKey.kt:186-209)
    def _check_fulfilled_by(self, keys):
        if any(isinstance(k, CompositeKey) for k in keys):
            return False
        total = 0
        for c in self.children:
            if isinstance(c.node, CompositeKey):
                ok = c.node._check_fulfilled_by(keys)
            else:
                ok = c.node in keys
            total = _int32(total + (c.weight if ok else 0))  # List<Int>.sum() wraps
        return total >= self.threshold

    def is_fulfilled_by(self, keys):
        if not isinstance(keys, (list, tuple, set, frozenset)):
            keys = [keys]
        if not self._validated:
            self.check_validity()
        return self._check_fulfilled_by(list(keys))

    @property
    def leaf_keys(self):
        out = set()
        for c in self.children:
            out |= c.node.leaf_keys if isinstance(c.node, CompositeKey) else {c.node}
        return out

    # ---- encoding (CompositeKey.kt:41-59, :172-181)
    @property
    def encoded(self):
        body = der.integer(self.threshold) + der.tlv(0x30, b"".join(c.to_der() for c in self.children))
        return der.spki(COMPOSITE_OID, b"", der.tlv(0x30, body))

    @staticmethod
    def get_instance(encoded):
        alg, _, bits = der.read_spki(encoded)
        if alg != COMPOSITE_OID:
            raise _iae("Failed requirement.")
        seq = der.read_seq(bits)
        threshold = der.read_integer(*seq[0])
        children = der.read_seq(der.tlv(seq[1][0], seq[1][1]))
        b = CompositeKey.Builder()
        for t, c in children:
            if t != 0x30:
                raise _iae("Failed requirement.")
            kv = der.read_seq(der.tlv(t, c))
            node = K.decode_spki_key(der.read_bit_string(*kv[0]))
            b.add_key(node, _int32(der.read_integer(*kv[1])))
        return b.build(_int32(threshold))

    def __eq__(self, other):
        return isinstance(other, CompositeKey) and self.threshold == other.threshold and \
            self.children == other.children

    def __hash__(self):
        return hash((self.threshold, tuple(self.children)))

    def __repr__(self):
        return "(" + ", ".join(repr(c) for c in self.children) + ")"

    class Builder:
        """CompositeKey.Builder (CompositeKey.kt:235-268)."""

        def __init__(self):
            self._children = []

        def add_key(self, key, weight=1):
            self._children.append(NodeAndWeight(key, weight))
            return self

        def add_keys(self, *keys):
            for k in keys:
                self.add_key(k)
            return self

        def build(self, threshold=None):
            n = len(self._children)
            if n > 1:
                t = threshold if threshold is not None else _int32(sum(c.weight for c in self._children))
                return CompositeKey(t, self._children)
            if n == 1:
                if threshold is not None and threshold != self._children[0].weight:
                    raise _iae("Trying to build invalid CompositeKey, threshold value different than weight of "
                               "single child node.")
                return self._children[0].node
            raise _iae("Trying to build CompositeKey without child nodes.")


def is_fulfilled_by(key, keys):
    """PublicKey.isFulfilledBy (CryptoUtils.kt:88-92)."""
    if isinstance(key, CompositeKey):
        return key.is_fulfilled_by(keys)
    if not isinstance(keys, (list, tuple, set, frozenset)):
        keys = [keys]
    return key in keys


def expanded(keys):
    """Iterable<PublicKey>.expandedCompositeKeys (CompositeKey.kt:276-277)."""
    out = set()
    for k in keys:
        out |= k.leaf_keys if isinstance(k, CompositeKey) else {k}
    return out


class CompositeSignaturesWithKeys:
    """CompositeSignaturesWithKeys(sigs: List<TransactionSignature>). ``serialize`` is the mirror's
    stand-in for its Kryo bytes (parity unpinned): b"CSWK" + count, then per signature the
    signature bytes, the key (scheme, format, bytes; composite keys as their DER) and the
    metadata (platformVersion, schemeNumberID)."""

    def __init__(self, sigs):
        self.sigs = list(sigs)

    def serialize(self):
        out = [b"CSWK", struct.pack("<I", len(self.sigs))]
        for s in self.sigs:
            kb = encoded_of(s.by) if isinstance(s.by, CompositeKey) else bytes(s.by.encoded)
            fmt = K.KEY_SPKI if isinstance(s.by, CompositeKey) else s.by.fmt
            out += [struct.pack("<I", len(s.bytes)), bytes(s.bytes), struct.pack("<BBI", s.by.scheme, fmt, len(kb)), kb,
                    struct.pack("<ii", s.platform_version, s.scheme_number_id)]
        return b"".join(out)

    @staticmethod
    def deserialize(b):
        from .crypto import PublicKey, SignatureException, TransactionSignature
        b = bytes(b)
        try:
            if b[:4] != b"CSWK":
                raise ValueError
            (n,), i, sigs = struct.unpack_from("<I", b, 4), 8, []
            for _ in range(n):
                (ls,) = struct.unpack_from("<I", b, i)
                sig = b[i + 4:i + 4 + ls]
                i += 4 + ls
                scheme, fmt, lk = struct.unpack_from("<BBI", b, i)
                kb = b[i + 6:i + 6 + lk]
                i += 6 + lk
                pv, sid = struct.unpack_from("<ii", b, i)
                i += 8
                key = CompositeKey.get_instance(kb) if scheme == 6 else PublicKey(scheme, kb, fmt)
                sigs.append(TransactionSignature(sig, key, pv, sid))
            if i != len(b):
                raise ValueError
            return CompositeSignaturesWithKeys(sigs)
        except (ValueError, struct.error, IndexError):
            # Kryo's KryoException on garbage; BC's JCA layer reports it as a SignatureException
            raise SignatureException("Could not deserialise CompositeSignaturesWithKeys") from None


def leaf_messages(sig_obj, clear):
    """The leaves' (TransactionSignature, clear data) pairs: clear = SignableData(txId, leaf
    metadata) with txId = SecureHash.SHA256(clear) (the 32 bytes themselves)."""
    from . import signable
    out = []
    for s in sig_obj.sigs:
        pre, suf = signable.template(s.platform_version, s.scheme_number_id)
        out.append((s, pre + bytes(clear) + suf))
    return out
