"""Batch layout shared by the host mirror, tests and bench: numpy views of the C ABI structs.

``KEY_DTYPE`` / ``ITEM_DTYPE`` / ``SPAN_DTYPE`` / ``COMPONENT_DTYPE`` / ``TX_DTYPE`` /
``TXSIG_DTYPE`` / ``TMPL_DTYPE`` are byte-for-byte ``cg_key`` / ``cg_item`` / ``cg_span`` /
``cg_component`` / ``cg_tx`` / ``cg_txsig`` / ``cg_signable_tmpl`` of include/cordagpu.h. ``BatchBuilder`` packs (key, sig, clear) triples the way a JVM
caller of ``Crypto.verifyBatch`` would: each distinct PublicKey object once in the key
table (as TransactionSignature.by references it), signatures and clear data appended to
one arena.
"""
import numpy as np

KEY_DTYPE = np.dtype([("off", "<u8"), ("len", "<u2"), ("scheme", "u1"), ("fmt", "u1"), ("reserved", "<u4")])
ITEM_DTYPE = np.dtype([("sig_off", "<u8"), ("msg_off", "<u8"), ("msg_len", "<u4"), ("key_idx", "<u4"),
                       ("sig_len", "<u2"), ("reserved0", "<u2"), ("reserved1", "<u4")])
SPAN_DTYPE = np.dtype([("off", "<u8"), ("len", "<u8")])
COMPONENT_DTYPE = np.dtype([("off", "<u8"), ("len", "<u4"), ("flags", "<u4")])
TX_DTYPE = np.dtype([("first", "<u8"), ("n", "<u4"), ("reserved", "<u4"), ("salt_off", "<u8")])
TXSIG_DTYPE = np.dtype([("sig_off", "<u8"), ("tx_idx", "<u4"), ("key_idx", "<u4"), ("sig_len", "<u2"),
                        ("tmpl", "<u2"), ("reserved", "<u4")])
TMPL_DTYPE = np.dtype([("prefix_off", "<u8"), ("suffix_off", "<u8"), ("prefix_len", "<u4"), ("suffix_len", "<u4")])
# cg_txsig_packed (round 6): the 12-byte table over a dense signature stream (each signature at the
# 4-byte-aligned end of the one before it)
TXSIG12_DTYPE = np.dtype([("tx_idx", "<u4"), ("key_idx", "<u4"), ("sig_len", "<u2"), ("tmpl", "<u2")])
assert TXSIG12_DTYPE.itemsize == 12
# tear-offs (cg_pmt_node / cg_filtered_leaf / cg_filtered_tx)
PMT_NODE_DTYPE = np.dtype([("hash_off", "<u8"), ("kind", "<u4"), ("reserved", "<u4")])
FLEAF_DTYPE = np.dtype([("off", "<u8"), ("nonce_off", "<u8"), ("len", "<u4"), ("flags", "<u4")])
FTX_DTYPE = np.dtype([("first_node", "<u8"), ("first_leaf", "<u8"), ("root_off", "<u8"), ("n_nodes", "<u4"),
                      ("n_leaves", "<u4"), ("flags", "<u4"), ("reserved", "<u4")])
assert PMT_NODE_DTYPE.itemsize == 16 and FLEAF_DTYPE.itemsize == 24 and FTX_DTYPE.itemsize == 40
PMT_NODE, PMT_LEAF, PMT_INCLUDED = 0, 1, 2
FLEAF_SALT, FLEAF_HASH = 1, 2
FTX_FILTERED = 1
assert TXSIG_DTYPE.itemsize == 24 and TMPL_DTYPE.itemsize == 24
assert KEY_DTYPE.itemsize == 16 and ITEM_DTYPE.itemsize == 32 and SPAN_DTYPE.itemsize == 16
assert COMPONENT_DTYPE.itemsize == 16 and TX_DTYPE.itemsize == 24

# status codes (include/cordagpu.h)
VALID, INVALID, SIG_MALFORMED, KEY_INVALID, UNSUPPORTED, EMPTY, NOT_RUN = 0, 1, 2, 3, 4, 5, 255
STATUS_NAMES = {VALID: "VALID", INVALID: "INVALID", SIG_MALFORMED: "SIG_MALFORMED", KEY_INVALID: "KEY_INVALID",
                UNSUPPORTED: "UNSUPPORTED", EMPTY: "EMPTY", NOT_RUN: "NOT_RUN"}
STATUS_BY_NAME = {v: k for k, v in STATUS_NAMES.items()}
ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256, EDDSA_ED25519_SHA512 = 2, 3, 4
KEY_RAW, KEY_SPKI, KEY_SEC1 = 0, 1, 2
MODE_DOVERIFY, MODE_ISVALID = 0, 1


# cg_item.sig_len / cg_txsig.sig_len are 16 bits, cg_item.msg_len 32 bits (include/cordagpu.h).
SIG_LEN_MAX = 0xFFFF
MSG_LEN_MAX = 0xFFFFFFFF
# A signature longer than SIG_LEN_MAX cannot be described to the engine. It is packed as a
# short surrogate whose verdict is the one the JVM gives the real bytes, with the same
# precedence (unsupported scheme, then key decode, then the signature):
#   Ed25519: any length != 64 -> SignatureException("signature length is wrong") (SIG_MALFORMED)
#   ECDSA:   BC 1.57 StdDSAEncoder.decode either rejects the DER (SIG_MALFORMED), or it is a
#            canonical SEQUENCE{INTEGER r, INTEGER s}, and then one INTEGER has more than 32
#            thousand content bytes: r or s is outside [1, n-1], isValid == false (INVALID).
SIG_SURROGATE_MALFORMED = b"\x00"
SIG_SURROGATE_INVALID = bytes.fromhex("3006020100020101")  # SEQUENCE{INTEGER 0, INTEGER 1}: r = 0


def _der_len_at(b, i):
    """(length, next index) of a minimal definite DER length at b[i], or None."""
    if i >= len(b):
        return None
    l0 = b[i]
    if l0 < 0x80:
        return l0, i + 1
    nb = l0 & 0x7F
    if nb == 0 or nb > 4 or i + 1 + nb > len(b) or b[i + 1] == 0:
        return None
    v = int.from_bytes(b[i + 1:i + 1 + nb], "big")
    if v < 0x80:
        return None
    return v, i + 1 + nb


def der_is_two_integers(sig):
    """True iff ``sig`` is exactly the canonical DER of SEQUENCE{INTEGER, INTEGER} (minimal
    lengths, minimal non-empty two's-complement contents, nothing trailing): the inputs BC 1.57's
    decode-and-re-encode check accepts."""
    b = bytes(sig)
    if len(b) < 2 or b[0] != 0x30:
        return False
    r = _der_len_at(b, 1)
    if r is None or r[1] + r[0] != len(b):
        return False
    i, n = r[1], 0
    while i < len(b):
        if b[i] != 0x02:
            return False
        r = _der_len_at(b, i + 1)
        if r is None or r[0] == 0 or r[1] + r[0] > len(b):
            return False
        ln, j = r
        if ln > 1 and ((b[j] == 0 and b[j + 1] < 0x80) or (b[j] == 0xFF and b[j + 1] >= 0x80)):
            return False
        i, n = j + ln, n + 1
    return n == 2


def sig_field(scheme, sig):
    """The bytes to pack for a signature: ``sig`` itself, or its surrogate when it is longer than
    the ABI's 16-bit length field (see SIG_SURROGATE_*)."""
    if len(sig) <= SIG_LEN_MAX:
        return sig
    if scheme in (ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256) and der_is_two_integers(sig):
        return SIG_SURROGATE_INVALID
    return SIG_SURROGATE_MALFORMED


def check_msg_len(msg):
    if len(msg) > MSG_LEN_MAX:  # a JVM byte[] holds at most 2^31 - 1 bytes: never a real input
        raise ValueError(f"clear data of {len(msg)} bytes exceeds the 32-bit cg_item.msg_len")


class Batch:
    """Packed batch: ``keys`` (KEY_DTYPE), ``items`` (ITEM_DTYPE), ``arena`` (uint8)."""

    def __init__(self, keys, items, arena):
        self.keys = keys
        self.items = items
        self.arena = arena

    @property
    def n(self):
        return len(self.items)

    def subset(self, idx):
        """The items ``idx`` over the same key table and arena (a re-queue of NOT_RUN items)."""
        return Batch(self.keys, np.ascontiguousarray(self.items[idx]), self.arena)


class BatchBuilder:
    def __init__(self):
        self._chunks = []
        self._size = 0
        self._keys = []
        self._key_index = {}
        self._items = []

    def _append(self, b, align=1):
        pad = (-self._size) % align
        if pad:
            self._chunks.append(bytes(pad))
            self._size += pad
        off = self._size
        if b:
            self._chunks.append(bytes(b))
            self._size += len(b)
        return off

    def key(self, scheme, fmt, key_bytes):
        """Registers a public key once (identity = (scheme, fmt, bytes)); returns its index."""
        k = (int(scheme), int(fmt), bytes(key_bytes))
        idx = self._key_index.get(k)
        if idx is None:
            if len(key_bytes) > SIG_LEN_MAX:
                # cg_key.len is 16 bits; no key encoding of a GPU scheme is that long, so the key
                # fails to decode either way: pack one byte, which decodes to KEY_INVALID too
                key_bytes = b"\x00"
            off = self._append(key_bytes, 4)
            idx = len(self._keys)
            self._keys.append((off, len(key_bytes), scheme, fmt))
            self._key_index[k] = idx
        return idx

    def add(self, key_idx, sig, msg):
        check_msg_len(msg)
        sig = sig_field(self._keys[key_idx][2], sig)
        sig_off = self._append(sig, 4)
        msg_off = self._append(msg, 4)
        self._items.append((sig_off, msg_off, len(msg), key_idx, len(sig)))
        return len(self._items) - 1

    def add_with_key(self, scheme, fmt, key_bytes, sig, msg):
        return self.add(self.key(scheme, fmt, key_bytes), sig, msg)

    def build(self):
        keys = np.zeros(len(self._keys), dtype=KEY_DTYPE)
        for i, (off, ln, scheme, fmt) in enumerate(self._keys):
            keys[i] = (off, ln, scheme, fmt, 0)
        items = np.zeros(len(self._items), dtype=ITEM_DTYPE)
        if self._items:
            arr = np.array(self._items, dtype=np.uint64)
            if arr[:, 4].max() > SIG_LEN_MAX or arr[:, 2].max() > MSG_LEN_MAX:
                raise ValueError("a length exceeds its cg_item field")  # add() never lets one through
            items["sig_off"] = arr[:, 0]
            items["msg_off"] = arr[:, 1]
            items["msg_len"] = arr[:, 2]
            items["key_idx"] = arr[:, 3]
            items["sig_len"] = arr[:, 4]
        arena = np.frombuffer(b"".join(self._chunks) + bytes(16), dtype=np.uint8).copy()
        return Batch(keys, items, arena)


class TxSigBatch:
    """Signatures over known transaction ids (cg_verify_tx_signatures): ``keys`` (KEY_DTYPE),
    ``ids`` (uint8 [n_ids * 32], the SecureHash bytes), ``sigs`` (TXSIG_DTYPE: tx_idx indexes ids,
    tmpl indexes tmpls), ``tmpls`` (TMPL_DTYPE: SignableData prefix / suffix per SignatureMetadata
    value, bytes in the arena), ``arena`` (uint8: key, template and signature bytes)."""

    def __init__(self, keys, ids, sigs, tmpls, arena):
        self.keys = keys
        self.ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1)
        self.sigs = sigs
        self.tmpls = tmpls
        self.arena = arena

    @property
    def n(self):
        return len(self.sigs)

    @property
    def n_ids(self):
        return self.ids.size // 32

    def subset(self, idx):
        """The signatures ``idx`` over the same keys, ids, templates and arena (a re-queue)."""
        return TxSigBatch(self.keys, self.ids, np.ascontiguousarray(self.sigs[idx]), self.tmpls, self.arena)

    def packed(self):
        """The same signatures as cg_verify_tx_signatures_packed input (PackedTxSigBatch): the 12-byte
        table and the dense signature stream. When the arena already holds the signatures back to back
        in table order, 4-byte aligned, after everything else (wl.tx_sig_stream, a JVM writer), the
        stream is a view of that tail and the arena is cut before it; otherwise the bytes are gathered."""
        n = len(self.sigs)
        sig12 = np.zeros(n, TXSIG12_DTYPE)
        for f in ("tx_idx", "key_idx", "sig_len", "tmpl"):
            sig12[f] = self.sigs[f]
        span = (self.sigs["sig_len"].astype(np.uint64) + np.uint64(3)) & ~np.uint64(3)
        rel = np.zeros(n, np.uint64)
        if n > 1:
            np.cumsum(span[:-1], out=rel[1:])
        total = int(rel[-1] + span[-1]) if n else 0
        start = int(self.sigs["sig_off"][0]) if n else int(self.arena.size)
        head_end = 0
        for k in self.keys:
            head_end = max(head_end, int(k["off"]) + int(k["len"]))
        for t in self.tmpls:
            head_end = max(head_end, int(t["prefix_off"]) + int(t["prefix_len"]), int(t["suffix_off"]) + int(t["suffix_len"]))
        if n and np.array_equal(self.sigs["sig_off"], np.uint64(start) + rel) and head_end <= start \
                and start + total <= self.arena.size:
            stream = self.arena[start:start + total]
            arena = self.arena[:start]
        else:
            stream = np.zeros(total, np.uint8)
            src = self.sigs["sig_off"].astype(np.int64)
            for j in range(n):
                ln = int(self.sigs["sig_len"][j])
                stream[int(rel[j]):int(rel[j]) + ln] = self.arena[src[j]:src[j] + ln]
            arena = self.arena
        return PackedTxSigBatch(self.keys, self.ids, sig12, stream, self.tmpls, arena)


class PackedTxSigBatch:
    """cg_verify_tx_signatures_packed input: ``sigs`` (TXSIG12_DTYPE), ``stream`` (uint8: signature i
    at the 4-byte-aligned end of signature i-1), ``arena`` (key and template bytes)."""

    def __init__(self, keys, ids, sigs, stream, tmpls, arena):
        self.keys, self.sigs, self.stream, self.tmpls, self.arena = keys, sigs, stream, tmpls, arena
        self.ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1)

    @property
    def n(self):
        return len(self.sigs)

    @property
    def n_ids(self):
        return self.ids.size // 32

    @property
    def h2d_bytes(self):
        return int(self.arena.size + self.stream.size + self.sigs.nbytes + self.ids.nbytes + self.keys.nbytes)


class TxSigBuilder(BatchBuilder):
    """Packs (tx id, TransactionSignature) pairs the way a JVM caller of cg_verify_tx_signatures
    would: one key per distinct PublicKey, one id per distinct tx id, one template per distinct
    SignatureMetadata (its SignableData prefix / suffix), then the signature bytes."""

    def __init__(self):
        super().__init__()
        self._ids, self._id_index = [], {}
        self._tmpls, self._tmpl_index = [], {}
        self._sigs = []

    def tx_id(self, tx_id):
        tx_id = bytes(tx_id)
        if len(tx_id) != 32:
            raise ValueError("a SecureHash.SHA256 id is 32 bytes")
        idx = self._id_index.get(tx_id)
        if idx is None:
            idx = self._id_index[tx_id] = len(self._ids)
            self._ids.append(tx_id)
        return idx

    def template(self, prefix, suffix):
        k = (bytes(prefix), bytes(suffix))
        idx = self._tmpl_index.get(k)
        if idx is None:
            if len(self._tmpls) >= 0x10000:
                raise ValueError("more than 65536 SignatureMetadata templates in one batch")
            idx = self._tmpl_index[k] = len(self._tmpls)
            self._tmpls.append((self._append(k[0], 4), self._append(k[1], 4), len(k[0]), len(k[1])))
        return idx

    def add_signature(self, key_idx, tx_idx, tmpl_idx, sig):
        sig = sig_field(self._keys[key_idx][2], sig)
        self._sigs.append((self._append(sig, 4), tx_idx, key_idx, len(sig), tmpl_idx))
        return len(self._sigs) - 1

    def build(self):
        b = super().build()
        sigs = np.zeros(len(self._sigs), dtype=TXSIG_DTYPE)
        if self._sigs:
            arr = np.array(self._sigs, dtype=np.uint64)
            sigs["sig_off"], sigs["tx_idx"], sigs["key_idx"] = arr[:, 0], arr[:, 1], arr[:, 2]
            sigs["sig_len"], sigs["tmpl"] = arr[:, 3], arr[:, 4]
        tmpls = np.zeros(len(self._tmpls), dtype=TMPL_DTYPE)
        for i, t in enumerate(self._tmpls):
            tmpls[i] = t
        ids = np.frombuffer(b"".join(self._ids), dtype=np.uint8).copy() if self._ids else np.zeros(0, np.uint8)
        return TxSigBatch(b.keys, ids, sigs, tmpls, b.arena)
