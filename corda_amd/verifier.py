"""Out-of-process verifier with a batch-signature request.

Reference: node-api/src/main/kotlin/net/corda/nodeapi/VerifierApi.kt:10-58 (request /
response messages keyed by a ``verificationId`` long property, reply to the request's
JMSReplyTo address) and verifier/src/main/kotlin/net/corda/verifier/Verifier.kt:69-84 (the
handler: decode, verify, reply with the exception or nothing, acknowledge). Today the verifier
runs ``LedgerTransaction.verify()`` and does no signature work; this module adds the message
pair INTEGRATION.md §4 specifies:

  * ``BatchSignatureRequest(verification_id, mode, keys, items, arena)`` -- the body is the
    C ABI's own tables (cg_key / cg_item / arena, include/cordagpu.h) behind a fixed header,
    so the verifier hands it to ``cg_verify_batch`` without re-encoding;
  * ``BatchSignatureResponse(verification_id, status, error)`` -- one status byte per item, or
    an error string when the request itself could not be run (the analogue of
    RESULT_EXCEPTION_FIELD_NAME carrying a serialised Throwable).

``VerifierWorker`` is the handler for one GPU: one process owns one device and one cg_ctx.
``serve`` consumes a shared request queue until it receives ``None`` -- several workers on one
queue are load-balanced the way Artemis balances consumers of ``verifier.requests``.
Transport is any object with ``get()`` / ``put()`` (``multiprocessing.Queue`` in tests); the
wire body is plain bytes, so an Artemis body buffer carries it unchanged.
"""
import struct
from dataclasses import dataclass

import numpy as np

from . import batch as B

VERIFICATION_REQUESTS_QUEUE_NAME = "verifier.requests"          # VerifierApi.kt:12
VERIFICATION_RESPONSES_QUEUE_NAME_PREFIX = "verifier.responses"  # VerifierApi.kt:13

_REQ_MAGIC = b"CGBQ"
_RSP_MAGIC = b"CGBR"
_REQ_HDR = struct.Struct("<4sHHqIIQQ")   # magic, version, mode, id, n_keys, reserved, n_items, arena_len
_RSP_HDR = struct.Struct("<4sHHqQI")     # magic, version, reserved, id, n_status, error_len
_VERSION = 1


class MalformedMessage(ValueError):
    pass


@dataclass
class BatchSignatureRequest:
    verification_id: int
    mode: int
    keys: np.ndarray    # KEY_DTYPE
    items: np.ndarray   # ITEM_DTYPE
    arena: np.ndarray   # uint8

    @staticmethod
    def from_batch(verification_id, batch, mode=B.MODE_DOVERIFY):
        return BatchSignatureRequest(int(verification_id), int(mode), batch.keys, batch.items, batch.arena)

    def to_bytes(self):
        if self.keys.dtype != B.KEY_DTYPE or self.items.dtype != B.ITEM_DTYPE:
            raise MalformedMessage("key / item tables must be KEY_DTYPE / ITEM_DTYPE")
        hdr = _REQ_HDR.pack(_REQ_MAGIC, _VERSION, self.mode, self.verification_id, len(self.keys), 0,
                            len(self.items), self.arena.size)
        return b"".join((hdr, self.keys.tobytes(), self.items.tobytes(), self.arena.tobytes()))

    @staticmethod
    def from_bytes(body):
        body = memoryview(bytes(body))
        if len(body) < _REQ_HDR.size:
            raise MalformedMessage("short request header")
        magic, ver, mode, vid, n_keys, _, n_items, arena_len = _REQ_HDR.unpack_from(body)
        if magic != _REQ_MAGIC or ver != _VERSION:
            raise MalformedMessage("not a batch-signature request")
        if mode not in (B.MODE_DOVERIFY, B.MODE_ISVALID):
            raise MalformedMessage(f"unknown mode {mode}")
        kb, ib = n_keys * B.KEY_DTYPE.itemsize, n_items * B.ITEM_DTYPE.itemsize
        if len(body) != _REQ_HDR.size + kb + ib + arena_len:
            raise MalformedMessage("body length does not match the header")
        o = _REQ_HDR.size
        keys = np.frombuffer(body[o:o + kb], dtype=B.KEY_DTYPE).copy()
        items = np.frombuffer(body[o + kb:o + kb + ib], dtype=B.ITEM_DTYPE).copy()
        arena = np.frombuffer(body[o + kb + ib:], dtype=np.uint8).copy()
        return BatchSignatureRequest(vid, mode, keys, items, arena)


@dataclass
class BatchSignatureResponse:
    verification_id: int
    status: np.ndarray          # uint8 per item (include/cordagpu.h status codes)
    error: str = None           # request-level failure: no status was produced

    def to_bytes(self):
        err = (self.error or "").encode()
        st = np.ascontiguousarray(self.status, dtype=np.uint8)
        return _RSP_HDR.pack(_RSP_MAGIC, _VERSION, 0, self.verification_id, st.size, len(err)) + st.tobytes() + err

    @staticmethod
    def from_bytes(body):
        body = bytes(body)
        if len(body) < _RSP_HDR.size:
            raise MalformedMessage("short response header")
        magic, ver, _, vid, n, elen = _RSP_HDR.unpack_from(body)
        if magic != _RSP_MAGIC or ver != _VERSION or len(body) != _RSP_HDR.size + n + elen:
            raise MalformedMessage("not a batch-signature response")
        o = _RSP_HDR.size
        st = np.frombuffer(body[o:o + n], dtype=np.uint8).copy()
        err = body[o + n:].decode() if elen else None
        return BatchSignatureResponse(vid, st, err)


class VerifierWorker:
    """The verifier process's handler for batch-signature requests on one GPU
    (Verifier.kt:69-84 with the request verified by cg_verify_batch instead of
    LedgerTransaction.verify). ``engine`` is a corda_amd.engine.Engine (one cg_ctx)."""

    def __init__(self, engine):
        self.engine = engine

    def handle(self, body):
        """Request body bytes -> response body bytes. A request that cannot be decoded or run is
        answered with an error and no statuses, never with statuses that read as valid."""
        try:
            req = BatchSignatureRequest.from_bytes(body)
        except MalformedMessage as e:
            vid = struct.unpack_from("<q", bytes(body), 8)[0] if len(body) >= 16 else -1
            return BatchSignatureResponse(vid, np.zeros(0, np.uint8), f"MalformedMessage: {e}").to_bytes()
        try:
            st = self.engine.verify(B.Batch(req.keys, req.items, req.arena), req.mode)
        except Exception as e:  # noqa: BLE001 - reported to the requester like Verifier.kt:73-78
            return BatchSignatureResponse(req.verification_id, np.zeros(0, np.uint8),
                                          f"{type(e).__name__}: {e}").to_bytes()
        return BatchSignatureResponse(req.verification_id, st).to_bytes()

    def serve(self, requests, responses):
        """Consume ``requests`` until a ``None`` sentinel; each message is (reply_to, body) and
        the reply is put on ``responses`` as (reply_to, body)."""
        n = 0
        while True:
            msg = requests.get()
            if msg is None:
                return n
            reply_to, body = msg
            responses.put((reply_to, self.handle(body)))
            n += 1


def serve_device(device, requests, responses):
    """Process entry point: one verifier process per GPU (Verifier.main, Verifier.kt:50-86)."""
    from .engine import Engine
    with Engine(device) as eng:
        return VerifierWorker(eng).serve(requests, responses)
