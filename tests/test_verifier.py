"""Verifier batch-signature messages (VerifierApi.kt:10-58, Verifier.kt:69-84).

CPU: the request / response wire format round-trips the C ABI tables, malformed bodies are
rejected, and workers sharing one request queue answer every request once (host logic, with a
stand-in engine that records what it was asked). GPU: a worker answers golden-fixture requests
through cg_verify_batch with the fixtures' expected verdicts.
"""
import queue
import threading

import numpy as np
import pytest

import golden_io
from corda_amd import batch as B
from corda_amd import verifier as V


def _batch(n=40, name="ed25519.json"):
    items = golden_io.load(name)[:n]
    b, exp, exp_iv = golden_io.sig_batch(items)
    return b, exp, exp_iv


def test_request_round_trip():
    b, _, _ = _batch()
    req = V.BatchSignatureRequest.from_batch(1234567890123, b, B.MODE_ISVALID)
    got = V.BatchSignatureRequest.from_bytes(req.to_bytes())
    assert got.verification_id == 1234567890123 and got.mode == B.MODE_ISVALID
    assert got.keys.tobytes() == b.keys.tobytes()
    assert got.items.tobytes() == b.items.tobytes()
    assert got.arena.tobytes() == b.arena.tobytes()


def test_response_round_trip():
    st = np.array([0, 1, 2, 3, 4, 5, 255], dtype=np.uint8)
    r = V.BatchSignatureResponse.from_bytes(V.BatchSignatureResponse(-7, st).to_bytes())
    assert r.verification_id == -7 and r.status.tolist() == st.tolist() and r.error is None
    r = V.BatchSignatureResponse.from_bytes(V.BatchSignatureResponse(9, np.zeros(0, np.uint8), "boom").to_bytes())
    assert r.error == "boom" and r.status.size == 0


def test_malformed_requests():
    b, _, _ = _batch(4)
    body = V.BatchSignatureRequest.from_batch(5, b).to_bytes()
    for bad in (body[:10], b"XXXX" + body[4:], body[:-1], body + b"\x00"):
        with pytest.raises(V.MalformedMessage):
            V.BatchSignatureRequest.from_bytes(bad)
    bad_mode = bytearray(body)
    bad_mode[6] = 9
    with pytest.raises(V.MalformedMessage):
        V.BatchSignatureRequest.from_bytes(bytes(bad_mode))


def _kotlin_long(x):
    """x as a JVM Long (64-bit two's complement)."""
    x &= (1 << 64) - 1
    return x - (1 << 64) if x >> 63 else x


def test_crafted_header_counts_are_rejected():
    """n_keys = 2^28, n_items = 1 and an arena_len that, read as a signed Long, cancels
    2^32 of key bytes: the lengths then add up modulo 2^64. Both parsers must refuse it: the Python
    one reads the counts unsigned and never wraps; VerifierBatchApi.parse (not compiled here)
    rejects a negative n_items / arena_len and any count whose table cannot fit a ByteBuffer."""
    import os
    import re
    import struct
    b, _, _ = _batch(1)
    real = V.BatchSignatureRequest.from_batch(5, b).to_bytes()
    n_keys, n_items = 1 << 28, 1
    body_len = len(real)
    # arena_len chosen so that 40 + 16 n_keys + 32 n_items + arena_len == body_len modulo 2^64
    arena_len = (body_len - 40 - 16 * n_keys - 32 * n_items) % (1 << 64)
    crafted = bytearray(real)
    struct.pack_into("<IIQQ", crafted, 16, n_keys, 0, n_items, arena_len)
    assert _kotlin_long(40 + 16 * n_keys + 32 * n_items + _kotlin_long(arena_len)) == body_len  # the wrap
    with pytest.raises(V.MalformedMessage):
        V.BatchSignatureRequest.from_bytes(bytes(crafted))
    for field, val in ((24, 1 << 63), (32, (1 << 64) - 1)):  # negative as a Long
        bad = bytearray(real)
        struct.pack_into("<Q", bad, field, val)
        with pytest.raises(V.MalformedMessage):
            V.BatchSignatureRequest.from_bytes(bytes(bad))
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    kt = open(os.path.join(root, "jvm/src/main/kotlin/net/corda/nodeapi/VerifierBatchApi.kt")).read()
    parse = kt[kt.index("fun parse("):kt.index("class BatchSignatureResponse")]
    assert "and 0xffffffffL" in parse  # n_keys read unsigned
    assert re.search(r"nItems < 0 \|\| arenaLen < 0", parse)
    assert "Int.MAX_VALUE / KEY_BYTES" in parse and "Int.MAX_VALUE / ITEM_BYTES" in parse
    # the Kotlin model of the same check: the crafted header fails the range test before the sum
    nk, ni, al = n_keys, n_items, _kotlin_long(arena_len)
    assert ni < 0 or al < 0 or nk > (2 ** 31 - 1) // 16 or ni > (2 ** 31 - 1) // 32 or al > 2 ** 31 - 1
    assert "Math.toIntExact" in kt[kt.index("private fun slice("):]


class _RecordingEngine:
    """Stand-in for corda_amd.engine.Engine in host-logic tests: answers NOT_RUN-free statuses
    derived from the item index, and fails on request."""

    def __init__(self, name):
        self.name, self.calls = name, 0

    def verify(self, batch, mode):
        self.calls += 1
        if batch.n == 3:
            raise RuntimeError("device lost")
        return (np.arange(batch.n) % 2).astype(np.uint8)


def test_worker_error_paths():
    w = V.VerifierWorker(_RecordingEngine("a"))
    r = V.BatchSignatureResponse.from_bytes(w.handle(b"garbage-garbage-garbage"))
    assert r.error.startswith("MalformedMessage") and r.status.size == 0
    b, _, _ = _batch(3)
    r = V.BatchSignatureResponse.from_bytes(w.handle(V.BatchSignatureRequest.from_batch(11, b).to_bytes()))
    assert r.verification_id == 11 and r.error == "RuntimeError: device lost" and r.status.size == 0


def test_workers_share_one_queue():
    reqs, rsps = queue.Queue(), queue.Queue()
    engines = [_RecordingEngine("gpu0"), _RecordingEngine("gpu1")]
    threads = [threading.Thread(target=V.VerifierWorker(e).serve, args=(reqs, rsps)) for e in engines]
    for t in threads:
        t.start()
    b, _, _ = _batch(10)
    for vid in range(50):
        reqs.put((f"{V.VERIFICATION_RESPONSES_QUEUE_NAME_PREFIX}.node{vid % 3}",
                  V.BatchSignatureRequest.from_batch(vid, b).to_bytes()))
    for _ in threads:
        reqs.put(None)
    for t in threads:
        t.join(30)
    got = {}
    while not rsps.empty():
        reply_to, body = rsps.get()
        r = V.BatchSignatureResponse.from_bytes(body)
        assert reply_to.endswith(f"node{r.verification_id % 3}")
        got[r.verification_id] = r.status
    assert sorted(got) == list(range(50))
    assert sum(e.calls for e in engines) == 50
    assert all(np.array_equal(s, np.arange(10) % 2) for s in got.values())


@pytest.mark.gpu
def test_worker_gpu_golden(engine):
    w = V.VerifierWorker(engine)
    for name in ("ed25519.json", "ecdsa.json"):
        b, exp, exp_iv = _batch(10 ** 6, name)
        for mode, want in ((B.MODE_DOVERIFY, exp), (B.MODE_ISVALID, exp_iv)):
            r = V.BatchSignatureResponse.from_bytes(w.handle(V.BatchSignatureRequest.from_batch(3, b, mode).to_bytes()))
            assert r.error is None and r.verification_id == 3
            assert np.array_equal(r.status, want)


def test_wire_format_matches_kotlin_constants():
    """jvm/.../VerifierBatchApi.kt (not compiled here: no JDK) encodes the same header as this
    module: magic words, header sizes and the C ABI record sizes agree."""
    import os
    import re
    from corda_amd import batch as B
    from corda_amd import verifier as V
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    kt = open(os.path.join(root, "jvm/src/main/kotlin/net/corda/nodeapi/VerifierBatchApi.kt")).read()
    const = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"const val (\w+) = (0x[0-9a-fA-F]+|\d+)", kt)}
    const.update({m.group(1): int(m.group(2), 0) for m in re.finditer(r"private const val (\w+) = (0x[0-9a-fA-F]+|\d+)", kt)})
    assert const["REQ_MAGIC"].to_bytes(4, "little") == V._REQ_MAGIC
    assert const["RSP_MAGIC"].to_bytes(4, "little") == V._RSP_MAGIC
    assert const["REQ_HEADER"] == V._REQ_HDR.size and const["RSP_HEADER"] == V._RSP_HDR.size
    assert const["KEY_BYTES"] == B.KEY_DTYPE.itemsize and const["ITEM_BYTES"] == B.ITEM_DTYPE.itemsize


def test_jni_exports_match_kotlin_externals():
    """Every `external fun` of CryptoBatch.kt has its JNI export in cordagpu_jni.c and vice versa."""
    import os
    import re
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    kt = open(os.path.join(root, "jvm/src/main/kotlin/net/corda/core/crypto/CryptoBatch.kt")).read()
    c = open(os.path.join(root, "jvm/jni/cordagpu_jni.c")).read()
    ext = set(re.findall(r"external fun (\w+)\(", kt))
    exp = set(re.findall(r"Java_net_corda_core_crypto_CryptoBatch_(\w+)\(", c))
    assert ext == exp and ext, (ext ^ exp)
