"""The 12-byte signature table (cg_txsig_packed, include/cordagpu.h) on the CPU: the packer's stream
layout rule (each signature at the 4-byte-aligned end of the one before it), both packing paths
(a view of a dense arena tail, a gather from an interleaved arena) agreeing, and the H2D bytes."""
import numpy as np

from corda_amd import batch as B


def _build(interleave):
    rng = np.random.default_rng(4)
    bld = B.TxSigBuilder()
    k = [bld.key(4, 0, rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(3)]
    t0 = bld.template(b"abc", b"de")
    tx = [bld.tx_id(rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(4)]
    for j in range(50):
        if interleave and j == 20:
            bld.template(b"x" * 9, b"")  # template bytes between signatures
        ln = int(rng.choice([64, 70, 71, 72, 1, 0]))
        bld.add_signature(k[j % 3], tx[j % 4], t0, rng.integers(0, 256, ln, dtype=np.uint8).tobytes())
    return bld.build()


def _check_stream(tb, pb):
    span = (pb.sigs["sig_len"].astype(np.int64) + 3) & ~3
    off = np.concatenate([[0], np.cumsum(span)[:-1]])
    for j in range(tb.n):
        a = int(tb.sigs["sig_off"][j])
        ln = int(tb.sigs["sig_len"][j])
        assert pb.stream[off[j]:off[j] + ln].tobytes() == tb.arena[a:a + ln].tobytes()
    assert pb.stream.size == int(span.sum())
    for f in ("tx_idx", "key_idx", "sig_len", "tmpl"):
        assert np.array_equal(pb.sigs[f], tb.sigs[f])


def test_dense_tail_is_a_view():
    tb = _build(False)
    pb = tb.packed()
    assert np.shares_memory(pb.stream, tb.arena)
    _check_stream(tb, pb)
    assert pb.arena.size == int(tb.sigs["sig_off"][0])


def test_interleaved_arena_is_gathered():
    tb = _build(True)
    pb = tb.packed()
    assert not np.shares_memory(pb.stream, tb.arena)
    _check_stream(tb, pb)


def test_twelve_bytes_per_signature():
    assert B.TXSIG12_DTYPE.itemsize == 12
    tb = _build(False)
    pb = tb.packed()
    full = tb.arena.size + tb.sigs.nbytes + tb.ids.nbytes + tb.keys.nbytes
    assert pb.h2d_bytes <= full - 12 * tb.n
    src = open(B.__file__.replace("corda_amd/batch.py", "include/cordagpu.h")).read()
    assert "} cg_txsig_packed;     /* 12 bytes */" in src
