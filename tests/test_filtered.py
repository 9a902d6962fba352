"""Tear-offs: FilteredTransaction.verify / PartialMerkleTree.build / verify.

CPU (no marker): the oracle restatement reproduces PartialMerkleTreeTest.kt's behaviours and the
committed fixtures (tests/golden/filtered.json, made by tests/golden/gen_filtered.py); the host
mirror's tree building and table packing (corda_amd/merkle.py) match the oracle.
GPU (@gpu): cg_verify_filtered through the C ABI against the fixtures, seeded random tear-offs
checked against the oracle, and the malformed inputs only the ABI can express (status 3).
"""
import hashlib
import json
import os
import random

import numpy as np
import pytest

from corda_amd import batch as B
from corda_amd import merkle as M
from oracle import corda as C

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "filtered.json")
HASHED = [hashlib.sha256(c.encode()).digest() for c in "abcdef"]


def _fixture():
    with open(GOLDEN) as f:
        return json.load(f)["items"]


def _decode(case):
    root = bytes.fromhex(case["root"])
    if case["filtered"]:
        leaves = [(bytes.fromhex(x["blob"]), bytes.fromhex(x["nonce"])) for x in case["leaves"]]
    else:
        leaves = [bytes.fromhex(x) for x in case["leaves"]]
    stream = [(k, bytes.fromhex(h) if h is not None else None) for k, h in case["pmt"]]
    return root, leaves, stream


class _PostOrder:
    """A partial tree given directly as its post-order stream (pack_filtered input)."""

    def __init__(self, stream):
        self.stream = stream

    def postorder(self):
        return self.stream


def _as_ftx(case):
    root, leaves, stream = _decode(case)
    pmt = _PostOrder(stream)
    if case["filtered"]:
        return M.FilteredTransaction(root, [b for b, _ in leaves], [n for _, n in leaves], pmt)
    return (root, leaves, None, pmt)


class _HashlibEngine:
    """Stands in for the GPU in host-logic tests (tree building only)."""

    @staticmethod
    def sha256(msgs):
        return [hashlib.sha256(bytes(m)).digest() for m in msgs]


# ----------------------------------------------------------------------------- CPU
def test_oracle_reference_build_behaviour():
    """PartialMerkleTreeTest.kt:86-96 (full-tree check) and :179-191 (duplicate leaves)."""
    mt = C.merkle_tree(HASHED)
    with pytest.raises(C.MerkleTreeException):
        C.partial_tree_build(mt, [HASHED[3], HASHED[5], HASHED[3], HASHED[5]])
    aaa = [hashlib.sha256(b"a").digest()] * 3
    with pytest.raises(C.MerkleTreeException):
        C.partial_tree_build(C.merkle_tree(aaa), aaa[:1])
    with pytest.raises(ValueError):
        C.partial_tree_build(mt, [C.ZERO_HASH])
    h = HASHED[0]
    left = ("N", h, ("N", h, ("L", h), ("L", h)), ("N", h, ("L", h), ("L", h)))
    right = ("N", h, ("L", h), ("L", h))
    with pytest.raises(C.MerkleTreeException):
        C.partial_tree_build(("N", h, left, right), [h])
    C.partial_tree_build(right, [h, h])
    C.partial_tree_build(("L", h), [h])


def test_oracle_matches_fixture():
    items = _fixture()
    assert {c["cls"] for c in items} >= {"ref_ok", "ref_too_many", "ref_too_few", "ref_duplicate", "ref_different",
                                         "ref_wrong_root", "ok", "tampered_blob", "tampered_nonce", "wrong_root",
                                         "missing_leaf", "extra_leaf", "shuffled", "empty"}
    for c in items:
        root, leaves, stream = _decode(c)
        assert C.filtered_status(root, leaves, C.partial_tree_from_postorder(stream), c["filtered"]) == c["expect"]


def test_host_mirror_build_matches_oracle():
    rng = random.Random(5)
    for n in (1, 2, 3, 5, 6, 8, 11, 17):
        hs = [rng.randbytes(32) for _ in range(n)]
        full = M.merkle_tree(hs, engine=_HashlibEngine)
        assert full.hash == C.merkle_root(hs)
        for _ in range(4):
            incl = rng.sample(hs, rng.randrange(0, n + 1))
            pmt = M.PartialMerkleTree.build(full, incl)
            want = C.partial_tree_postorder(C.partial_tree_build(C.merkle_tree(hs), incl))
            assert pmt.postorder() == want
    with pytest.raises(M.MerkleTreeException):
        M.merkle_tree([], engine=_HashlibEngine)
    with pytest.raises(ValueError):
        M.PartialMerkleTree.build(M.merkle_tree(HASHED, engine=_HashlibEngine), [bytes(32)])


def test_pack_filtered_layout():
    items = _fixture()[:20]
    t, n, lv, arena = M.pack_filtered([_as_ftx(c) for c in items])
    assert t.dtype == B.FTX_DTYPE and n.dtype == B.PMT_NODE_DTYPE and lv.dtype == B.FLEAF_DTYPE
    assert len(t) == 20 and int(t["n_nodes"].sum()) == len(n) and int(t["n_leaves"].sum()) == len(lv)
    for j, c in enumerate(items):
        root, leaves, stream = _decode(c)
        assert arena[t[j]["root_off"]:t[j]["root_off"] + 32].tobytes() == root
        assert bool(t[j]["flags"] & B.FTX_FILTERED) == c["filtered"]
        for q, (kind, h) in enumerate(stream):
            row = n[t[j]["first_node"] + q]
            assert row["kind"] == kind
            if h is not None:
                assert arena[row["hash_off"]:row["hash_off"] + 32].tobytes() == h
    assert arena.size % 4 == 0 or arena[-8:].tobytes() == bytes(8)


# ----------------------------------------------------------------------------- GPU
@pytest.mark.gpu
def test_filtered_fixture_gpu(engine):
    items = _fixture()
    st = M.verify_filtered_batch([_as_ftx(c) for c in items], engine)
    want = np.array([c["expect"] for c in items], dtype=np.uint8)
    bad = np.nonzero(st != want)[0]
    assert len(bad) == 0, [(items[i]["cls"], int(st[i]), int(want[i])) for i in bad[:10]]


@pytest.mark.gpu
def test_filtered_random_vs_oracle(engine):
    """Seeded tear-offs of random transactions (1-40 components, every corruption class)."""
    rng = random.Random(77)
    ftxs, want = [], []
    for k in range(3000):
        n = rng.randrange(1, 40)
        blobs = [rng.randbytes(rng.randrange(0, 300)) for _ in range(n)]
        salt = rng.randbytes(32)
        nonces = [C.compute_nonce(salt, i) for i in range(n)]
        hashes = [C.sha256(b + x) for b, x in zip(blobs, nonces)] + [C.sha256(b"\x01" + salt)]
        mt = C.merkle_tree(hashes)
        vis = sorted(rng.sample(range(n), rng.randrange(0, n + 1)))
        pt = C.partial_tree_build(mt, [hashes[i] for i in vis])
        leaves = [(blobs[i], nonces[i]) for i in vis]
        root = mt[1]
        r = rng.random()
        if r < 0.1 and leaves:
            leaves[0] = (leaves[0][0] + b"\x00", leaves[0][1])
        elif r < 0.2:
            root = bytes(32)
        elif r < 0.3 and leaves:
            leaves.append(leaves[-1])
        elif r < 0.4:
            rng.shuffle(leaves)
        want.append(C.filtered_status(root, leaves, pt))
        ftxs.append(M.FilteredTransaction(root, [b for b, _ in leaves], [x for _, x in leaves],
                                          _PostOrder(C.partial_tree_postorder(pt))))
    st = M.verify_filtered_batch(ftxs, engine)
    want = np.array(want, dtype=np.uint8)
    assert np.array_equal(st, want), np.nonzero(st != want)[0][:10]
    assert set(np.unique(want).tolist()) == {0, 1, 2}


@pytest.mark.gpu
def test_filtered_host_api_gpu(engine):
    """The host mirror end to end on the GPU: tree building (GPU SHA-256 levels), build,
    PartialMerkleTree.verify and FilteredTransaction.verify / its MerkleTreeException."""
    full = M.merkle_tree(HASHED, engine)
    assert full.hash == C.merkle_root(HASHED)
    pmt = M.PartialMerkleTree.build(full, [HASHED[3], HASHED[5]])
    assert pmt.verify(full.hash, [HASHED[3], HASHED[5]], engine)
    assert not pmt.verify(full.hash, [HASHED[5], HASHED[3], HASHED[0]], engine)
    assert not pmt.verify(C.hash_concat(HASHED[3], HASHED[5]), [HASHED[3], HASHED[5]], engine)
    salt = bytes(range(32))
    blobs = [b"input", b"output-state", b"command", b"notary", b"time-window"]
    nonces = [C.compute_nonce(salt, i) for i in range(len(blobs))]
    hashes = [C.sha256(b + x) for b, x in zip(blobs, nonces)] + [C.sha256(b"\x01" + salt)]
    wfull = M.merkle_tree(hashes, engine)
    vis = [0, 3, 4]
    ftx = M.FilteredTransaction(wfull.hash, [blobs[i] for i in vis], [nonces[i] for i in vis],
                                M.PartialMerkleTree.build(wfull, [hashes[i] for i in vis]))
    assert ftx.verify(engine) is True
    empty = M.FilteredTransaction(wfull.hash, [], [], M.PartialMerkleTree.build(wfull, []))
    with pytest.raises(M.MerkleTreeException):
        empty.verify(engine)


@pytest.mark.gpu
def test_filtered_malformed_gpu(engine):
    """Inputs a JVM PartialTree cannot express are status 3, never 'valid'."""
    h = HASHED
    good = [(B.PMT_LEAF, h[0]), (B.PMT_INCLUDED, h[1]), (B.PMT_NODE, None)]
    root = C.hash_concat(h[0], h[1])
    deep = [(B.PMT_LEAF, h[0])] * (C_MAX_DEPTH + 1) + [(B.PMT_NODE, None)] * C_MAX_DEPTH
    cases = [
        (good, 0),
        ([(B.PMT_NODE, None)], 3),                                   # underflow
        ([(B.PMT_LEAF, h[0]), (B.PMT_INCLUDED, h[1])], 3),           # two roots left
        ([(B.PMT_LEAF, h[0]), (7, h[1]), (B.PMT_NODE, None)], 3),    # unknown kind
        ([], 3),                                                     # no nodes
        (deep, 3),                                                   # deeper than CG_PMT_MAX_DEPTH
    ]
    ftxs = [(root, [h[1]], None, _PostOrder(s)) for s, _ in cases]
    st = M.verify_filtered_batch(ftxs, engine, filtered=False)
    assert st.tolist() == [w for _, w in cases]
    # a hash / leaf / root offset outside the arena, through the raw tables
    t, n, lv, arena = M.pack_filtered(ftxs[:1], filtered=False)
    t2, n2, lv2 = t.copy(), n.copy(), lv.copy()
    t2["root_off"] = arena.size
    assert engine.verify_filtered(t2, n, lv, arena).tolist() == [3]
    n2[0]["hash_off"] = arena.size - 4
    assert engine.verify_filtered(t, n2, lv, arena).tolist() == [3]
    lv2[0]["len"] = 31
    assert engine.verify_filtered(t, n, lv2, arena).tolist() == [3]
    t3 = t.copy()
    t3["n_nodes"] = len(n) + 1
    assert engine.verify_filtered(t3, n, lv, arena).tolist() == [3]


C_MAX_DEPTH = 64
