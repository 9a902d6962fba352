"""Whole-chain resolution: ResolveTransactionsFlow.topologicalSort restated on
the host, and the downloaded chain verified as one GPU call with the serial loop's failure
semantics (ResolveTransactionsFlow.kt:36-96, SignedTransaction.kt:143-149)."""
import random

import pytest

from corda_amd import signable
from corda_amd import transactions as T
from corda_amd.crypto import IllegalArgumentException, PublicKey, SignatureException
from oracle import corda as C
from oracle import ed25519_i2p as ed


class _Stx:
    def __init__(self, inputs):
        self.inputs = inputs


def _kotlin_topological_sort(stxs, ids):
    """Literal recursive restatement of ResolveTransactionsFlow.topologicalSort (:36-62), the
    check for the iterative host version."""
    forward = {}
    for t, s in enumerate(stxs):
        for h in s.inputs:
            forward.setdefault(h, [])
            if t not in forward[h]:
                forward[h].append(t)
    visited, result = set(), []

    def visit(t):
        if ids[t] not in visited:
            visited.add(ids[t])
            for d in forward.get(ids[t], []):
                visit(d)
            result.append(t)

    for t in range(len(stxs)):
        visit(t)
    result.reverse()
    assert len(result) == len(stxs)
    return result


def _random_dag(rng, n):
    ids = [rng.randbytes(32) for _ in range(n)]
    stxs = []
    for t in range(n):
        k = rng.randrange(0, min(t, 3) + 1)
        deps = rng.sample(range(t), k) if t else []
        stxs.append(_Stx([ids[d] for d in deps] + ([rng.randbytes(32)] if rng.random() < 0.2 else [])))
    perm = list(range(n))
    rng.shuffle(perm)
    return [stxs[p] for p in perm], [ids[p] for p in perm]


def test_topological_sort_matches_reference_order():
    rng = random.Random(3)
    for n in (1, 2, 5, 17, 60):
        for _ in range(5):
            stxs, ids = _random_dag(rng, n)
            order = T.topological_sort(stxs, ids)
            assert order == _kotlin_topological_sort(stxs, ids)
            pos = {t: i for i, t in enumerate(order)}
            idx = {h: t for t, h in enumerate(ids)}
            for t, s in enumerate(stxs):
                for h in s.inputs:
                    if h in idx:
                        assert pos[idx[h]] < pos[t]


def test_topological_sort_deep_chain_and_duplicates():
    n = 5000   # deeper than Python's default recursion limit: the host sort is iterative
    ids = [i.to_bytes(32, "big") for i in range(n)]
    stxs = [_Stx([ids[t - 1]] if t else []) for t in range(n)]
    order = T.topological_sort(stxs[::-1], ids[::-1])
    assert order == list(range(n))[::-1]
    with pytest.raises(IllegalArgumentException):
        T.topological_sort([_Stx([]), _Stx([])], [ids[0], ids[0]])


def _chain(n, seed, bad=None, missing=None):
    """A chain of signed wire transactions (tx t spends tx t-1), listed shuffled. ``bad``: index
    (chain position) whose second signature is corrupted; ``missing``: index lacking a required
    signer."""
    rng = random.Random(seed)
    seeds = [ed.entropy_seed(40 + i) for i in range(3)]
    keys = [PublicKey(4, ed.public_from_seed(s)) for s in seeds]
    stxs, ids = [], []
    for t in range(n):
        comps = [rng.randbytes(rng.randrange(20, 200)) for _ in range(rng.randrange(1, 6))]
        if t:
            comps[0] = ids[t - 1] + b"\x00\x00\x00\x00"       # the input StateRef (txhash, index)
        salt = rng.randbytes(32)
        wtx = T.WireTransactionData(comps, salt, b"\x01" + salt)
        tid = C.tx_id(comps, salt, b"\x01" + salt)
        msg = signable.serialize(tid, 1, 4)
        sigs = [T.TransactionSignature(ed.sign(s, msg), k, 1, 4) for s, k in zip(seeds, keys)]
        if t == bad:
            b = bytearray(sigs[1].bytes)
            b[40] ^= 4
            sigs[1] = T.TransactionSignature(bytes(b), keys[1], 1, 4)
        req = set(keys)
        if t == missing:
            sigs = sigs[:2]
        stxs.append(T.SignedWireTransaction(wtx, sigs, req, [ids[t - 1]] if t else []))
        ids.append(tid)
    perm = list(range(n))
    rng.shuffle(perm)
    return [stxs[p] for p in perm], [ids[p] for p in perm], perm


@pytest.mark.gpu
def test_verify_chain_gpu():
    stxs, ids, perm = _chain(40, 1)
    seen = []
    order = T.verify_chain(stxs, on_verified=lambda t, i: seen.append((t, i)))
    assert [perm[t] for t in order] == list(range(40))       # dependencies first
    assert [i for _, i in seen] == [ids[t] for t in order]


@pytest.mark.gpu
def test_verify_chain_first_failure_gpu():
    stxs, ids, perm = _chain(30, 2, bad=17, missing=9)
    seen = []
    with pytest.raises(T.SignaturesMissingException) as ei:
        T.verify_chain(stxs, on_verified=lambda t, i: seen.append(perm[t]))
    assert seen == list(range(9))                               # the serial loop stops at chain position 9
    assert ei.value.tx_id == ids[perm.index(9)]
    stxs, ids, perm = _chain(30, 2, bad=17)
    seen = []
    with pytest.raises(SignatureException):
        T.verify_chain(stxs, on_verified=lambda t, i: seen.append(perm[t]))
    assert seen == list(range(17))
    seen = []
    T.verify_chain(_chain(30, 2, missing=9)[0], check_sufficient_signatures=False,
                   on_verified=lambda t, i: seen.append(t))
    assert len(seen) == 30
    with pytest.raises(T.ExcessivelyLargeTransactionGraph):
        T.verify_chain(stxs, limit=10)
