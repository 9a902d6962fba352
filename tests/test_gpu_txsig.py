"""GPU tests of cg_verify_tx_signatures(_device) / cg_pool_verify_tx_signatures: the batch form of
Crypto.doVerify(txId, TransactionSignature) (Crypto.kt:499-502), each signature's clear data
SignableData(id, metadata) = prefix || id || suffix spliced on the device.

Parity: the C oracle verifies the same signatures over the materialised SignableData bytes
(tests/txsig_util.py); at full size (> 8M signatures, the configs[4] per-GPU shard in one call)
through idempotence: every draw's verdict equals its pool item's, which equals the oracle's."""
import os

import numpy as np
import pytest

from corda_amd import batch as B
from oracle import c_oracle

import txsig_util

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def spool():
    from corda_amd import signable
    from tools.workload import wl
    b, labels, schemes = wl.notary_pool(1 << 16, ed_keys=512, ec_keys=128, seed=91, nthreads=16, sig_group=4)
    pre, _ = signable.template(1, 4)
    ids, id_idx = wl.pool_ids(b, len(pre))
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    return b, labels, schemes, ids, id_idx, ref


def test_tx_signatures_host_and_device_vs_oracle(spool):
    import torch
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    idx = np.random.default_rng(3).integers(0, b.n, 150_000)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    # the oracle on the materialised messages of a sample agrees with the pool verdicts
    sub = np.random.default_rng(4).choice(tb.n, 4000, replace=False)
    tsub = B.TxSigBatch(tb.keys, tb.ids, tb.sigs[sub], tb.tmpls, tb.arena)
    assert np.array_equal(c_oracle.verify_batch(txsig_util.to_message_batch(tsub), 0, 16), ref[idx[sub]])
    for chunk in (0, 40_001):
        with Engine(0, chunk_items=chunk) as eng:
            st = eng.verify_tx_signatures(tb)
            assert np.array_equal(st, ref[idx]), f"host path (chunk {chunk}): {np.count_nonzero(st != ref[idx])} differ"
            dev = torch.device("cuda", 0)
            up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
            kd, ijd, sgd, ad = up(tb.keys), up(tb.ids), up(tb.sigs), up(tb.arena)
            sd = torch.full((tb.n,), 255, dtype=torch.uint8, device=dev)
            eng.verify_tx_signatures_device(kd.data_ptr(), len(tb.keys), ijd.data_ptr(), tb.n_ids, sgd.data_ptr(), tb.n,
                                            tb.tmpls, ad.data_ptr(), tb.arena.size, sd.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(sd.cpu().numpy(), ref[idx]), "device path"
            # message-form call on the same items gives the same verdicts
            st_m = eng.verify(txsig_util.to_message_batch(B.TxSigBatch(tb.keys, tb.ids, tb.sigs[:20000], tb.tmpls,
                                                                        tb.arena)))
            assert np.array_equal(st_m, st[:20000])


def test_registered_host_buffers_and_thread_budgets(spool):
    """Zero-copy ingestion (cg_host_register) and the host thread budget change only how the bytes
    reach the device: the verdicts equal the oracle's with the caller's arena / signature table / ids
    registered, for host budgets of 1, 2 and 16 threads, and after unregistering (pageable again)."""
    from corda_amd import _lib
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    idx = np.random.default_rng(5).integers(0, b.n, 300_000)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    L = _lib.lib()
    arrs = (tb.arena, tb.sigs, tb.ids)
    for a in arrs:
        assert _lib.host_register(a)
        assert L.cg_host_registered(a.ctypes.data, a.nbytes) == 1
    # overlapping and unknown ranges are refused
    assert L.cg_host_register(tb.arena.ctypes.data + 8, 16) != 0
    assert L.cg_host_unregister(tb.arena.ctypes.data + 8) != 0
    try:
        for threads in (1, 2, 16):
            with Engine(0, chunk_items=70_001 if threads == 2 else 0, host_threads=threads) as eng:
                st = eng.verify_tx_signatures(tb)
                assert np.array_equal(st, ref[idx]), f"registered, {threads} threads: {np.count_nonzero(st != ref[idx])} differ"
    finally:
        for a in arrs:
            _lib.host_unregister(a)
    assert L.cg_host_registered(tb.arena.ctypes.data, tb.arena.nbytes) == 0
    with Engine(0) as eng:
        assert np.array_equal(eng.verify_tx_signatures(tb), ref[idx]), "pageable after unregistering"


def test_tx_signatures_edges():
    """Out-of-range id / template index -> NOT_RUN; templates of any length (odd, empty prefix or
    suffix); isValid mode; an empty call; signatures before the keys in the arena."""
    from corda_amd.engine import Engine
    from corda_amd.batch import TxSigBuilder
    import golden_io
    items = [it for it in golden_io.load("ed25519.json") if it["expect"] in ("VALID", "INVALID")][:6]
    rng = np.random.default_rng(8)
    bld = TxSigBuilder()
    tx = [bld.tx_id(rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(3)]
    tm = [bld.template(b"\x01\x02\x03", b""), bld.template(b"", b"\xfe" * 7), bld.template(b"p" * 233, b"s" * 5)]
    for it in items:
        bld.key(4, 0, bytes.fromhex(it["key"]))
    # synthetic signatures: whatever the verdict, the engine must agree with the oracle on the
    # materialised bytes
    for j in range(60):
        k = bld.key(4, 0, bytes.fromhex(items[j % len(items)]["key"]))
        bld.add_signature(k, tx[j % 3], tm[j % 3], bytes.fromhex(items[(j * 7) % len(items)]["sig"]))
    tb = bld.build()
    tb.sigs[5]["tx_idx"] = 99        # no such id
    tb.sigs[6]["tmpl"] = 40          # no such template
    with Engine(0) as eng:
        for mode in (B.MODE_DOVERIFY, B.MODE_ISVALID):
            st = eng.verify_tx_signatures(tb, mode)
            ref = c_oracle.verify_batch(txsig_util.to_message_batch(tb), mode, 4)
            assert st[5] == B.NOT_RUN and st[6] == B.NOT_RUN
            assert np.array_equal(st, ref)
        empty = B.TxSigBatch(tb.keys, tb.ids, tb.sigs[:0], tb.tmpls, tb.arena)
        assert eng.verify_tx_signatures(empty).size == 0


def test_tx_signatures_valid_signable_data():
    """Real signatures over SignableData(id, SignatureMetadata(1, 4)): VALID through the splice,
    INVALID under another id or another metadata template."""
    from corda_amd import signable
    from corda_amd.batch import TxSigBuilder
    from corda_amd.engine import Engine
    from oracle import ed25519_i2p as ed
    rng = np.random.default_rng(12)
    bld = TxSigBuilder()
    pre, suf = signable.template(1, 4)
    pre3, suf3 = signable.template(1, 3)
    t4, t3 = bld.template(pre, suf), bld.template(pre3, suf3)
    expect = []
    for j in range(24):
        seed = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        pub = ed.public_from_seed(seed)
        txid = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        sig = ed.sign(seed, signable.serialize(txid, 1, 4))
        k = bld.key(4, 0, pub)
        other = bld.tx_id(rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        tid = bld.tx_id(txid)
        bld.add_signature(k, tid, t4, sig)
        bld.add_signature(k, other, t4, sig)
        bld.add_signature(k, tid, t3, sig)
        expect += [B.VALID, B.INVALID, B.INVALID]
    with Engine(0) as eng:
        assert list(eng.verify_tx_signatures(bld.build())) == expect


def test_tx_signatures_8m_one_call(spool):
    """> 8M signatures (configs[4] per-GPU shape) in ONE cg_verify_tx_signatures call from host
    buffers: two device chunks, signature bytes copied per chunk. Idempotence vs the oracle."""
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    n = 8_400_000
    idx = np.random.default_rng(21).integers(0, b.n, n)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    with Engine(0) as eng:
        st = eng.verify_tx_signatures(tb)
    assert not np.any(st == B.NOT_RUN)
    bad = np.nonzero(st != ref[idx])[0]
    assert bad.size == 0, f"{bad.size} of {n} verdicts differ from the oracle's verdict on the same pool item"
    assert np.all(st[labels[idx] == 0] == B.VALID)


def test_pool_tx_signatures(spool):
    from corda_amd.engine import EnginePool
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    idx = np.random.default_rng(5).integers(0, b.n, 100_000)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    with EnginePool([0, 0], chunk_items=30000) as ep:
        assert np.array_equal(ep.verify_tx_signatures(tb), ref[idx])
        assert ep.last_stats["shards"] == 2
        ep.inject_fault(0)
        assert np.array_equal(ep.verify_tx_signatures(tb), ref[idx])
        assert ep.last_stats["reruns"] == 1


def test_tx_signatures_ecdsa_template_lengths():
    """ECDSA through the splice with SHA-256 resuming from the template prefix's midstate, for
    prefixes of 0, 63, 64, 127, 128, 200 and 234 bytes (0, 0, 1, 1, 2, 3, 3 absorbed blocks) and
    suffixes of 0-9 bytes: verdicts equal the oracle's on the materialised bytes and the labels."""
    from corda_amd.batch import TMPL_DTYPE, TXSIG_DTYPE
    from corda_amd.engine import Engine
    from tools.workload import wl
    rng = np.random.default_rng(31)
    parts, tm = [], []
    lens = [(0, 5), (63, 9), (64, 0), (127, 3), (128, 1), (200, 7), (234, 3)]
    for j, (pl, sl) in enumerate(lens):
        pre = rng.integers(0, 256, pl, dtype=np.uint8).tobytes()
        suf = rng.integers(0, 256, sl, dtype=np.uint8).tobytes()
        with wl.signable_mode(pre, suf, group=3, id_seed=j + 1):
            b, lab = wl.ecdsa_batch(j & 1, 400, n_keys=20, msg_len=pl + 32 + sl, corrupt_permille=150, seed=40 + j,
                                    nthreads=8)
        parts.append((b, lab, pre, suf))
    big, _ = wl.concat([p[0] for p in parts])
    labels = np.concatenate([p[1] for p in parts])
    # template bytes behind the arena; ids = the 32 bytes after each message's prefix
    arena = [big.arena]
    off = big.arena.size
    tmpls = np.zeros(len(parts), TMPL_DTYPE)
    for j, (_, _, pre, suf) in enumerate(parts):
        tmpls[j] = (off, off + len(pre), len(pre), len(suf))
        arena.append(np.frombuffer(pre + suf, np.uint8))
        off += len(pre) + len(suf)
    arena = np.concatenate(arena + [np.zeros(64, np.uint8)])
    tm = np.repeat(np.arange(len(parts)), [p[0].n for p in parts])
    pl = np.array([len(parts[t][2]) for t in tm])
    rows = arena[big.items["msg_off"].astype(np.int64)[:, None] + pl[:, None] + np.arange(32)]
    sigs = np.zeros(big.n, TXSIG_DTYPE)
    sigs["sig_off"], sigs["sig_len"], sigs["key_idx"] = big.items["sig_off"], big.items["sig_len"], big.items["key_idx"]
    sigs["tx_idx"] = np.arange(big.n)
    sigs["tmpl"] = tm
    tb = B.TxSigBatch(big.keys, rows.reshape(-1), sigs, tmpls, arena)
    ref = c_oracle.verify_batch(txsig_util.to_message_batch(tb), B.MODE_DOVERIFY, 8)
    assert np.array_equal(ref, c_oracle.verify_batch(big, B.MODE_DOVERIFY, 8))
    assert np.all(ref[labels == 0] == B.VALID) and np.all(ref[labels == 1] == B.INVALID)
    with Engine(0) as eng:
        st = eng.verify_tx_signatures(tb)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} differ"


def test_tx_signatures_mixed_table_modes(spool):
    """One family hot (every key wide, so the host counts skip its row-0 / full table builds) and
    the other two cold (row-0 tables for unsampled keys, wide for sampled ones), for each family in
    turn, through one host-buffer call each: verdicts equal the oracle's on the same pool items."""
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    rng = np.random.default_rng(44)
    with Engine(0) as eng:
        for hot in (4, 3, 2):  # Ed25519, secp256r1, secp256k1 (Corda scheme numbers)
            h, c = np.nonzero(schemes == hot)[0], np.nonzero(schemes != hot)[0]
            idx = np.concatenate([rng.choice(h, 1_500_000), rng.choice(c, 30_000)])
            rng.shuffle(idx)
            tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
            st = eng.verify_tx_signatures(tb)
            bad = np.nonzero(st != ref[idx])[0]
            assert bad.size == 0, f"hot scheme {hot}: {bad.size} verdicts differ, first at {bad[:5]}"


def test_every_table_mode_in_one_call(spool):
    """Keys drawn 1, 2, 3, 6, 12, 31, 40 and 1900 times in one call, so that every table mode
    (keyws.h: row 0, quarter, full, wide) and the boundaries between them carry items of every
    scheme: the host-buffer tx-signature path (fewer than 256 uses a key on average: the exact
    host count), the device one and the message form all give the oracle's verdicts on the same
    pool items."""
    import torch
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    rng = np.random.default_rng(77)
    per_key = [1, 2, 3, 6, 12, 31, 40, 1900]
    key_of = b.items["key_idx"]
    order = np.argsort(key_of, kind="stable")
    starts = np.searchsorted(key_of[order], np.arange(len(b.keys) + 1))
    draws = []
    for k in range(len(b.keys)):
        mine = order[starts[k]:starts[k + 1]]
        if mine.size:
            draws.append(rng.choice(mine, per_key[k % len(per_key)]))
    idx = np.concatenate(draws)
    rng.shuffle(idx)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    with Engine(0) as eng:
        st = eng.verify_tx_signatures(tb)
        assert np.array_equal(st, ref[idx]), f"host path: {np.count_nonzero(st != ref[idx])} differ"
        dev = torch.device("cuda", 0)
        up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
        kd, ijd, sgd, ad = up(tb.keys), up(tb.ids), up(tb.sigs), up(tb.arena)
        sd = torch.full((tb.n,), 255, dtype=torch.uint8, device=dev)
        eng.verify_tx_signatures_device(kd.data_ptr(), len(tb.keys), ijd.data_ptr(), tb.n_ids, sgd.data_ptr(), tb.n,
                                        tb.tmpls, ad.data_ptr(), tb.arena.size, sd.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(sd.cpu().numpy(), ref[idx]), "device path"
        from corda_amd.batch import Batch
        assert np.array_equal(eng.verify(Batch(b.keys, b.items[idx], b.arena)), ref[idx]), "message form"


def test_skipped_modes_are_reported_not_run():
    """the host skips a family's row-0 / quarter / full builds and ladders when its counts
    prove no key needs them (verify.hip families_needing_full). If the device classification ever
    disagrees, the items of those modes must come back CG_NOT_RUN, never a verdict from stale
    tables. CG_TEST_SKIP_FAMILIES forces the skip for every family (in a child process: the library
    reads it once): every verdict equals the oracle's or is NOT_RUN, and the skipped modes' items
    are NOT_RUN; without it, every verdict is the oracle's."""
    import json
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    for mask, expect_skip in (("7", True), ("0", False)):
        env = dict(os.environ, CG_TEST_SKIP_FAMILIES=mask)
        r = subprocess.run([sys.executable, os.path.join(here, "mode_guard_probe.py")], env=env, capture_output=True,
                           text=True, timeout=240)
        assert r.returncode == 0, r.stderr[-2000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
        assert out["wide"]["n"] > 0 and out["wide"]["oracle"] == out["wide"]["n"], out
        assert out["other"]["n"] > 0 and out["other"]["other"] == 0, out
        if expect_skip:
            # every item is the oracle's verdict or NOT_RUN, never a verdict from tables that were not
            # built; the items of the skipped modes are NOT_RUN. (Keys the sampled host count puts on
            # wide tables -- a sampled key in a hot call is raised to the wide threshold -- keep
            # their verdicts: their work is not skipped.)
            o = out["other"]
            assert o["not_run"] > 0 and o["not_run"] + o["oracle"] == o["n"], out
        else:
            assert out["other"]["oracle"] == out["other"]["n"], out


# ---- round 6: the 12-byte signature table over a dense signature stream (cg_txsig_packed,
# VERDICT r5 item 4). Every verdict equals the 24-byte form's on the same signatures.
def test_packed_host_device_pool_vs_oracle(spool):
    import torch
    from corda_amd.engine import Engine, EnginePool
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    idx = np.random.default_rng(61).integers(0, b.n, 150_000)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    pb = tb.packed()
    assert np.shares_memory(pb.stream, tb.arena)  # the generator's tail is already the dense stream
    assert pb.h2d_bytes < tb.arena.size + tb.sigs.nbytes + tb.ids.nbytes + tb.keys.nbytes - 11 * tb.n
    for chunk in (0, 40_001):
        with Engine(0, chunk_items=chunk) as eng:
            st = eng.verify_tx_signatures_packed(pb)
            assert np.array_equal(st, ref[idx]), f"packed host (chunk {chunk}): {np.count_nonzero(st != ref[idx])}"
            # device form: the stream inside the one HBM arena (tb.arena = head || stream)
            dev = torch.device("cuda", 0)
            up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
            kd, ijd, sgd, ad = up(pb.keys), up(pb.ids), up(pb.sigs), up(tb.arena)
            sd = torch.full((pb.n,), 255, dtype=torch.uint8, device=dev)
            eng.verify_tx_signatures_packed_device(kd.data_ptr(), len(pb.keys), ijd.data_ptr(), pb.n_ids,
                                                   sgd.data_ptr(), pb.n, pb.arena.size, pb.stream.size, pb.tmpls,
                                                   ad.data_ptr(), tb.arena.size, sd.data_ptr())
            torch.cuda.synchronize()
            assert np.array_equal(sd.cpu().numpy(), ref[idx]), "packed device"
    with EnginePool([0, 0], chunk_items=30000) as ep:
        assert np.array_equal(ep.verify_tx_signatures_packed(pb), ref[idx])
        assert ep.last_stats["shards"] == 2
        ep.inject_fault(1)
        assert np.array_equal(ep.verify_tx_signatures_packed(pb), ref[idx])
        assert ep.last_stats["reruns"] == 1


def test_packed_edges():
    """The 24-byte form's edge cases through the 12-byte table: out-of-range id / template -> NOT_RUN,
    odd template lengths, isValid mode, an empty call; plus the packed form's own: signature bytes
    gathered from an interleaved arena, a stream cut short (the signatures past its end NOT_RUN, the
    rest unchanged), a key outside the caller's arena (as in the 24-byte form), and a JVM signature
    longer than 65 535 bytes through its surrogate."""
    from corda_amd.batch import TxSigBuilder
    from corda_amd.engine import Engine
    import golden_io
    items = [it for it in golden_io.load("ed25519.json") if it["expect"] in ("VALID", "INVALID")][:6]
    ec = [it for it in golden_io.load("ecdsa.json") if it["expect"] in ("VALID", "INVALID")][:6]
    rng = np.random.default_rng(18)
    bld = TxSigBuilder()
    tx = [bld.tx_id(rng.integers(0, 256, 32, dtype=np.uint8).tobytes()) for _ in range(3)]
    tm = [bld.template(b"\x01\x02\x03", b""), bld.template(b"", b"\xfe" * 7), bld.template(b"p" * 233, b"s" * 5)]
    for j in range(90):
        if j % 3 == 2:  # ECDSA, DER of 70-72 bytes: the stream's spans are not all 64
            it = ec[j % len(ec)]
            k = bld.key(it["scheme"], it["key_fmt"], bytes.fromhex(it["key"]))
            bld.add_signature(k, tx[j % 3], tm[j % 3], bytes.fromhex(ec[(j * 5) % len(ec)]["sig"]))
        else:
            k = bld.key(4, 0, bytes.fromhex(items[j % len(items)]["key"]))
            bld.add_signature(k, tx[j % 3], tm[j % 3], bytes.fromhex(items[(j * 7) % len(items)]["sig"]))
        if j == 40:  # a signature past the 16-bit length: packed as its surrogate
            bld.add_signature(k, tx[0], tm[0], b"\x30" + bytes(70000))
    tb = bld.build()
    tb.sigs[5]["tx_idx"] = 99
    tb.sigs[6]["tmpl"] = 40
    pb = tb.packed()
    assert not np.shares_memory(pb.stream, tb.arena)  # templates interleave: the bytes were gathered
    with Engine(0) as eng:
        for mode in (B.MODE_DOVERIFY, B.MODE_ISVALID):
            want = eng.verify_tx_signatures(tb, mode)
            assert np.array_equal(want, c_oracle.verify_batch(txsig_util.to_message_batch(tb), mode, 4))
            st = eng.verify_tx_signatures_packed(pb, mode)
            assert st[5] == B.NOT_RUN and st[6] == B.NOT_RUN
            assert np.array_equal(st, want)
        # the stream cut inside signature 70: it and every later one NOT_RUN, the rest as before
        span = (pb.sigs["sig_len"].astype(np.int64) + 3) & ~3
        o70 = int(span[:70].sum())
        short = B.PackedTxSigBatch(pb.keys, pb.ids, pb.sigs, pb.stream[:o70 + 10], pb.tmpls, pb.arena)
        st = eng.verify_tx_signatures_packed(short)
        assert np.all(st[70:] == B.NOT_RUN) and np.array_equal(st[:70], want[:70])
        # a key outside the caller's arena: the 24-byte form's verdicts for that key's signatures
        keys = pb.keys.copy()
        keys[1]["off"] = pb.arena.size + 8  # would land inside the stream on the device
        st = eng.verify_tx_signatures_packed(B.PackedTxSigBatch(keys, pb.ids, pb.sigs, pb.stream, pb.tmpls, pb.arena))
        keys24 = tb.keys.copy()
        keys24[1]["off"] = tb.arena.size + 8
        want_k = eng.verify_tx_signatures(B.TxSigBatch(keys24, tb.ids, tb.sigs, tb.tmpls, tb.arena))
        assert np.array_equal(st, want_k)
        assert np.any(st[pb.sigs["key_idx"] == 1] != want[pb.sigs["key_idx"] == 1])
        empty = B.PackedTxSigBatch(pb.keys, pb.ids, pb.sigs[:0], pb.stream[:0], pb.tmpls, pb.arena)
        assert eng.verify_tx_signatures_packed(empty).size == 0


def test_packed_8m_one_call(spool):
    """The configs[4]-shaped call (> 8M signatures, one call) through the 12-byte table: idempotence
    against the oracle's pool verdicts, as test_tx_signatures_8m_one_call."""
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, schemes, ids, id_idx, ref = spool
    n = 8_400_000
    idx = np.random.default_rng(22).integers(0, b.n, n)
    pb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16).packed()
    with Engine(0) as eng:
        st = eng.verify_tx_signatures_packed(pb)
    assert not np.any(st == B.NOT_RUN)
    bad = np.nonzero(st != ref[idx])[0]
    assert bad.size == 0, f"{bad.size} of {n} verdicts differ"


@pytest.mark.parametrize("bridge", ["1", "0"])
def test_device_call_ordered_on_caller_stream(bridge):
    """A device call enqueued on a caller's (torch) stream: the kernels run on the context's own
    stream, bridged by events (cordagpu.cpp stream_of), and work the caller enqueues on its stream
    afterwards sees the finished verdicts without any synchronisation in between; CG_STREAM_BRIDGE=0
    runs the call on the caller's stream itself. Both in a child process (the switch is read once)."""
    import subprocess
    import sys
    import textwrap
    code = textwrap.dedent(f"""
        import os, sys, numpy as np, torch
        os.environ["CG_STREAM_BRIDGE"] = "{bridge}"
        sys.path.insert(0, {ROOT!r})
        sys.path.insert(0, os.path.join({ROOT!r}, "tests"))
        from corda_amd.engine import Engine
        from corda_amd import signable
        from oracle import c_oracle
        from corda_amd import batch as B
        from tools.workload import wl
        pool, labels, schemes = wl.notary_pool(1 << 14, ed_keys=24, ec_keys=12, seed=707, nthreads=16, sig_group=4)
        ids, id_idx = wl.pool_ids(pool, len(signable.template(1, 4)[0]))
        idx = np.random.default_rng(708).integers(0, pool.n, 90_000)
        tb = wl.tx_sig_stream(pool, schemes, idx, ids, id_idx, nthreads=16)
        pb = tb.packed()
        ref = c_oracle.verify_batch(pool, B.MODE_DOVERIFY, 16)[idx]
        dev = torch.device("cuda", 0)
        up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)
        kd, ijd, sgd, ad = up(pb.keys), up(pb.ids), up(pb.sigs), up(tb.arena)
        s = torch.cuda.Stream(device=dev)
        with Engine(0) as eng:
            outs = []
            for rep in range(3):
                sd = torch.full((pb.n,), 255, dtype=torch.uint8, device=dev)
                torch.cuda.synchronize()
                with torch.cuda.stream(s):
                    eng.verify_tx_signatures_packed_device(kd.data_ptr(), len(pb.keys), ijd.data_ptr(), pb.n_ids,
                                                           sgd.data_ptr(), pb.n, pb.arena.size, pb.stream.size,
                                                           pb.tmpls, ad.data_ptr(), tb.arena.size, sd.data_ptr(),
                                                           stream=s.cuda_stream)
                    outs.append(sd.clone())  # enqueued on the caller's stream right after the call
            torch.cuda.synchronize()
        for o in outs:
            got = o.cpu().numpy()
            assert np.array_equal(got, ref), int(np.count_nonzero(got != ref))
        print("ORDERED_OK")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "ORDERED_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
