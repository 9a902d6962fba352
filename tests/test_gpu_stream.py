"""GPU tests of the streaming paths (include/cordagpu.h, ABI v2):
  * chunked verify calls: one key-table build, items in chunks (device and host-buffer forms,
    arena windows copied by extent, any item order / layout), against the C oracle;
  * a BASELINE configs[4]-shaped call of more than 8M items through cg_verify_batch (the JNI
    path): every occurrence of a pool item gets the pool item's verdict, and the pool's verdicts
    equal the C oracle's;
  * async device calls on two streams sharing one context (ordered by the context);
  * cg_pool on one GPU (two contexts on device 0), including a drill fault and its re-run."""
import numpy as np
import pytest

from corda_amd import batch as B
from oracle import c_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pool():
    from tools.workload import wl
    b, labels, schemes = wl.notary_pool(1 << 16, ed_keys=512, ec_keys=128, seed=77, nthreads=16)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    return b, labels, schemes, ref


def test_chunked_device_and_host_paths(pool):
    import torch
    from corda_amd.batch import Batch
    from corda_amd.engine import Engine
    b, labels, schemes, ref = pool
    # reverse the item order: chunk extents then run backwards through the arena
    rb = Batch(b.keys, b.items[::-1].copy(), b.arena)
    with Engine(0, chunk_items=7001) as eng:
        st = eng.verify(b)
        assert np.array_equal(st, ref), f"host path: {np.count_nonzero(st != ref)} mismatches"
        st_r = eng.verify(rb)
        assert np.array_equal(st_r, ref[::-1]), "host path, reversed items"
        dev = torch.device("cuda", 0)
        kd = torch.from_numpy(b.keys.view(np.uint8)).to(dev)
        idd = torch.from_numpy(b.items.view(np.uint8)).to(dev)
        ad = torch.from_numpy(b.arena).to(dev)
        sd = torch.full((b.n,), 255, dtype=torch.uint8, device=dev)
        eng.verify_device(kd.data_ptr(), len(b.keys), idd.data_ptr(), b.n, ad.data_ptr(), b.arena.size, sd.data_ptr())
        torch.cuda.synchronize()
        assert np.array_equal(sd.cpu().numpy(), ref), "device path"


def test_host_window_keys_after_items(pool):
    """Keys stored behind every item in the arena: the window spans both; verdicts unchanged."""
    from corda_amd.batch import Batch
    from corda_amd.engine import Engine
    b, _, _, ref = pool
    keys = b.keys.copy()
    parts, off = [b.arena], b.arena.size
    for j in range(len(keys)):
        o, n = int(keys[j]["off"]), int(keys[j]["len"])
        pad = (-off) % 4
        parts.append(np.zeros(pad, np.uint8))
        off += pad
        parts.append(b.arena[o:o + n])
        keys[j]["off"] = off
        off += n
    b2 = Batch(keys, b.items, np.concatenate(parts + [np.zeros(64, np.uint8)]))
    with Engine(0, chunk_items=9000) as eng:
        assert np.array_equal(eng.verify(b2), ref)


def test_notary_shard_over_8m_items_one_call(pool):
    """> 8M items (BASELINE configs[4] per-GPU shape, 70/20/10) in ONE cg_verify_batch call: several
    device chunks and host pipeline chunks. Bit-exact at full size through idempotence: each item
    is a draw from the pool, so its verdict must equal the pool item's, which equals the oracle's."""
    from corda_amd.engine import Engine
    from tools.workload import wl
    b, labels, _, ref = pool
    n = 8_400_000
    big, idx = wl.index_stream(b, n, seed=5)
    with Engine(0) as eng:
        st = eng.verify(big)
    assert not np.any(st == B.NOT_RUN)
    bad = np.nonzero(st != ref[idx])[0]
    assert bad.size == 0, f"{bad.size} of {n} verdicts differ from the oracle's verdict on the same pool item"
    assert np.all(st[labels[idx] == 0] == B.VALID)


def test_async_calls_on_two_streams_share_one_context(pool):
    """two device calls enqueued back to back on different streams of one context share
    its workspace; the context orders them, so both results are exact."""
    import torch
    from corda_amd.batch import Batch
    from corda_amd.engine import Engine
    b, _, _, ref = pool
    dev = torch.device("cuda", 0)
    half = b.n // 2
    parts = [Batch(b.keys, b.items[:half].copy(), b.arena), Batch(b.keys, b.items[half:].copy(), b.arena)]
    kd = torch.from_numpy(b.keys.view(np.uint8)).to(dev)
    ad = torch.from_numpy(b.arena).to(dev)
    streams = [torch.cuda.Stream(device=dev), torch.cuda.Stream(device=dev)]
    with Engine(0) as eng:
        outs = []
        for p, s in zip(parts, streams):
            idd = torch.from_numpy(p.items.view(np.uint8)).to(dev)
            sd = torch.full((p.n,), 255, dtype=torch.uint8, device=dev)
            torch.cuda.synchronize()
            outs.append((idd, sd))
        for (idd, sd), p, s in zip(outs, parts, streams):
            eng.verify_device(kd.data_ptr(), len(b.keys), idd.data_ptr(), p.n, ad.data_ptr(), b.arena.size,
                              sd.data_ptr(), stream=s.cuda_stream)
        torch.cuda.synchronize()
        got = np.concatenate([sd.cpu().numpy() for _, sd in outs])
    assert np.array_equal(got, ref)


def test_pool_two_contexts_and_drill_fault(pool):
    from corda_amd._lib import EngineUnavailable
    from corda_amd.engine import EnginePool
    b, _, _, ref = pool
    with EnginePool([0, 0], chunk_items=20000) as ep:
        assert np.array_equal(ep.verify(b), ref)
        assert ep.last_stats["shards"] == 2 and ep.last_stats["reruns"] == 0
        ep.inject_fault(1)
        assert np.array_equal(ep.verify(b), ref)           # slot 1's shard re-ran on slot 0
        assert ep.last_stats["reruns"] == 1 and ep.healthy() == [True, False]
        assert np.array_equal(ep.verify(b), ref)           # unhealthy slot skipped
        assert ep.last_stats["shards"] == 1
        ep.inject_fault(0)
        st = ep.verify(b, allow_partial=True)              # nothing healthy: every item NOT_RUN
        assert np.all(st == B.NOT_RUN)
        with pytest.raises(EngineUnavailable):
            ep.verify(b)
        ep.inject_fault(0, False)
        ep.inject_fault(1, False)
        assert ep.healthy() == [True, True]
        assert np.array_equal(ep.verify(b), ref)
