"""The N > 1 path on CPU: world_size 2 over gloo (127.0.0.1). Each rank verifies its
contiguous shard (with the C oracle standing in for the GPU engine: there is no GPU here)
and the verdict bytes are all-gathered; the result must equal one unsharded run."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import golden_io
from corda_amd import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist

    from oracle import c_oracle
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        items = golden_io.load("ed25519.json") + golden_io.load("ecdsa.json")
        b, exp, _ = golden_io.sig_batch(items)
        full = shard.verify_sharded(b, lambda s: c_oracle.verify_batch(s, 0, 2), world, rank)
        q.put((rank, full.tobytes(), exp.tobytes()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_verify_matches_unsharded(world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, full, exp in res:
        assert np.array_equal(np.frombuffer(full, np.uint8), np.frombuffer(exp, np.uint8)), rank


def test_shard_ranges_cover_exactly():
    for n in (0, 1, 7, 1000, 1 << 20):
        for w in (1, 2, 3, 8):
            spans = [shard.shard_range(n, w, r) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in spans]
            assert max(sizes) - min(sizes) <= 1
