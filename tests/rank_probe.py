"""One rank of the N-process world that `bench.py --gpus N` starts (bench.spawn_cmd), run here on
CPU over gloo: each rank verifies its contiguous shard of the golden batch with the C oracle
(standing in for the engine: no GPU), the verdict bytes are all-gathered as in the bench
(corda_amd/shard.py), and rank 0 prints one JSON line, the last on stdout, as bench.py does."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import numpy as np
    import torch.distributed as dist

    import bench
    import golden_io
    from corda_amd import shard
    from oracle import c_oracle

    a = bench.parse(sys.argv[1:])
    how, world = bench.launch_plan(a.gpus, os.environ, a.gpus)
    assert how == "inline", how
    rank = int(os.environ["RANK"])
    dist.init_process_group("gloo")
    try:
        items = golden_io.load("ed25519.json") + golden_io.load("ecdsa.json")
        b, exp, _ = golden_io.sig_batch(items)
        full = shard.verify_sharded(b, lambda s: c_oracle.verify_batch(s, 0, 1), world, rank)
        ok = bool(np.array_equal(full, exp))
        if rank == 0:
            print(json.dumps({"n_gpus": world, "items": int(b.n), "equal_unsharded": ok}), flush=True)
    finally:
        dist.destroy_process_group()
    sys.exit(0 if ok else 3)


if __name__ == "__main__":
    main()
