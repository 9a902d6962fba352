#!/usr/bin/env python3
"""One key-distribution leg of bench.py on its own (for rocprofv3 traces and counter passes): the
headline call shape (cg_verify_tx_signatures, host arena -> host verdicts, 12.5M signatures) with
'distinct' (every pool item its own key: 2^20 keys) or 'zipf' keys. Prints the leg's JSON.
usage: python3 tools/keydist_probe.py [distinct|zipf] [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from corda_amd.engine import Engine
    dist = sys.argv[1] if len(sys.argv) > 1 else "distinct"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    a = bench.parse([])
    threads = bench.host_threads(0)
    with Engine(0, stage_timing=True) as eng:
        out = bench.bench_key_dist(a, eng, dist, 0, threads, steps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
