#!/bin/bash
# what 8 ranks' host sides do to one rank, on one GPU. The headline runs at one
# rank's share of the 16-CPU quota (--threads 2 --engine-threads 2) while 7 GPU-free processes
# (stage_load: 2 threads each, ~1.06 GB memcpy per 36-ms step, what the HIP runtime's pageable
# staging does on each other rank) load the host; pageable copies vs registered (--host-register 1,
# DMA straight from the caller's pages: no staging memcpy on any rank, so the loaders then only read
# their 1.06 GB per step, the other ranks' DMA traffic on host memory). Interleaved, ROUNDS times.
# usage: bash tools/host8/run.sh <tag> <rounds>
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ROUNDS=${2:-2}
OUT=gpurun_out/host8_$TAG
mkdir -p $OUT
B="python3 -u bench.py --steps 5 --warmup 2 --threads 2 --engine-threads 2 --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 --no-cpu-baseline"
run() {  # name, loaders (0 none / copy / read), bench args
  local name=$1 load=$2; shift 2
  local pids=()
  if [ "$load" != 0 ]; then
    for q in 1 2 3 4 5 6 7; do
      ./tools/host8/stage_load 2 1060 36 400 $load > $OUT/${name}_load$q.json 2>&1 &
      pids+=($!)
    done
  fi
  timeout -k 10 400 $B "$@" --secondary-out $OUT/${name}_sec.json > $OUT/$name.log 2> $OUT/$name.err
  local rc=$?
  for p in "${pids[@]}"; do kill $p 2>/dev/null; done
  wait 2>/dev/null
  [ $rc = 0 ] || { echo FAIL $name rc=$rc; tail -20 $OUT/$name.err; exit 1; }
  python3 - $OUT/$name.log $OUT/${name}_sec.json $name <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sec = json.load(open(sys.argv[2]))
h = sec.get("headline_h2d", {}).get("cg_stats_ms_mean", {})
print(sys.argv[3], "value", d["value"], "ms", d["ms_per_step"], "h2d", h.get("ms_h2d"), "prep", h.get("ms_key_prep"), flush=True)
PY
}
for r in $(seq 1 $ROUNDS); do
  run quiet_pageable_$r 0
  run load_pageable_$r copy
  run load_registered_$r read --host-register 1
  run quiet_registered_$r 0 --host-register 1
done
echo HOST8_DONE
