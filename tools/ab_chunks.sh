#!/bin/bash
# Headline-only bench at several device chunk sizes (whole-node call), one process each.
# usage: bash tools/ab_chunks.sh <tag> <chunk> [<chunk> ...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for ch in "$@"; do
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --chunk-items $ch --device-steps 0 --host-steps 0 \
    --key-dists '' --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 \
    --no-cpu-baseline > $OUT/chunk_$ch.log 2>&1 || { echo FAIL $ch; tail -20 $OUT/chunk_$ch.log; exit 1; }
  python - $OUT/chunk_$ch.log $ch <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["secondary"]["headline_h2d"]["cg_stats_ms_mean"]
print("chunk", sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "h2d", s["ms_h2d"], "verify", s["ms_verify"],
      "mism", d["verdicts"]["label_mismatches"])
PY
done
echo AB_DONE
