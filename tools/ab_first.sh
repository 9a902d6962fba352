#!/bin/bash
# Headline-only bench with CG_TXSIG_FIRST_DIV set to each value (0 = equal chunks).
# usage: bash tools/ab_first.sh <tag> <div> [<div> ...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for dv in "$@"; do
  CG_TXSIG_FIRST_DIV=$dv timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --device-steps 0 --host-steps 0 \
    --key-dists '' --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 \
    --no-cpu-baseline > $OUT/first_$dv.log 2>&1 || { echo FAIL $dv; tail -20 $OUT/first_$dv.log; exit 1; }
  python - $OUT/first_$dv.log $dv <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
s = d["secondary"]["headline_h2d"]["cg_stats_ms_mean"]
print("first_div", sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "plan", s.get("ms_key_prep"), "h2d",
      s["ms_h2d"], "verify", s["ms_verify"], "mism", d["verdicts"]["label_mismatches"])
PY
done
echo AB_DONE
