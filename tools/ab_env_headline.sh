#!/bin/bash
# Headline-only bench under each environment setting given as NAME=VALUE ("-" = none).
# usage: bash tools/ab_env_headline.sh <tag> <NAME=VALUE[+NAME=VALUE...]|-> [...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for kv in "$@"; do
  name=$(echo "$kv" | tr '=' '_')
  if [ "$kv" = "-" ]; then E=""; else E=$(echo "$kv" | tr '+' ' '); fi
  env $E timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --device-steps 0 --host-steps 0 \
    --key-dists '' --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 \
    --no-cpu-baseline --secondary-out $OUT/h_${name}_sec.json > $OUT/h_$name.log 2> $OUT/h_$name.err || { echo FAIL $kv; tail -20 $OUT/h_$name.err; exit 1; }
  python - $OUT/h_$name.log "$kv" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sec = json.load(open(sys.argv[1][:-4] + "_sec.json"))
s = sec["headline_h2d"]["cg_stats_ms_mean"]
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "plan", s.get("ms_key_prep"), "h2d", s["ms_h2d"],
      "verify", s["ms_verify"], "mism", sec["verdicts"]["label_mismatches"])
PY
done
echo AB_DONE
