#!/bin/bash
# Interleaved A/B of headline configurations on one GPU box (bench.py headline leg only).
# usage: bash tools/ab_cfg.sh <tag> <rounds> "name|ENV=v ENV2=v|--bench-args" ["name2|...|..." ...]
#   ENV may name CORDA_AMD_LIB=tools/variants/<v>.so (a library variant, tools/build_variant.sh).
# Each run: timeout 300 s; a failing run ends the script (no retry on the GPU).
set -o pipefail
export TMPDIR=/tmp
TAG=$1; ROUNDS=$2; shift 2
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B="python3 -u bench.py --steps 5 --warmup 2 --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 --no-cpu-baseline"
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sec = json.load(open(sys.argv[1][:-4] + "_sec.json"))
st = {k: round(v["ms_per_step"], 2) for k, v in sec["stages"].items() if v["ms_per_step"] > 0.5}
h = sec.get("headline_h2d", {}).get("cg_stats_ms_mean", {})
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "mism", sec["verdicts"]["label_mismatches"],
      "h2d", h.get("ms_h2d"), "prep", h.get("ms_key_prep"), st, flush=True)
PY
}
for round in $(seq 1 $ROUNDS); do
  for cfg in "$@"; do
    IFS='|' read -r name envs args <<< "$cfg"
    f=$OUT/${name}_$round
    env $envs timeout -k 10 300 $B $args --secondary-out ${f}_sec.json > $f.log 2> $f.err || { echo FAIL $name; tail -20 $f.err; exit 1; }
    summ $f.log ${name}_$round
  done
done
echo AB_DONE
