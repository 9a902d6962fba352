#!/bin/bash
# A/B of library builds on one GPU box: the whole-node headline (bench.py headline only) with the
# in-tree libcordagpu.so and each variant .so (tools/build_variant.sh), interleaved, two rounds.
# usage: bash tools/ab_lib.sh <tag> variantB.so [variantC.so ...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B="python3 -u bench.py --steps 5 --warmup 2 --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 --no-cpu-baseline"
summ() {  # the compact stdout line + the secondary file bench.py wrote beside it
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
sec = json.load(open(sys.argv[1][:-4] + "_sec.json"))
st = {k: v["ms_per_step"] for k, v in sec["stages"].items() if v["ms_per_step"] > 0.5}
print(sys.argv[2], "value", d["value"], "ms", d["ms_per_step"], "mism", sec["verdicts"]["label_mismatches"], st)
PY
}
for round in 1 2; do
  timeout -k 10 300 $B --secondary-out $OUT/base_${round}_sec.json > $OUT/base_$round.log 2> $OUT/base_$round.err || { echo FAIL base; tail -20 $OUT/base_$round.err; exit 1; }
  summ $OUT/base_$round.log base_$round
  i=0
  for v in "$@"; do
    i=$((i+1))
    CORDA_AMD_LIB=$v timeout -k 10 300 $B --secondary-out $OUT/v${i}_${round}_sec.json > $OUT/v${i}_$round.log 2> $OUT/v${i}_$round.err || { echo FAIL $v; tail -20 $OUT/v${i}_$round.err; exit 1; }
    summ $OUT/v${i}_$round.log "v${i}_$round($(basename $v))"
  done
done
echo AB_DONE
