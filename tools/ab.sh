#!/bin/bash
# A/B kernel experiment on one GPU box: bench the in-tree library and the variants given as
# arguments (paths to alternative libcordagpu.so builds), interleaved, Ed25519 headline only.
# usage: bash tools/ab.sh out_tag variantB.so [variantC.so ...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 10 --no-cpu-baseline ${BENCH_ARGS:---ecdsa-items 0 --mixed-items 0 --pipeline-txs 0}"
for round in 1 2; do
  timeout -k 10 200 $B > $OUT/base_$round.log 2>&1 || exit 1
  i=0
  for v in "$@"; do
    i=$((i+1))
    CORDA_AMD_LIB=$v timeout -k 10 200 $B > $OUT/v${i}_$round.log 2>&1 || exit 1
  done
done
python3 tools/ab_summary.py $OUT/*.log
