#!/bin/bash
# GPU-box bench pass: a small smoke run of every bench leg, then the default run.
# usage: bash tools/gpu_bench.sh <tag> [skip_small]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ "$2" != "skip_small" ]; then
timeout -k 10 300 python -u bench.py --items 2000000 --pool 262144 --steps 3 --warmup 1 --configs1-items 262144 \
  --ecdsa-items 131072 --pipeline-txs 65536 --tear-offs 65536 --configs0-txs 2000 --cpu-seconds 2 \
  > $OUT/bench_small.log 2>&1 || { echo SMALL_FAIL; tail -30 $OUT/bench_small.log; exit 1; }
tail -c 3000 $OUT/bench_small.log
fi
timeout -k 10 600 python -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log > $OUT/bench.json
echo BENCH_DONE
