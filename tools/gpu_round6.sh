#!/bin/bash
# Round 6 GPU pass: the parity suite, smoke, then the full bench (default args) with its line and
# secondary file under gpurun_out/<tag>/.  usage: bash tools/gpu_round6.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-r6}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 900 python -u bench.py --secondary-out $OUT/bench_secondary.json > $OUT/bench_line.json 2> $OUT/bench.err || { echo BENCH_FAIL; tail -30 $OUT/bench.err; exit 1; }
cat $OUT/bench_line.json
echo R6_DONE
