#!/bin/bash
# One GPU-box pass: parity tests, smoke, default bench line, then rocprofv3 passes.
# usage: bash tools/gpu_check.sh <tag> [skip_prof]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench.log 2>&1 || { echo BENCH_FAIL; tail -30 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
if [ "$2" != "skip_prof" ]; then
  bash tools/profile_r01.sh $TAG || { echo PROF_FAIL; exit 1; }
fi
echo ALL_DONE
