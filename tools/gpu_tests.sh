#!/bin/bash
# GPU-box pass: parity tests (one process, per-test timeout), then smoke.
# usage: bash tools/gpu_tests.sh <tag> [pytest -k expr]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}
OUT=gpurun_out/$TAG
mkdir -p $OUT
K=()
[ -n "$2" ] && K=(-k "$2")
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
echo TESTS_DONE
