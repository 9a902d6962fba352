#!/bin/bash
# Round 6, device-resident headline: the first two chunks' items and plans before the table builds
# (default) vs inside each front (CG_DEV_PRE_PLAN=0); interleaved, 3 rounds; then one kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/preplan
timeout -k 10 300 python -u -m pytest tests/test_gpu_txsig.py tests/test_gpu_tables.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/preplan/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/preplan/pytest.log; exit 1; }
tail -1 gpurun_out/preplan/pytest.log
bash tools/ab_cfg.sh preplan 3 "pre||--h2h-steps 0" "inline|CG_DEV_PRE_PLAN=0|--h2h-steps 0" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/preplan/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --device-steps 0 --host-steps 0 --h2h-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 > gpurun_out/preplan/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo PREPLAN_DONE
