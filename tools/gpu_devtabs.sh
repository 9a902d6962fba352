#!/bin/bash
# Round 6, device-resident headline: table builds after the first chunk's plan (default) vs before it
# (CG_DEV_TABS_FIRST=1), and 4M-item device chunks; interleaved, 3 rounds; then one kernel trace.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/devtabs
timeout -k 10 300 python -u -m pytest tests/test_gpu_txsig.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/devtabs/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/devtabs/pytest.log; exit 1; }
tail -1 gpurun_out/devtabs/pytest.log
bash tools/ab_cfg.sh devtabs 3 "after||--h2h-steps 0" "first|CG_DEV_TABS_FIRST=1|--h2h-steps 0" "c4m||--h2h-steps 0 --chunk-items 4194304" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/devtabs/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --device-steps 0 --host-steps 0 --h2h-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 > gpurun_out/devtabs/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo DEVTABS_DONE
