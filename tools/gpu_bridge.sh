#!/bin/bash
# Round 6: device calls on a caller's stream bridged to the context's stream (cordagpu.cpp
# stream_of): the GPU suites that use caller streams, then an interleaved A/B of the device-resident
# headline with and without the bridge (CG_STREAM_BRIDGE=0), then one kernel trace of the bridged form.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/bridge
timeout -k 10 400 python -u -m pytest tests/test_gpu_stream.py tests/test_gpu_txsig.py tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/bridge/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/bridge/pytest.log; exit 1; }
tail -1 gpurun_out/bridge/pytest.log
bash tools/ab_cfg.sh bridge 3 "bridge||--h2h-steps 0" "nobridge|CG_STREAM_BRIDGE=0|--h2h-steps 0" || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/bridge/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --device-steps 0 --host-steps 0 --h2h-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 > gpurun_out/bridge/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo BRIDGE_DONE
