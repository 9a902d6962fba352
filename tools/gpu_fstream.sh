#!/bin/bash
# Round 6, device-resident headline: chunk 1's hashes and ECDSA fronts on a front stream of their own
# (CG_DEV_FRONT_STREAM=1) so chunk 0's ladders start when the key tables are built; parity under the
# switch, then an interleaved A/B, 3 rounds, then one kernel trace with it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fstream
CG_DEV_FRONT_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_txsig.py tests/test_gpu_tables.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/fstream/pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/fstream/pytest.log; exit 1; }
tail -1 gpurun_out/fstream/pytest.log
bash tools/ab_cfg.sh fstream 3 "main||--h2h-steps 0 --ctx2-steps 0" "fs|CG_DEV_FRONT_STREAM=1|--h2h-steps 0 --ctx2-steps 0" || exit 1
CG_DEV_FRONT_STREAM=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fstream/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --device-steps 0 --host-steps 0 --h2h-steps 0 --ctx2-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 > gpurun_out/fstream/trace.log 2>&1 || { echo TRACE_FAIL; exit 1; }
echo FSTREAM_DONE
