#!/bin/bash
# Round 6, device-resident headline: the first of the two device chunks at 50% (default) / 60% / 67%
# of the call (CG_DEV_FIRST_PCT); interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
CG_DEV_FIRST_PCT=67 timeout -k 10 300 python -u -m pytest tests/test_gpu_txsig.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/firstpct_pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/firstpct_pytest.log; exit 1; }
tail -1 gpurun_out/firstpct_pytest.log
bash tools/ab_cfg.sh firstpct 3 "p50||--h2h-steps 0 --ctx2-steps 0" "p60|CG_DEV_FIRST_PCT=60|--h2h-steps 0 --ctx2-steps 0" "p67|CG_DEV_FIRST_PCT=67|--h2h-steps 0 --ctx2-steps 0" || exit 1
echo FIRSTPCT_DONE
