#!/bin/bash
# Round 6, device-resident headline: the Ed25519 wide-row builds with independent column chains
# (FE9_ROWS_ILP=1, tools/variants/rowsilp.so) against the pinned chains; interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
CORDA_AMD_LIB=tools/variants/rowsilp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/rowsilp_pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/rowsilp_pytest.log; exit 1; }
tail -1 gpurun_out/rowsilp_pytest.log
bash tools/ab_cfg.sh rowsilp 3 "pin||--h2h-steps 0 --ctx2-steps 0" "ilp|CORDA_AMD_LIB=tools/variants/rowsilp.so|--h2h-steps 0 --ctx2-steps 0" || exit 1
echo ROWSILP_DONE
