#!/bin/bash
# Round 6: the final GPU pass (suite, smoke, full bench) on the main build, then an interleaved A/B
# of k_ed_ladder_wide at 5 waves per SIMD (tools/variants/w5.so: 96 VGPRs, 36 B scratch).
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu_round6.sh final_c || exit 1
CORDA_AMD_LIB=tools/variants/w5.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/final_c/pytest_w5.log 2>&1 || { echo W5_TESTS_FAIL; tail -20 gpurun_out/final_c/pytest_w5.log; exit 1; }
tail -1 gpurun_out/final_c/pytest_w5.log
bash tools/ab_cfg.sh w5 3 "w4||--h2h-steps 0" "w5|CORDA_AMD_LIB=tools/variants/w5.so|--h2h-steps 0" || exit 1
echo FINAL_W5_DONE
