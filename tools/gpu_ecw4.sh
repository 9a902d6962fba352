#!/bin/bash
# Round 6: the ECDSA wide ladders at 4 waves per SIMD (128 VGPRs, ~180 B of scratch;
# tools/variants/ecw4.so) against 3 (159 / 168 VGPRs); parity, then an interleaved A/B, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
CORDA_AMD_LIB=tools/variants/ecw4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/ecw4_pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/ecw4_pytest.log; exit 1; }
tail -1 gpurun_out/ecw4_pytest.log
bash tools/ab_cfg.sh ecw4 3 "w3||--h2h-steps 0 --ctx2-steps 0" "w4|CORDA_AMD_LIB=tools/variants/ecw4.so|--h2h-steps 0 --ctx2-steps 0" || exit 1
echo ECW4_DONE
