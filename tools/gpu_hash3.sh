#!/bin/bash
# Round 6, device-resident headline: k_ed_hash at 3 waves per SIMD (tools/variants/hash3.so) against 4.
set -o pipefail
export TMPDIR=/tmp
CORDA_AMD_LIB=tools/variants/hash3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/hash3_pytest.log 2>&1 || { echo TESTS_FAIL; tail -20 gpurun_out/hash3_pytest.log; exit 1; }
tail -1 gpurun_out/hash3_pytest.log
bash tools/ab_cfg.sh hash3 3 "h4||--h2h-steps 0 --ctx2-steps 0" "h3|CORDA_AMD_LIB=tools/variants/hash3.so|--h2h-steps 0 --ctx2-steps 0" || exit 1
echo HASH3_DONE
