#!/bin/bash
# Round 6, device-resident headline: phase-1 issue priorities. Default: Ed25519 wide-row builds at
# s_setprio 2, the challenge hash at 0. rp0: the row builds at 0; fp3: the hash at 3 (above the rows).
set -o pipefail
export TMPDIR=/tmp
for v in rp0 fp3; do
  CORDA_AMD_LIB=tools/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${v}_pytest.log 2>&1 || { echo TESTS_FAIL $v; tail -20 gpurun_out/${v}_pytest.log; exit 1; }
  tail -1 gpurun_out/${v}_pytest.log
done
bash tools/ab_cfg.sh rowprio 3 "def||--h2h-steps 0 --ctx2-steps 0" "rp0|CORDA_AMD_LIB=tools/variants/rp0.so|--h2h-steps 0 --ctx2-steps 0" "fp3|CORDA_AMD_LIB=tools/variants/fp3.so|--h2h-steps 0 --ctx2-steps 0" || exit 1
echo ROWPRIO_DONE
