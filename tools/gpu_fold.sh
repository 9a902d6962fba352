#!/bin/bash
# Round 6: the Ed25519 wide ladder's sign fold (fe9.h ge9_madd_half_flip) on the GPU: the parity
# suites that run it, an interleaved A/B against the select form (tools/variants/nofold.so), then
# the round's headline profiling passes (tools/profile_r06.sh).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/fold
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_txsig.py tests/test_gpu_tables.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/fold/pytest.log 2>&1 || { echo TESTS_FAIL; tail -30 gpurun_out/fold/pytest.log; exit 1; }
tail -1 gpurun_out/fold/pytest.log
bash tools/ab_cfg.sh fold 3 "fold||" "sel|CORDA_AMD_LIB=tools/variants/nofold.so|" || exit 1
bash tools/profile_r06.sh a headline
