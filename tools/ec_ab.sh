set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ec_ab
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/ec_ab/pytest_main.log 2>&1 || { echo MAIN_TESTS_FAIL; tail -30 gpurun_out/ec_ab/pytest_main.log; exit 1; }
tail -1 gpurun_out/ec_ab/pytest_main.log
CORDA_AMD_LIB=tools/variants/ecacc.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_txsig.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/ec_ab/pytest_acc.log 2>&1 || { echo ACC_TESTS_FAIL; tail -30 gpurun_out/ec_ab/pytest_acc.log; exit 1; }
tail -1 gpurun_out/ec_ab/pytest_acc.log
bash tools/ab_cfg.sh ec 3 "main||" "acc|CORDA_AMD_LIB=tools/variants/ecacc.so|" "r5|CORDA_AMD_LIB=tools/variants/ecr5.so|"
