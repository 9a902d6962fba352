#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration passes (tools/microbench/fetch_calib.hip), one PMC counter per
# run.  usage: bash tools/fetch_calib.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/fetch_calib}
mkdir -p $OUT
./tools/microbench/fetch_calib > $OUT/expected.jsonl || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $OUT/$c -o run --output-format csv -- ./tools/microbench/fetch_calib > $OUT/$c.log 2>&1 || { echo FAIL $c; tail -5 $OUT/$c.log; exit 1; }
done
echo CALIB_DONE
