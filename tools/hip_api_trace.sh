#!/bin/bash
# Host-side HIP API time of the headline (rocprofv3 --hip-trace --stats, no counters): which runtime
# calls the enqueuing thread spends its time in.  usage: bash tools/hip_api_trace.sh <tag> [bench args]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}; shift
OUT=gpurun_out/hipapi_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --device-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 "$@" > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name '*hip_api_stats.csv' | head -1)
head -40 "$f"
echo HIPAPI_DONE
