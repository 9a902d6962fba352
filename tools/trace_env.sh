#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of the headline under one environment setting, for
# a step timeline (tools/timeline.py).  usage: bash tools/trace_env.sh <tag> [NAME=VALUE]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; KV=${2:-}
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0"
if [ -n "$KV" ]; then export "$KV"; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
echo trace_ok
