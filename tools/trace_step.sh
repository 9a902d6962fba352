#!/bin/bash
# One rocprofv3 kernel-trace pass of the headline (bench.py --steps 3) and the per-step timeline
# of its last step (tools/timeline.py).  usage: bash tools/trace_step.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}; shift
OUT=gpurun_out/trace_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
f=$(find $OUT/trace -name '*kernel_trace.csv' | head -1)
python3 tools/timeline.py "$f" -1 > $OUT/timeline_step.txt && echo TRACE_DONE
