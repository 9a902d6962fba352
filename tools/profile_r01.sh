#!/bin/bash
# Round-1 profiling recipe (run on the GPU box from the repo root). Each rocprofv3 pass is
# its own process; counter passes never combine --pmc with tracing domains.
# usage: bash tools/profile_r01.sh <tag>
set -e
export TMPDIR=/tmp
TAG=${1:-v}
OUT=gpurun_out/prof_r01_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ecdsa-items 0 --mixed-items 0 --pipeline-txs 0 --tear-offs 0 --host-buffers 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1
echo PROFILE_DONE
