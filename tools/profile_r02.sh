#!/bin/bash
# Round-2 profiling recipe for the headline (run on the GPU box from the repo root). Each rocprofv3
# pass is its own process; counter passes never combine --pmc with tracing domains; each pass has
# its own time limit.  usage: bash tools/profile_r02.sh <tag> [bench args...]
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}; shift
OUT=gpurun_out/prof_r02_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --host-steps 0 --device-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
echo trace_ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; tail -5 $OUT/fetch.log; exit 1; }
echo fetch_ok
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { echo WRITE_FAIL; tail -5 $OUT/write.log; exit 1; }
echo write_ok
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1 || { echo VALU_FAIL; tail -5 $OUT/valu.log; exit 1; }
echo valu_ok
echo PROFILE_DONE
