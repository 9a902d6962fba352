#!/bin/bash
# rocprofv3 passes over the configs[3] transaction pipeline (1M WireTransactions: tx ids, SignableData
# splice, verify) with a small headline: kernel trace + stats, then FETCH_SIZE / WRITE_SIZE / SQ
# passes, each its own process with its own time limit.  usage: bash tools/profile_tx.sh <tag>
set -o pipefail
export TMPDIR=/tmp
TAG=${1:-v}
OUT=gpurun_out/prof_tx_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --items 1048576 --no-cpu-baseline --host-steps 0 --configs1-items 0 --ecdsa-items 0 --tear-offs 0 --configs0-txs 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
echo trace_ok
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $B > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $B > $OUT/write.log 2>&1 || { echo WRITE_FAIL; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $B > $OUT/valu.log 2>&1 || { echo VALU_FAIL; exit 1; }
echo PROFILE_TX_DONE
