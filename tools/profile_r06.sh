#!/bin/bash
# Round-6 profiling passes (GPU box, repo root), each its own process with its own time limit;
# counter passes never combine --pmc with tracing domains.
# usage: bash tools/profile_r06.sh <tag> <what...>
#   headline  configs[4] shard (bench.py --steps 3): kernel trace + stats, FETCH_SIZE, WRITE_SIZE,
#             the memory-side read requests by size (TCC_EA0_RDREQ_32B / _64B / _128B, _DRAM), SQ
#   tx        the configs[3] transaction pipeline with a small headline: the same passes
#   calib     tools/microbench/fetch_calib (known byte counts) under the same trio
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
TRIO="TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_DRAM_sum"
SQ="SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
passes() {  # <outdir> <command...>
  local OUT=$1; shift
  mkdir -p $OUT
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- "$@" > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; return 1; }
  echo trace_ok
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- "$@" > $OUT/fetch.log 2>&1 || { echo FETCH_FAIL; return 1; }
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- "$@" > $OUT/write.log 2>&1 || { echo WRITE_FAIL; return 1; }
  timeout -s KILL 240 rocprofv3 --pmc $TRIO -d $OUT/tcc -o run --output-format csv -- "$@" > $OUT/tcc.log 2>&1 || { echo TCC_FAIL; return 1; }
  timeout -s KILL 240 rocprofv3 --pmc $SQ -d $OUT/valu -o run --output-format csv -- "$@" > $OUT/valu.log 2>&1 || { echo VALU_FAIL; return 1; }
  echo pmc_ok
}
for what in "$@"; do
  case $what in
    headline)
      passes gpurun_out/prof_r06_$TAG python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --device-steps 0 --host-steps 0 --h2h-steps 0 \
        --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 || exit 1 ;;
    tx)
      passes gpurun_out/prof_r06_tx_$TAG python3 bench.py --steps 2 --warmup 1 --items 1048576 --no-cpu-baseline \
        --host-steps 0 --device-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --tear-offs 0 --configs0-txs 0 || exit 1 ;;
    calib)
      OUT=gpurun_out/prof_r06_calib_$TAG; mkdir -p $OUT
      ./tools/microbench/fetch_calib > $OUT/expected.jsonl || exit 1
      for c in FETCH_SIZE WRITE_SIZE "$TRIO"; do
        d=$(echo $c | cut -d' ' -f1)
        timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $OUT/$d -o run --output-format csv -- ./tools/microbench/fetch_calib > $OUT/$d.log 2>&1 || { echo CALIB_FAIL $c; exit 1; }
      done
      echo calib_ok ;;
  esac
done
echo PROFILE_R06_DONE
