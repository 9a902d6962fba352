#!/bin/bash
# Round-4 profiling passes (GPU box, repo root). usage: bash tools/profile_r04.sh <tag> <what...>
#   keydist  kernel trace of the distinct-key leg alone (tools/keydist_probe.py)
#   headline bash tools/profile_r03.sh (trace + FETCH_SIZE / WRITE_SIZE / SQ passes) on the headline
#   tx       bash tools/profile_tx.sh (the configs[3] transaction pipeline: k_tx_* kernels)
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
for what in "$@"; do
  case $what in
    keydist)
      OUT=gpurun_out/prof_r04_kd_$TAG; mkdir -p $OUT
      K="python3 tools/keydist_probe.py distinct 2"
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $K > $OUT/trace.log 2>&1 || { echo KD_FAIL; tail -20 $OUT/trace.log; exit 1; }
      echo keydist_ok
      if [ -n "$KD_PMC" ]; then
        timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- $K > $OUT/fetch.log 2>&1 || { echo KD_FETCH_FAIL; exit 1; }
        timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- $K > $OUT/write.log 2>&1 || { echo KD_WRITE_FAIL; exit 1; }
        timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d $OUT/valu -o run --output-format csv -- $K > $OUT/valu.log 2>&1 || { echo KD_VALU_FAIL; exit 1; }
        echo keydist_pmc_ok
      fi ;;
    headline)
      bash tools/profile_r03.sh r04_$TAG || exit 1 ;;
    tx)
      bash tools/profile_tx.sh r04_$TAG || exit 1 ;;
  esac
done
echo PROFILE_R04_DONE
