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
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/keydist_probe.py distinct 2 > $OUT/trace.log 2>&1 || { echo KD_FAIL; tail -20 $OUT/trace.log; exit 1; }
      echo keydist_ok ;;
    headline)
      bash tools/profile_r03.sh r04_$TAG || exit 1 ;;
    tx)
      bash tools/profile_tx.sh r04_$TAG || exit 1 ;;
  esac
done
echo PROFILE_R04_DONE
