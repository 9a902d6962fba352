#!/bin/bash
# k_tx_leaves A/B: for each library (in-tree and the named variants), a kernel trace of the configs[3]
# pipeline leg (small headline) and one counter pass (L2 hit / miss, memory-side read requests).
# usage: bash tools/ab_tx.sh <outdir> [variant ...]
set -o pipefail
export TMPDIR=/tmp
OUT=$1; shift
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 1 --items 262144 --pool 65536 --no-cpu-baseline --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --tear-offs 0 --configs0-txs 0"
for v in base "$@"; do
  if [ "$v" = base ]; then L=""; else L="tools/variants/$v.so"; fi
  mkdir -p $OUT/$v
  CORDA_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$v/trace -o run --output-format csv -- $B --secondary-out $OUT/$v/sec.json > $OUT/$v/trace.log 2>&1 || { echo TRACE_FAIL $v; tail -5 $OUT/$v/trace.log; exit 1; }
  CORDA_AMD_LIB=$L timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d $OUT/$v/pmc -o run --output-format csv -- $B > $OUT/$v/pmc.log 2>&1 || { echo PMC_FAIL $v; exit 1; }
  echo done $v
done
echo AB_TX_DONE
