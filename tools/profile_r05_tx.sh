#!/bin/bash
# Counter passes over the configs[3] transaction pipeline (1M WireTransactions) for k_tx_leaves'
# traffic: L2 hit / miss, the memory-side read requests by size (128-B
# "bubble", 64-B, 32-B: the exact EA read bytes, where FETCH_SIZE counts every request as 64 B)
# and the requests destined for DRAM. Each pass its own process and time limit.
# usage: bash tools/profile_r05_tx.sh <outdir>
set -o pipefail
export TMPDIR=/tmp
OUT=${1:-gpurun_out/prof_tx5}
mkdir -p $OUT
B="python3 bench.py --steps 1 --warmup 1 --items 262144 --pool 65536 --no-cpu-baseline --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --tear-offs 0 --configs0-txs 0 --secondary-out $OUT/sec.json"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || { echo TRACE_FAIL; tail -20 $OUT/trace.log; exit 1; }
i=0
for P in "TCC_HIT_sum TCC_MISS_sum" "TCC_BUBBLE_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" "TCC_EA0_RDREQ_DRAM_sum WRITE_SIZE" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P -d $OUT/pmc$i -o run --output-format csv -- $B > $OUT/pmc$i.log 2>&1 || { echo PMC_FAIL $i; tail -5 $OUT/pmc$i.log; exit 1; }
done
echo PROFILE_TX5_DONE
