#!/bin/bash
# Phase-1 markers (CG_HOST_TRACE: chunk 0's front done, every table built, first copies landed) and
# the step time for every (library, environment) pair, R rounds interleaved.
# usage: bash tools/ab_phase1.sh <tag> <rounds> "<lib.so|base> ..." "<NAME=VALUE[+...]|-> ..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; R=$2; LIBS=$3; ENVS=$4
OUT=gpurun_out/p1_$TAG
mkdir -p $OUT
B="python3 -u bench.py --steps 5 --warmup 2 --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 --no-cpu-baseline"
for r in $(seq 1 $R); do
  for lib in $LIBS; do
    for kv in $ENVS; do
      n=$(basename $lib .so)_$(echo "$kv" | tr '=+' '__')_$r
      L=""; [ "$lib" != base ] && L=$lib
      E=""; [ "$kv" != - ] && E=$(echo "$kv" | tr '+' ' ')
      env CG_HOST_TRACE=1 CORDA_AMD_LIB=$L $E timeout -k 10 300 $B --secondary-out $OUT/${n}_sec.json > $OUT/$n.log 2> $OUT/$n.err || { echo FAIL $n; tail -5 $OUT/$n.err; exit 1; }
      python3 - $OUT/$n.log $OUT/$n.err $n <<'PY'
import json, re, statistics, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
f0, tb = [], []
for l in open(sys.argv[2]):
    m = re.search(r"chunk 0 front done ([\d.]+), tables built ([\d.]+)", l)
    if m:
        f0.append(float(m.group(1))); tb.append(float(m.group(2)))
print(sys.argv[3], d["value"], d["ms_per_step"], "front0", round(statistics.median(f0[-5:]), 2), "tables", round(statistics.median(tb[-5:]), 2))
PY
    done
  done
done
echo P1_DONE
