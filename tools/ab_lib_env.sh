#!/bin/bash
# Headline-only bench for every (library, environment) pair, two rounds.
# usage: bash tools/ab_lib_env.sh <tag> "<lib1.so|base> ..." "<NAME=VALUE[+...]|-> ..."
set -o pipefail
export TMPDIR=/tmp
TAG=$1; LIBS=$2; ENVS=$3
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B="python3 -u bench.py --steps 5 --warmup 2 --device-steps 0 --host-steps 0 --key-dists= --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0 --no-cpu-baseline"
for r in 1 2; do
  for lib in $LIBS; do
    for kv in $ENVS; do
      n=$(basename $lib .so)_$(echo "$kv" | tr '=+' '__')_$r
      L=""; [ "$lib" != base ] && L=$lib
      E=""; [ "$kv" != - ] && E=$(echo "$kv" | tr '+' ' ')
      env CORDA_AMD_LIB=$L $E timeout -k 10 300 $B --secondary-out $OUT/${n}_sec.json > $OUT/$n.log 2> $OUT/$n.err || { echo FAIL $n; tail -5 $OUT/$n.err; exit 1; }
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=json.load(open(sys.argv[2]))['headline_h2d']['cg_stats_ms_mean']; print(sys.argv[3], d['value'], d['ms_per_step'], s)" $OUT/$n.log $OUT/${n}_sec.json $n
    done
  done
done
echo AB_DONE
