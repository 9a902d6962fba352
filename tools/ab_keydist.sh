#!/bin/bash
# Key-distribution legs (tools/keydist_probe.py) with the in-tree library and each variant .so,
# interleaved, two rounds.  usage: bash tools/ab_keydist.sh <tag> <dists> variantB.so [...]
#   dists: comma list of distinct,zipf
set -o pipefail
export TMPDIR=/tmp
TAG=$1; DISTS=$2; shift 2
OUT=gpurun_out/abkd_$TAG
mkdir -p $OUT
for r in 1 2; do
  for v in base "$@"; do
    n=$(basename $v .so)
    for d in ${DISTS//,/ }; do
      L=""; [ $v != base ] && L=$v
      CORDA_AMD_LIB=$L timeout -k 10 200 python3 tools/keydist_probe.py $d 2 > $OUT/${n}_${d}_$r.json 2> $OUT/${n}_${d}_$r.err || { echo FAIL $v $d; tail -5 $OUT/${n}_${d}_$r.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_call'], {k: v for k, v in d.get('table_modes_items', {}).items() if k != 'max_uses'})" $OUT/${n}_${d}_$r.json "$n $d $r"
    done
  done
done
echo ABKD_DONE
