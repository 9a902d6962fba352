#!/bin/bash
# A/B of bench-argument variants on one GPU box (same library): the headline bench without the
# secondaries, interleaved, two rounds.  usage: bash tools/ab_args.sh out_tag "--chunk-items 0" ["ARGS" ...]
# ("-" = no extra arguments)
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/ab_$TAG
mkdir -p $OUT
B="python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --host-steps 0 --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0"
for round in 1 2; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    [ "$v" = "-" ] && v=""
    timeout -k 10 200 $B $v > $OUT/v${i}_$round.log 2>&1 || exit 1
    echo "v$i ($v) round $round: $(grep -o '"value": [0-9.]*' $OUT/v${i}_$round.log | head -1) $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print({k: v['ms_per_step'] for k, v in d['secondary']['stages'].items() if v['ms_per_step'] > 0.2})" $OUT/v${i}_$round.log)"
  done
done
