set -o pipefail
OUT=gpurun_out/ab_stream; mkdir -p $OUT
B="python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --host-steps 0 --configs1-items 0 --ecdsa-items 0 --pipeline-txs 0 --tear-offs 0 --configs0-txs 0"
for r in 1 2; do for s in ctx torch; do
  timeout -k 10 200 $B --stream $s > $OUT/${s}_$r.log 2>&1 || exit 1
  echo "$s $r $(grep -o '"value": [0-9.]*' $OUT/${s}_$r.log | head -1)"
done; done
