#!/bin/bash
# Round 6, host form (host arena -> host verdicts): the library's default chunking (a 1/6 first chunk,
# then 4) against 3 and 4 chunks in all (cg_config.chunk_items); interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_cfg.sh h2hchunks 3 "c5||--headline host --ctx2-steps 0" "c3||--headline host --ctx2-steps 0 --chunk-items 6250000" "c4||--headline host --ctx2-steps 0 --chunk-items 4200000" || exit 1
echo H2H_CHUNKS_DONE
