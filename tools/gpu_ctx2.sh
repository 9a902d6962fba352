#!/bin/bash
# Round 6: device-form steps over two contexts on one GPU (a call's key-table phase beside the previous
# call's ladders) vs one; interleaved, 3 rounds; plus side streams on dedicated queues for two contexts.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_cfg.sh ctx2 3 "c1||--h2h-steps 0" "c2||--h2h-steps 0 --contexts 2" "c2m|CG_MASKED_SIDE_STREAMS=1|--h2h-steps 0 --contexts 2" || exit 1
echo CTX2_DONE
