#!/bin/bash
# Round 6, device-resident headline: the context's stream at the device's highest priority
# (CG_STREAM_PRIORITY=1) against the default; interleaved, 3 rounds.
set -o pipefail
export TMPDIR=/tmp
bash tools/ab_cfg.sh sprio 3 "def||--h2h-steps 0 --ctx2-steps 0" "prio|CG_STREAM_PRIORITY=1|--h2h-steps 0 --ctx2-steps 0" || exit 1
echo SPRIO_DONE
