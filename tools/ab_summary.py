"""Summarise tools/ab.sh logs: headline value, ms/step and item-kernel ms per run."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f"{f}: {d['value'] / 1e6:.1f} M sigs/s, {d['ms_per_step']} ms/step, kernels {d['roofline']['kernel_ms']} ms, frac {d['roofline']['frac']}")
