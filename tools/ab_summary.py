"""Summarise tools/ab.sh logs: headline value, ms/step and the per-stage ms per step of each run."""
import json
import sys

for f in sys.argv[1:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = {k: v["ms_per_step"] for k, v in d.get("secondary", {}).get("stages", {}).items() if v["ms_per_step"] > 0.2}
    print(f"{f}: {d['value'] / 1e6:.1f} M sigs/s, {d['ms_per_step']} ms/step, frac {d['roofline']['frac']}, {st}")
