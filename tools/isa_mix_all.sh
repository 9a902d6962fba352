#!/bin/bash
# Hottest-loop VALU mixes of the priced item kernels (tools/isa_mix.py) in one file, the input of
# tools/pmc_traffic.py.  usage: bash tools/isa_mix_all.sh profiles/r02/isa_mix_<version>.json
set -eo pipefail
DEST=$1
T=$(mktemp -d)
cd "$(dirname "$0")/.."
F="-O3 -std=c++17 --offload-arch=gfx950 --cuda-device-only -S -Icorda_amd/csrc -Iinclude"
/opt/rocm/bin/hipcc $F corda_amd/csrc/verify_ed.hip -o $T/ed.s
/opt/rocm/bin/hipcc $F corda_amd/csrc/verify_ec.hip -o $T/ec.s
python3 - "$T" "$DEST" <<'EOF'
import json, subprocess, sys
t, dest = sys.argv[1], sys.argv[2]
# kernel (pmc_traffic.py name) -> (assembly, mangled symbol prefix); curve 0 = secp256k1, 1 = secp256r1
K = {"k_ed_ladder_wide": ("ed", "_ZN2cg16k_ed_ladder_wide"), "k_ed_ladder_pf": ("ed", "_ZN2cg14k_ed_ladder_pf"),
     "k_ed_hash": ("ed", "_ZN2cg9k_ed_hash"), "k_ed_finish": ("ed", "_ZN2cg11k_ed_finish"),
     "k_ec_ladder_wide<1>": ("ec", "_ZN2cg16k_ec_ladder_wideILi1E"), "k_ec_ladder_wide<0>": ("ec", "_ZN2cg16k_ec_ladder_wideILi0E"),
     "k_ec_prep<1>": ("ec", "_ZN2cg9k_ec_prepILi1E"), "k_ec_prep<0>": ("ec", "_ZN2cg9k_ec_prepILi0E"),
     "k_ec_inv<1>": ("ec", "_ZN2cg8k_ec_invILi1E"), "k_ec_inv<0>": ("ec", "_ZN2cg8k_ec_invILi0E")}
out = {}
for name, (f, sym) in K.items():
    r = subprocess.run([sys.executable, "tools/isa_mix.py", f"{t}/{f}.s", sym], capture_output=True, text=True, check=True)
    out[name] = json.loads(r.stdout)["loop"]
json.dump(out, open(dest, "w"), indent=1)
print({k: round(v["mean_ns_per_wave_instr"], 4) for k, v in out.items()})
EOF
rm -rf $T
