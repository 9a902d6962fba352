"""VALU instruction mix of a kernel's hottest loop from its gfx950 assembly, priced with the measured
per-instruction chip rates (profiles/r04/ubench/, round 1's in profiles/r01/ubench_int.json), to turn rocprof's SQ_INSTS_VALU count into
an issue-time estimate that does not assume every wave64 VALU op costs the same (VERDICT r1:
"replace the 4-cycle issue_frac with per-opcode costs").

The hottest loop = the backward branch enclosing the most VALU instructions (for k_ed_ladder_pf the
69-op mixed-addition loop; for k_ec_ladder the digit loop). Costs are nanoseconds of one SIMD per
wave64 instruction, 64 lanes x 1024 SIMDs / chip lane-rate: measured for v_mad_u64_u32, v_add_u32,
v_add_co/addc, v_mul_lo/hi, v_lshl_add, v_alignbit, v_lshlrev_b64; other VOP1/VOP2 ops (32-bit
encoding: and/or/xor/shifts/mov/cndmask) are priced as v_add_u32, other VOP3 ops as v_lshl_add.

usage: python tools/isa_mix.py <file.s> <kernel symbol prefix>   (build the .s with
       hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S corda_amd/csrc/verify_ed.hip)
"""
import collections
import json
import re
import sys

SIMD_NS = lambda rate: 64 * 1024 / rate * 1e9  # noqa: E731
# round 4 (profiles/r04/ubench/ubench_peak_summary.json: 16 chains, 8 waves per SIMD); addc and
# mul_hi priced as their measured siblings
RATES = {"v_mad_u64_u32": 3.6412e13, "v_add_u32": 5.3575e13, "v_add_co_u32": 3.7041e13,
         "v_addc_co_u32": 3.7041e13, "v_mul_lo_u32": 3.4681e13, "v_mul_hi_u32": 3.4681e13,
         "v_lshl_add_u32": 3.6414e13, "v_alignbit_b32": 3.3392e13, "v_lshlrev_b64": 3.6807e13}
FAST_VOP = SIMD_NS(RATES["v_add_u32"])
SLOW_VOP3 = SIMD_NS(RATES["v_lshl_add_u32"])


def cost_ns(op, vop3):
    if op in RATES:
        return SIMD_NS(RATES[op])
    if op.startswith(("v_sub_co", "v_subb_co", "v_subrev_co", "v_add_co", "v_addc")):
        return SIMD_NS(RATES["v_add_co_u32"])
    if op.startswith(("v_mad_u64", "v_mad_i64")):
        return SIMD_NS(RATES["v_mad_u64_u32"])
    if op.startswith(("v_mul_hi", "v_mul_lo")):
        return SIMD_NS(RATES["v_mul_lo_u32"])
    if op.endswith("_b64") or op.endswith("_u64"):
        return SIMD_NS(RATES["v_lshlrev_b64"])
    return SLOW_VOP3 if vop3 else FAST_VOP


def kernel_lines(lines, prefix):
    start = next(i for i, l in enumerate(lines) if re.match(rf"^{re.escape(prefix)}\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    return lines[start:end]


def hottest_loop(body):
    labels = {m.group(1): i for i, l in enumerate(body) for m in [re.match(r"^(\.LBB\w+):", l)] if m}
    best = None
    for i, l in enumerate(body):
        m = re.match(r"^\s+s_(?:cbranch_\w+|branch)\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] < i:
            a = labels[m.group(1)]
            n = sum(1 for x in body[a:i] if re.match(r"^\s+v_", x))
            if best is None or n > best[0]:
                best = (n, a, i)
    return body[best[1]:best[2]] if best else body


def mix(body):
    ops = collections.Counter()
    ns = 0.0
    for l in body:
        m = re.match(r"^\s+(v_\w+)(_e64)?\s", l + " ")
        if not m or m.group(1).startswith(("v_readfirstlane", "v_readlane", "v_writelane")):
            continue
        op = m.group(1)
        # the assembler prints VOP3-only forms without _e64; 3-source or 64-bit-result ops are VOP3
        vop3 = bool(m.group(2)) or op in ("v_cndmask_b32",) and l.count(",") >= 3 or l.count(",") >= 3
        ops[op] += 1
        ns += cost_ns(op, vop3)
    n = sum(ops.values())
    return {"valu_static": n, "mean_ns_per_wave_instr": round(ns / max(n, 1), 4),
            "v_mad_u64_u32_frac": round(ops["v_mad_u64_u32"] / max(n, 1), 4),
            "top": dict(ops.most_common(12))}


def main():
    lines = open(sys.argv[1]).read().splitlines()
    body = kernel_lines(lines, sys.argv[2])
    out = {"kernel": sys.argv[2], "loop": mix(hottest_loop(body)), "whole_kernel": mix(body)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
