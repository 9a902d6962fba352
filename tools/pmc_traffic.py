"""Per-launch HBM traffic of the Ed25519 item kernels from two rocprofv3 PMC passes
(tools/profile_r01.sh: --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate runs), written to
profiles/r01/pmc_traffic.json for bench.py's roofline.traffic.

gfx950 correction (MI355X_MICROARCH.md, HBM section): FETCH_SIZE tallies 128-B requests at 64 B,
so a wide streaming read reports half its bytes; hbm = 2*FETCH_SIZE + WRITE_SIZE (KB * 1024).
The doubling is calibrated for streaming reads, not 16-B table gathers, so the figure is an
upper estimate.

usage: pmc_traffic.py <prof_dir> <kernel_version> <items> <dest_profile_dir>
"""
import collections
import csv
import json
import os
import shutil
import sys

KERNELS = ("cg::k_ed_hash", "cg::k_ed_ladder", "cg::k_ed_finish")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def per_kernel_kb(path):
    """Average KB per launch of each kernel; the two table modes' ladders (k_ed_ladder_pf for
    full-table keys, k_ed_ladder<false> for row-0 keys, both launched every step) are summed
    under k_ed_ladder."""
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        full = r["Kernel_Name"].split("(")[0].replace("void ", "")
        name = full.split("<")[0]
        if name.startswith("cg::k_ed_ladder"):  # k_ed_ladder_pf (full tables) + k_ed_ladder<false>
            name = "cg::k_ed_ladder"
        if name in KERNELS:
            acc[(name, full)].append(float(r["Counter_Value"]))
    out = collections.defaultdict(float)
    for (name, _), v in acc.items():
        out[name] += sum(v) / len(v)
    return dict(out)


def valu_issue(path, items):
    """VALU issue occupancy of the Ed25519 item kernels from the SQ pass (tools/profile_r01.sh):
    VALU wave-instructions x 4 cycles (a wave64 VALU op holds a SIMD16 for 4 cycles) over the
    SIMD-cycles the kernel ran (GRBM_GUI_ACTIVE is summed over the 8 XCDs; 1024 SIMDs). ~1.0
    means the kernel is bound by instruction issue, whatever its MAC fraction."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        if name.startswith(("cg::k_ed_ladder_pf", "cg::k_ed_hash", "cg::k_ed_finish")):
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for name, cs in acc.items():
        m = {k: sum(v) / len(v) for k, v in cs.items()}
        clk = m["GRBM_GUI_ACTIVE"] / 8
        out[name.split("::")[1]] = {
            "valu_insts_per_item": round(m["SQ_INSTS_VALU"] * 64 / items, 1),
            "xcd_cycles": round(clk),
            "issue_frac": round(m["SQ_INSTS_VALU"] * 4 / (1024 * clk), 3),
            "wait_frac": round(m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"], 3)}
    return out


def main():
    prof, version, items, dest = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    fetch = per_kernel_kb(os.path.join(prof, "fetch", "run_counter_collection.csv"))
    write = per_kernel_kb(os.path.join(prof, "write", "run_counter_collection.csv"))
    assert set(fetch) == set(KERNELS) and set(write) == set(KERNELS), (fetch, write)
    hbm = int(round((2 * sum(fetch.values()) + sum(write.values())) * 1024))
    os.makedirs(dest, exist_ok=True)
    for src, dst in (("trace/run_kernel_stats.csv", "kernel_stats.csv"),
                     ("fetch/run_counter_collection.csv", "pmc_fetch_size.csv"),
                     ("write/run_counter_collection.csv", "pmc_write_size.csv"),
                     ("valu/run_counter_collection.csv", "pmc_valu.csv")):
        if os.path.exists(os.path.join(prof, src)):
            shutil.copy(os.path.join(prof, src), os.path.join(dest, dst))
    rel = os.path.relpath(dest, ROOT)
    out = {"items": items, "kernel": " + ".join(k.split("::")[1] for k in KERNELS),
           "source": f"{rel}/pmc_fetch_size.csv, pmc_write_size.csv (rocprofv3 --pmc FETCH_SIZE / "
                     "WRITE_SIZE, separate passes, bench.py --steps 3)",
           "fetch_size_kb": fetch, "write_size_kb": write,
           "correction": "gfx950 FETCH_SIZE reads half the bytes of wide streaming reads "
                         "(MI355X_MICROARCH.md HBM): hbm = 2*FETCH_SIZE + WRITE_SIZE (KB*1024); "
                         "uncalibrated for 16-B table gathers, so an upper estimate",
           "hbm_bytes_per_launch": hbm, "kernel_version": version}
    vpath = os.path.join(prof, "valu", "run_counter_collection.csv")
    if os.path.exists(vpath):
        out["valu_issue"] = valu_issue(vpath, items)
    with open(os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
