"""Per-launch HBM traffic and VALU issue of the item kernels from rocprofv3 passes
(tools/profile_r02.sh: --kernel-trace --stats, then --pmc FETCH_SIZE, --pmc WRITE_SIZE and an SQ pass,
each its own process), written to profiles/r04/pmc_traffic.json (PMC_TRAFFIC_FILE) for bench.py's roofline.

HBM bytes (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE = TCC_EA0_RDREQ x 64 B, so a
wide streaming read (128-B requests) reports half its bytes while a table gather (64-B requests)
may report them exactly or at half (profiles/r05/calib: fetch_calib's stream, 112-B-entry gathers
and 16-B gathers against their known byte counts). Round 5: with the read-requests-by-size pass
(tcc/: TCC_EA0_RDREQ_32B / _64B / _128B, and _DRAM) each request is priced at its own size,
hbm = 32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B + WRITE_SIZE (TCC_BUBBLE, documented as the
128-B requests, reads 0 on gfx950); without it, round 4's upper estimate 2 FETCH_SIZE + WRITE_SIZE.

VALU issue: SQ_INSTS_VALU wave-instructions of the kernel priced per opcode (tools/isa_mix.py: the
hottest loop's static instruction mix x the measured chip rate of each opcode,
profiles/r01/ubench_int.json) and spread over the 1024 SIMDs, against the kernel's own duration in
the counter pass. ``issue_frac_4cyc`` keeps round 1's flat 4-cycles-per-op figure for comparison.

usage: pmc_traffic.py <prof_dir> <kernel_version> <items> <dest_profile_dir> [isa_mix.json]
"""
import collections
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = ("k_ed_hash", "k_ed_hash<true>", "k_ed_hash<false>", "k_ec_prep<1, true>", "k_ec_prep<0, true>",
           "k_ec_prep<1, false>", "k_ec_prep<0, false>", "k_ed_ladder_pf", "k_ed_ladder_wide", "k_ed_finish", "k_ec_prep<1>", "k_ec_inv<1>",
           "k_ec_ladder<1, true>", "k_ec_ladder_wide<1>", "k_ec_prep<0>", "k_ec_inv<0>", "k_ec_ladder<0, true>",
           "k_ec_ladder_wide<0>", "k_ed_wide_fwd", "k_ed_wide_inv", "k_ed_wide_bwd", "k_ec_wide_fwd<1>",
           "k_ec_wide_bwd<1>", "k_ec_wide_fwd<0>", "k_ec_wide_bwd<0>", "k_ec_wide_inv<1>", "k_ec_wide_inv<0>",
           # configs[3] transaction pipeline (tools/profile_tx.sh)
           "k_tx_map", "k_tx_leaf_count", "k_tx_leaf_scatter", "k_tx_leaves", "k_tx_roots", "k_txsig_items", "k_splice")


def short(name):
    return name.split("(")[0].replace("void ", "").replace("cg::", "")


def first_n():
    """PMC_FIRST_N=N keeps each kernel's first N dispatches: the headline leg runs first in bench.py
    (warmup + steps calls x chunks), so the averages are the headline's launches only, not a mix with
    the secondary legs' (device-resident, key-distribution) launches of other sizes."""
    n = int(os.environ.get("PMC_FIRST_N", "0"))
    return n if n > 0 else None


def per_launch(path, counter_names):
    rows = collections.defaultdict(lambda: collections.defaultdict(dict))
    for r in csv.DictReader(open(path)):
        n = short(r["Kernel_Name"])
        if n not in KERNELS or r["Counter_Name"] not in counter_names:
            continue
        d = rows[n][int(r["Dispatch_Id"])]
        d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        d["ms"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6
    out = {}
    for n, by_id in rows.items():
        ds = [by_id[i] for i in sorted(by_id)][:first_n()]
        out[n] = {k: sum(d.get(k, 0.0) for d in ds) / len(ds) for k in list(counter_names) + ["ms"]}
        out[n]["launches"] = len(ds)
    return out


def trace_stats(path):
    out = {}
    tpath = path.replace("run_kernel_stats.csv", "run_kernel_trace.csv")
    if first_n() and os.path.exists(tpath):  # the headline's launches only (see first_n)
        by = collections.defaultdict(list)
        for r in csv.DictReader(open(tpath)):
            n = short(r["Kernel_Name"])
            if n in KERNELS:
                by[n].append((int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-6))
        for n, v in by.items():
            d = [x[1] for x in sorted(v)][:first_n()]
            out[n] = {"calls": len(d), "avg_ms": sum(d) / len(d), "min_ms": min(d), "max_ms": max(d)}
        return out
    for r in csv.DictReader(open(path)):
        n = short(r["Name"])
        if n in KERNELS:
            out[n] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) * 1e-6,
                      "min_ms": float(r["MinNs"]) * 1e-6, "max_ms": float(r["MaxNs"]) * 1e-6}
    return out


def main():
    prof, version, items, dest = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
    mixes = json.load(open(sys.argv[5])) if len(sys.argv) > 5 else {}
    fetch = per_launch(os.path.join(prof, "fetch", "run_counter_collection.csv"), ["FETCH_SIZE"])
    write = per_launch(os.path.join(prof, "write", "run_counter_collection.csv"), ["WRITE_SIZE"])
    sq_names = ["SQ_INSTS_VALU", "SQ_WAVE_CYCLES", "SQ_WAIT_INST_ANY", "GRBM_GUI_ACTIVE", "SQ_WAVES",
                "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_INT64"]
    vpath = os.path.join(prof, "valu", "run_counter_collection.csv")
    valu = per_launch(vpath, sq_names) if os.path.exists(vpath) else {}
    trio = ["TCC_EA0_RDREQ_32B_sum", "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_DRAM_sum"]
    tpath = os.path.join(prof, "tcc", "run_counter_collection.csv")
    tcc = per_launch(tpath, trio) if os.path.exists(tpath) else {}
    trace = trace_stats(os.path.join(prof, "trace", "run_kernel_stats.csv"))
    os.makedirs(dest, exist_ok=True)
    for src, dst in (("trace/run_kernel_stats.csv", "kernel_stats.csv"),
                     ("fetch/run_counter_collection.csv", "pmc_fetch_size.csv"),
                     ("write/run_counter_collection.csv", "pmc_write_size.csv"),
                     ("valu/run_counter_collection.csv", "pmc_valu.csv"),
                     ("tcc/run_counter_collection.csv", "pmc_tcc_trio.csv")):
        if os.path.exists(os.path.join(prof, src)):
            shutil.copy(os.path.join(prof, src), os.path.join(dest, dst))
    kern = {}
    for n in KERNELS:
        k = {}
        if n in trace:
            k["trace"] = trace[n]
        if n in fetch and n in write:
            k["fetch_kb"] = round(fetch[n]["FETCH_SIZE"], 1)
            k["write_kb"] = round(write[n]["WRITE_SIZE"], 1)
            k["hbm_bytes_2x_fetch"] = int(round((2 * fetch[n]["FETCH_SIZE"] + write[n]["WRITE_SIZE"]) * 1024))
            k["hbm_bytes_per_launch"] = k["hbm_bytes_2x_fetch"]
            if n in tcc:
                t = tcc[n]
                r32, r64, r128 = t["TCC_EA0_RDREQ_32B_sum"], t["TCC_EA0_RDREQ_64B_sum"], t["TCC_EA0_RDREQ_128B_sum"]
                k["read_requests"] = {"32b": r32, "64b": r64, "128b": r128, "dram": t["TCC_EA0_RDREQ_DRAM_sum"]}
                k["read_bytes_trio"] = int(round(32 * r32 + 64 * r64 + 128 * r128))
                k["hbm_bytes_per_launch"] = int(round(k["read_bytes_trio"] + write[n]["WRITE_SIZE"] * 1024))
        if n in valu:
            v = valu[n]
            clk = v["GRBM_GUI_ACTIVE"] / 8
            # a launch under 0.1 ms is shorter than the counters' sampling of GRBM_GUI_ACTIVE resolves
            # (round 5 derived 7.5 GHz for a 0.03-ms launch): no clock and no issue fraction for it
            short = v["ms"] < 0.1
            k["valu"] = {"insts_per_launch": v["SQ_INSTS_VALU"], "ms_in_counter_pass": round(v["ms"], 3),
                         "clock_GHz": None if short else round(clk / (v["ms"] * 1e6), 3),
                         "issue_frac_4cyc": None if short else round(v["SQ_INSTS_VALU"] * 4 / (1024 * clk), 3),
                         "wait_frac": round(v["SQ_WAIT_INST_ANY"] / v["SQ_WAVE_CYCLES"], 3)}
            if short:
                k["valu"]["note"] = "launch < 0.1 ms: derived clock and issue fraction suppressed"
            if "SQ_INSTS_VALU_INT64" in v:
                k["valu"]["int64_frac"] = round(v["SQ_INSTS_VALU_INT64"] / v["SQ_INSTS_VALU"], 3)
                k["valu"]["int32_frac"] = round(v["SQ_INSTS_VALU_INT32"] / v["SQ_INSTS_VALU"], 3)
            mix = mixes.get(n) or mixes.get(n.replace(", true>", ">").replace(", false>", ">").replace("<true>", "")
                                            .replace("<false>", ""))
            if mix:
                t = v["SQ_INSTS_VALU"] / 1024 * mix["mean_ns_per_wave_instr"] * 1e-6
                k["valu"]["issue_ms_per_opcode_model"] = round(t, 3)
                k["valu"]["issue_frac"] = None if v["ms"] < 0.1 else round(t / v["ms"], 3)
                k["valu"]["mix"] = mix
        if k:
            kern[n] = k
    rel = os.path.relpath(dest, ROOT)
    out = {"items": items, "kernel_version": version,
           "source": f"{rel}/ (rocprofv3 --kernel-trace --stats; --pmc FETCH_SIZE; --pmc WRITE_SIZE; SQ pass; "
                     "separate processes, bench.py --steps 3 on the headline workload)",
           "launches_kept": f"first {first_n()} dispatches per kernel (the headline leg)" if first_n() else "all",
           "correction": ("hbm = 32 TCC_EA0_RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B + WRITE_SIZE (each memory-side "
                          "read request at its size; gfx950 FETCH_SIZE = RDREQ x 64 B), checked on "
                          "tools/microbench/fetch_calib (profiles/r05/calib)" if tcc else
                          "hbm = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE counts 128-B requests at 64 B); upper "
                          "estimate for table gathers"),
           "kernels": kern,
           "hbm_bytes_per_launch": {n: k["hbm_bytes_per_launch"] for n, k in kern.items() if "hbm_bytes_per_launch" in k},
           "valu_issue": {n: k["valu"] for n, k in kern.items() if "valu" in k}}
    with open(os.path.join(dest, "pmc_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    if os.environ.get("PMC_TRAFFIC_HEADLINE", "1") == "1":  # the file bench.py's roofline reads (TRAFFIC_FILE)
        head = os.path.join(ROOT, os.environ.get("PMC_TRAFFIC_FILE", "profiles/r06/pmc_traffic.json"))
        os.makedirs(os.path.dirname(head), exist_ok=True)
        with open(head, "w") as f:
            json.dump(out, f, indent=1)
    print(json.dumps({n: (k.get("hbm_bytes_per_launch"), k.get("valu", {}).get("issue_frac"),
                          k.get("trace", {}).get("avg_ms")) for n, k in kern.items()}))


if __name__ == "__main__":
    main()
