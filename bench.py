#!/usr/bin/env python3
"""Headline benchmark: verified signatures / second for the whole node (BASELINE.json).

Workload (BASELINE.json configs[1]): per GPU, a batch of
2^20 Ed25519 (EDDSA_ED25519_SHA512) signatures over 4096 keys and 270-byte
SignableData-sized messages, 12% corrupted across Appendix A classes A1-A7, seeded
synthetic data (no network, no JVM). One step = one full pass of the hot path over the
batch with every input already resident in HBM: key prep (decode + tables for every key)
-> verify every item -> status bytes in HBM, plus (N > 1) the RCCL all-gather of the
per-GPU verdict vectors, the engine's only collective.

Launch: ``python bench.py`` (N = 1) or ``torchrun --nproc-per-node N bench.py --gpus N``;
one process per GPU, each verifying its own shard (weak scaling). Rank 0 prints ONE JSON
line. ``roofline`` prices the dominant kernel (k_ed_verify) in 32x32->64 multiply-
accumulates against the measured v_mad_u64_u32 peak (profiles/r01/ubench_int.json);
``cpu_baseline`` is the C restatement of the reference's algorithms (oracle/c, "port")
timed on a bounded sample on the host cores (rank 0, N = 1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "verified sigs/sec (whole node), Ed25519 + ECDSA-P256, at 1/2/4/8 MI355X"
# Reference-algorithm work per Ed25519 verify, frozen from the C restatement of i2p 0.2.0
# (oracle/c/ed25519_i2p.c counters): 1601 field multiplies + 1258
# squarings per engineVerify (key decode excluded), each priced at 64 MAC32. Reported as
# `i2p_equiv`: the rate at which the GPU retires the reference's own work.
N_FE_ED25519 = 2859
MAC32_PER_ED25519 = N_FE_ED25519 * 64
# Executed work of the GPU path per Ed25519 item, counted by the host build of the same lane
# code (tests/native/host_kernels.cpp t_ed_verify_wb / t_ed_count_w6; pinned by
# tests/test_host_kernels.py::test_executed_work_constants_match_lane_code).
# (field multiplies, field squarings):
ED_VERIFY_FE = (500, 24)   # k_ed_ladder: 43 + 26 mixed additions (-A rows W=6 in 2 windows, radix-2^10 B) + 6 doublings
ED_FINISH_FE = (5, 0)      # k_ed_finish: prefix product, unwinding, encode
ED_INVERT_FE = (11, 254)   # one fe_invert, shared by ED_FINISH_K items
ED_FINISH_K = 16
# 32x32->64 products per operation in the radix-2^25.5 representation (fe25519.h)
MAC_PER_MUL, MAC_PER_SQ = 100, 55
MAC32_EXEC_PER_ED25519 = ((ED_VERIFY_FE[0] + ED_FINISH_FE[0]) * MAC_PER_MUL +
                          (ED_VERIFY_FE[1] + ED_FINISH_FE[1]) * MAC_PER_SQ +
                          (ED_INVERT_FE[0] * MAC_PER_MUL + ED_INVERT_FE[1] * MAC_PER_SQ) / ED_FINISH_K)
# v_mad_u64_u32 chip throughput measured on MI355X (profiles/r01/ubench_int.json)
PEAK_MAC32_PER_S = 2.7944e13
# kernel generation whose PMC traffic profile is committed (profiles/r01/pmc_traffic.json)
KERNEL_VERSION = "ed25519_v12"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--items", type=int, default=1 << 20, help="items per GPU")
    ap.add_argument("--keys", type=int, default=4096)
    ap.add_argument("--msg-len", type=int, default=270)
    ap.add_argument("--corrupt-permille", type=int, default=120)
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU work for the baseline sample")
    ap.add_argument("--threads", type=int, default=0, help="host threads for data generation / CPU baseline")
    ap.add_argument("--ecdsa-items", type=int, default=1 << 18,
                    help="items of the secondary ECDSA measurement (N = 1 only; 0 disables)")
    ap.add_argument("--pipeline-txs", type=int, default=1 << 18,
                    help="WireTransactions of the secondary config-4 pipeline measurement (N = 1 only; 0 disables)")
    ap.add_argument("--tear-offs", type=int, default=1 << 18, help="FilteredTransaction.verify secondary (0: off)")
    ap.add_argument("--host-buffers", type=int, default=1, help="PCIe-inclusive cg_verify_batch secondary (0: off)")
    ap.add_argument("--mixed-items", type=int, default=1 << 20,
                    help="items of the secondary config-5-shaped mixed batch (N = 1 only; 0 disables)")
    return ap.parse_args()


def host_threads(req):
    if req > 0:
        return req
    env = os.environ.get("OMP_NUM_THREADS")
    n = int(env) if env and env.isdigit() else 16
    return max(1, min(n, os.cpu_count() or 1, 16))


def cpu_baseline(batch, seconds, threads):
    """oracle/c (C restatement of i2p 0.2.0 / BC 1.57 semantics) on a bounded sample."""
    from corda_amd.batch import Batch
    from oracle import c_oracle
    probe = min(batch.n, 256 * threads)
    sub = Batch(batch.keys, batch.items[:probe], batch.arena)
    t = time.perf_counter()
    c_oracle.verify_batch(sub, 0, threads)
    dt = time.perf_counter() - t
    n = int(min(batch.n, max(probe, probe * seconds / max(dt, 1e-6))))
    sub = Batch(batch.keys, batch.items[:n], batch.arena)
    t = time.perf_counter()
    st = c_oracle.verify_batch(sub, 0, threads)
    dt = time.perf_counter() - t
    return {"value": round(n / dt, 1), "unit": "sigs/s", "cores": threads, "kind": "port",
            "sample": f"first {n} items of the rank-0 batch (incl. key decode for all {len(batch.keys)} keys), "
                      f"oracle/c or_verify_batch over {threads} threads, {dt:.1f} s; JVM reference "
                      f"unavailable (no JDK / i2p / BouncyCastle jars on the box)"}, st


def bench_mixed(a, wl, eng, dev, stream, run, threads):
    """BASELINE configs[4] shape on one GPU: 70% Ed25519 / 20% secp256r1 / 10% secp256k1,
    shuffled, no deduplication (ECDSA items are tiled from 65 536-item pools)."""
    import torch
    n = a.mixed_items
    ne, nr = int(n * 0.7), int(n * 0.2)
    nk = n - ne - nr
    e, _ = wl.ed25519_batch(ne, n_keys=a.keys, msg_len=a.msg_len, corrupt_permille=a.corrupt_permille,
                            seed=a.seed + 101, nthreads=threads)
    parts = [e]
    for curve, cnt in ((1, nr), (0, nk)):
        pool, _ = wl.ecdsa_batch(curve, min(cnt, 65536), n_keys=1024, msg_len=a.msg_len, corrupt_permille=100,
                                 seed=a.seed + 103 + curve, nthreads=threads)
        pool.items = np.resize(pool.items, cnt)
        parts.append(pool)
    b, _ = wl.concat(parts, shuffle_seed=a.seed + 107)
    kd = torch.from_numpy(b.keys.view(np.uint8)).to(dev)
    idd = torch.from_numpy(b.items.view(np.uint8)).to(dev)
    ad = torch.from_numpy(b.arena).to(dev)
    sd = torch.full((b.n,), 255, dtype=torch.uint8, device=dev)
    steps = max(2, a.steps // 2)
    el, km = run(kd, len(b.keys), idd, b.n, ad, int(b.arena.size), sd, steps, 1, False)
    st = sd.cpu().numpy()
    return {"value": round(b.n * steps / el, 1), "unit": "sigs/s", "items": b.n, "keys": len(b.keys),
            "mix": {"ed25519": ne, "secp256r1": nr, "secp256k1": nk}, "kernel_ms": round(km, 3),
            "ms_per_step": round(el / steps * 1e3, 3),
            "verdicts": {str(int(k)): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}


def bench_ecdsa_mixed(a, wl, dev, run, pools, n):
    """BASELINE configs[2] shape: one shuffled batch of n ECDSA items, half secp256r1 and half
    secp256k1, 2048 keys per curve, ~10% corrupted (items tiled from the 65 536-item pools)."""
    import torch
    from corda_amd.batch import Batch
    parts = [Batch(pools[c].keys, np.resize(pools[c].items, n // 2), pools[c].arena) for c in (1, 0)]
    b, _ = wl.concat(parts, shuffle_seed=a.seed + 29)
    kd = torch.from_numpy(b.keys.view(np.uint8)).to(dev)
    idd = torch.from_numpy(b.items.view(np.uint8)).to(dev)
    ad = torch.from_numpy(b.arena).to(dev)
    sd = torch.full((b.n,), 255, dtype=torch.uint8, device=dev)
    steps = max(2, a.steps // 2)
    el, km = run(kd, len(b.keys), idd, b.n, ad, int(b.arena.size), sd, steps, 1, False)
    st = sd.cpu().numpy()
    return {"value": round(b.n * steps / el, 1), "unit": "sigs/s", "items": b.n, "keys": len(b.keys),
            "kernel_ms": round(km, 3), "ms_per_step": round(el / steps * 1e3, 3),
            "verdicts": {str(int(k)): int(v) for k, v in zip(*np.unique(st, return_counts=True))}}


def bench_pipeline(a, wl, eng, dev, stream, threads):
    """BASELINE configs[3] shape: WireTransaction ids (SHA-256 Merkle) for every transaction,
    SignableData(id) spliced from the template, every signature verified -- one
    cg_verify_transactions_device call per step. Also times the id pass alone (cg_tx_ids_device)
    and reports its input bytes / time."""
    import torch
    from corda_amd import _lib
    t0 = time.time()
    w = wl.tx_pipeline(a.pipeline_txs, n_keys=1024, seed=a.seed + 211, corrupt_permille=20, nthreads=threads)
    gen = time.time() - t0
    up = lambda x: torch.from_numpy(x.view(np.uint8)).to(dev)  # noqa: E731
    txd, cd, kd, sgd, ad = up(w.txs), up(w.comps), up(w.keys), up(w.sigs), up(w.arena)
    n_tx, n_sig = len(w.txs), len(w.sigs)
    idd = torch.zeros(32 * n_tx, dtype=torch.uint8, device=dev)
    tsd = torch.zeros(n_tx, dtype=torch.uint8, device=dev)
    ssd = torch.full((n_sig,), 255, dtype=torch.uint8, device=dev)
    sptr = stream.cuda_stream
    L = _lib.lib()
    steps = max(2, a.steps // 2)

    def timed(fn):
        fn()
        torch.cuda.synchronize(dev)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        e0.record(stream)
        for _ in range(steps):
            fn()
        e1.record(stream)
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / steps, e0.elapsed_time(e1) / steps

    def ids_only():
        _lib.check(L.cg_tx_ids_device(eng._h, txd.data_ptr(), n_tx, cd.data_ptr(), len(w.comps), ad.data_ptr(),
                                      len(w.arena), idd.data_ptr(), tsd.data_ptr(), sptr), "cg_tx_ids_device")

    def full():
        eng.verify_transactions_device(txd.data_ptr(), n_tx, cd.data_ptr(), len(w.comps), kd.data_ptr(), len(w.keys),
                                       sgd.data_ptr(), n_sig, w.tmpls, ad.data_ptr(), len(w.arena), idd.data_ptr(),
                                       tsd.data_ptr(), ssd.data_ptr(), stream=sptr)

    _, ids_ms = timed(ids_only)
    el, full_ms = timed(full)
    ids = idd.cpu().numpy().reshape(-1, 32)
    sst = ssd.cpu().numpy()
    comp_bytes = int(w.comps["len"].astype(np.int64).sum())
    parity = bool(np.array_equal(ids, w.ids) and np.all(sst[w.labels == 0] == 0) and np.all(sst[w.labels == 1] == 1))
    return {"value": round(n_sig / el, 1), "unit": "sigs/s", "txs": n_tx, "sigs": n_sig,
            "components": len(w.comps), "component_bytes": comp_bytes,
            "tx_per_s": round(n_tx / el, 1), "ms_per_step": round(el * 1e3, 3), "kernel_ms": round(full_ms, 3),
            "tx_ids": {"ms": round(ids_ms, 3), "tx_per_s": round(n_tx / (ids_ms * 1e-3), 1),
                       "input_GBps": round(comp_bytes / (ids_ms * 1e-3) / 1e9, 1)},
            "parity_vs_generator": parity, "gen_s": round(gen, 1),
            "note": "BASELINE configs[3] is 1M txs; default 2^18 keeps host-side signing within the bench budget"}


def bench_tear_offs(a, wl, eng, dev, stream):
    """the non-validating notary's FilteredTransaction.verify for a batch of
    tear-offs (inputs + notary visible out of ~11 components), one cg_verify_filtered_device call
    per step. 4096 unique tear-offs are tiled to --tear-offs rows (no deduplication in the
    engine). Work: SHA-256 compressions (visible leaves + 2 per partial-tree node)."""
    import torch
    from corda_amd import merkle as M
    from corda_amd.batch import PMT_NODE
    pool, expect = wl.filtered_pool(4096, seed=a.seed + 307)
    t, n, lv, arena = M.pack_filtered(pool)
    reps = max(1, a.tear_offs // len(t))
    tt = np.tile(t, reps)
    up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
    td, nd, ld, ad = up(tt), up(n), up(lv), up(arena)
    sd = torch.full((len(tt),), 255, dtype=torch.uint8, device=dev)
    sptr = stream.cuda_stream

    def once():
        eng.verify_filtered_device(td.data_ptr(), len(tt), nd.data_ptr(), len(n), ld.data_ptr(), len(lv),
                                   ad.data_ptr(), int(arena.size), sd.data_ptr(), sptr)

    once()
    torch.cuda.synchronize(dev)
    steps = max(2, a.steps // 2)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        once()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    km = e0.elapsed_time(e1) / steps
    st = sd.cpu().numpy()
    comp_leaf = int(((lv["len"].astype(np.int64) + 32 + 9 + 63) // 64).sum())
    comp_node = 2 * int(np.count_nonzero(n["kind"] == PMT_NODE))
    comp_per = (comp_leaf + comp_node) / len(t)
    return {"value": round(len(tt) / el, 1), "unit": "tear-offs/s", "tear_offs": len(tt), "unique": len(t),
            "ms_per_step": round(el * 1e3, 3), "kernel_ms": round(km, 3),
            "sha256_compressions_per_tear_off": round(comp_per, 2),
            "sha256_compressions_per_s": round(len(tt) * comp_per / (km * 1e-3), 1),
            "parity_vs_generator": bool(np.array_equal(st, np.tile(expect, reps)))}


def bench_host_buffers(eng, batch, steps=3):
    """The PCIe-inclusive rate: cg_verify_batch from pageable host buffers (H2D of keys, items
    and arena, key prep, verify, D2H of the status bytes) on the headline batch."""
    eng.verify(batch)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.verify(batch)
    el = (time.perf_counter() - t0) / steps
    st = eng.last_stats
    return {"value": round(batch.n / el, 1), "unit": "sigs/s", "items": batch.n,
            "bytes_h2d": int(batch.arena.size + batch.items.nbytes + batch.keys.nbytes),
            "ms_per_call": round(el * 1e3, 3), "cg_stats_ms": {k: round(v, 3) for k, v in st.items()
                                                               if k.startswith("ms_")}}


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    threads = host_threads(a.threads)

    from corda_amd import shard
    from corda_amd.engine import Engine
    from tools.workload import wl

    # ---- synthetic shard for this rank (outside the timed region) ----
    t0 = time.time()
    batch, labels = wl.ed25519_batch(a.items, n_keys=a.keys, msg_len=a.msg_len,
                                     corrupt_permille=a.corrupt_permille, seed=a.seed + 7919 * rank,
                                     nthreads=threads)
    gen_s = time.time() - t0
    eng = Engine(local)
    eng.reserve(len(batch.keys), batch.n)
    keys_d = torch.from_numpy(batch.keys.view(np.uint8)).to(dev)
    items_d = torch.from_numpy(batch.items.view(np.uint8)).to(dev)
    arena_d = torch.from_numpy(batch.arena).to(dev)
    status_d = torch.full((batch.n,), 255, dtype=torch.uint8, device=dev)
    gathered_out = []
    n_keys, n_items, arena_len = len(batch.keys), batch.n, int(batch.arena.size)
    # one explicit stream for the engine, the timing events and the RCCL all-gather
    stream = torch.cuda.Stream(device=dev)
    sptr = stream.cuda_stream
    torch.cuda.set_stream(stream)

    def run(keys_t, n_keys_, items_t, n_items_, arena_t, arena_len_, status_t, steps, warmup, gather):
        ev = []

        def step(timed, prepare=True):
            if prepare:
                # one-shot cg_verify_batch_device: key prep sized by each key's use count, then items
                eng.verify_device(keys_t.data_ptr(), n_keys_, items_t.data_ptr(), n_items_, arena_t.data_ptr(),
                                  arena_len_, status_t.data_ptr(), 0, sptr)
            else:
                # item kernels alone against the tables the last one-shot step built
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                eng.verify_items_device(keys_t.data_ptr(), n_keys_, items_t.data_ptr(), n_items_,
                                        arena_t.data_ptr(), arena_len_, status_t.data_ptr(), 0, sptr)
                e1.record(stream)
                ev.append((e0, e1))
            if gather and prepare:
                # the engine's only collective: RCCL all-gather of the per-GPU verdict bytes
                gathered_out.append(shard.gather_verdicts(status_t, world * n_items_, world))

        for _ in range(warmup):
            step(False)
        torch.cuda.synchronize(dev)
        if gather:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(steps):
            step(False)
        torch.cuda.synchronize(dev)
        if gather:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t
        if gather:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        # item kernels alone (key tables already built by the last step), HIP events on the
        # engine stream: the duration the roofline is priced on. Key preparation overlaps the
        # item work inside a step, so a step's events would mix the two.
        for _ in range(max(2, steps // 2)):
            step(True, prepare=False)
        torch.cuda.synchronize(dev)
        return el, float(np.mean([a.elapsed_time(b) for a, b in ev])) if ev else float("nan")

    elapsed, kern_ms = run(keys_d, n_keys, items_d, n_items, arena_d, arena_len, status_d, a.steps, a.warmup,
                           world > 1)

    extra = {}
    if world == 1 and a.ecdsa_items > 0:
        # BASELINE configs[2] shape (secp256r1 / secp256k1 batches), outside the headline value
        pools = {}
        for curve, name in ((1, "ecdsa_secp256r1"), (0, "ecdsa_secp256k1")):
            pool = min(a.ecdsa_items, 65536)
            eb, _ = wl.ecdsa_batch(curve, pool, n_keys=2048, msg_len=a.msg_len, corrupt_permille=100,
                                   seed=a.seed + 17 + curve, nthreads=threads)
            pools[curve] = eb
            reps = max(1, a.ecdsa_items // pool)
            items_rep = np.tile(eb.items, reps)
            ek = torch.from_numpy(eb.keys.view(np.uint8)).to(dev)
            ei = torch.from_numpy(items_rep.view(np.uint8)).to(dev)
            ea = torch.from_numpy(eb.arena).to(dev)
            es = torch.full((len(items_rep),), 255, dtype=torch.uint8, device=dev)
            el, km = run(ek, len(eb.keys), ei, len(items_rep), ea, int(eb.arena.size), es, max(2, a.steps // 2), 1,
                         False)
            n_e = len(items_rep)
            extra[name] = {"value": round(n_e * max(2, a.steps // 2) / el, 1), "unit": "sigs/s",
                           "items": n_e, "unique_items": pool, "kernel_ms": round(km, 3)}
        # configs[2] proper: one shuffled batch, half secp256r1 / half secp256k1, 4x --ecdsa-items
        extra["ecdsa_mixed"] = bench_ecdsa_mixed(a, wl, dev, run, pools, 4 * a.ecdsa_items)
    if world == 1 and a.mixed_items > 0:
        extra["notary_mixed"] = bench_mixed(a, wl, eng, dev, stream, run, threads)
    if world == 1 and a.pipeline_txs > 0:
        extra["tx_pipeline"] = bench_pipeline(a, wl, eng, dev, stream, threads)
    if world == 1 and a.tear_offs > 0:
        extra["tear_offs"] = bench_tear_offs(a, wl, eng, dev, stream)
    if world == 1 and a.host_buffers:
        extra["host_buffers"] = bench_host_buffers(eng, batch)

    st = status_d.cpu().numpy()
    counts = {str(int(k)): int(v) for k, v in zip(*np.unique(st, return_counts=True))}
    # label sanity (full parity lives in tests/test_gpu_parity.py)
    valid_ok = bool(np.all(st[labels == 0] == 0))

    total_items = n_items * world * a.steps
    value = total_items / elapsed
    achieved = n_items * MAC32_EXEC_PER_ED25519 / (kern_ms * 1e-3)
    i2p_equiv = n_items * MAC32_PER_ED25519 / (kern_ms * 1e-3)
    roof = {"bound": "valu-int", "achieved": round(achieved / 1e12, 3), "peak": round(PEAK_MAC32_PER_S / 1e12, 3),
            "unit": "TMAC32/s", "frac": round(achieved / PEAK_MAC32_PER_S, 4), "traffic": None,
            "kernel": "k_ed_hash + k_ed_ladder + k_ed_finish (+ plan, k_misc_status, empty ECDSA launches)",
            "kernel_ms": round(kern_ms, 3),
            "work_per_item": f"executed: {MAC32_EXEC_PER_ED25519:.0f} MAC32 (field products the lane code "
                             f"runs: {ED_VERIFY_FE[0] + ED_FINISH_FE[0]} mul x {MAC_PER_MUL} + "
                             f"{ED_VERIFY_FE[1]} sq x {MAC_PER_SQ} + inversion/{ED_FINISH_K})",
            "i2p_equiv": {"achieved": round(i2p_equiv / 1e12, 3), "unit": "TMAC32/s",
                          "work_per_item": f"{N_FE_ED25519} i2p field mul/sq x 64 MAC32 = {MAC32_PER_ED25519}",
                          "note": "reference algorithm's work / GPU time; exceeds peak because the row "
                                  "tables do ~2.6x less work than i2p's sliding window"}}
    traffic_file = os.path.join(ROOT, "profiles", "r01", "pmc_traffic.json")
    if os.path.exists(traffic_file):
        with open(traffic_file) as f:
            tr = json.load(f)
        if tr.get("items") == n_items and tr.get("kernel_version") == KERNEL_VERSION:
            roof["traffic"] = tr.get("hbm_bytes_per_launch")
            if "valu_issue" in tr:  # PMC SQ pass of the same build: issue-slot occupancy per kernel
                roof["valu_issue"] = tr["valu_issue"]

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu, cst = cpu_baseline(batch, a.cpu_seconds, threads)
        cpu["parity_on_sample"] = bool(np.array_equal(cst, st[:cst.size]))

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 1), "unit": "sigs/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: seeded RFC 8032 Ed25519 signatures (tools/workload), no JVM capture",
            "config": {"workload": "BASELINE configs[1]: 2^20 Ed25519 sigs per GPU, bit-exact verdicts incl. "
                                   "corrupted sigs", "items_per_gpu": n_items, "keys": n_keys,
                       "msg_len": a.msg_len, "corrupt_permille": a.corrupt_permille,
                       "parallelism": f"shard{world}" + ("+rccl_allgather(verdicts)" if world > 1 else "")},
            "roofline": roof, "cpu_baseline": cpu, "secondary": extra,
            "verdicts": {"counts": counts, "valid_labels_all_valid": valid_ok},
            "gen_s": round(gen_s, 1),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()


if __name__ == "__main__":
    main()
