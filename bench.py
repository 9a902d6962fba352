#!/usr/bin/env python3
"""Headline benchmark: verified signatures / second for the whole node (BASELINE.json metric).

Workload (BASELINE configs[4], SURVEY.md §8(d) config 5, one GPU's shard): the notary-style
mixed batch, 70% Ed25519 / 20% ECDSA secp256r1 / 10% ECDSA secp256k1, 12.5M signatures per GPU
(100M over 8 GPUs), drawn by a seeded index stream from a 2^20-item unique pool with every
Appendix A corruption class (~11% corrupted). Every signature signs SignableData(txId,
SignatureMetadata(1, scheme)) -- the clear data Crypto.doVerify(txId, sig) checks -- with
--sigs-per-tx signatures per transaction id, 4096 Ed25519 keys and 1024 keys per curve.
Synthetic data (no network, no JVM).

One step = ONE cg_verify_tx_signatures_packed_device call over the whole shard with its inputs
already resident in HBM when the timed region starts (the key table, ids, the 12-byte signature
table, the dense signature stream, the template bytes; the task's measurement rule: `value` is never
a PCIe-inclusive rate): key-use counts sampled on the device, key tables, SignableData spliced on
the device, verify, verdicts left in HBM; plus (N > 1) the RCCL all-gather of the per-GPU verdict
vectors, the engine's only collective. `value` = signatures of all ranks / max-over-ranks time.
The same shard through the host form (cg_verify_tx_signatures_packed: host arena -> host verdicts,
the key-use count pass, ~85 B per signature over PCIe, D2H of the verdicts) is timed right after
it on every rank and reported as summary.host_to_host (--headline host makes it the timed form).

Launch: ``python bench.py`` (N = 1), ``python bench.py --gpus N`` (this process checks that N
devices are visible and starts ``torch.distributed.run --nproc-per-node N`` as a child before
anything touches the GPU, then exits with its code) or ``torchrun --nproc-per-node N bench.py
--gpus N`` (the driver's form); one process per GPU, each verifying its own shard (weak scaling).
Rank 0 prints ONE compact JSON line (<= 4 KB, the last line on stdout): the headline, `roofline`
and a `cpu_baseline` summary. Everything else (secondary legs, per-stage maps, the full CPU
baseline) goes to --secondary-out (default gpurun_out/bench_secondary.json) and to stderr.
  roofline      the dominant kernel (k_ed_ladder_wide: the shard's keys have wide tables; else
                k_ed_ladder_pf), priced in the 32x32->64 multiply-accumulates
                its lane code executes (host-counted) over its per-launch time from HIP events
                recorded on the stream it runs on, during the timed region (CG_FLAG_STAGE_TIMING);
                peak = the measured v_mad_u64_u32 chip rate. traffic = PMC FETCH/WRITE bytes per
                launch (profiles/, tools/pmc_traffic.py) when the committed profile matches.
  cpu_baseline  the C restatement of the reference algorithms (oracle/c, "port") on a bounded sample
                of the same workload, on the box's CPU quota (16 CPUs of a 256-thread EPYC) and on
                one thread; plus BASELINE configs[0] (10k SignedTransactions, fail-fast
                checkSignaturesAreValid) on the port and on OpenSSL, next to the GPU on that shape.
  secondary     device-resident forms of the same shard (inputs in HBM: cg_verify_batch_device over
                materialised messages, cg_verify_tx_signatures_device), the message-form host call
                (cg_verify_batch), per-stage times, key-distribution legs (2^20 distinct keys; Zipf),
                and at N = 1 the other BASELINE configs: [1] 2^20 Ed25519, [2] 2^20 ECDSA 50/50,
                [3] 1M-transaction pipeline, tear-offs.
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
# (oracle/c/ed25519_i2p.c counters): 1601 field multiplies + 1258 squarings
# per engineVerify (key decode excluded), each priced at 64 MAC32. Reported as `i2p_equiv`.
N_FE_ED25519 = 2859
MAC32_PER_ED25519 = N_FE_ED25519 * 64
# Executed work of the GPU path, counted by the host build of the same lane code
# (tests/native/host_kernels.cpp; pinned by tests/test_host_kernels.py::test_executed_work_*).
# Ed25519 (field multiplies, squarings) in the radix-2^25.5 representation (fe25519.h):
ED_VERIFY_FE = (319, 24)   # k_ed_ladder_pf: 43 mixed additions + 6 doublings in radix 2^25.5 ...
ED_VERIFY_FE9 = 69         # ... then the 10 B additions (radix-2^26 table) in radix 2^29 (fe9.h products)
ED_WIDE_FE = (287, 0)      # k_ed_ladder_wide: 32 + 10 signed entries, no doublings (keys with wide tables), all fe9; the first entry is one product (identity + q0)
ED_WIDE_BUILD_FE = (62279, 9120)  # one key's wide table: 248-doubling chain, then per row one lane walking its 128 entries, one inversion, the walk back (k_ed_wide_rows, ED_WIDE_ROW_LANES 1)
ED_FINISH_FE = (5, 0)      # k_ed_finish: prefix product, unwinding, encode
ED_INVERT_FE = (11, 254)   # one fe_invert, shared by ED_FINISH_K items
ED_FINISH_K = 16
MAC_PER_MUL, MAC_PER_SQ = 100, 55
MAC_PER_MUL9 = 81 + 16 + 1  # fe9.h: 81 products, 8 columns x 2 fold MACs, the top carry's 1216 T_lo
MAC32_ED_LADDER = ED_VERIFY_FE[0] * MAC_PER_MUL + ED_VERIFY_FE[1] * MAC_PER_SQ + ED_VERIFY_FE9 * MAC_PER_MUL9
MAC32_ED_WIDE = ED_WIDE_FE[0] * MAC_PER_MUL9
MAC32_EXEC_PER_ED25519 = ED_VERIFY_FE9 * MAC_PER_MUL9 + ((ED_VERIFY_FE[0] + ED_FINISH_FE[0]) * MAC_PER_MUL +
                          (ED_VERIFY_FE[1] + ED_FINISH_FE[1]) * MAC_PER_SQ +
                          (ED_INVERT_FE[0] * MAC_PER_MUL + ED_INVERT_FE[1] * MAC_PER_SQ) / ED_FINISH_K)
# ECDSA: field products (mont29.h) per item: (k_ec_ladder full tables mod p, k_ec_inv mod n
# per 16 items). A Montgomery product = 81 a*b MACs + 9 per non-zero 29-bit limb of the modulus
# (q*m); secp256r1's p telescopes its all-ones limbs (q*m = 4 MACs: 2^9, 2^18, limbs 7 and 8);
# secp256k1's p is folded instead (pseudo-Mersenne, plain form): 81 + 9 + 2 MACs.
# The ladder figure is its full schedule (every digit non-zero): a lane whose digit is zero skips
# its addition, but the wave issues it for the other 63 lanes, so the full schedule is what the
# SIMD executes (per-item mean 1% lower).
EC_LADDER_MUL = {"secp256r1": 719, "secp256k1": 701}
EC_WIDE_MUL = {"secp256r1": 454, "secp256k1": 454}  # k_ec_ladder_wide: 33 + 10 mixed additions (G radix 2^26) + x-check
# of those, the squares (round 6, ec9.h ec9_sqr*: 45 a*a MACs against a doubled copy instead of 81),
# priced at EC_MAC_PER_SQR_P: the same reduction as a product, 36 fewer multiply MACs
EC_WIDE_SQR = {"secp256r1": 123, "secp256k1": 123}  # 3 per addition (Z1^2, H^2, r^2 + E) x 41
# table modes (corda_amd/csrc/keyws.h): quarter tables from 3 items per key, full from 32, wide from
# KEY_WIDE_MIN_USES (1536 Ed25519 / 512 ECDSA)
KEY_QUARTER_MIN_USES, KEY_FULL_MIN_USES, KEY_WIDE_MAX = 3, 32, 8192  # keyws.h
KEY_WIDE_MIN_USES = {4: int(os.environ.get("CG_WIDE_MIN_USES_ED", 1536)), 3: int(os.environ.get("CG_WIDE_MIN_USES_EC", 512)),
                     2: int(os.environ.get("CG_WIDE_MIN_USES_EC", 512))}
EC_INV_K = 16  # items per k_ec_inv lane (corda_amd/csrc/ecdsa_rows.h; round 6: 16)
EC_INV_MUL_K = {"secp256r1": 421, "secp256k1": 428}  # products of one lane: prefix, inversion, unwinding
EC_MAC_PER_MUL_P = {"secp256r1": 117, "secp256k1": 92}
EC_MAC_PER_SQR_P = {"secp256r1": 45 + 36, "secp256k1": 45 + 11}
# executed MAC32 per k_ec_ladder_wide item: r1 48 690, k1 37 340 (round 5 priced every product at
# the general MAC count, 53 118 / 41 768, which round 6's squares would overstate by 9-11%)
EC_WIDE_MAC32 = {c: (EC_WIDE_MUL[c] - EC_WIDE_SQR[c]) * EC_MAC_PER_MUL_P[c] + EC_WIDE_SQR[c] * EC_MAC_PER_SQR_P[c]
                 for c in EC_WIDE_MUL}
EC_MAC_PER_MUL_N = {"secp256r1": 162, "secp256k1": 162}
# v_mad_u64_u32 chip throughput measured on MI355X (profiles/r04/ubench/ubench_peak_summary.json:
# 16 independent chains per lane, 8 waves per SIMD: 15.05 lanes/clk/SIMD at the measured shader
# clock). Round 1's 2.79e13 came from a latency-limited harness (8 chains, short launches).
PEAK_MAC32_PER_S = 3.6412e13
PEAK_MAC32_SPEC = 16 * 1024 * 2.4e9  # 4 cycles per wave64 v_mad_u64_u32 on a SIMD-32, 2.4 GHz
PEAK_SOURCE = "measured v_mad_u64_u32 chip rate, profiles/r04/ubench (spec-derived 3.93e13: frac_spec)"
# kernel generation whose PMC traffic profile is committed (profiles/r03/pmc_traffic.json)
KERNEL_VERSION = "r06_final"
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "r06", "pmc_traffic.json")

# Appendix A labels (tools/workload) -> the verdict Crypto.doVerify gives them (key decodes)
ED_LABEL_EXPECT = {0: 0, 1: 1, 2: 1, 3: 1, 4: 0, 6: 1, 7: 2}       # A5 (high S) depends on slide()
EC_LABEL_EXPECT = {0: 0, 1: 1, 2: 0, 3: 1, 6: 2, 7: 2}  # E5 (pad byte) is minimal when r >= 2^255


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--pool-devices", default="",
                    help="one process drives several devices through cg_pool_verify_tx_signatures (comma-separated "
                         "device ordinals, a device may repeat; weak scaling: --items per slot). Off: the torchrun form")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--items", type=int, default=12_500_000, help="items per GPU (configs[4]: 100M / 8)")
    ap.add_argument("--pool", type=int, default=1 << 20, help="unique items the index stream draws from")
    ap.add_argument("--ed-keys", type=int, default=4096)
    ap.add_argument("--ec-keys", type=int, default=1024, help="keys per ECDSA curve")
    ap.add_argument("--msg-len", type=int, default=270)
    ap.add_argument("--chunk-items", type=int, default=0, help="device chunk (0: CG_DEFAULT_CHUNK_ITEMS = 8M)")
    ap.add_argument("--seed", type=int, default=20251015)
    ap.add_argument("--sigs-per-tx", type=int, default=5,
                    help="signatures per transaction id (GeneratedLedger: 1+Poisson(3) signers + the notary)")
    ap.add_argument("--device-steps", type=int, default=4, help="device-resident secondary calls (0: off)")
    ap.add_argument("--key-dists", default="distinct,zipf",
                    help="key-distribution secondaries on the headline shape ('' : off): distinct = every pool item "
                         "its own key (2^20 keys, ~12 uses each), zipf = Zipf(1.1) over 2^20 keys")
    ap.add_argument("--host-steps", type=int, default=3, help="message-form cg_verify_batch calls (0: off)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="target CPU work of the baseline sample")
    ap.add_argument("--threads", type=int, default=0,
                    help="host threads of this rank (0: the CPU quota / LOCAL_WORLD_SIZE, at most 16)")
    ap.add_argument("--engine-threads", type=int, default=0,
                    help="cg_config.host_threads of the headline context (0: this rank's share when ranks "
                         "share the node, else the library's budget)")
    ap.add_argument("--txsig-table", type=int, default=12, choices=(12, 24),
                    help="the headline's signature table: 12 = cg_verify_tx_signatures_packed (12-byte records over "
                         "the dense signature stream, round 6), 24 = cg_verify_tx_signatures (24-byte cg_txsig)")
    ap.add_argument("--headline", default="device", choices=("device", "host"),
                    help="the timed form: device = inputs resident in HBM when the timed region starts (keys, ids, "
                         "12-byte table, signature stream, templates; verdicts left in HBM): "
                         "cg_verify_tx_signatures_packed_device; host = host arena -> host verdicts through "
                         "cg_verify_tx_signatures_packed (PCIe-inclusive; always measured beside the headline as "
                         "summary.host_to_host)")
    ap.add_argument("--contexts", type=int, default=1,
                    help="device-form steps alternate over this many contexts on the GPU (each call on its "
                         "context's own stream, so a call's key-table phase can overlap the previous call's "
                         "ladders: several verifiers on one device); 1: one context, calls in order")
    ap.add_argument("--ctx2-steps", type=int, default=-1,
                    help="with one headline context: the same device-form call timed again over two contexts on "
                         "the GPU, reported as summary.two_contexts (-1: --steps; 0: off)")
    ap.add_argument("--h2h-steps", type=int, default=-1,
                    help="host arena -> host verdicts calls timed beside a device headline (-1: --steps; 0: off)")
    ap.add_argument("--host-register", type=int, default=-1,
                    help="1: register the headline's host buffers once (cg_host_register: DMA straight from "
                         "them, no CPU staging copy), as a JVM node registers its persistent direct buffers; "
                         "2: the same after copying them into 2 MB transparent huge pages; 0: pageable; "
                         "-1 (default): the library's rule for the ranks on this node (register_advised: "
                         "pageable for 1-3 ranks per node, registered from 4, profiles/r06/host8)")
    ap.add_argument("--configs1-items", type=int, default=1 << 20, help="configs[1] Ed25519 secondary (0: off)")
    ap.add_argument("--ecdsa-items", type=int, default=1 << 20, help="configs[2] ECDSA 50/50 secondary (0: off)")
    ap.add_argument("--pipeline-txs", type=int, default=1 << 20, help="configs[3] transaction pipeline (0: off)")
    ap.add_argument("--tear-offs", type=int, default=1 << 18, help="FilteredTransaction.verify secondary (0: off)")
    ap.add_argument("--configs0-txs", type=int, default=10_000, help="configs[0] SignedTransactions (0: off)")
    ap.add_argument("--secondary-out", default=os.path.join(ROOT, "gpurun_out", "bench_secondary.json"),
                    help="where the secondary legs' JSON goes ('' : stderr only)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------ launcher
def launch_plan(gpus, env, visible):
    """How `bench.py --gpus N` runs (no GPU call is made to decide it).
    -> ("inline", world): this process is one rank of a world of `world` (WORLD_SIZE from torchrun,
       or N = 1); ("spawn", N): start torch.distributed.run with N processes, one per GPU.
    Raises SystemExit with a message when the request cannot be met: fewer than N visible devices,
    or a torchrun world that disagrees with --gpus (never report n_gpus = 1 for --gpus 8)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus}: need at least 1")
    if "WORLD_SIZE" in env:
        world = int(env["WORLD_SIZE"])
        if world != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: launch one process per GPU")
        return "inline", world
    if visible < gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} requested but only {visible} device(s) are visible")
    return ("spawn", gpus) if gpus > 1 else ("inline", 1)


def spawn_cmd(nproc, argv, port, script=None):
    """The driver's own N-GPU command line (one rank per GPU, rendezvous on 127.0.0.1)."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr=127.0.0.1", f"--master-port={port}", script or os.path.abspath(__file__)] + list(argv)


def free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _lib_mod():
    from corda_amd import _lib
    return _lib


def hugepage_copy(arr):
    """A copy of `arr` in an anonymous mapping advised MADV_HUGEPAGE, 2 MB aligned (so the kernel can
    back it with transparent huge pages); returns (view, mapping)."""
    import mmap
    huge = 2 << 20
    size = (arr.nbytes + 2 * huge - 1) // huge * huge
    m = mmap.mmap(-1, size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    if hasattr(mmap, "MADV_HUGEPAGE"):
        m.madvise(mmap.MADV_HUGEPAGE)
    base = np.frombuffer(m, dtype=np.uint8)
    off = (-base.ctypes.data) % huge
    view = base[off:off + arr.nbytes].view(arr.dtype).reshape(arr.shape)
    view[...] = arr
    return view, m


def anon_huge_kb():
    """AnonHugePages of this process (kB), from /proc/self/smaps_rollup (0 if unreadable)."""
    try:
        with open("/proc/self/smaps_rollup") as f:
            for l in f:
                if l.startswith("AnonHugePages:"):
                    return int(l.split()[1])
    except OSError:
        pass
    return 0


def kfd_gpus(sysfs="/sys/class/kfd/kfd/topology/nodes", env=None):
    """GPUs this process may use, counted without any HIP / HSA call: the KFD topology nodes with a
    gfx target (CPU nodes have gfx_target_version 0), cut down by ROCR_VISIBLE_DEVICES /
    HIP_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES the way the runtime applies them (a list of ordinals)."""
    env = os.environ if env is None else env
    n = 0
    try:
        for node in sorted(os.listdir(sysfs), key=lambda x: int(x) if x.isdigit() else 1 << 30):
            try:
                with open(os.path.join(sysfs, node, "properties")) as f:
                    props = dict(l.split(None, 1) for l in f if len(l.split(None, 1)) == 2)
            except OSError:
                continue
            if int(props.get("gfx_target_version", "0").strip() or 0) != 0:
                n += 1
    except OSError:
        return 0
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = env.get(var)
        if v is not None:
            ids = [x for x in v.split(",") if x.strip() != ""]
            n = min(n, len(ids))
    return n


def gpu_initialised(fd_dir="/proc/self/fd"):
    """True once this process has opened /dev/kfd, i.e. the HSA runtime under HIP has initialised
    (loading libamdhip64 with `import torch` does not open it; the first HIP call does). A process
    that has initialised the GPU must not exec or fork a GPU world from its own image."""
    try:
        for fd in os.listdir(fd_dir):
            try:
                if os.readlink(os.path.join(fd_dir, fd)) == "/dev/kfd":
                    return True
            except OSError:
                continue
    except OSError:
        return False
    return False


def rank_host_threads(req, env=None):
    """Host threads of this rank: the process's CPU quota (host_threads) divided among the ranks on
    the node (LOCAL_WORLD_SIZE under torchrun), at least 1; --threads wins when given."""
    env = os.environ if env is None else env
    if req > 0:
        return req
    ranks = max(1, int(env.get("LOCAL_WORLD_SIZE", "1") or 1))
    return max(1, host_threads(0) // ranks)


HOST_REGISTER_MIN_RANKS = 4  # corda_amd/csrc/host_budget.h kHostRegisterMinContexts


def register_advised(env=None):
    """--host-register -1: register the headline's buffers when 4 or more ranks share the node
    (LOCAL_WORLD_SIZE), the rule cg_host_register_advised states (profiles/r06/host8/summary.json:
    registered -10% alone, +5% beside 7 other ranks' host copies). HIP-free."""
    env = os.environ if env is None else env
    ranks = max(1, int(env.get("LOCAL_WORLD_SIZE", "1") or 1))
    return 1 if ranks >= HOST_REGISTER_MIN_RANKS else 0


def spawn_world(nproc, argv):
    """Start the N-rank world as a CHILD process (this process has not touched the GPU: the device
    count comes from sysfs, and gpu_initialised() is checked) and return its exit code; rank 0's
    stdout passes through."""
    import subprocess
    if gpu_initialised():
        raise SystemExit("bench.py: the GPU runtime is already initialised in the launcher process; "
                         "refusing to start the world from it")
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(spawn_cmd(nproc, argv, free_port()), env=env)


# ------------------------------------------------------------------------------------ the line
LINE_MAX = 4096
LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline")
ROOF_KEYS = ("kernel", "bound", "achieved", "peak", "unit", "frac", "frac_spec", "traffic", "traffic_source", "launch_ms",
             "items_per_launch", "work_per_item", "peak_source")
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "host", "jvm", "parity_on_sample")


def _trim(d, keys):
    return None if d is None else {k: d[k] for k in keys if k in d}


def compact_line(head, roof, cpu, summary):
    """The ONE stdout line the driver parses: headline keys, the dominant kernel's roofline,
    a cpu_baseline summary and a few secondary values; <= LINE_MAX bytes (BENCH_r03's 17.8-KB
    line was not parsed). Secondaries are dropped before the required keys are."""
    line = dict(head)
    line["roofline"] = _trim(roof, ROOF_KEYS)
    if cpu is not None and "error" not in cpu:
        c = _trim(cpu, CPU_KEYS)
        o = cpu.get("openssl")
        if isinstance(o, dict):
            c["openssl"] = {"value": o.get("value"), "threads": o.get("threads"),
                            "value_1thread": o.get("value_1thread")}
        if isinstance(cpu.get("serial_1thread"), dict):
            c["value_1thread"] = cpu["serial_1thread"].get("value")
        c0 = cpu.get("configs0")
        if isinstance(c0, dict) and "port" in c0:
            c["configs0"] = {"port_sigs_per_s": c0["port"]["sigs_per_s"],
                             "gpu_sigs_per_s": c0.get("gpu", {}).get("sigs_per_s"),
                             "first_failures_equal_port": c0.get("gpu", {}).get("first_failures_equal_port")}
        line["cpu_baseline"] = c
    else:
        line["cpu_baseline"] = cpu
    line["summary"] = summary
    s = json.dumps(line, separators=(",", ":"))
    for drop in ("summary", ("cpu_baseline", "configs0"), ("cpu_baseline", "openssl"), ("cpu_baseline", "host"),
                 ("config", "workload")):
        if len(s) <= LINE_MAX:
            break
        if isinstance(drop, tuple):
            if isinstance(line.get(drop[0]), dict):
                line[drop[0]].pop(drop[1], None)
        else:
            line.pop(drop, None)
        s = json.dumps(line, separators=(",", ":"))
    assert len(s) <= LINE_MAX, len(s)
    return s


def write_secondary(path, obj):
    """Secondary legs: a file (merged back by gpurun from gpurun_out/) and stderr."""
    s = json.dumps(obj, separators=(",", ":"), default=str)
    if path:
        try:
            os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
            with open(path, "w") as f:
                f.write(s + "\n")
        except OSError as e:
            print(f"bench.py: could not write {path}: {e}", file=sys.stderr)
    print("SECONDARY " + s, file=sys.stderr, flush=True)


def guarded(out, name, fn):
    """Run one secondary leg; a failure is recorded and never voids the headline line."""
    try:
        out[name] = fn()
    except Exception as e:  # noqa: BLE001
        out[name] = {"error": f"{type(e).__name__}: {e}"}


def host_threads(req):
    if req > 0:
        return req
    n = os.cpu_count() or 1
    try:  # the container's CPU quota (the GPU box: 16 CPUs of a 256-thread host)
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(n, 16))


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            return next(l.split(":", 1)[1].strip() for l in f if l.startswith("model name"))
    except (OSError, StopIteration):
        return "unknown"


def expected_verdicts(labels, schemes):
    """Label -> verdict the reference gives (keys all decode in these workloads); 255 = no fixed
    expectation (A5: the slide() carry rule decides)."""
    exp = np.full(labels.size, 255, np.uint8)
    ed = schemes == 4
    for lab, v in ED_LABEL_EXPECT.items():
        exp[ed & (labels == lab)] = v
    for lab, v in EC_LABEL_EXPECT.items():
        exp[~ed & (labels == lab)] = v
    return exp


def check_verdicts(st, exp):
    m = exp != 255
    bad = int(np.count_nonzero(st[m] != exp[m]))
    return {"counts": {str(int(k)): int(v) for k, v in zip(*np.unique(st, return_counts=True))},
            "checked_vs_labels": int(m.sum()), "label_mismatches": bad,
            "not_run": int(np.count_nonzero(st == 255))}


# ------------------------------------------------------------------------------------ CPU legs
def cpu_baseline(batch, st_gpu, seconds, threads):
    """oracle/c (C restatement of i2p 0.2.0 / BC 1.57 semantics) on a bounded sample of the
    headline items, on `threads` threads and on one thread."""
    from corda_amd.batch import Batch
    from oracle import c_oracle
    probe = min(batch.n, 256 * threads)
    sub = Batch(batch.keys, batch.items[:probe], batch.arena)
    t = time.perf_counter()
    c_oracle.verify_batch(sub, 0, threads)
    dt = time.perf_counter() - t
    n = int(min(batch.n, max(probe, probe * seconds / max(dt, 1e-6))))
    for _ in range(3):  # the probe includes every key's decode: grow the sample until it fills the target
        sub = Batch(batch.keys, batch.items[:n], batch.arena)
        t = time.perf_counter()
        st = c_oracle.verify_batch(sub, 0, threads)
        dt = time.perf_counter() - t
        if dt >= 0.6 * seconds or n >= batch.n:
            break
        n = int(min(batch.n, n * seconds / max(dt, 1e-6)))
    n1 = max(64, min(n, int(n / threads / 2)))
    sub1 = Batch(batch.keys, batch.items[:n1], batch.arena)
    t = time.perf_counter()
    c_oracle.verify_batch(sub1, 0, 1)
    dt1 = time.perf_counter() - t
    ossl = openssl_items(sub, st, threads)
    return {"value": round(n / dt, 1), "unit": "sigs/s", "cores": threads, "kind": "port",
            "sample": f"first {n} items of the rank-0 headline batch (70/20/10 mix; incl. decoding all "
                      f"{len(batch.keys)} keys), oracle/c or_verify_batch over {threads} threads, {dt:.1f} s",
            "host": f"{cpu_model()}; CPU quota {threads} CPUs (cgroup cpu.max) of {os.cpu_count()} hardware threads",
            "serial_1thread": {"value": round(n1 / dt1, 1), "items": n1, "seconds": round(dt1, 2)},
            "parity_on_sample": bool(np.array_equal(st, st_gpu[:n])),
            "openssl": ossl,
            "jvm": "JVM reference unavailable: no JDK, no i2p / BouncyCastle jars, no network"}


def openssl_items(sub, st_port, threads):
    """OpenSSL 3 EVP_DigestVerify on the same headline sample (Ed25519 + both ECDSA curves, each key
    decoded once per call and shared by the workers), on the CPU quota and on one thread: an
    industrial CPU point beside the port. Its verdicts differ from the reference's exactly where
    i2p 0.2.0 does: Ed25519 signatures with S >= L (workload labels A4 / A5), which i2p accepts."""
    import ctypes
    so = os.path.join(ROOT, "tools", "cpu_baseline", "libosslcheck.so")
    if not os.path.exists(so):
        return "absent: tools/cpu_baseline not built"
    O = ctypes.CDLL(so)
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    O.ob_verify_items.argtypes = [vp, u32, vp, u64, vp, u64, vp, i32]
    O.ob_verify_items.restype = ctypes.c_int64
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    st = np.zeros(sub.n, np.uint8)
    t = time.perf_counter()
    if O.ob_verify_items(p(sub.keys), len(sub.keys), p(sub.items), sub.n, p(sub.arena), sub.arena.size, p(st),
                         threads) < 0:
        return "absent: libcrypto.so.3 could not be loaded"
    dt = time.perf_counter() - t
    n1 = max(64, sub.n // threads // 2)
    st1 = np.zeros(n1, np.uint8)
    t = time.perf_counter()
    O.ob_verify_items(p(sub.keys), len(sub.keys), p(sub.items[:n1]), n1, p(sub.arena), sub.arena.size, p(st1), 1)
    dt1 = time.perf_counter() - t
    valid_port = st_port == 0
    return {"value": round(sub.n / dt, 1), "unit": "sigs/s", "threads": threads, "items": int(sub.n),
            "value_1thread": round(n1 / dt1, 1),
            "valid_verdicts_differing_from_port": int(np.count_nonzero((st == 0) != valid_port)),
            "note": "OpenSSL 3.0.2 EVP_DigestVerify per item, keys decoded once per call (Ed25519 raw keys; "
                    "ECDSA raw X||Y wrapped in the curve's SPKI); rejects Ed25519 S >= L (labels A4 / A5), "
                    "which i2p 0.2.0 accepts: the only differing verdicts"}


def configs0(a, eng, wl, threads):
    """BASELINE configs[0]: 10k SignedTransactions (GeneratedLedger shape: 1+Poisson(3) command
    signers + the notary, ~5 Ed25519 signatures each over SignableData(id, metadata)), verified
    with checkSignaturesAreValid semantics (serial per transaction, fail-fast,
    TransactionWithSignatures.kt:58-61), transactions taken by workers from a shared counter
    (Injectors.kt:18-55). CPU: oracle/c port and OpenSSL, on the CPU quota and on one thread.
    GPU: every signature of every transaction in one cg_verify_batch call, the first failure per
    transaction rebuilt in list order (corda_amd/transactions.py), checked against the port."""
    import ctypes
    from oracle import c_oracle
    c0, tx_first, _ = wl.configs0(a.configs0_txs, seed=a.seed + 401, nthreads=threads)
    n_tx, n_sig = len(tx_first) - 1, c0.n
    L = c_oracle.lib()
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.or_check_txs.argtypes = [vp, u32, vp, vp, u64, vp, u64, vp, i32]
    L.or_check_txs.restype = u64
    p = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    tf = np.ascontiguousarray(tx_first, np.uint64)

    def run(fn, nt, ntx):
        ff = np.zeros(ntx, np.int64)
        t = time.perf_counter()
        done = fn(p(c0.keys), len(c0.keys), p(c0.items), p(tf), ntx, p(c0.arena), c0.arena.size, p(ff), nt)
        return done, time.perf_counter() - t, ff

    out = {"txs": n_tx, "sigs": n_sig, "shape": "GeneratedLedger-like: 1+Poisson(1) inputs, Poisson(3) outputs, "
                                                 "1+Poisson(3) command signers + notary; Ed25519; 2% corrupted"}
    done, dt, ff_port = run(L.or_check_txs, threads, n_tx)
    out["port"] = {"sigs_per_s": round(done / dt, 1), "tx_per_s": round(n_tx / dt, 1), "threads": threads,
                   "seconds": round(dt, 2)}
    n1 = max(1, n_tx // 8)
    done, dt, _ = run(L.or_check_txs, 1, n1)
    out["port_1thread"] = {"sigs_per_s": round(done / dt, 1), "tx_per_s": round(n1 / dt, 1), "txs": n1}
    so = os.path.join(ROOT, "tools", "cpu_baseline", "libosslcheck.so")
    if os.path.exists(so):
        O = ctypes.CDLL(so)
        O.ob_check_txs.argtypes = [vp, u32, vp, vp, u64, vp, u64, vp, i32]
        O.ob_check_txs.restype = ctypes.c_int64
        done, dt, ff_ossl = run(O.ob_check_txs, threads, n_tx)
        if done < 0:
            out["openssl"] = "absent: libcrypto.so.3 could not be loaded"
        else:
            d1, dt1, _ = run(O.ob_check_txs, 1, n1)
            out["openssl"] = {"sigs_per_s": round(done / dt, 1), "tx_per_s": round(n_tx / dt, 1),
                              "threads": threads, "sigs_per_s_1thread": round(d1 / dt1, 1),
                              "same_first_failures_as_port": bool(np.array_equal(ff_ossl, ff_port)),
                              "note": "OpenSSL 3.0.2 EVP_DigestVerify, fresh EVP_PKEY per signature; rejects "
                                      "S >= L where i2p 0.2.0 accepts it"}
    else:
        out["openssl"] = "absent: tools/cpu_baseline not built"
    # GPU: one batch of all signatures, fail-fast rebuilt per transaction
    eng.verify(c0)
    t = time.perf_counter()
    st = eng.verify(c0)
    dt = time.perf_counter() - t
    ff_gpu = np.full(n_tx, -1, np.int64)
    bad = np.nonzero(st != 0)[0]
    owner = np.searchsorted(tf, bad, side="right") - 1
    for i, o in zip(bad[::-1], owner[::-1]):
        ff_gpu[o] = i - tf[o]
    out["gpu"] = {"sigs_per_s": round(n_sig / dt, 1), "tx_per_s": round(n_tx / dt, 1), "ms": round(dt * 1e3, 3),
                  "path": "cg_verify_batch (host buffers, PCIe included), one call",
                  "first_failures_equal_port": bool(np.array_equal(ff_gpu, ff_port))}
    return out


# ------------------------------------------------------------------------------------ GPU legs
def upload(dev, b):
    import torch
    up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
    return up(b.keys), up(b.items), up(b.arena), torch.full((b.n,), 255, dtype=torch.uint8, device=dev)


def timed_device(eng, bufs, b, steps, warmup, stream, dev, gather=None, ctx_stream=False):
    """ctx_stream: enqueue on the engine context's own stream (hip_stream = NULL, the form a JNI
    caller uses) instead of torch's; the verdict gather then waits for it (device sync)."""
    import torch
    kd, idd, ad, sd = bufs
    sptr = 0 if ctx_stream else stream.cuda_stream

    def step():
        eng.verify_device(kd.data_ptr(), len(b.keys), idd.data_ptr(), b.n, ad.data_ptr(), b.arena.size,
                          sd.data_ptr(), 0, sptr)
        if gather is not None and ctx_stream:
            torch.cuda.synchronize(dev)
        if gather is not None:
            gather(sd)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize(dev)
    return step


def stage_summary(times, steps_per_read):
    out = {}
    for name, (ms, n) in times.items():
        if n:
            out[name] = {"ms_per_step": round(ms / steps_per_read, 3), "launches": int(n),
                         "ms_per_launch": round(ms / n, 3)}
    return out


def headline_chunk(a, n):
    """Items per verify chunk of the headline call: cg_verify_tx_signatures splits a large host call
    into at least 3 chunks (besides the first) unless the caller sets cg_config.chunk_items (cordagpu.cpp)."""
    chunk = eng_chunk(a)
    k = max(1, -(-n // chunk))
    per = -(-n // k)
    if not a.chunk_items and n >= 3 * (1 << 20):
        per = min(per, -(-n // 3))
    return per


def ladder_units(b, labels, schemes, chunk):
    """Items that reach each ladder, per device chunk and table mode: Ed25519 items with a 64-byte
    signature, ECDSA items whose DER parses and whose r, s are in range (labels 0-2). The mode of a
    key follows its item count in the call (keyws.h; the engine samples the counts, so a key
    within 20% of a threshold makes the split approximate: `exact` says whether any is)."""
    sig64 = b.items["sig_len"] == 64
    ok_ec = np.isin(labels, (0, 1, 2))
    uses = np.bincount(b.items["key_idx"], minlength=len(b.keys))
    thr = np.array([KEY_WIDE_MIN_USES.get(int(s), 1 << 30) for s in b.keys["scheme"]])
    cap = min(len(b.keys), b.n // min(KEY_WIDE_MIN_USES.values()), KEY_WIDE_MAX)
    wide_key = uses >= thr
    full_key = (uses >= KEY_FULL_MIN_USES) & ~wide_key
    near = ((np.abs(uses - thr) < 0.2 * thr) |
            (np.abs(uses - KEY_FULL_MIN_USES) < 0.2 * KEY_FULL_MIN_USES)) & (uses > 0)
    exact = not near.any() and all(int((wide_key & (b.keys["scheme"] == s)).sum()) <= cap for s in (2, 3, 4))
    kw, kf = wide_key[b.items["key_idx"]], full_key[b.items["key_idx"]]
    n = b.n
    k = max(1, -(-n // chunk)) if chunk else 1
    per = -(-n // k)
    f = lambda m: [int(m[i:i + per].sum()) for i in range(0, n, per)]  # noqa: E731
    out = {"exact": exact}
    for name, sel in (("ed", (schemes == 4) & sig64), ("r1", (schemes == 3) & ok_ec), ("k1", (schemes == 2) & ok_ec)):
        out[name] = f(sel & kf)
        out[name + "_wide"] = f(sel & kw)
    return out


def roofline(stages, units, steps):
    """Each ladder's executed MAC32 over its average launch time (HIP events on its stream). The
    headline block is the Ed25519 ladder with the most time per step (k_ed_ladder_wide when the
    keys have wide tables, else k_ed_ladder_pf); the ECDSA ladders are reported beside it."""
    def block(stage, per_item, unit_counts, label):
        ms, n = stages.get(stage, (0.0, 0))
        if not n or not sum(unit_counts):
            return None
        launch_ms = ms / n
        # per launch: the step's items over its launches (the stage timer counts the launches, so a
        # first chunk of another size, CG_TXSIG_FIRST_DIV, is averaged in correctly)
        items = sum(unit_counts) * max(steps, 1) / n
        ach = items * per_item / (launch_ms * 1e-3)
        return {"kernel": label, "bound": "valu-int", "achieved": round(ach / 1e12, 3),
                "peak": round(PEAK_MAC32_PER_S / 1e12, 3), "unit": "TMAC32/s", "frac": round(ach / PEAK_MAC32_PER_S, 4),
                "frac_spec": round(ach / PEAK_MAC32_SPEC, 4),
                "launch_ms": round(launch_ms, 3), "launches": int(n), "items_per_launch": int(items),
                "work_per_item": per_item, "ms_per_step": round(ms / max(steps, 1), 3),
                "units_exact": units["exact"]}
    eds = [x for x in (block("ed_ladder", MAC32_ED_LADDER, units["ed"], "k_ed_ladder_pf"),
                       block("ed_ladder_wide", MAC32_ED_WIDE, units["ed_wide"], "k_ed_ladder_wide")) if x]
    ed = max(eds, key=lambda x: x["ms_per_step"]) if eds else None
    ec = {}
    for c, tag in (("secp256r1", "r1"), ("secp256k1", "k1")):
        ec[c] = block(tag + "_ladder", EC_LADDER_MUL[c] * EC_MAC_PER_MUL_P[c], units[tag], f"k_ec_ladder<{c}, full>")
        ec[c + "_wide"] = block(tag + "_ladder_wide", EC_WIDE_MAC32[c], units[tag + "_wide"], f"k_ec_ladder_wide<{c}>")
    return ed, ec


def run_secondary_device(eng, dev, stream, b, steps=4):
    """Device-resident rate of a secondary batch plus its item-kernel time (tables prebuilt)."""
    import torch
    bufs = upload(dev, b)
    step = timed_device(eng, bufs, b, steps, 1, stream, dev, ctx_stream=True)
    eng.stage_times()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t) / steps
    stg = eng.stage_times()
    st = bufs[3].cpu().numpy()
    return el, st, stg


def bench_configs1(a, eng, dev, stream, wl, threads):
    b, labels = wl.ed25519_batch(a.configs1_items, n_keys=4096, msg_len=a.msg_len, corrupt_permille=120,
                                 seed=a.seed + 7, nthreads=threads)
    el, st, stg = run_secondary_device(eng, dev, stream, b)
    units = ladder_units(b, labels, np.full(b.n, 4, np.uint8), eng_chunk(a))
    ed, _ = roofline(stg, units, 4)
    ver = check_verdicts(st, expected_verdicts(labels, np.full(b.n, 4, np.uint8)))
    return {"value": round(b.n / el, 1), "unit": "sigs/s", "items": b.n, "keys": 4096, "ms_per_step": round(el * 1e3, 3),
            "roofline": ed, "stages": stage_summary(stg, 4), "verdicts": ver}


def eng_chunk(a):
    return a.chunk_items or (8 << 20)


def bench_ecdsa(a, eng, dev, stream, wl, threads):
    """configs[2]: one shuffled batch, half secp256r1 / half secp256k1, 2048 keys per curve, ~10%
    corrupted, every item unique."""
    b, labels, schemes = wl.notary_pool(a.ecdsa_items, ec_keys=2048, msg_len=a.msg_len, seed=a.seed + 29,
                                        nthreads=threads, mix=(0.0, 0.5, 0.5))
    el, st, stg = run_secondary_device(eng, dev, stream, b)
    units = ladder_units(b, labels, schemes, eng_chunk(a))
    _, ec = roofline(stg, units, 4)
    return {"value": round(b.n / el, 1), "unit": "sigs/s", "items": b.n, "keys": len(b.keys),
            "ms_per_step": round(el * 1e3, 3), "roofline": ec, "stages": stage_summary(stg, 4),
            "verdicts": check_verdicts(st, expected_verdicts(labels, schemes)),
            "work_per_item_mac32": {c: EC_LADDER_MUL[c] * EC_MAC_PER_MUL_P[c] + EC_INV_MUL_K[c] * EC_MAC_PER_MUL_N[c] / EC_INV_K
                                    for c in EC_LADDER_MUL}}


def bench_pipeline(a, eng, dev, stream, wl, threads):
    """configs[3]: WireTransaction ids (SHA-256 Merkle) for every transaction, SignableData(id)
    spliced from the template, every signature verified -- one cg_verify_transactions_device call
    per step; the id pass alone timed too (SHA-256 compressions/s against the integer-VALU bound)."""
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
    steps = 3

    def timed(fn):
        fn()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t) / steps

    def ids_only():
        _lib.check(L.cg_tx_ids_device(eng._h, txd.data_ptr(), n_tx, cd.data_ptr(), len(w.comps), ad.data_ptr(),
                                      len(w.arena), idd.data_ptr(), tsd.data_ptr(), sptr), "cg_tx_ids_device")

    def full():
        eng.verify_transactions_device(txd.data_ptr(), n_tx, cd.data_ptr(), len(w.comps), kd.data_ptr(), len(w.keys),
                                       sgd.data_ptr(), n_sig, w.tmpls, ad.data_ptr(), len(w.arena), idd.data_ptr(),
                                       tsd.data_ptr(), ssd.data_ptr(), stream=sptr)

    ids_s = timed(ids_only)
    eng.stage_times()
    el = timed(full)
    stg = eng.stage_times()
    ids = idd.cpu().numpy().reshape(-1, 32)
    sst = ssd.cpu().numpy()
    lens = w.comps["len"].astype(np.int64)
    comp_bytes = int(lens.sum())
    # SHA-256 compressions of the id pass: per component nonce (1) + leaf (blob || nonce, or the
    # salt blob alone), then 2 per Merkle node over the padded leaves
    salt = (w.comps["flags"] & 1) == 1
    leaf_blocks = np.where(salt, (lens + 9 + 63) // 64, (lens + 32 + 9 + 63) // 64)
    nonce_blocks = np.where(salt, 0, 1)
    ncomp = w.txs["n"].astype(np.int64)
    padded = 1 << np.ceil(np.log2(np.maximum(ncomp, 1))).astype(np.int64)
    comps_total = int(leaf_blocks.sum() + nonce_blocks.sum() + 2 * (padded - 1).sum())
    rate = comps_total / ids_s
    parity = bool(np.array_equal(ids, w.ids) and np.all(sst[w.labels == 0] == 0) and np.all(sst[w.labels == 1] == 1))
    return {"value": round(n_sig / el, 1), "unit": "sigs/s", "txs": n_tx, "sigs": n_sig, "components": len(w.comps),
            "component_bytes": comp_bytes, "tx_per_s": round(n_tx / el, 1), "ms_per_step": round(el * 1e3, 3),
            "stages": stage_summary(stg, steps),
            "tx_ids": {"ms": round(ids_s * 1e3, 3), "tx_per_s": round(n_tx / ids_s, 1),
                       "input_GBps": round(comp_bytes / ids_s / 1e9, 1),
                       "hbm_frac": round(comp_bytes / ids_s / 8e12, 4),
                       "sha256_compressions": comps_total,
                       "valu_roofline": {"bound": "valu-int", "achieved_compressions_per_s": round(rate, 1),
                                         "int_ops_per_compression": 2720,
                                         "achieved_Tops": round(rate * 2720 / 1e12, 2),
                                         "peak_Tops": 59.0, "frac": round(rate * 2720 / 59e12, 4),
                                         "note": "peak = v_add_u32 chip rate (profiles/r01/ubench_int.json); "
                                                 "2 720 32-bit ops per SHA-256 compression (SURVEY §8(d))"}},
            "parity_vs_generator": parity, "gen_s": round(gen, 1)}


def bench_tear_offs(a, eng, dev, stream, wl):
    """the non-validating notary's FilteredTransaction.verify for a batch of
    tear-offs, one cg_verify_filtered_device call per step (4096 unique tiled, no dedup)."""
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
    steps = 4
    t0 = time.perf_counter()
    for _ in range(steps):
        once()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t0) / steps
    st = sd.cpu().numpy()
    comp_leaf = int(((lv["len"].astype(np.int64) + 32 + 9 + 63) // 64).sum())
    comp_node = 2 * int(np.count_nonzero(n["kind"] == PMT_NODE))
    comp_per = (comp_leaf + comp_node) / len(t)
    return {"value": round(len(tt) / el, 1), "unit": "tear-offs/s", "tear_offs": len(tt), "unique": len(t),
            "ms_per_step": round(el * 1e3, 3), "sha256_compressions_per_tear_off": round(comp_per, 2),
            "sha256_compressions_per_s": round(len(tt) * comp_per / el, 1),
            "parity_vs_generator": bool(np.array_equal(st, np.tile(expect, reps)))}


def bench_device(eng, dev, stream, b, tb, st_ref, steps):
    """Device-resident forms of the headline shard (inputs already in HBM, status left in HBM):
    cg_verify_batch_device over the materialised messages, and cg_verify_tx_signatures_device over
    (id, template) pairs. The PCIe-free ceiling of the whole-node headline."""
    import torch
    out = {}
    bufs = upload(dev, b)
    step = timed_device(eng, bufs, b, steps, 1, stream, dev, ctx_stream=True)
    eng.stage_times()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t) / steps
    stg = eng.stage_times()
    out["message_form"] = {"value": round(b.n / el, 1), "unit": "sigs/s", "ms_per_step": round(el * 1e3, 3),
                           "path": "cg_verify_batch_device, one call per step (SignableData bytes resident in HBM)",
                           "stages": stage_summary(stg, steps),
                           "verdicts_equal_headline": bool(np.array_equal(bufs[3].cpu().numpy(), st_ref))}
    del bufs
    up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
    kd, ijd, sgd, ad = up(tb.keys), up(tb.ids), up(tb.sigs), up(tb.arena)
    sd = torch.full((tb.n,), 255, dtype=torch.uint8, device=dev)

    def once():
        eng.verify_tx_signatures_device(kd.data_ptr(), len(tb.keys), ijd.data_ptr(), tb.n_ids, sgd.data_ptr(), tb.n,
                                        tb.tmpls, ad.data_ptr(), tb.arena.size, sd.data_ptr())
    once()
    torch.cuda.synchronize(dev)
    eng.stage_times()
    t = time.perf_counter()
    for _ in range(steps):
        once()
    torch.cuda.synchronize(dev)
    el = (time.perf_counter() - t) / steps
    stg = eng.stage_times()
    out["tx_signatures"] = {"value": round(tb.n / el, 1), "unit": "sigs/s", "ms_per_step": round(el * 1e3, 3),
                            "path": "cg_verify_tx_signatures_device, one call per step",
                            "stages": stage_summary(stg, steps),
                            "verdicts_equal_headline": bool(np.array_equal(sd.cpu().numpy(), st_ref))}
    del kd, ijd, sgd, ad, sd
    torch.cuda.empty_cache()
    return out


def table_modes(b, schemes):
    """Items per key-table mode (keyws.h thresholds on the exact use counts): row 0 (< 3 uses),
    quarter (3 .. 31), full (32 .. wide threshold), wide (>= 1536 Ed25519 / 512 ECDSA uses, up to
    the pool cap). The library decides on its own (sampled) counts, so this is the intended split."""
    uses = np.bincount(b.items["key_idx"], minlength=len(b.keys))
    thr = np.array([KEY_WIDE_MIN_USES.get(int(s), 1 << 30) for s in b.keys["scheme"]])
    ku = uses[b.items["key_idx"]]
    kt = thr[b.items["key_idx"]]
    out = {}
    for name, sel in (("ed25519", schemes == 4), ("secp256r1", schemes == 3), ("secp256k1", schemes == 2)):
        out[name] = {"row0": int((sel & (ku < KEY_QUARTER_MIN_USES)).sum()),
                     "quarter": int((sel & (ku >= KEY_QUARTER_MIN_USES) & (ku < KEY_FULL_MIN_USES)).sum()),
                     "full": int((sel & (ku >= KEY_FULL_MIN_USES) & (ku < kt)).sum()),
                     "wide": int((sel & (ku >= kt)).sum())}
    out["keys_used"] = int((uses > 0).sum())
    out["max_uses"] = int(uses.max()) if uses.size else 0
    return out


def bench_key_dist(a, eng, dist, rank, threads, steps):
    """The headline call (cg_verify_tx_signatures, host arena -> host verdicts) on the headline
    shape with another key distribution: 'distinct' (every pool item its own key: 2^20 keys, each
    drawn ~12 times by the 12.5M-item stream) or 'zipf' (Zipf(1.1) over 2^20 keys: a few hot keys,
    a long tail). GeneratedLedger.kt:48-54 draws the signers per command."""
    from corda_amd import signable
    from tools.workload import wl
    t0 = time.time()
    pool, pl, ps = wl.notary_pool(a.pool, seed=a.seed + 7919 * rank + 17, nthreads=threads, sig_group=a.sigs_per_tx,
                                  key_dist=dist)
    ids, id_idx = wl.pool_ids(pool, len(signable.template(1, 4)[0]))
    idx = wl.tx_ordered_draws(pool.n, a.items, id_idx, seed=a.seed + 5)
    tb = wl.tx_sig_stream(pool, ps, idx, ids, id_idx, nthreads=threads)
    gen = time.time() - t0
    from corda_amd.batch import Batch
    modes = table_modes(Batch(pool.keys, pool.items[idx], pool.arena), ps[idx])
    pb = tb.packed() if a.txsig_table == 12 else None
    call = (lambda: eng.verify_tx_signatures_packed(pb)) if pb is not None else (lambda: eng.verify_tx_signatures(tb))
    call()
    eng.stage_times()
    t = time.perf_counter()
    for _ in range(steps):
        st = call()
    el = (time.perf_counter() - t) / steps
    stg = eng.stage_times()
    ver = check_verdicts(st, expected_verdicts(pl[idx], ps[idx]))
    return {"value": round(tb.n / el, 1), "unit": "sigs/s", "ms_per_call": round(el * 1e3, 3), "keys": len(pool.keys),
            "table_modes_items": modes, "stages": stage_summary(stg, steps), "verdicts": ver,
            "cg_stats_ms": {k: round(v, 3) for k, v in eng.last_stats.items() if k.startswith("ms_")},
            "gen_s": round(gen, 1)}


def bench_host(eng, b, st_dev, steps):
    """PCIe-inclusive message form: host arena -> host verdicts through cg_verify_batch on the
    headline shard with every SignableData materialised: keys, items and ~370 B per item copied,
    chunk k+1's copy overlapping chunk k."""
    st = eng.verify(b)
    t0 = time.perf_counter()
    for _ in range(steps):
        st = eng.verify(b)
    el = (time.perf_counter() - t0) / steps
    s = eng.last_stats
    return {"value": round(b.n / el, 1), "unit": "sigs/s", "items": b.n, "ms_per_call": round(el * 1e3, 3),
            "bytes_h2d": int(b.arena.size + b.items.nbytes + b.keys.nbytes),
            "h2d_GBps_effective": round((b.arena.size + b.items.nbytes) / el / 1e9, 1),
            "cg_stats_ms": {k: round(v, 3) for k, v in s.items() if k.startswith("ms_")},
            "verdicts_equal_headline": bool(np.array_equal(st, st_dev)),
            "path": "cg_verify_batch from pageable host memory, SignableData bytes materialised per signature"}


def main_pool(a):
    """The library's own multi-device form (one JVM process drives every GPU of the
    node): cg_pool_verify_tx_signatures over the slots in --pool-devices, contiguous equal shards of
    one signature table (--items per slot), each slot's H2D, verify and D2H on its own host thread.
    Prints the same JSON line; `value` = all slots' signatures / call time."""
    from corda_amd import signable
    from corda_amd.engine import EnginePool
    from tools.workload import wl
    devices = [int(x) for x in a.pool_devices.split(",") if x != ""]
    threads = host_threads(a.threads)
    n = a.items * len(devices)
    t0 = time.time()
    pool, pl, ps = wl.notary_pool(a.pool, ed_keys=a.ed_keys, ec_keys=a.ec_keys, msg_len=a.msg_len, seed=a.seed,
                                  nthreads=threads, sig_group=a.sigs_per_tx)
    ids, id_idx = wl.pool_ids(pool, len(signable.template(1, 4)[0]))
    idx = wl.tx_ordered_draws(pool.n, n, id_idx, seed=a.seed + 1)
    tb = wl.tx_sig_stream(pool, ps, idx, ids, id_idx, nthreads=threads)
    gen_s = time.time() - t0
    pb = tb.packed() if a.txsig_table == 12 else None
    with EnginePool(devices, chunk_items=a.chunk_items) as ep:
        call = (lambda: ep.verify_tx_signatures_packed(pb)) if pb is not None else (lambda: ep.verify_tx_signatures(tb))
        for _ in range(a.warmup):
            st = call()
        t = time.perf_counter()
        for _ in range(a.steps):
            st = call()
        el = (time.perf_counter() - t) / a.steps
        stats = dict(ep.last_stats)
    ver = check_verdicts(st, expected_verdicts(pl[idx], ps[idx]))
    line = {"metric": METRIC, "value": round(n / el, 1), "unit": "sigs/s", "n_gpus": len(set(devices)),
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(el * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32", "data": "synthetic (as the headline)",
            "config": {"workload": f"BASELINE configs[4], whole node from one process: {a.items} signatures per slot "
                                   f"over slots {devices} through cg_pool_verify_tx_signatures"
                                   + ("_packed" if pb is not None else ""),
                       "items": n, "parallelism": f"cg_pool{len(devices)}"},
            "pool_stats": stats, "verdicts": ver, "gen_s": round(gen_s, 1)}
    print(json.dumps(line), flush=True)
    if ver["label_mismatches"] or ver["not_run"]:
        sys.exit(3)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    a = parse(argv)
    if a.pool_devices:
        return main_pool(a)
    # decide the world before any GPU call, and before torch is imported: the device count comes
    # from the KFD topology in sysfs (no HIP / HSA call), so the launcher never initialises the GPU
    visible = kfd_gpus() if "WORLD_SIZE" not in os.environ else a.gpus
    how, world = launch_plan(a.gpus, os.environ, visible)
    if how == "spawn":
        sys.exit(spawn_world(world, argv))
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    # this rank's share of the host: the CPU quota / the ranks on the node (the engine's scans and
    # the workload generator both use it)
    threads = rank_host_threads(a.threads)

    from corda_amd import shard
    from corda_amd.engine import Engine
    from tools.workload import wl

    # ---- this rank's shard (outside the timed region)
    t0 = time.time()
    from corda_amd import signable
    pool, pool_labels, pool_schemes = wl.notary_pool(a.pool, ed_keys=a.ed_keys, ec_keys=a.ec_keys, msg_len=a.msg_len,
                                                     seed=a.seed + 7919 * rank, nthreads=threads,
                                                     sig_group=a.sigs_per_tx)
    ids, id_idx = wl.pool_ids(pool, len(signable.template(1, 4)[0]))
    draws = wl.tx_ordered_draws(pool.n, a.items, id_idx, seed=a.seed + 31 * rank + 1)
    batch, idx = wl.index_stream(pool, a.items, replicate=True, idx=draws)
    tb = wl.tx_sig_stream(pool, pool_schemes, idx, ids, id_idx, nthreads=threads)
    labels, schemes = pool_labels[idx], pool_schemes[idx]
    gen_s = time.time() - t0
    # the engine's host threads: --engine-threads, else this rank's share when ranks share the node,
    # else 0 (the library's own budget: the CPU quota / the contexts in this process)
    eng_threads = a.engine_threads or (threads if world > 1 else 0)
    eng = Engine(local, chunk_items=a.chunk_items, stage_timing=True, host_threads=eng_threads)
    eng.reserve(len(batch.keys), batch.n)
    engs = [eng]
    if a.headline == "device":
        for _ in range(max(a.contexts, 1) - 1):
            e2 = Engine(local, chunk_items=a.chunk_items, stage_timing=True, host_threads=eng_threads)
            e2.reserve(len(batch.keys), batch.n)
            engs.append(e2)
    stream = torch.cuda.Stream(device=dev)
    torch.cuda.set_stream(stream)
    holder = {}
    # zero-copy ingestion: the caller's persistent buffers registered once, outside the timed region
    # (a JVM node registers its direct-buffer arena once; cg_host_register, include/cordagpu.h)
    registered, huge_maps = [], []
    if a.host_register < 0:
        a.host_register = register_advised()
    # the 12-byte table: the generator's arena tail is already the dense stream (a view, no copy)
    pb = tb.packed() if a.txsig_table == 12 else None
    if a.host_register and hasattr(_lib_mod().lib(), "cg_host_register"):
        if a.host_register == 2:  # the same bytes in 2 MB transparent huge pages first
            from corda_amd import batch as _B
            cp = {}
            for name in ("arena", "sigs", "ids"):
                cp[name], m = hugepage_copy(getattr(tb, name))
                huge_maps.append(m)
            tb = _B.TxSigBatch(tb.keys, cp["ids"], cp["sigs"], tb.tmpls, cp["arena"])
            pb = tb.packed() if a.txsig_table == 12 else None
        for arr in ((tb.arena, pb.sigs, pb.ids) if pb is not None else (tb.arena, tb.sigs, tb.ids)):
            if _lib_mod().host_register(arr):
                registered.append(arr)

    def host_step():
        # host arena -> host verdicts, one cg_verify_tx_signatures(_packed) call (synchronous)
        holder["st_host"] = eng.verify_tx_signatures_packed(pb) if pb is not None else eng.verify_tx_signatures(tb)
        if world > 1:  # RCCL all-gather of the per-GPU verdict vectors
            holder["all"] = shard.gather_verdicts(torch.from_numpy(holder["st_host"]).to(dev), world * tb.n, world)

    dbuf = {}
    if a.headline == "device":
        # inputs resident in HBM before the timed region starts: the key table, ids, signature table and
        # one arena with the key / template bytes and (12-byte table) the signature stream at a 16-B
        # aligned offset; verdicts stay in HBM (the all-gather at N > 1 reads them there)
        up = lambda x: torch.from_numpy(np.ascontiguousarray(x).view(np.uint8)).to(dev)  # noqa: E731
        if pb is not None:
            off = -(-pb.arena.size // 16) * 16
            har = np.zeros(off + pb.stream.size, np.uint8)
            har[:pb.arena.size] = pb.arena
            har[off:] = pb.stream
            dbuf.update(k=up(pb.keys), i=up(pb.ids), s=up(pb.sigs), a=up(har), off=off, alen=har.size)
            del har
        else:
            dbuf.update(k=up(tb.keys), i=up(tb.ids), s=up(tb.sigs), a=up(tb.arena), off=0, alen=tb.arena.size)
        dbuf["st"] = torch.full((tb.n,), 255, dtype=torch.uint8, device=dev)
        dbuf["sts"] = [dbuf["st"]] + [torch.full((tb.n,), 255, dtype=torch.uint8, device=dev) for _ in engs[1:]]
        torch.cuda.synchronize(dev)

    def device_step():
        d = dbuf
        k = holder.get("k", 0)
        holder["k"] = k + 1
        e, st_k = engs[k % len(engs)], d["sts"][k % len(engs)]
        # one context: on torch's stream (bridged to the context's); several: each on its own stream
        sp = stream.cuda_stream if len(engs) == 1 else 0
        if pb is not None:
            e.verify_tx_signatures_packed_device(d["k"].data_ptr(), len(pb.keys), d["i"].data_ptr(), pb.n_ids,
                                                 d["s"].data_ptr(), pb.n, d["off"], pb.stream.size, pb.tmpls,
                                                 d["a"].data_ptr(), d["alen"], st_k.data_ptr(), stream=sp)
        else:
            e.verify_tx_signatures_device(d["k"].data_ptr(), len(tb.keys), d["i"].data_ptr(), tb.n_ids,
                                          d["s"].data_ptr(), tb.n, tb.tmpls, d["a"].data_ptr(), d["alen"],
                                          st_k.data_ptr(), stream=sp)
        if world > 1:  # RCCL all-gather of the per-GPU verdict vectors, device to device
            if len(engs) > 1:
                torch.cuda.synchronize(dev)
            holder["all"] = shard.gather_verdicts(st_k, world * tb.n, world)

    def all_stage_times():
        out = {}
        for e in engs:
            for name, (ms, n) in e.stage_times().items():
                m0, n0 = out.get(name, (0.0, 0))
                out[name] = (m0 + ms, n0 + n)
        return out

    def timed(step, steps, warmup, host_stats):
        """W untimed steps, then K steps between a barrier + synchronize on both sides; the max over ranks."""
        for _ in range(warmup):
            step()
        torch.cuda.synchronize(dev)
        all_stage_times()  # drop the warmup's records
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        cg = []
        for _ in range(steps):
            step()
            if host_stats:
                cg.append(dict(eng.last_stats))
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        el = time.perf_counter() - t
        if world > 1:
            tt = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            el = float(tt.item())
        return el, all_stage_times(), cg

    h2h_steps = a.steps if a.h2h_steps < 0 else a.h2h_steps
    h2h = None
    if a.headline == "device":
        elapsed, stages, _ = timed(device_step, a.steps, a.warmup, False)
        st = dbuf["st"].cpu().numpy()
        for other in dbuf["sts"][1:]:  # every context's last verdicts agree
            if not np.array_equal(other.cpu().numpy(), st):
                st = np.full_like(st, 255)
        c2_steps = a.steps if a.ctx2_steps < 0 else a.ctx2_steps
        if len(engs) == 1 and c2_steps > 0:
            # two verifier contexts on the device, calls alternating (each on its own stream): a call's
            # key-table phase runs beside the other call's ladders. Reported, not the headline: the
            # overlap stretches every kernel's launch time, so the roofline would no longer be per kernel
            e2 = Engine(local, chunk_items=a.chunk_items, stage_timing=True, host_threads=eng_threads)
            e2.reserve(len(batch.keys), batch.n)
            engs.append(e2)
            dbuf["sts"].append(torch.full((tb.n,), 255, dtype=torch.uint8, device=dev))
            holder["k"] = 0
            el2, _, _ = timed(device_step, c2_steps, 2, False)
            same = all(np.array_equal(x.cpu().numpy(), st) for x in dbuf["sts"])
            holder["ctx2"] = {"value": round(a.items * world * c2_steps / el2, 1), "unit": "sigs/s",
                              "ms_per_step": round(el2 / c2_steps * 1e3, 3), "steps": c2_steps,
                              "verdicts_equal": bool(same)}
        if h2h_steps > 0:  # the same call shape from host buffers, PCIe-inclusive (never `value`)
            el_h, stg_h, cg_ms = timed(host_step, h2h_steps, 1, True)
            h2h = {"value": round(a.items * world * h2h_steps / el_h, 1), "unit": "sigs/s",
                   "ms_per_step": round(el_h / h2h_steps * 1e3, 3), "steps": h2h_steps,
                   "path": ("cg_verify_tx_signatures_packed" if pb is not None else "cg_verify_tx_signatures")
                   + ": host arena -> host verdicts (pageable or registered per --host-register)",
                   "stages": stage_summary(stg_h, h2h_steps),
                   "verdicts_equal_device": bool(np.array_equal(holder["st_host"], st))}
        for k in ("k", "i", "s", "a", "st", "sts"):
            dbuf.pop(k, None)
        for e in engs[1:]:
            e.close()
        torch.cuda.empty_cache()
    else:
        elapsed, stages, cg_ms = timed(host_step, a.steps, a.warmup, True)
        el_h, h2h_steps = elapsed, a.steps
        st = holder["st_host"]

    # ---- verdict checks: labels, and every draw of a pool item gets that item's verdict
    ver = check_verdicts(st, expected_verdicts(labels, schemes))
    per_pool = np.full(pool.n, 255, np.uint8)
    per_pool[idx] = st
    ver["draws_consistent"] = bool(np.array_equal(per_pool[idx], st))
    if world > 1:  # every rank's verdicts are checked; rank 0 reports the worst
        bad = torch.tensor([ver["label_mismatches"] + ver["not_run"] + (0 if ver["draws_consistent"] else 1)],
                           dtype=torch.int64, device=dev)
        dist.all_reduce(bad, op=dist.ReduceOp.SUM)
        ver["world_bad"] = int(bad.item())
        ver["gathered_not_run"] = int((holder["all"] == 255).sum().item())

    units = ladder_units(batch, labels, schemes, headline_chunk(a, batch.n))
    roof, ec_roof = roofline(stages, units, a.steps)
    if roof is not None:
        roof["i2p_equiv_TMAC32"] = round(roof["achieved"] * MAC32_PER_ED25519 / roof["work_per_item"], 3)
        roof["peak_source"] = PEAK_SOURCE
        roof["traffic"] = None
        if os.path.exists(TRAFFIC_FILE):
            with open(TRAFFIC_FILE) as f:
                tr = json.load(f)
            if tr.get("kernel_version") == KERNEL_VERSION and tr.get("items") == a.items:
                roof["traffic"] = tr.get("hbm_bytes_per_launch", {}).get(roof["kernel"])
                roof["traffic_source"] = tr.get("source")
                if "valu_issue" in tr:
                    roof["valu_issue"] = tr["valu_issue"]

    h2d_bytes = pb.h2d_bytes if pb is not None else int(tb.arena.size + tb.sigs.nbytes + tb.ids.nbytes + tb.keys.nbytes)
    extra = {"headline": a.headline, "stages": stage_summary(stages, a.steps), "ecdsa_ladders": ec_roof,
             "roofline_full": roof, "verdicts": ver, "gen_s": round(gen_s, 1), "host_to_host": h2h,
             "two_contexts": holder.get("ctx2")}
    if a.headline == "host" or h2h is not None:
        extra["headline_h2d"] = {
            "bytes_per_call": h2d_bytes, "bytes_per_sig": round(h2d_bytes / tb.n, 1),
            "GBps_effective": round(h2d_bytes * h2h_steps / el_h / 1e9, 1),
            "cg_stats_ms_mean": {k: round(float(np.mean([c[k] for c in cg_ms])), 3)
                                 for k in ("ms_key_prep", "ms_h2d", "ms_verify", "ms_d2h", "ms_total")},
            "note": "the host arena -> host verdicts calls: ms_key_prep = host-side planning (the key-use "
                    "count pass), ms_h2d = until the first chunk's bytes are resident, ms_verify = the rest"}
    extra["table_modes_items"] = table_modes(batch, schemes)
    extra["host"] = {"threads": threads, "engine_host_threads": eng_threads or "library budget",
                     "registered_bytes": int(sum(x.nbytes for x in registered)), "host_register": a.host_register,
                     "anon_huge_pages_kB": anon_huge_kb()}
    cpu = None
    if rank == 0 and world == 1:
        if a.device_steps > 0:
            guarded(extra, "device_resident", lambda: bench_device(eng, dev, stream, batch, tb, st, a.device_steps))
        if a.host_steps > 0:
            guarded(extra, "host_message_form", lambda: bench_host(eng, batch, st, a.host_steps))
        if not a.no_cpu_baseline:
            try:
                cpu = cpu_baseline(batch, st, a.cpu_seconds, threads)
                if a.configs0_txs > 0:
                    guarded(cpu, "configs0", lambda: configs0(a, eng, wl, threads))
            except Exception as e:  # noqa: BLE001
                cpu = {"error": f"{type(e).__name__}: {e}"}
        torch.cuda.empty_cache()
        for kd in [d for d in a.key_dists.split(",") if d]:
            guarded(extra, "key_dist_" + kd, lambda: bench_key_dist(a, eng, kd, rank, threads, 2))
            torch.cuda.empty_cache()
        for name, on, fn in (("configs1_ed25519", a.configs1_items, lambda: bench_configs1(a, eng, dev, stream, wl, threads)),
                             ("configs2_ecdsa", a.ecdsa_items, lambda: bench_ecdsa(a, eng, dev, stream, wl, threads)),
                             ("configs3_tx_pipeline", a.pipeline_txs,
                              lambda: bench_pipeline(a, eng, dev, stream, wl, threads)),
                             ("tear_offs", a.tear_offs, lambda: bench_tear_offs(a, eng, dev, stream, wl))):
            if on > 0:
                guarded(extra, name, fn)
                torch.cuda.empty_cache()

    failed = bool(ver["label_mismatches"] or ver["not_run"] or not ver["draws_consistent"] or ver.get("world_bad"))
    if rank == 0:
        total = a.items * world * a.steps
        n_ed, n_r1 = int((schemes == 4).sum()), int((schemes == 3).sum())
        head = {
            "metric": METRIC, "value": round(total / elapsed, 1), "unit": "sigs/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(elapsed / a.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic: seeded Ed25519 + ECDSA (secp256r1/k1) signatures over SignableData(txId, "
                    "SignatureMetadata(1, scheme)) with every Appendix A corruption class (tools/workload)",
            "config": {"workload": "BASELINE configs[4] per-GPU shard, whole node: notary-style mixed batch 70% "
                                   "Ed25519 / 20% secp256r1 / 10% secp256k1, one "
                                   + ("cg_verify_tx_signatures_packed" if pb is not None else "cg_verify_tx_signatures")
                                   + ("_device call per step, inputs resident in HBM when the timed region starts "
                                      "(keys, ids, signature table and stream, templates; verdicts left in HBM); "
                                      "host arena -> host verdicts (PCIe-inclusive) in summary.host_to_host"
                                      if a.headline == "device" else
                                      " call per step, host arena -> host verdicts (PCIe-inclusive)")
                                   + " (batch Crypto.doVerify(txId, sig))",
                       "boundary": a.headline, "contexts": max(a.contexts, 1) if a.headline == "device" else 1,
                       "items_per_gpu": a.items, "unique_pool": a.pool,
                       "mix": [n_ed, n_r1, a.items - n_ed - n_r1], "keys": len(batch.keys),
                       "sigs_per_tx": a.sigs_per_tx, "h2d_bytes_per_gpu": h2d_bytes, "txsig_table": a.txsig_table,
                       "parallelism": f"shard{world}" + ("+rccl_allgather(verdicts)" if world > 1 else "")},
        }
        summary = {"verdicts_checked": ver["checked_vs_labels"], "label_mismatches": ver["label_mismatches"],
                   "not_run": ver["not_run"], "draws_consistent": ver["draws_consistent"],
                   "secondary_file": os.path.relpath(a.secondary_out, ROOT) if a.secondary_out else None}
        if holder.get("ctx2"):
            summary["two_contexts"] = holder["ctx2"]["value"]
            summary["two_contexts_equal"] = holder["ctx2"]["verdicts_equal"]
        if h2h is not None:
            summary["host_to_host"] = h2h["value"]
            summary["host_to_host_ms"] = h2h["ms_per_step"]
            summary["host_verdicts_equal"] = h2h["verdicts_equal_device"]
        if ec_roof:
            summary["ecdsa_wide_frac"] = {c: (ec_roof.get(c + "_wide") or {}).get("frac") for c in ("secp256r1", "secp256k1")}
        for k in ("device_resident", "key_dist_distinct", "key_dist_zipf", "configs1_ed25519", "configs2_ecdsa",
                  "configs3_tx_pipeline", "tear_offs"):
            v = extra.get(k)
            if isinstance(v, dict):
                if k == "device_resident":
                    v = v.get("tx_signatures", {})
                summary[k] = v.get("value", v.get("error", "")[:80] if "error" in v else None)
        extra["cpu_baseline_full"] = cpu
        write_secondary(a.secondary_out, extra)
        print(compact_line(head, roof, cpu, summary), flush=True)
    if world > 1:
        dist.destroy_process_group()
    eng.close()
    for arr in registered:
        _lib_mod().host_unregister(arr)
    if failed:
        sys.exit(3)  # a wrong verdict voids the number


if __name__ == "__main__":
    main()
