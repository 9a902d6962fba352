"""ctypes wrapper of tools/workload/libworkload.so: seeded synthetic batches in the
include/cordagpu.h layout (bench.py and the GPU parity tests). Not product, not oracle."""
import ctypes
import os

import numpy as np

from corda_amd.batch import ITEM_DTYPE, KEY_DTYPE, Batch

_SO = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libworkload.so")
_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            raise RuntimeError(f"workload generator not built: {_SO} (make -C tools/workload)")
        L = ctypes.CDLL(_SO)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.wl_ed25519_keys.argtypes = [u32, u64, u32, vp, vp, i32]
        L.wl_ed25519_keys.restype = i32
        L.wl_ed25519_items.argtypes = [u64, u32, vp, vp, u32, u32, u64, vp, vp, vp, vp, i32]
        L.wl_ed25519_arena_bytes.argtypes = [u64, u32, u32]
        L.wl_ed25519_arena_bytes.restype = u64
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


class signable_mode:
    """Context manager: items generated inside get SignableData clear data, pre || id || suf
    (pre, suf = corda_amd.signable.template(...)), `group` consecutive items sharing one 32-byte
    id derived from id_seed; msg_len must be len(pre) + 32 + len(suf)."""

    def __init__(self, pre, suf, group=4, id_seed=0):
        self.pre, self.suf, self.group, self.id_seed = bytes(pre), bytes(suf), group, id_seed

    def __enter__(self):
        L = lib()
        L.wl_set_signable.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32,
                                      ctypes.c_uint32, ctypes.c_uint64]
        L.wl_set_signable(self.pre, len(self.pre), self.suf, len(self.suf), self.group, self.id_seed)
        return self

    def __exit__(self, *exc):
        lib().wl_set_signable(None, 0, None, 0, 1, 0)


def ed25519_batch(n_items, n_keys=4096, msg_len=270, corrupt_permille=120, seed=1, bad_key_every=0, nthreads=8):
    """Config 2 shape: n_items Ed25519 items over n_keys keys, ~msg_len-byte
    messages, corrupt_permille/1000 corrupted across classes A1-A7. Returns (Batch, labels)."""
    L = lib()
    seeds = np.zeros(32 * n_keys, dtype=np.uint8)
    pubs = np.zeros(32 * n_keys, dtype=np.uint8)
    L.wl_ed25519_keys(n_keys, seed, bad_key_every, _p(seeds), _p(pubs), nthreads)
    arena = np.zeros(int(L.wl_ed25519_arena_bytes(n_items, n_keys, msg_len)), dtype=np.uint8)
    keys = np.zeros(n_keys, dtype=KEY_DTYPE)
    items = np.zeros(n_items, dtype=ITEM_DTYPE)
    labels = np.zeros(n_items, dtype=np.uint8)
    L.wl_ed25519_items(n_items, n_keys, _p(seeds), _p(pubs), msg_len, corrupt_permille, seed, _p(arena), _p(keys),
                       _p(items), _p(labels), nthreads)
    return Batch(keys, items, arena), labels


def ecdsa_batch(curve, n_items, n_keys=2048, msg_len=270, corrupt_permille=100, seed=2, nthreads=8):
    """Config 3 shape: ECDSA over secp256k1 (curve 0, scheme 2) or secp256r1 (curve 1,
    scheme 3), DER signatures, corruption classes E1/E2/E3/E5/E6/E7. Returns (Batch, labels)."""
    L = lib()
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.wl_ecdsa_keys.argtypes = [i32, u32, u64, vp, vp, i32]
    L.wl_ecdsa_items.argtypes = [i32, u64, u32, vp, vp, u32, u32, u64, vp, vp, vp, vp, i32]
    L.wl_ecdsa_arena_bytes.argtypes = [u64, u32, u32]
    L.wl_ecdsa_arena_bytes.restype = u64
    ds = np.zeros(32 * n_keys, dtype=np.uint8)
    pubs = np.zeros(64 * n_keys, dtype=np.uint8)
    L.wl_ecdsa_keys(curve, n_keys, seed, _p(ds), _p(pubs), nthreads)
    arena = np.zeros(int(L.wl_ecdsa_arena_bytes(n_items, n_keys, msg_len)), dtype=np.uint8)
    keys = np.zeros(n_keys, dtype=KEY_DTYPE)
    items = np.zeros(n_items, dtype=ITEM_DTYPE)
    labels = np.zeros(n_items, dtype=np.uint8)
    L.wl_ecdsa_items(curve, n_items, n_keys, _p(ds), _p(pubs), msg_len, corrupt_permille, seed, _p(arena), _p(keys),
                     _p(items), _p(labels), nthreads)
    return Batch(keys, items, arena), labels


def concat(batches, shuffle_seed=None):
    """One batch from several (keys/items re-based into one arena); optional item shuffle.
    Returns (Batch, perm) where perm[j] = index of item j in the concatenation order."""
    arenas, keys, items = [], [], []
    a_off, k_off = 0, 0
    for b in batches:
        pad = (-a_off) % 16
        if pad:
            arenas.append(np.zeros(pad, dtype=np.uint8))
            a_off += pad
        k = b.keys.copy()
        k["off"] += a_off
        it = b.items.copy()
        it["sig_off"] += a_off
        it["msg_off"] += a_off
        it["key_idx"] += k_off
        arenas.append(b.arena)
        keys.append(k)
        items.append(it)
        a_off += b.arena.size
        k_off += len(b.keys)
    keys = np.concatenate(keys)
    items = np.concatenate(items)
    perm = np.arange(len(items))
    if shuffle_seed is not None:
        perm = np.random.default_rng(shuffle_seed).permutation(len(items))
        items = items[perm]
    return Batch(keys, items, np.concatenate(arenas + [np.zeros(64, dtype=np.uint8)])), perm


class key_choice:
    """Context manager: items generated inside sign with key k[i] instead of a uniform draw."""

    def __init__(self, k):
        self.k = None if k is None else np.ascontiguousarray(k, dtype=np.uint32)

    def __enter__(self):
        L = lib()
        L.wl_set_key_choice.argtypes = [ctypes.c_void_p, ctypes.c_uint64]
        if self.k is not None:
            L.wl_set_key_choice(_p(self.k), self.k.size)
        return self

    def __exit__(self, *exc):
        lib().wl_set_key_choice(None, 0)


def _key_draw(dist, n_items, n_keys, seed):
    """Key index per item: 'uniform' (None: the generator's own draw), 'distinct' (item i -> key i),
    'zipf' (Zipf(s = 1.1) over n_keys, rank 0 the hottest)."""
    if dist == "uniform":
        return None
    if dist == "distinct":
        return np.arange(n_items, dtype=np.uint32) % n_keys
    if dist == "zipf":
        w = 1.0 / np.arange(1, n_keys + 1, dtype=np.float64) ** 1.1
        c = np.cumsum(w)
        u = np.random.default_rng(seed).random(n_items) * c[-1]
        return np.minimum(np.searchsorted(c, u), n_keys - 1).astype(np.uint32)
    raise ValueError(dist)


def _signable_or_not(sig_group, scheme, seed):
    if not sig_group:
        import contextlib
        return contextlib.nullcontext()
    from corda_amd import signable
    pre, suf = signable.template(1, scheme)
    return signable_mode(pre, suf, sig_group, id_seed=(seed * 0x9E3779B1 + scheme) & (2 ** 64 - 1))


def notary_pool(n_unique, ed_keys=4096, ec_keys=1024, msg_len=270, seed=9, nthreads=8,
                mix=(0.7, 0.2, 0.1), ed_corrupt_permille=120, ec_corrupt_permille=100, sig_group=0,
                key_dist="uniform"):
    """BASELINE configs[4]'s unique pool: n_unique items, 70% Ed25519 /
    20% secp256r1 / 10% secp256k1 by default, every corruption class of Appendix A, shuffled.
    sig_group > 0: every item's clear data is SignableData(id, SignatureMetadata(1, scheme)), groups
    of sig_group items of one scheme signing one id (msg_len is then the template's, 269 bytes).
    key_dist: 'uniform' (ed_keys / ec_keys keys drawn uniformly), 'distinct' (ed_keys / ec_keys are
    ignored: every item its own key) or 'zipf' (Zipf(1.1) over as many keys as the part has items).
    Returns (Batch, labels, scheme_of_item)."""
    ne = int(n_unique * mix[0])
    nr = int(n_unique * mix[1])
    nk = n_unique - ne - nr
    if sig_group:
        from corda_amd import signable
        pre, suf = signable.template(1, 4)
        msg_len = len(pre) + 32 + len(suf)
    parts, labs, sch = [], [], []
    if key_dist != "uniform":
        ed_keys, ec_keys = max(1, ne), max(1, nr, nk)
    if ne:
        with _signable_or_not(sig_group, 4, seed), key_choice(_key_draw(key_dist, ne, ed_keys, seed + 11)):
            e, le = ed25519_batch(ne, n_keys=ed_keys, msg_len=msg_len, corrupt_permille=ed_corrupt_permille, seed=seed,
                                  nthreads=nthreads)
        parts.append(e), labs.append(le), sch.append(np.full(ne, 4, np.uint8))
    for curve, cnt, scheme in ((1, nr, 3), (0, nk, 2)):
        if cnt:
            nkc = cnt if key_dist != "uniform" else ec_keys
            with _signable_or_not(sig_group, scheme, seed), key_choice(_key_draw(key_dist, cnt, nkc, seed + 13 + curve)):
                b, lb = ecdsa_batch(curve, cnt, n_keys=nkc, msg_len=msg_len, corrupt_permille=ec_corrupt_permille,
                                    seed=seed + 1 + curve, nthreads=nthreads)
            parts.append(b), labs.append(lb), sch.append(np.full(cnt, scheme, np.uint8))
    b, perm = concat(parts, shuffle_seed=seed + 7)
    return b, np.concatenate(labs)[perm], np.concatenate(sch)[perm]


def tx_ordered_draws(pool_n, n_items, id_idx, seed):
    """The index stream's draws (as index_stream draws them), reordered so that within each pass over
    the pool (draw i belongs to copy i // pool_n) the signatures of one transaction id are adjacent:
    the layout a caller of cg_verify_tx_signatures produces when it lists each transaction's
    signatures together (TransactionWithSignatures.checkSignaturesAreValid walks one tx at a time)."""
    idx = np.random.default_rng(seed).integers(0, pool_n, n_items)
    copy = np.arange(n_items, dtype=np.int64) // pool_n
    return idx[np.lexsort((id_idx[idx], copy))]


def index_stream(pool, n_items, seed=10, replicate=False, idx=None):
    """n_items items drawn from `pool` by a seeded index stream (the engine sees every draw as
    its own item: nothing is deduplicated). replicate=False: the items point into the pool's
    arena. replicate=True: the arena holds one physical copy of the pool per 2^k draws, item i
    pointing into copy i // len(pool), so every item has its own bytes and a host-buffer call
    moves ~370 B per item over PCIe, as a real notary batch would. Returns (Batch, pool_index)."""
    if idx is None:
        idx = np.random.default_rng(seed).integers(0, pool.n, n_items)
    items = pool.items[idx]
    arena = pool.arena
    if replicate:
        n_copies = (n_items + pool.n - 1) // pool.n
        step = (pool.arena.size + 15) & ~15
        arena = np.zeros(step * n_copies + 64, np.uint8)
        for c in range(n_copies):
            arena[c * step:c * step + pool.arena.size] = pool.arena
        copy = (np.arange(n_items, dtype=np.uint64) // np.uint64(pool.n)) * np.uint64(step)
        items["sig_off"] += copy
        items["msg_off"] += copy
        # keys stay in copy 0 (key table offsets unchanged)
    return Batch(pool.keys, items, arena), idx


def pool_ids(pool, pre_len):
    """The distinct 32-byte ids inside a signable pool's messages: (ids [m, 32], id index per item)."""
    rows = pool.arena[pool.items["msg_off"].astype(np.int64)[:, None] + pre_len + np.arange(32)]
    v = np.ascontiguousarray(rows).view(np.dtype((np.void, 32))).reshape(-1)
    uniq, inv = np.unique(v, return_inverse=True)
    return np.frombuffer(uniq.tobytes(), np.uint8).reshape(-1, 32), inv.astype(np.uint32)


def tx_sig_stream(pool, schemes, idx, ids, id_idx, nthreads=8):
    """The index stream `idx` over a signable pool, as cg_verify_tx_signatures input (the form a
    JVM caller of checkSignaturesAreValid holds: tx id + TransactionSignature): a compact arena of
    key bytes, the three SignatureMetadata(1, scheme) templates and every drawn item's own copy of
    its signature bytes; one id table copy per pass over the pool (draw i of copy i // pool.n),
    so no two items share bytes unless they share a transaction. Returns batch.TxSigBatch."""
    from corda_amd import signable
    from corda_amd.batch import KEY_DTYPE, TMPL_DTYPE, TXSIG_DTYPE, TxSigBatch
    L = lib()
    vp, u64, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
    L.wl_gather.argtypes = [vp, vp, vp, u64, vp, vp, i32]
    n, m = len(idx), len(ids)
    al4 = lambda x: (x.astype(np.uint64) + np.uint64(3)) & ~np.uint64(3)  # noqa: E731
    # keys
    keys = pool.keys.copy()
    klen = keys["len"].astype(np.uint16)
    koff = np.concatenate([[0], np.cumsum(al4(klen))[:-1]]).astype(np.uint64)
    kend = int(koff[-1] + al4(klen[-1:])[0]) if len(keys) else 0
    # templates, one per scheme id (2, 3, 4) -> index scheme - 2
    parts, tmpls, off = [], np.zeros(3, TMPL_DTYPE), (kend + 15) & ~15
    for j, sch in enumerate((2, 3, 4)):
        pre, suf = signable.template(1, sch)
        tmpls[j] = (off, off + len(pre), len(pre), len(suf))
        parts.append((off, pre + suf))
        off += (len(pre) + len(suf) + 3) & ~3
    sig_base = (off + 15) & ~15
    it = pool.items[idx]
    slen = it["sig_len"].astype(np.uint16)
    soff = np.uint64(sig_base) + np.concatenate([[0], np.cumsum(al4(slen))[:-1]]).astype(np.uint64)
    total = int(soff[-1] + al4(slen[-1:])[0]) if n else sig_base
    arena = np.zeros(total + 64, np.uint8)
    L.wl_gather(_p(pool.arena), _p(np.ascontiguousarray(keys["off"])), _p(klen), len(keys), _p(arena), _p(koff), nthreads)
    keys["off"] = koff
    for o, b in parts:
        arena[o:o + len(b)] = np.frombuffer(b, np.uint8)
    src = np.ascontiguousarray(it["sig_off"])
    L.wl_gather(_p(pool.arena), _p(src), _p(slen), n, _p(arena), _p(soff), nthreads)
    n_copies = max(1, -(-n // pool.n))
    sigs = np.zeros(n, TXSIG_DTYPE)
    sigs["sig_off"] = soff
    sigs["sig_len"] = slen
    sigs["key_idx"] = it["key_idx"]
    sigs["tx_idx"] = id_idx[idx].astype(np.uint64) + (np.arange(n, dtype=np.uint64) // np.uint64(pool.n)) * np.uint64(m)
    sigs["tmpl"] = schemes[idx].astype(np.uint16) - 2
    return TxSigBatch(keys, np.tile(ids.reshape(-1), n_copies), sigs, tmpls, arena)


class TxPipeline:
    """A packed config-4 workload: WireTransactions + their signatures (include/cordagpu.h
    layouts) and the generator's own tx ids and corruption labels."""

    def __init__(self, txs, comps, keys, sigs, tmpls, arena, ids, labels):
        self.txs, self.comps, self.keys, self.sigs, self.tmpls, self.arena = txs, comps, keys, sigs, tmpls, arena
        self.ids, self.labels = ids, labels


def tx_pipeline(n_tx, n_keys=1024, seed=4, corrupt_permille=20, nthreads=8, comp_len=(80, 600)):
    """Config 4 shape: n_tx WireTransactions with 1+Poisson(1) inputs,
    Poisson(3) outputs, 1+Poisson(3) commands, a notary and the privacy-salt leaf (~11
    components), component blobs uniform in comp_len bytes; one Ed25519 signature per command
    (random signer among keys 1..n_keys-1) plus the notary's (key 0), each over
    SignableData(id, SignatureMetadata(1, 4)) (corda_amd/signable.py template)."""
    from corda_amd import signable
    from corda_amd.batch import COMPONENT_DTYPE, KEY_DTYPE, TMPL_DTYPE, TX_DTYPE, TXSIG_DTYPE
    L = lib()
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    L.wl_tx_sign.argtypes = [u64, vp, vp, vp, u64, u64, vp, vp, vp, vp, u32, vp, u32, u32, u64, vp, vp, i32]
    rng = np.random.default_rng(seed)
    n_in = 1 + rng.poisson(1, n_tx)
    n_out = rng.poisson(3, n_tx)
    n_cmd = 1 + rng.poisson(3, n_tx)
    ncomp = (n_in + n_out + n_cmd + 2).astype(np.int64)  # + notary + salt leaf
    first = np.concatenate([[0], np.cumsum(ncomp)[:-1]])
    total = int(ncomp.sum())
    lens = rng.integers(comp_len[0], comp_len[1] + 1, total).astype(np.int64)
    is_salt = np.zeros(total, dtype=bool)
    is_salt[first + ncomp - 1] = True
    lens[is_salt] = 40
    pre, suf = signable.template(1, 4)
    # arena: [keys][template][components][salts][signatures]
    key_base = 0
    tmpl_base = 32 * n_keys
    comp_base = (tmpl_base + len(pre) + len(suf) + 3 + 15) & ~15
    aligned = (lens + 3) & ~3
    comp_off = comp_base + np.concatenate([[0], np.cumsum(aligned)[:-1]])
    salt_base = int(comp_base + aligned.sum())
    n_sig_tx = n_cmd + 1
    n_sigs = int(n_sig_tx.sum())
    sig_base = salt_base + 32 * n_tx
    arena_len = sig_base + 64 * n_sigs
    arena = np.zeros(arena_len + 64, dtype=np.uint8)
    body = salt_base - comp_base
    arena[comp_base:salt_base] = np.random.default_rng(seed + 1).integers(
        0, 2 ** 63, (body + 7) // 8, dtype=np.int64).view(np.uint8)[:body]
    arena[salt_base:sig_base] = rng.integers(0, 256, 32 * n_tx, dtype=np.uint8)
    arena[tmpl_base:tmpl_base + len(pre)] = np.frombuffer(pre, np.uint8)
    arena[tmpl_base + len(pre):tmpl_base + len(pre) + len(suf)] = np.frombuffer(suf, np.uint8)
    comps = np.zeros(total, dtype=COMPONENT_DTYPE)
    comps["off"] = comp_off
    comps["len"] = lens
    comps["flags"] = is_salt.astype(np.uint32)
    txs = np.zeros(n_tx, dtype=TX_DTYPE)
    txs["first"] = first
    txs["n"] = ncomp
    txs["salt_off"] = salt_base + 32 * np.arange(n_tx)
    seeds = np.zeros(32 * n_keys, dtype=np.uint8)
    pubs = np.zeros(32 * n_keys, dtype=np.uint8)
    L.wl_ed25519_keys(n_keys, seed, 0, _p(seeds), _p(pubs), nthreads)
    arena[key_base:key_base + 32 * n_keys] = pubs
    keys = np.zeros(n_keys, dtype=KEY_DTYPE)
    keys["off"] = 32 * np.arange(n_keys)
    keys["len"] = 32
    keys["scheme"] = 4
    sigs = np.zeros(n_sigs, dtype=TXSIG_DTYPE)
    sigs["tx_idx"] = np.repeat(np.arange(n_tx), n_sig_tx)
    signer = rng.integers(1, max(2, n_keys), n_sigs)
    last = np.cumsum(n_sig_tx) - 1
    signer[last] = 0  # the notary signs last
    sigs["key_idx"] = signer
    sigs["sig_off"] = sig_base + 64 * np.arange(n_sigs)
    sigs["sig_len"] = 64
    tmpls = np.zeros(1, dtype=TMPL_DTYPE)
    tmpls[0] = (tmpl_base, tmpl_base + len(pre), len(pre), len(suf))
    ids = np.zeros(32 * n_tx, dtype=np.uint8)
    labels = np.zeros(n_sigs, dtype=np.uint8)
    L.wl_tx_sign(n_tx, _p(txs), _p(comps), _p(arena), arena_len, n_sigs, _p(sigs), _p(seeds), _p(pubs),
                 _p(arena[tmpl_base:]), len(pre), _p(arena[tmpl_base + len(pre):]), len(suf), corrupt_permille,
                 seed, _p(ids), _p(labels), nthreads)
    return TxPipeline(txs, comps, keys, sigs, tmpls, arena[:arena_len + 64], ids.reshape(-1, 32), labels)


def configs0(n_tx, seed=11, nthreads=8, n_keys=1024, corrupt_permille=20):
    """BASELINE configs[0]: n_tx SignedTransactions of the tx_pipeline shape, each signature's
    clear data materialised as SignableData(id, metadata) bytes (prefix || id || suffix), items of
    a transaction contiguous and in list order. Returns (Batch, tx_first [n_tx + 1], labels)."""
    from corda_amd.batch import ITEM_DTYPE
    w = tx_pipeline(n_tx, n_keys=n_keys, seed=seed, corrupt_permille=corrupt_permille, nthreads=nthreads)
    t = w.tmpls[0]
    pre = w.arena[int(t["prefix_off"]):int(t["prefix_off"]) + int(t["prefix_len"])]
    suf = w.arena[int(t["suffix_off"]):int(t["suffix_off"]) + int(t["suffix_len"])]
    mlen = pre.size + 32 + suf.size
    stride = (64 + mlen + 3) & ~3
    n = len(w.sigs)
    kbytes = 32 * n_keys
    base = (kbytes + 15) & ~15
    rows = np.zeros((n, stride), np.uint8)
    so = w.sigs["sig_off"].astype(np.int64)
    rows[:, :64] = w.arena[so[:, None] + np.arange(64)]
    rows[:, 64:64 + pre.size] = pre
    rows[:, 64 + pre.size:64 + pre.size + 32] = w.ids[w.sigs["tx_idx"]]
    rows[:, 64 + pre.size + 32:64 + mlen] = suf
    arena = np.concatenate([w.arena[:kbytes], np.zeros(base - kbytes, np.uint8), rows.reshape(-1),
                            np.zeros(64, np.uint8)])
    items = np.zeros(n, ITEM_DTYPE)
    items["sig_off"] = base + stride * np.arange(n)
    items["msg_off"] = items["sig_off"] + 64
    items["msg_len"] = mlen
    items["key_idx"] = w.sigs["key_idx"]
    items["sig_len"] = 64
    tx_first = np.concatenate([[0], np.cumsum(np.bincount(w.sigs["tx_idx"], minlength=n_tx))]).astype(np.uint64)
    return Batch(w.keys, items, arena), tx_first, w.labels


class _Sha256Host:
    """hashlib stand-in for the engine when building bench inputs (tree node hashes)."""

    @staticmethod
    def sha256(msgs):
        import hashlib
        return [hashlib.sha256(bytes(m)).digest() for m in msgs]


def filtered_pool(n_unique, seed=5, comp_len=(80, 600), corrupt_permille=50):
    """Notary tear-offs (NonValidatingNotaryFlow.kt:22-27): WireTransactions of the
    config-4 shape (1+Poisson(1) inputs, Poisson(3) outputs, 1+Poisson(3) commands, notary, salt)
    filtered down to inputs + notary, as a non-validating notary receives them. Returns the list
    of corda_amd.merkle.FilteredTransaction and the expected status per tear-off (a corrupted
    one has a flipped bit in a visible component: status 1)."""
    import hashlib
    import struct
    from corda_amd import merkle as M
    rng = np.random.default_rng(seed)
    out, expect = [], []
    for _ in range(n_unique):
        n_in, n_out, n_cmd = 1 + rng.poisson(1), rng.poisson(3), 1 + rng.poisson(3)
        n = n_in + n_out + n_cmd + 1
        blobs = [rng.integers(0, 256, int(rng.integers(comp_len[0], comp_len[1] + 1)), dtype=np.uint8).tobytes()
                 for _ in range(n)]
        salt = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        nonces = [hashlib.sha256(salt + struct.pack(">i", i)).digest() for i in range(n)]
        hashes = [hashlib.sha256(b + x).digest() for b, x in zip(blobs, nonces)]
        hashes.append(hashlib.sha256(b"\x01" + salt).digest())
        full = M.merkle_tree(hashes, engine=_Sha256Host)
        vis = list(range(n_in)) + [n - 1]
        pmt = M.PartialMerkleTree.build(full, [hashes[i] for i in vis])
        vb = [blobs[i] for i in vis]
        bad = rng.integers(0, 1000) < corrupt_permille
        if bad:
            j = int(rng.integers(0, len(vb)))
            b = bytearray(vb[j])
            b[int(rng.integers(0, len(b)))] ^= 1
            vb[j] = bytes(b)
        out.append(M.FilteredTransaction(full.hash, vb, [nonces[i] for i in vis], pmt))
        expect.append(1 if bad else 0)
    return out, np.array(expect, dtype=np.uint8)
