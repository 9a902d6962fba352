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
