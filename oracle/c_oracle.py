"""ctypes binding of the C oracle (oracle/c/liboracle.so). TEST INFRASTRUCTURE ONLY.

Used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg; never by the
product path. Build with ``make -C oracle/c`` (``__graft_entry__.build()`` does it).
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# CG_SANITIZE=address (tests/test_sanitizers.py): the -fsanitize=address,undefined build (make asan)
_SAN = os.environ.get("CG_SANITIZE", "") == "address"
_LIB_PATH = os.path.join(_HERE, "c", "liboracle_asan.so" if _SAN else "liboracle.so")
_lib = None


class Counters(ctypes.Structure):
    _fields_ = [("fe_mul", ctypes.c_uint64), ("fe_sq", ctypes.c_uint64), ("sc_mul", ctypes.c_uint64),
                ("sha256_blocks", ctypes.c_uint64), ("sha512_blocks", ctypes.c_uint64)]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            raise RuntimeError(f"C oracle not built: {_LIB_PATH} (run make -C oracle/c)")
        L = ctypes.CDLL(_LIB_PATH)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.or_verify_batch.argtypes = [vp, u32, vp, u64, vp, u64, u32, vp, i32]
        L.or_verify_batch.restype = i32
        L.or_merkle_root.argtypes = [vp, ctypes.c_size_t, vp]
        L.or_tx_ids_batch.argtypes = [vp, u64, vp, vp, vp, i32]
        L.or_sha256.argtypes = [vp, ctypes.c_size_t, vp]
        L.or_sha512.argtypes = [vp, ctypes.c_size_t, vp]
        L.or_counters_get.restype = Counters
        L.or_ed_slide_escapes.argtypes = [vp]
        L.or_ed_slide_escapes.restype = i32
        _lib = L
    return _lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None


def verify_batch(batch, mode=0, nthreads=0):
    st = np.full(batch.n, 255, dtype=np.uint8)
    lib().or_verify_batch(_ptr(batch.keys), len(batch.keys), _ptr(batch.items), batch.n, _ptr(batch.arena),
                          batch.arena.size, mode, _ptr(st), nthreads)
    return st


def counters_reset():
    lib().or_counters_reset()


def counters():
    c = lib().or_counters_get()
    return {k: getattr(c, k) for k, _ in Counters._fields_}


def sha256(b):
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    lib().or_sha256(_ptr(a), len(b), _ptr(out))
    return out.tobytes()


def sha512(b):
    a = np.frombuffer(bytes(b) + b"\0", dtype=np.uint8)
    out = np.zeros(64, dtype=np.uint8)
    lib().or_sha512(_ptr(a), len(b), _ptr(out))
    return out.tobytes()


def merkle_root(leaves):
    a = np.frombuffer(b"".join(leaves) + b"\0", dtype=np.uint8)
    out = np.zeros(32, dtype=np.uint8)
    r = lib().or_merkle_root(_ptr(a), len(leaves), _ptr(out))
    if r != 0:
        raise ValueError("Cannot calculate Merkle root on empty hash list.")
    return out.tobytes()


def tx_ids(txs, comps, arena, nthreads=0):
    out = np.zeros(32 * len(txs), dtype=np.uint8)
    lib().or_tx_ids_batch(_ptr(txs), len(txs), _ptr(comps), _ptr(arena), _ptr(out), nthreads)
    return out.reshape(-1, 32)


def slide_escapes(s32):
    a = np.frombuffer(bytes(s32), dtype=np.uint8).copy()
    return bool(lib().or_ed_slide_escapes(_ptr(a)))
