"""ctypes binding of libcordagpu.so (include/cordagpu.h).

The library is built in-tree (``make -C corda_amd/csrc`` or ``__graft_entry__.build()``)
and loaded from ``corda_amd/libcordagpu.so``. There is no fallback: if the library is
missing, or the device cannot run it, every entry point raises ``EngineUnavailable``.
"""
import ctypes
import os
import re
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
# CORDA_AMD_LIB: an alternative in-tree build (A/B kernel experiments on one GPU box)
LIB_PATH = os.environ.get("CORDA_AMD_LIB") or os.path.join(_HERE, "libcordagpu.so")
HEADER_PATH = os.path.join(os.path.dirname(_HERE), "include", "cordagpu.h")

_lib = None
_lock = threading.Lock()


class EngineUnavailable(RuntimeError):
    pass


class cg_stats(ctypes.Structure):
    _fields_ = [("n_items", ctypes.c_uint64), ("n_keys", ctypes.c_uint64), ("ms_h2d", ctypes.c_double),
                ("ms_key_prep", ctypes.c_double), ("ms_verify", ctypes.c_double), ("ms_d2h", ctypes.c_double),
                ("ms_total", ctypes.c_double)]


class cg_config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32), ("max_items", ctypes.c_uint64),
                ("max_arena", ctypes.c_uint64), ("chunk_items", ctypes.c_uint64), ("host_threads", ctypes.c_uint32),
                ("reserved0", ctypes.c_uint32), ("table_bytes_max", ctypes.c_uint64), ("reserved1", ctypes.c_uint64)]


class cg_info(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("fixed_base_bits", ctypes.c_uint32), ("table_bytes", ctypes.c_uint64),
                ("host_threads", ctypes.c_uint32), ("reserved", ctypes.c_uint32), ("chunk_items", ctypes.c_uint64)]


class cg_pool_stats(ctypes.Structure):
    _fields_ = [("shards", ctypes.c_uint32), ("reruns", ctypes.c_uint32), ("failed_slots", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("not_run", ctypes.c_uint64), ("ms_total", ctypes.c_double)]


ABI_VERSION = 2
FLAG_STAGE_TIMING = 1
STAGE_NAMES = ["plan", "ed_hash", "ed_ladder", "ed_ladder_row0", "ed_finish", "r1_front", "r1_ladder",
               "r1_ladder_row0", "k1_front", "k1_ladder", "k1_ladder_row0", "ed_ladder_wide", "r1_ladder_wide",
               "k1_ladder_wide"]


def declared_symbols():
    """Function names declared in include/cordagpu.h."""
    with open(HEADER_PATH) as f:
        src = f.read()
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\*?\s+\*?(cg_\w+)\s*\(", src, re.M)))


def lib():
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise EngineUnavailable(f"{LIB_PATH} not built (run __graft_entry__.build() or make -C corda_amd/csrc)")
            L = ctypes.CDLL(LIB_PATH)
            vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
            L.cg_abi_version.restype = i32
            L.cg_build_info.restype = ctypes.c_char_p
            L.cg_device_count.restype = i32
            L.cg_last_error.restype = ctypes.c_char_p
            L.cg_open.argtypes = [ctypes.POINTER(vp), ctypes.POINTER(cg_config)]
            L.cg_open.restype = i32
            L.cg_close.argtypes = [vp]
            L.cg_close.restype = None
            L.cg_reserve.argtypes = [vp, u32, u64]
            L.cg_verify_batch.argtypes = [vp, vp, u32, vp, u64, vp, u64, u32, vp, ctypes.POINTER(cg_stats)]
            L.cg_verify_batch_device.argtypes = [vp, vp, u32, vp, u64, vp, u64, u32, vp, vp]
            L.cg_prepare_keys_device.argtypes = [vp, vp, u32, vp, u64, vp]
            L.cg_prepare_keys_device.restype = i32
            L.cg_verify_items_device.argtypes = [vp, vp, u32, vp, u64, vp, u64, u32, vp, vp]
            L.cg_verify_items_device.restype = i32
            L.cg_sha256_batch.argtypes = [vp, vp, u64, vp, u64, vp]
            L.cg_sha512_batch.argtypes = [vp, vp, u64, vp, u64, vp]
            L.cg_sha256_batch_device.argtypes = [vp, vp, u64, vp, u64, vp, vp]
            L.cg_merkle_roots.argtypes = [vp, vp, vp, vp, u64, vp, vp]
            L.cg_tx_ids.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, vp]
            L.cg_tx_ids_device.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, vp, vp]
            L.cg_verify_transactions.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp, u64, vp, u32, vp, u64, u32, vp,
                                                 vp, vp]
            L.cg_verify_transactions_device.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp, u64, vp, u32, vp, u64,
                                                        u32, vp, vp, vp, vp]
            L.cg_verify_tx_signatures.argtypes = [vp, vp, u32, vp, u64, vp, u64, vp, u32, vp, u64, u32, vp,
                                                  ctypes.POINTER(cg_stats)]
            L.cg_verify_tx_signatures.restype = i32
            L.cg_verify_tx_signatures_device.argtypes = [vp, vp, u32, vp, u64, vp, u64, vp, u32, vp, u64, u32, vp, vp]
            L.cg_verify_tx_signatures_device.restype = i32
            L.cg_verify_filtered.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, u64, vp]
            L.cg_verify_filtered_device.argtypes = [vp, vp, u64, vp, u64, vp, u64, vp, u64, vp, vp]
            if hasattr(L, "cg_stage_times"):
                L.cg_stage_times.argtypes = [vp, vp, vp, u32]
                L.cg_stage_times.restype = i32
            if hasattr(L, "cg_host_register"):  # older builds (A/B variants) lack the registration
                L.cg_host_register.argtypes = [vp, u64]
                L.cg_host_register.restype = i32
                L.cg_host_unregister.argtypes = [vp]
                L.cg_host_unregister.restype = i32
                L.cg_host_registered.argtypes = [vp, u64]
                if hasattr(L, "cg_host_register_advised"):
                    L.cg_host_register_advised.argtypes = [u32]
                    L.cg_host_register_advised.restype = i32
                L.cg_host_registered.restype = i32
            pool = hasattr(L, "cg_pool_open")  # older builds (A/B variants) lack the pool
            if pool:
                L.cg_pool_open.argtypes = [ctypes.POINTER(vp), vp, u32, ctypes.POINTER(cg_config)]
                L.cg_pool_open.restype = i32
                L.cg_pool_close.argtypes = [vp]
                L.cg_pool_close.restype = None
                L.cg_pool_slots.argtypes = [vp]
                L.cg_pool_slots.restype = u32
                L.cg_pool_slot_healthy.argtypes = [vp, u32]
                L.cg_pool_slot_healthy.restype = i32
                L.cg_pool_verify_batch.argtypes = [vp, vp, u32, vp, u64, vp, u64, u32, vp, ctypes.POINTER(cg_pool_stats)]
                L.cg_pool_verify_batch.restype = i32
                L.cg_pool_verify_tx_signatures.argtypes = [vp, vp, u32, vp, u64, vp, u64, vp, u32, vp, u64, u32, vp,
                                                           ctypes.POINTER(cg_pool_stats)]
                L.cg_pool_verify_tx_signatures.restype = i32
                L.cg_pool_inject_fault.argtypes = [vp, u32, i32]
                L.cg_pool_inject_fault.restype = i32
                if hasattr(L, "cg_pool_verify_transactions"):
                    L.cg_pool_verify_transactions.argtypes = [vp, vp, u64, vp, u64, vp, u32, vp, u64, vp, u32, vp, u64,
                                                              u32, vp, vp, vp, ctypes.POINTER(cg_pool_stats)]
                    L.cg_pool_verify_transactions.restype = i32
            if hasattr(L, "cg_verify_tx_signatures_packed"):  # round 6: the 12-byte signature table
                L.cg_verify_tx_signatures_packed.argtypes = [vp, vp, u32, vp, u64, vp, u64, vp, u64, vp, u32, vp, u64,
                                                             u32, vp, ctypes.POINTER(cg_stats)]
                L.cg_verify_tx_signatures_packed.restype = i32
                L.cg_verify_tx_signatures_packed_device.argtypes = [vp, vp, u32, vp, u64, vp, u64, u64, u64, vp, u32,
                                                                    vp, u64, u32, vp, vp]
                L.cg_verify_tx_signatures_packed_device.restype = i32
                if pool:
                    L.cg_pool_verify_tx_signatures_packed.argtypes = [vp, vp, u32, vp, u64, vp, u64, vp, u64, vp, u32,
                                                                      vp, u64, u32, vp, ctypes.POINTER(cg_pool_stats)]
                    L.cg_pool_verify_tx_signatures_packed.restype = i32
            if hasattr(L, "cg_context_info"):  # round 6: the fixed-base table budget
                L.cg_context_info.argtypes = [vp, ctypes.POINTER(cg_info)]
                L.cg_context_info.restype = i32
                L.cg_table_bytes.argtypes = [u32]
                L.cg_table_bytes.restype = u64
                L.cg_table_choice.argtypes = [u64, u64]
                L.cg_table_choice.restype = u32
            for name in ("cg_verify_filtered", "cg_verify_filtered_device", "cg_verify_transactions", "cg_verify_transactions_device", "cg_reserve", "cg_verify_batch", "cg_verify_batch_device", "cg_sha256_batch",
                         "cg_sha512_batch", "cg_sha256_batch_device", "cg_merkle_roots", "cg_tx_ids",
                         "cg_tx_ids_device"):
                getattr(L, name).restype = i32
            _lib = L
        return _lib


def host_register(arr):
    """cg_host_register over a numpy array's bytes (kept alive and unchanged by the caller until
    host_unregister): the host entry points then copy out of it by DMA, without CPU staging."""
    if arr is None or arr.size == 0:
        return False
    check(lib().cg_host_register(arr.ctypes.data, arr.nbytes), "cg_host_register")
    return True


def host_unregister(arr):
    check(lib().cg_host_unregister(arr.ctypes.data), "cg_host_unregister")


def last_error():
    return lib().cg_last_error().decode(errors="replace")


def check(rc, what):
    if rc != 0:
        raise EngineUnavailable(f"{what} failed ({rc}): {last_error()}")
