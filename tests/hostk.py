"""ctypes access to tests/native/libhostkernels.so (host build of the HIP lane code)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# CG_HOSTK_DEFS="-DFOO ...": extra defines for a variant's host build (its own .so)
DEFS = os.environ.get("CG_HOSTK_DEFS", "").split()
# CG_SANITIZE=address (tests/test_sanitizers.py): an -fsanitize=address,undefined build of its own
SAN = ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"] \
    if os.environ.get("CG_SANITIZE", "") == "address" else []
SO = os.path.join(HERE, "native", "libhostkernels%s%s.so" % ("_" + "_".join(d.lstrip("-D") for d in DEFS) if DEFS else "",
                                                            "_asan" if SAN else ""))
P = 2 ** 255 - 19
L = 2 ** 252 + 27742317777372353535851937790883648493
OFFS = [0, 26, 51, 77, 102, 128, 153, 179, 204, 230]


def build():
    build_so()
    return ctypes.CDLL(SO)


def build_so():
    src = os.path.join(HERE, "native", "host_kernels.cpp")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(
            os.path.getmtime(os.path.join(HERE, "..", "corda_amd", "csrc", f))
            for f in os.listdir(os.path.join(HERE, "..", "corda_amd", "csrc")) if f.endswith(".h")) or \
            os.path.getmtime(SO) < os.path.getmtime(src):
        tmp = f"{SO}.{os.getpid()}.tmp"  # build aside and rename: parallel test workers never load a partial .so
        subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", "-DFE_BOUNDS_CHECK", "-DFE_OP_COUNT", *DEFS, *SAN,
                               "-fPIC", "-shared", "-o", tmp, src])
        os.replace(tmp, SO)


_lib = None


def lib():
    global _lib
    if _lib is None:
        L = build()
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.t_ecdsa_verify_rows.argtypes = [i32, vp, u64, u64, u32, u32, u64, u32, u64, u64]
        L.t_ed_verify.argtypes = [vp, vp, vp, u64]
        L.t_sha512_prefix.argtypes = [vp, vp, u64, u64, vp]
        L.t_sha256_suffix.argtypes = [vp, u64, u64, vp, vp]
        L.t_ed_count_w6.argtypes = [vp, vp, vp, u64, vp]
        _lib = L
    return _lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def limbs_to_int(v):
    return sum(int(x) << o for x, o in zip(v, OFFS))


def int_to_limbs(x):
    out = []
    for i, o in enumerate(OFFS):
        w = 26 if i % 2 == 0 else 25
        out.append((x >> o) & ((1 << w) - 1))
    return np.array(out, dtype=np.uint32)


def words(b):
    return np.frombuffer(bytes(b), dtype="<u4").copy()
