"""The host thread pool of the tx-signature path (corda_amd/csrc/host_pool.h: the key-use count
pass and each chunk's extent scan run on it, cordagpu.cpp cg_verify_tx_signatures) on the CPU:
every part of a run executes exactly once and before run returns, for run sizes from 0 to many times
the thread count, with a pool of no workers, and with several threads sharing one pool
(tests/native/host_pool_test.cpp)."""
import ctypes
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
# CG_SANITIZE=thread (tests/test_sanitizers.py): a -fsanitize=thread build of its own
TSAN = os.environ.get("CG_SANITIZE", "") == "thread"
SO = os.path.join(HERE, "native", "libhostpooltest%s.so" % ("_tsan" if TSAN else ""))


def build():
    src = os.path.join(HERE, "native", "host_pool_test.cpp")
    hdr = os.path.join(HERE, "..", "corda_amd", "csrc", "host_pool.h")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", *(["-fsanitize=thread"] if TSAN else []), "-fPIC",
                               "-shared", "-o", SO, src, "-lpthread"])


def _lib():
    build()
    L = ctypes.CDLL(SO)
    L.hp_check.argtypes = [ctypes.c_uint32] * 3
    L.hp_check.restype = ctypes.c_uint64
    L.hp_threads.argtypes = [ctypes.c_uint32]
    L.hp_threads.restype = ctypes.c_uint32
    return L


@pytest.mark.parametrize("workers", [0, 1, 3, 15])
def test_every_part_once_before_return(workers):
    assert _lib().hp_check(workers, 200, 1) == 0


@pytest.mark.parametrize("callers", [2, 4])
def test_callers_sharing_a_pool_take_turns(callers):
    assert _lib().hp_check(7, 100, callers) == 0


def test_thread_count():
    L = _lib()
    assert L.hp_threads(0) == 1
    assert L.hp_threads(15) == 16
