"""Multi-device shard plan and failure handling (corda_amd/csrc/pool.h, cg_pool_verify_batch) on
the CPU: the library's own pool_run, with every slot verifying its shard through the C oracle and
failing on demand (tests/native/pool_test.cpp). The GPU form (two contexts on one device, a drill
fault) is tests/test_gpu_pool.py."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

import golden_io
from oracle import c_oracle

HERE = os.path.dirname(os.path.abspath(__file__))
# CG_SANITIZE=thread (tests/test_sanitizers.py): a -fsanitize=thread build of its own
TSAN = os.environ.get("CG_SANITIZE", "") == "thread"
SO = os.path.join(HERE, "native", "libpooltest%s.so" % ("_tsan" if TSAN else ""))
ORACLE_DIR = os.path.join(HERE, "..", "oracle", "c")


def build():
    src = os.path.join(HERE, "native", "pool_test.cpp")
    hdr = os.path.join(HERE, "..", "corda_amd", "csrc", "pool.h")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        c_oracle.lib()  # builds oracle/c if needed
        subprocess.check_call(["g++", "-O1", "-g", "-std=c++17", *(["-fsanitize=thread"] if TSAN else []), "-fPIC",
                               "-shared", "-o", SO, src,
                               f"-L{ORACLE_DIR}", "-loracle", f"-Wl,-rpath,{os.path.abspath(ORACLE_DIR)}",
                               "-lpthread"])


def _lib():
    build()
    L = ctypes.CDLL(SO)
    vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
    L.pt_pool_verify.argtypes = [vp, u32, vp, u64, vp, u64, u32, vp, u32, vp, u32, u32, u32, u32, vp, vp]
    L.pt_pool_verify.restype = ctypes.c_int
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


@pytest.fixture(scope="module")
def batch():
    items = golden_io.load("ed25519.json") + golden_io.load("ecdsa.json")
    b, exp, _ = golden_io.sig_batch(items)
    return b, exp


def _run(L, b, n_slots, healthy=None, fail_always=0, fail_once=0, fail_arg=0, probe_ok=0):
    st = np.full(b.n, 7, dtype=np.uint8)
    h = np.ones(n_slots, np.uint8) if healthy is None else np.array(healthy, np.uint8)
    calls = np.zeros(n_slots, np.uint32)
    rep = np.zeros(4, np.uint64)
    rc = L.pt_pool_verify(_p(b.keys), len(b.keys), _p(b.items), b.n, _p(b.arena), b.arena.size, 0, _p(st), n_slots,
                          _p(h), fail_always, fail_once, fail_arg, probe_ok, _p(calls), _p(rep))
    return rc, st, h, calls, rep


@pytest.mark.parametrize("n_slots", [1, 2, 3, 4, 8])
def test_shards_gather_equal_one_run(batch, n_slots):
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, n_slots)
    assert rc == 0
    assert np.array_equal(st, exp)
    assert list(calls) == [1] * n_slots and int(rep[0]) == n_slots and int(rep[1]) == 0 and int(rep[3]) == 0


def test_failed_slot_is_rerun_on_a_healthy_one(batch):
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 4, fail_always=0b0100)
    assert rc == 0 and np.array_equal(st, exp)
    assert list(h) == [1, 1, 0, 1]
    assert int(rep[1]) == 1 and int(rep[2]) == 1 and int(rep[3]) == 0
    assert calls[2] == 1 and int(calls.sum()) == 5


def test_transient_fault_partial_write_is_discarded(batch):
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 2, fail_once=0b01)
    assert rc == 0 and np.array_equal(st, exp)
    assert list(h) == [0, 1] and int(rep[1]) == 1


def test_more_failures_than_healthy_slots_run_in_passes(batch):
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 5, fail_always=0b01110)
    assert rc == 0 and np.array_equal(st, exp)
    assert list(h) == [1, 0, 0, 0, 1] and int(rep[1]) == 3 and int(rep[2]) == 3


def test_unhealthy_slots_are_skipped_next_call(batch):
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 3, healthy=[1, 0, 1])
    assert rc == 0 and np.array_equal(st, exp)
    assert calls[1] == 0 and int(rep[0]) == 2


def test_every_slot_failing_leaves_not_run(batch):
    L = _lib()
    b, _ = batch
    rc, st, h, calls, rep = _run(L, b, 3, fail_always=0b111)
    assert rc != 0
    assert np.all(st == 255) and int(rep[3]) == b.n and list(h) == [0, 0, 0]
    rc, st, _, calls, rep = _run(L, b, 2, healthy=[0, 0])
    assert rc != 0 and np.all(st == 255) and int(calls.sum()) == 0


def test_empty_batch(batch):
    L = _lib()
    b, _ = batch
    from corda_amd.batch import Batch
    e = Batch(b.keys, b.items[:0], b.arena)
    rc, st, _, calls, rep = _run(L, e, 2)
    assert rc == 0 and st.size == 0 and int(calls.sum()) == 0


def test_capacity_error_reruns_elsewhere_and_keeps_the_slot(batch):
    """A slot that cannot allocate (CG_ERR_NOMEM: e.g. another process holds its device's memory)
    hands its shard to another live slot and stays healthy: the call completes."""
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 3, fail_arg=0b010)
    assert rc == 0 and np.array_equal(st, exp)
    assert list(h) == [1, 1, 1] and int(rep[2]) == 0 and int(rep[1]) == 1 and calls[1] == 1
    rc, st, h, calls, rep = _run(L, b, 3)
    assert rc == 0 and np.array_equal(st, exp)


def test_capacity_error_on_every_slot_leaves_not_run(batch):
    """Only a shard every live slot refused stays CG_NOT_RUN, and the call returns CG_ERR_NOMEM;
    no slot is marked unhealthy for it (the device is fine)."""
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 3, fail_arg=0b111)
    assert rc == -3 and list(h) == [1, 1, 1] and int(rep[2]) == 0
    assert int(rep[3]) == b.n and np.all(st == 255) and list(calls) == [3, 3, 3]
    # two slots refuse: everything runs on the third
    rc, st, h, calls, rep = _run(L, b, 3, fail_arg=0b011)
    assert rc == 0 and np.array_equal(st, exp) and list(h) == [1, 1, 1]


def test_unhealthy_slot_rejoins_after_probe(batch):
    """An unhealthy slot is re-probed at the start of a call and rejoins the plan if it answers."""
    L = _lib()
    b, exp = batch
    rc, st, h, calls, rep = _run(L, b, 3, healthy=[1, 0, 0], probe_ok=0b010)
    assert rc == 0 and np.array_equal(st, exp)
    assert list(h) == [1, 1, 0] and calls[1] == 1 and calls[2] == 0 and int(rep[0]) == 2
