"""The host-side budget for N GPUs, decided before any GPU call, on the CPU:

- corda_amd/csrc/host_budget.h through tests/native/host_budget_test.cpp: the cgroup v2 / v1 CPU
  quota parser (whole CPUs, bounded by the affinity mask) and the per-context thread budget
  (cg_config.host_threads, else CG_HOST_THREADS, else quota / contexts open; clamped to [1, 64]);
- bench.py's HIP-free launcher helpers: kfd_gpus() counts GPUs from the KFD sysfs topology and the
  visibility variables, gpu_initialised() looks for an open /dev/kfd, rank_host_threads() divides the
  quota among LOCAL_WORLD_SIZE ranks — and none of them initialises the GPU runtime.
"""
import ctypes
import os
import subprocess
import sys

import pytest

import bench

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "native", "libhostbudgettest.so")


def _lib():
    src = os.path.join(HERE, "native", "host_budget_test.cpp")
    hdr = os.path.join(HERE, "..", "corda_amd", "csrc", "host_budget.h")
    if not os.path.exists(SO) or os.path.getmtime(SO) < max(os.path.getmtime(src), os.path.getmtime(hdr)):
        subprocess.check_call(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-o", SO, src])
    L = ctypes.CDLL(SO)
    L.hb_quota_from.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_uint]
    L.hb_threads_for.argtypes = [ctypes.c_uint] * 4
    for f in (L.hb_quota_from, L.hb_threads_for, L.hb_quota, L.hb_max):
        f.restype = ctypes.c_uint
    return L


@pytest.mark.parametrize("cpu_max, v1, affinity, want", [
    (b"max 100000", None, 256, 256),        # no v2 limit: the affinity mask
    (b"1600000 100000", None, 256, 16),     # the GPU box: 16 CPUs of a 256-thread host
    (b"1600000 100000", None, 8, 8),        # affinity tighter than the quota
    (b"150000 100000", None, 64, 1),        # fractional quota rounds down ...
    (b"50000 100000", None, 64, 1),         # ... to at least one CPU
    (None, (b"400000", b"100000"), 64, 4),  # cgroup v1
    (None, (b"-1", b"100000"), 12, 12),     # v1 without a limit
    (None, None, 0, 1),                     # nothing known: one thread
])
def test_cpu_quota_parser(cpu_max, v1, affinity, want):
    q, p = v1 if v1 else (None, None)
    assert _lib().hb_quota_from(cpu_max, q, p, affinity) == want


@pytest.mark.parametrize("requested, env, quota, contexts, want", [
    (4, 9, 16, 1, 4),     # cg_config.host_threads wins
    (0, 9, 16, 1, 9),     # then CG_HOST_THREADS
    (0, 0, 16, 1, 16),    # one context: the whole quota
    (0, 0, 16, 8, 2),     # 8 contexts (a cg_pool over 8 GPUs) share it
    (0, 0, 16, 32, 1),    # never below one
    (0, 0, 0, 0, 1),      # degenerate inputs
    (0, 0, 256, 1, 64),   # clamped to kHostThreadsMax
    (500, 0, 16, 1, 64),
])
def test_thread_budget(requested, env, quota, contexts, want):
    L = _lib()
    assert L.hb_max() == 64
    assert L.hb_threads_for(requested, env, quota, contexts) == want


def test_quota_of_this_container_is_sane():
    q = _lib().hb_quota()
    assert 1 <= q <= (os.cpu_count() or 1)


def _node(root, i, gfx):
    d = root / str(i)
    d.mkdir(parents=True)
    (d / "properties").write_text(f"cpu_cores_count 0\ngfx_target_version {gfx}\nsimd_count 1024\n")


def test_kfd_gpu_count_from_sysfs(tmp_path):
    nodes = tmp_path / "nodes"
    _node(nodes, 0, 0)           # the CPU node
    for i in range(1, 9):
        _node(nodes, i, 90500)   # eight gfx950 GPUs
    assert bench.kfd_gpus(str(nodes), env={}) == 8
    assert bench.kfd_gpus(str(nodes), env={"HIP_VISIBLE_DEVICES": "0,1"}) == 2
    assert bench.kfd_gpus(str(nodes), env={"ROCR_VISIBLE_DEVICES": "3"}) == 1
    assert bench.kfd_gpus(str(nodes), env={"CUDA_VISIBLE_DEVICES": ""}) == 0
    assert bench.kfd_gpus(str(tmp_path / "absent"), env={}) == 0


def test_gpu_initialised_looks_for_an_open_kfd(tmp_path):
    fds = tmp_path / "fd"
    fds.mkdir()
    os.symlink("/dev/null", fds / "0")
    os.symlink("/tmp/x", fds / "1")
    assert not bench.gpu_initialised(str(fds))
    os.symlink("/dev/kfd", fds / "7")
    assert bench.gpu_initialised(str(fds))
    assert not bench.gpu_initialised(str(tmp_path / "absent"))


def test_rank_host_threads_divides_the_quota():
    full = bench.host_threads(0)
    assert bench.rank_host_threads(5, env={"LOCAL_WORLD_SIZE": "8"}) == 5
    assert bench.rank_host_threads(0, env={}) == full
    assert bench.rank_host_threads(0, env={"LOCAL_WORLD_SIZE": "2"}) == max(1, full // 2)
    assert bench.rank_host_threads(0, env={"LOCAL_WORLD_SIZE": str(4 * full)}) == 1


def test_launcher_helpers_do_not_initialise_the_gpu():
    """The device count and the budget come before any HIP call: in a fresh interpreter, importing
    bench (which imports torch lazily) and calling the helpers leaves /dev/kfd unopened."""
    code = ("import bench; bench.kfd_gpus(); bench.rank_host_threads(0); "
            "import sys; sys.exit(1 if bench.gpu_initialised() else 0)")
    r = subprocess.run([sys.executable, "-c", code], cwd=os.path.dirname(HERE), capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr


def test_host_register_rule_matches_library_and_bench():
    """the registration default depends on the contexts per node (host_budget.h
    host_register_advised, exported as cg_host_register_advised); bench.py's --host-register -1 mirrors
    it from LOCAL_WORLD_SIZE before any GPU call (profiles/r06/host8/summary.json has the A/B)."""
    import bench
    from corda_amd import _lib
    L = _lib.lib()
    for n in range(0, 17):
        assert L.cg_host_register_advised(n) == (1 if n >= 4 else 0), n
        assert bench.register_advised({"LOCAL_WORLD_SIZE": str(max(n, 1))}) == (1 if n >= 4 else 0), n
    assert bench.register_advised({}) == 0  # one process, one GPU: pageable
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "corda_amd", "csrc",
                            "host_budget.h")).read()
    assert "kHostRegisterMinContexts = 4" in src and bench.HOST_REGISTER_MIN_RANKS == 4
