"""Sanitizer runs of the host code (SURVEY §5 "race detection / sanitizers"), CPU
only -- no GPU sanitizer exists on this pool and none is asked for:

- ThreadSanitizer over the threaded host code: corda_amd/csrc/host_pool.h (the scans' thread pool,
  tests/native/host_pool_test.cpp) and corda_amd/csrc/pool.h (cg_pool's shard threads, re-runs and
  failure handling, tests/native/pool_test.cpp), each built with -fsanitize=thread and driven by its
  own CPU tests in a child Python with the TSan runtime preloaded;
- AddressSanitizer + UBSan over the lane code's host build (tests/native/host_kernels.cpp: the
  field, point, scalar and SHA code the kernels run, with FE_BOUNDS_CHECK) and the C oracle
  (oracle/c, `make asan`), driven by their golden-vector and big-integer tests.

A sanitizer report fails the child (halt_on_error) and its text fails the test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    if not p or not os.path.isabs(p) or not os.path.exists(p):
        pytest.skip(f"{name} not available")
    return p


def _build(mode, code):
    """Build the sanitized libraries in a child WITHOUT the sanitizer runtime preloaded (a preloaded
    runtime would also load into g++ / make and their children)."""
    env = dict(os.environ, CG_SANITIZE=mode)
    env.pop("LD_PRELOAD", None)
    subprocess.check_call([sys.executable, "-c", "import sys; sys.path.insert(0, 'tests'); " + code], cwd=ROOT, env=env,
                          timeout=600)


def _child(env_extra, args, timeout):
    env = dict(os.environ, **env_extra)
    env.pop("PYTEST_ADDOPTS", None)
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider", "-m", "not gpu", *args],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    return r.returncode, out


def test_thread_sanitizer_host_pools():
    _build("thread", "import test_host_pool as a, test_pool as b; from oracle import c_oracle; a.build(); b.build()")
    rc, out = _child({"CG_SANITIZE": "thread", "LD_PRELOAD": _runtime("libtsan.so"),
                      "TSAN_OPTIONS": "halt_on_error=1 exitcode=66 report_signal_unsafe=0"},
                     ["tests/test_host_pool.py", "tests/test_pool.py"], 600)
    assert "ThreadSanitizer" not in out, out[-4000:]
    assert rc == 0, out[-4000:]
    assert " passed" in out, out[-2000:]


def test_address_sanitizer_lane_code_and_oracle():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle", "c"), "asan"])
    _build("address", "import hostk; hostk.build_so()")
    preload = _runtime("libasan.so")
    rc, out = _child({"CG_SANITIZE": "address", "LD_PRELOAD": preload,
                      "ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=0",
                      "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"},
                     ["tests/test_host_kernels.py", "tests/test_oracle_golden.py",
                      # the slowest cases under ASan are left to the plain run (the rows-form ECDSA lane
                      # verify, the signed-digit B variant, the pure-Python oracle): the wide ECDSA
                      # lane verify, both madd forms and every Ed25519 lane verify stay in
                      "-k", "not executed_work and not wide_row_build and not three_pass and not "
                            "t_ecdsa_verify_rows and not signed and not python_oracle"], 900)
    for marker in ("AddressSanitizer", "runtime error:", "UndefinedBehaviorSanitizer"):
        assert marker not in out, out[-4000:]
    assert rc == 0, out[-4000:]
    assert " passed" in out, out[-2000:]
