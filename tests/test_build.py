"""The host-side native trees __graft_entry__.build() compiles still compile from the current lane
headers (the tests load prebuilt .so files, so a header change that breaks one of them would
otherwise surface only in build()). Syntax-only compiles into nothing: no artefact is replaced."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = "/opt/rocm/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG) and shutil.which("g++") is None, reason="no host C++ compiler")
def test_workload_generator_compiles():
    cxx = CLANG if os.path.exists(CLANG) else "g++"
    subprocess.run([cxx, "-fsyntax-only", "-std=c++17", "-march=x86-64-v3", "-Wno-unknown-pragmas",
                    os.path.join(ROOT, "tools", "workload", "workload.cpp")], check=True)


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_oracle_and_cpu_baseline_compile():
    for src in ("oracle/c/oracle.c", "oracle/c/ed25519_i2p.c", "oracle/c/ecdsa_bc.c", "oracle/c/sha2.c",
                "oracle/c/bn.c", "tools/cpu_baseline/ossl_check.c"):
        subprocess.run(["gcc", "-fsyntax-only", "-std=gnu11", os.path.join(ROOT, src)], check=True)


def _make_var(mk, name):
    """The value of `name = ...` in a Makefile (one line)."""
    import re
    m = re.search(rf"^{name}\s*=\s*(.*)$", mk, re.M)
    assert m, name
    return m.group(1).split()


def test_makefile_lists_every_header_the_library_includes():
    """every local header cordagpu.cpp and the .hip sources include is a
    dependency of their objects, so an edit to one rebuilds libcordagpu.so (build() would otherwise
    link a stale object)."""
    import re
    csrc = os.path.join(ROOT, "corda_amd", "csrc")
    mk = open(os.path.join(csrc, "Makefile")).read()
    hdrs = set(_make_var(mk, "HDRS"))
    cpp_hdrs = set(_make_var(mk, "CPP_HDRS"))
    rule = re.search(r"^build/cordagpu\.o:(.*)$", mk, re.M).group(1)
    assert "$(HDRS)" in rule and "$(CPP_HDRS)" in rule

    def local_includes(path, seen):
        for inc in re.findall(r'^\s*#include\s+"([^"]+)"', open(path).read(), re.M):
            full = os.path.normpath(os.path.join(os.path.dirname(path), inc))
            rel = os.path.relpath(full, csrc)
            if rel not in seen:
                seen.add(rel)
                local_includes(full, seen)
        return seen

    got = local_includes(os.path.join(csrc, "cordagpu.cpp"), set())
    assert got - hdrs - cpp_hdrs == set(), "cordagpu.o does not depend on: %s" % sorted(got - hdrs - cpp_hdrs)
    for src in ("verify.hip", "verify_ed.hip", "verify_ec.hip", "hash.hip", "txpipe.hip", "plan_sort.hip",
                "filtered.hip"):
        got = local_includes(os.path.join(csrc, src), set())
        assert got - hdrs == set(), f"{src}: missing from HDRS: {sorted(got - hdrs)}"
    # the radix builds: each variant object of each radix-dependent source
    assert set(_make_var(mk, "VARIANT_SRCS")) == {"verify", "verify_ed", "verify_ec", "plan_sort"}
    assert set(_make_var(mk, "VARIANTS")) == {"24", "22"}
