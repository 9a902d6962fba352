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
