"""The constant fixed-base tables' budget (corda_amd/csrc/table_budget.h), CPU
only: the C ABI's HIP-free cg_table_bytes / cg_table_choice against the rule include/cordagpu.h
documents for cg_config.table_bytes_max."""
import ctypes

import pytest

from corda_amd import _lib

G = 1 << 30
HEADROOM = 16 * G


@pytest.fixture(scope="module")
def L():
    return _lib.lib()


def test_table_sizes(L):
    """Ed25519 B at 128-B entries, each curve's G at 72-B entries, plus the radix-2^10 tables."""
    sizes = {b: L.cg_table_bytes(b) for b in (26, 24, 22)}
    small = 1.6e6 + 2 * 0.96e6  # the radix-2^10 tables every set carries
    for bits, rows in ((26, 10), (24, 11), (22, 12)):
        wide = rows * (1 << (bits - 1)) * (128 + 2 * 72)
        assert abs(sizes[bits] - wide - small) < 5e6, (bits, sizes[bits], wide)
    assert sizes[26] > sizes[24] > sizes[22] > 0
    assert 90e9 < sizes[26] < 92e9 and 24e9 < sizes[24] < 26e9 and 6e9 < sizes[22] < 7.5e9
    assert L.cg_table_bytes(20) == 0 and L.cg_table_bytes(0) == 0


def test_explicit_budget(L):
    s26, s24, s22 = (L.cg_table_bytes(b) for b in (26, 24, 22))
    for budget, want in ((s26, 26), (s26 - 1, 24), (s24, 24), (s24 - 1, 22), (s22, 22), (s22 - 1, 0),
                         (1 << 62, 26), (1, 0)):
        # an explicit budget ignores the device's free memory
        for free in (0, 1 << 40):
            assert L.cg_table_choice(budget, free) == want, (budget, free)


def test_automatic_choice_leaves_headroom(L):
    s26, s24, s22 = (L.cg_table_bytes(b) for b in (26, 24, 22))
    assert L.cg_table_choice(0, 287 * 10**9) == 26          # a fresh MI355X
    assert L.cg_table_choice(0, s26 + HEADROOM) == 26
    assert L.cg_table_choice(0, s26 + HEADROOM - 1) == 24
    assert L.cg_table_choice(0, s24 + HEADROOM) == 24
    assert L.cg_table_choice(0, s24 + HEADROOM - 1) == 22
    assert L.cg_table_choice(0, s22 + HEADROOM) == 22
    assert L.cg_table_choice(0, 0) == 22                     # nothing fits: the smallest (the build decides)


def test_verifier_processes_sharing_one_device(L):
    """The reference starts 4 verifiers against one node (VerifierTests.kt:54-70): four processes
    opening a context on one 288-GB device in turn, each holding its tables plus ~15 GB of call
    workspace, all get tables (round 5: the third failed cg_open)."""
    free, got = 288 * 10**9, []
    for _ in range(4):
        bits = L.cg_table_choice(0, free)
        assert bits
        got.append(bits)
        free -= L.cg_table_bytes(bits) + 15 * 10**9
    assert got[0] == 26 and got[-1] in (24, 22) and free > 0, got


def test_config_field_replaces_a_reserved_word():
    """cg_config stays 56 bytes; table_bytes_max sits where reserved[0] was (ABI v2 callers that
    zeroed it get the automatic choice)."""
    assert ctypes.sizeof(_lib.cg_config) == 56
    assert _lib.cg_config.table_bytes_max.offset == 40 and _lib.cg_config.reserved1.offset == 48
    assert ctypes.sizeof(_lib.cg_info) == 32
    src = open(_lib.HEADER_PATH).read()
    assert "uint64_t table_bytes_max;" in src and "#define CG_TABLE_HEADROOM (16ull << 30)" in src
