"""The exact lane arithmetic of the HIP kernels (corda_amd/csrc/*.h), compiled for the
host with FE_BOUNDS_CHECK (every limb bound assumed by fe25519.h is asserted; a violated
bound aborts the process), checked against Python big integers and the oracle.
CPU only: this is where kernel arithmetic is debugged before it reaches a GPU."""
import ctypes
import random

import numpy as np
import pytest

import golden_io
import hostk
from hostk import L, P, limbs_to_int, ptr, words
from oracle import c_oracle, ed25519_i2p as ed

TIGHT = [(1 << 26) - 1 if i % 2 == 0 else (1 << 25) + (1 << 18) for i in range(10)]


def test_fe_mul_sq_bounds_and_values():
    lib = hostk.lib()
    rng = random.Random(1)
    out = np.zeros(10, dtype=np.uint32)
    for trial in range(4000):
        fm, gm = rng.choice([1, 2, 3, 5]), rng.choice([1, 2, 3])
        if trial < 64:
            f = np.array([t * fm for t in TIGHT], dtype=np.uint32)
            g = np.array([t * gm for t in TIGHT], dtype=np.uint32)
        else:
            f = np.array([rng.randrange(0, t * fm + 1) for t in TIGHT], dtype=np.uint32)
            g = np.array([rng.randrange(0, t * gm + 1) for t in TIGHT], dtype=np.uint32)
        lib.t_fe_mul(ptr(f), ptr(g), ptr(out))
        assert limbs_to_int(out) % P == limbs_to_int(f) * limbs_to_int(g) % P
        if fm <= 2:
            lib.t_fe_sq(ptr(f), ptr(out))
            assert limbs_to_int(out) % P == limbs_to_int(f) ** 2 % P


def test_fe_tobytes_canonical():
    lib = hostk.lib()
    rng = random.Random(2)
    w = np.zeros(8, dtype=np.uint32)
    for trial in range(3000):
        m = rng.choice([1, 2, 3, 5])
        f = np.array([rng.randrange(0, t * m + 1) for t in TIGHT], dtype=np.uint32)
        if trial < 40:  # values near p and 2p
            v = (P + rng.randrange(-40, 40)) % (1 << 255)
            f = hostk.int_to_limbs(v)
        lib.t_fe_tobytes(ptr(f), ptr(w))
        assert int.from_bytes(w.tobytes(), "little") == limbs_to_int(f) % P


def test_fe_invert():
    lib = hostk.lib()
    rng = random.Random(3)
    out = np.zeros(10, dtype=np.uint32)
    for _ in range(50):
        x = rng.randrange(1, P)
        lib.t_fe_invert(ptr(hostk.int_to_limbs(x)), ptr(out))
        assert limbs_to_int(out) * x % P == 1


def test_sc_reduce512():
    lib = hostk.lib()
    rng = random.Random(4)
    o = np.zeros(8, dtype=np.uint32)
    for trial in range(3000):
        x = rng.getrandbits(512) if trial > 6 else [0, 2 ** 512 - 1, L, 2 * L, L - 1, 2 ** 256, L * L][trial]
        lib.t_sc_reduce512(ptr(words(x.to_bytes(64, "little"))), ptr(o))
        assert int.from_bytes(o.tobytes(), "little") == x % L


def test_slide_escape_matches_literal_slide():
    lib = hostk.lib()
    rng = random.Random(5)
    for trial in range(3000):
        s = rng.getrandbits(256) | (1 << 255) if trial % 3 else rng.getrandbits(256)
        if trial < 4:
            s = [2 ** 256 - 1, 2 ** 255, 2 ** 256 - L, 2 ** 255 + 2 ** 251][trial]
        sb = s.to_bytes(32, "little")
        assert bool(lib.t_slide_escapes(ptr(words(sb)))) == (ed.slide_value(sb) < 0)


def test_recode16():
    lib = hostk.lib()
    rng = random.Random(6)
    d = np.zeros(64, dtype=np.int32)
    for _ in range(500):
        a = rng.randrange(0, L)
        lib.t_recode16(ptr(words(a.to_bytes(32, "little"))), ptr(d))
        assert sum(int(x) << (4 * i) for i, x in enumerate(d)) == a
        assert d.min() >= -8 and d.max() <= 8


def test_ed25519_lane_verify_on_fixtures():
    lib = hostk.lib()
    n = 0
    for it in golden_io.load("ed25519.json"):
        key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
        if it["key_fmt"] != 0 or len(key) != 32 or len(sig) != 64:
            continue
        m = np.frombuffer(msg + bytes(8), dtype=np.uint8).copy()
        st = lib.t_ed_verify(ptr(words(key)), ptr(words(sig)), ptr(m), len(msg))
        got = {0: "VALID", 1: "INVALID", 3: "KEY_INVALID"}[st]
        assert got == it["expect_isvalid"], it["note"]
        n += 1
    assert n > 200


def test_abyte_without_square_root():
    """k_ed_key_abyte's Abyte (no decode) equals the decoded point's re-encoding for every key
    that decodes: fixtures, random y, y >= p, y = +-1 (x = 0) with either sign bit."""
    import ctypes
    lib = hostk.lib()
    lib.t_ed_abyte_fast.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    lib.t_ed_keyprep.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    cands = [bytes.fromhex(it["key"]) for it in golden_io.load("ed25519.json")
             if it["key_fmt"] == 0 and len(bytes.fromhex(it["key"])) == 32]
    rng = np.random.default_rng(5)
    cands += [rng.integers(0, 256, 32, dtype=np.uint8).tobytes() for _ in range(400)]
    P = 2 ** 255 - 19
    for y in (1, P - 1, P + 1, 2 ** 255 - 1, P, 0, 2 ** 255 - 20):
        for sign in (0, 1):
            cands.append(((y % 2 ** 255) | (sign << 255)).to_bytes(32, "little"))
    n = 0
    for key in cands:
        ref = np.zeros(8, dtype=np.uint32)
        got = np.zeros(8, dtype=np.uint32)
        st = lib.t_ed_keyprep(ptr(words(key)), ptr(ref))
        lib.t_ed_abyte_fast(ptr(words(key)), ptr(got))
        if st == 0:
            assert got.tobytes() == ref.tobytes(), key.hex()
            n += 1
    assert n > 300


def test_sha_lane_code():
    import ctypes
    lib = hostk.lib()
    rng = np.random.default_rng(7)
    out = np.zeros(16, dtype=np.uint32)
    for ln in list(range(0, 300, 7)) + [111, 112, 239, 240]:
        msg = rng.integers(0, 256, ln, dtype=np.uint8).tobytes()
        pre = rng.integers(0, 256, 64, dtype=np.uint8).tobytes()
        for off in (0, 1, 2, 3):
            buf = np.frombuffer(bytes(off) + msg + bytes(16), dtype=np.uint8).copy()
            lib.t_sha512_prefix(ptr(words(pre)), ptr(buf), ctypes.c_uint64(off), ctypes.c_uint64(ln), ptr(out))
            assert out.tobytes() == c_oracle.sha512(pre + msg)
            sfx = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
            o8 = np.zeros(8, dtype=np.uint32)
            sw = np.frombuffer(sfx, dtype=">u4").astype(np.uint32)
            lib.t_sha256_suffix(ptr(buf), ctypes.c_uint64(off), ctypes.c_uint64(ln), ptr(sw), ptr(o8))
            assert o8.astype(">u4").tobytes() == c_oracle.sha256(msg + sfx)


@pytest.mark.parametrize("w", [4, 6])
def test_ed25519_row_table_lane_verify_on_fixtures(w):
    """The radix-2^W row-table double-scalar path (k_ed_verify's arithmetic) on the fixtures."""
    import ctypes
    lib = hostk.lib()
    lib.t_ed_verify_w.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                  ctypes.c_uint64]
    n = 0
    for it in golden_io.load("ed25519.json"):
        key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
        if it["key_fmt"] != 0 or len(key) != 32 or len(sig) != 64:
            continue
        m = np.frombuffer(msg + bytes(8), dtype=np.uint8).copy()
        st = lib.t_ed_verify_w(w, ptr(words(key)), ptr(words(sig)), ptr(m), len(msg))
        got = {0: "VALID", 1: "INVALID", 3: "KEY_INVALID"}[st]
        assert got == it["expect_isvalid"], it["note"]
        n += 1
    assert n > 200


@pytest.mark.parametrize("fn", ["t_ed_verify_wb", "t_ed_verify_wb_signed"])
def test_ed25519_wide_b_lane_verify_on_fixtures(fn):
    """k_ed_ladder's arithmetic: -A rows (W=6, K=2) + the radix-2^10 B table (ed25519_rows.h);
    the _signed form is k_ed_ladder_pf's (entries by |digit|, sign through ge_madd_signed), with
    every limb bound asserted."""
    import ctypes
    lib = hostk.lib()
    f = getattr(lib, fn)
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    n = 0
    for it in golden_io.load("ed25519.json"):
        key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
        if it["key_fmt"] != 0 or len(key) != 32 or len(sig) != 64:
            continue
        m = np.frombuffer(msg + bytes(8), dtype=np.uint8).copy()
        st = f(ptr(words(key)), ptr(words(sig)), ptr(m), len(msg), None)
        got = {0: "VALID", 1: "INVALID", 3: "KEY_INVALID"}[st]
        assert got == it["expect_isvalid"], it["note"]
        n += 1
    assert n > 200


def test_executed_work_constants_match_lane_code():
    """bench.py prices k_ed_verify + k_ed_finish with the field products the lane code
    executes; the constants there must equal what the host build of that code counts."""
    import bench
    lib = hostk.lib()
    it = next(i for i in golden_io.load("ed25519.json") if i["expect"] == "VALID" and i["key_fmt"] == 0)
    key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
    m = np.frombuffer(msg + bytes(8), dtype=np.uint8).copy()
    out = np.zeros(8, dtype=np.uint64)
    assert lib.t_ed_count_w6(ptr(words(key)), ptr(words(sig)), ptr(m), len(msg), ptr(out)) == 0
    _, _, mul_f, sq_f, mul_i, sq_i = (int(x) for x in out[:6])
    import ctypes
    lib.t_ed_verify_wb.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    lad = np.zeros(3, dtype=np.uint64)
    assert lib.t_ed_verify_wb(ptr(words(key)), ptr(words(sig)), ptr(m), len(msg), ptr(lad)) == 0
    mul_v, sq_v, mul9 = int(lad[0]), int(lad[1]), int(lad[2])
    assert (mul_v, sq_v) == bench.ED_VERIFY_FE, (mul_v, sq_v)
    assert mul9 == bench.ED_VERIFY_FE9, mul9
    assert (mul_f, sq_f) == bench.ED_FINISH_FE, (mul_f, sq_f)
    assert (mul_i, sq_i) == bench.ED_INVERT_FE, (mul_i, sq_i)


def test_executed_work_constants_ecdsa():
    """bench.py prices the ECDSA ladders and batched inversions with the Montgomery products the
    lane code executes; those constants must equal what the host build counts, and the MACs per
    product must follow from the moduli's 29-bit limbs: 81 a*b + 9 per non-zero limb of q*m, except
    secp256r1's p (the all-ones run telescopes: 4 MACs per digit) and secp256k1's p (folded:
    81 + 9 + 2, mont29.h)."""
    import ctypes
    import bench
    lib = hostk.lib()
    lib.t_ecdsa_count.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint32,
                                  ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_uint64,
                                  ctypes.c_void_p]
    moduli = {"secp256r1": (2**256 - 2**224 + 2**192 + 2**96 - 1,
                            0xffffffff00000000ffffffffffffffffbce6faada7179e84f3b9cac2fc632551),
              "secp256k1": (2**256 - 2**32 - 977, 0xfffffffffffffffffffffffffffffffebaaedce6af48a03bbfd25e8cd0364141)}
    nnz = lambda m: sum(1 for i in range(9) if (m >> (29 * i)) & (2**29 - 1))  # noqa: E731
    for name, scheme in (("secp256r1", 3), ("secp256k1", 2)):
        p, n = moduli[name]
        assert bench.EC_MAC_PER_MUL_P[name] == {"secp256r1": 81 + 9 * 4, "secp256k1": 81 + 9 + 2}[name]
        assert bench.EC_MAC_PER_MUL_N[name] == 81 + 9 * nnz(n)
        from tools.workload import wl
        b, _ = wl.ecdsa_batch(1 if scheme == 3 else 0, 256, n_keys=8, corrupt_permille=0, seed=3, nthreads=4)
        lad = []
        for i in range(b.n):
            it = b.items[i]
            k = b.keys[it["key_idx"]]
            out = np.zeros(6, np.uint64)
            assert lib.t_ecdsa_count(scheme, ptr(b.arena), b.arena.size, int(k["off"]), int(k["len"]), int(k["fmt"]),
                                     int(it["sig_off"]), int(it["sig_len"]), int(it["msg_off"]), int(it["msg_len"]),
                                     ptr(out)) == 0
            assert int(out[5]) == 0 and int(out[2]) == 0 and int(out[0]) == 0 and int(out[1]) == 0, (name, out)
            assert int(out[3]) == bench.EC_INV_MUL_K[name], (name, out)
            lad.append(int(out[4]))
        # the wave's schedule: a mixed addition is skipped only when all 64 lanes' digits are zero,
        # so a wave issues the per-item maximum over random items (the mean is ~1% lower)
        assert max(lad) == bench.EC_LADDER_MUL[name] and np.mean(lad) > 0.97 * max(lad), (name, lad)


@pytest.mark.parametrize("fn", ["t_ecdsa_verify_rows"])
def test_ecdsa_lane_verify_on_fixtures(fn):
    """ECDSA lane code (the row-table pipeline: key decode -> rows -> prep -> batched
    inverse -> ladder + x-check, 29-bit Montgomery arithmetic) on every ECDSA fixture,
    isValid semantics."""
    lib = hostk.lib()
    f = getattr(lib, fn)
    names = {0: "VALID", 1: "INVALID", 2: "SIG_MALFORMED", 3: "KEY_INVALID"}
    n = 0
    for it in golden_io.load("ecdsa.json"):
        key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
        if it["scheme"] not in (2, 3):
            continue
        arena = np.frombuffer(key + sig + msg + bytes(8), dtype=np.uint8).copy()
        st = f(it["scheme"], ptr(arena), len(key) + len(sig) + len(msg), 0, len(key), it["key_fmt"], len(key),
               len(sig), len(key) + len(sig), len(msg))
        assert names[st] == it["expect_isvalid"], (it["class"], it["note"])
        n += 1
    assert n > 300


M29_MODS = {(1, 0): 2 ** 256 - 2 ** 224 + 2 ** 192 + 2 ** 96 - 1,
            (1, 1): 0xFFFFFFFF00000000FFFFFFFFFFFFFFFFBCE6FAADA7179E84F3B9CAC2FC632551,
            (0, 0): 2 ** 256 - 2 ** 32 - 977,
            (0, 1): 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141}


@pytest.mark.parametrize("curve,n", sorted(M29_MODS))
def test_mont29_ops(curve, n):
    """mont29.h (ECDSA field / scalar arithmetic; secp256k1's p by the pseudo-Mersenne fold) against
    Python integers, including values
    in [m, 2m) (the reduced range) and the lazy-sum operands, with every column bound asserted."""
    import ctypes
    lib = hostk.lib()
    lib.t_m29_op.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                             ctypes.c_void_p]
    m = M29_MODS[(curve, n)]
    # R = 2^261 (Montgomery) or 1 (secp256k1 p in plain form, folded products)
    rinv = 1 if lib.t_m29_plain(curve, n) else pow(2 ** 261, -1, m)
    rng = random.Random(curve * 2 + n)
    edge = [0, 1, m - 1, m, m + 1, 2 * m - 1, 2 ** 256 - 1 if 2 ** 256 - 1 < 2 * m else 2 * m - 2]
    vals = edge + [rng.randrange(0, 2 * m) for _ in range(300)]
    out = np.zeros(8, dtype=np.uint32)

    def w(x):
        return np.frombuffer(x.to_bytes(32, "little"), dtype=np.uint32).copy()

    for t in range(len(vals)):
        a, b = vals[t], vals[(t * 7 + 3) % len(vals)]
        if a >= 2 ** 256 or b >= 2 ** 256:
            continue
        lib.t_m29_op(curve, n, 0, ptr(w(a)), ptr(w(b)), ptr(out))
        assert int.from_bytes(out.tobytes(), "little") == a * b * rinv % m
        lib.t_m29_op(curve, n, 1, ptr(w(a)), ptr(w(b)), ptr(out))
        assert int.from_bytes(out.tobytes(), "little") == 4 * a * b * rinv % m
        lib.t_m29_op(curve, n, 2, ptr(w(a)), ptr(w(b)), ptr(out))
        assert int.from_bytes(out.tobytes(), "little") == (a + b) % m
        lib.t_m29_op(curve, n, 3, ptr(w(a)), ptr(w(b)), ptr(out))
        assert int.from_bytes(out.tobytes(), "little") == (a - b) % m


def test_ed25519_wide_tables_lane_verify_on_fixtures():
    """k_ed_ladder_wide's arithmetic (keys with many items: 32 rows x 128 multiples of 2^{8j}(-A),
    B over 22 radix-2^12 rows, 54 signed additions, no doublings) on the fixtures, every limb
    bound asserted."""
    import ctypes
    lib = hostk.lib()
    lib.t_ed_verify_wide.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    n = 0
    for it in golden_io.load("ed25519.json"):
        key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
        if it["key_fmt"] != 0 or len(key) != 32 or len(sig) != 64:
            continue
        m = np.frombuffer(msg + bytes(8), dtype=np.uint8).copy()
        st = lib.t_ed_verify_wide(ptr(words(key)), ptr(words(sig)), ptr(m), len(msg), None)
        got = {0: "VALID", 1: "INVALID", 3: "KEY_INVALID"}[st]
        assert got == it["expect_isvalid"], it["note"]
        n += 1
    assert n > 200


def test_ecdsa_wide_tables_lane_verify_on_fixtures():
    """k_ec_ladder_wide's arithmetic (33 rows x 128 multiples of 2^{8j} Q, G over 22 radix-2^12
    rows, no doublings) on every ECDSA and SPKI fixture, isValid semantics."""
    import ctypes
    lib = hostk.lib()
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.t_ecdsa_verify_wide.argtypes = [i32, vp, u64, u64, u32, u32, u64, u32, u64, u64, vp]
    names = {0: "VALID", 1: "INVALID", 2: "SIG_MALFORMED", 3: "KEY_INVALID"}
    n = 0
    for it in golden_io.load("ecdsa.json") + golden_io.load("spki.json"):
        key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
        if it["scheme"] not in (2, 3):
            continue
        arena = np.frombuffer(key + sig + msg + bytes(8), dtype=np.uint8).copy()
        st = lib.t_ecdsa_verify_wide(it["scheme"], ptr(arena), len(key) + len(sig) + len(msg), 0, len(key),
                                     it["key_fmt"], len(key), len(sig), len(key) + len(sig), len(msg), None)
        assert names[st] == it["expect_isvalid"], (it["class"], it["note"])
        n += 1
    assert n > 300


def test_executed_work_constants_wide():
    """bench.py prices k_ed_ladder_wide / k_ec_ladder_wide with the products their lane code
    executes (full schedule: every digit non-zero) and the wide-table build per key."""
    import ctypes
    import bench
    from tools.workload import wl
    lib = hostk.lib()
    lib.t_ed_verify_wide.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p]
    it = next(i for i in golden_io.load("ed25519.json") if i["expect"] == "VALID" and i["key_fmt"] == 0)
    key, sig, msg = bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"])
    m = np.frombuffer(msg + bytes(8), dtype=np.uint8).copy()
    out = np.zeros(4, dtype=np.uint64)
    assert lib.t_ed_verify_wide(ptr(words(key)), ptr(words(sig)), ptr(m), len(msg), ptr(out)) == 0
    assert (int(out[0]), int(out[1])) == bench.ED_WIDE_FE
    assert (int(out[2]), int(out[3])) == bench.ED_WIDE_BUILD_FE
    vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
    lib.t_ecdsa_verify_wide.argtypes = [i32, vp, u64, u64, u32, u32, u64, u32, u64, u64, vp]
    for name, scheme, curve in (("secp256r1", 3, 1), ("secp256k1", 2, 0)):
        b, _ = wl.ecdsa_batch(curve, 96, n_keys=2, corrupt_permille=0, seed=3, nthreads=4)
        lad, sqr = [], []
        for i in range(b.n):
            itm = b.items[i]
            k = b.keys[itm["key_idx"]]
            o = np.zeros(3, np.uint64)
            assert lib.t_ecdsa_verify_wide(scheme, ptr(b.arena), b.arena.size, int(k["off"]), int(k["len"]),
                                           int(k["fmt"]), int(itm["sig_off"]), int(itm["sig_len"]),
                                           int(itm["msg_off"]), int(itm["msg_len"]), ptr(o)) == 0
            lad.append(int(o[0]))
            sqr.append(int(o[2]))
        # of those products, the squares (ec9.h ec9_sqr*: 45 a*a MACs): priced at EC_MAC_PER_SQR_P
        assert int(np.median(sqr)) == bench.EC_WIDE_SQR[name], (name, sqr)
        # a square: the 36 pairs i < j once plus the 9 diagonal terms, then the product's reduction
        assert bench.EC_MAC_PER_SQR_P[name] == 36 + 9 + (bench.EC_MAC_PER_MUL_P[name] - 81)
        assert bench.EC_WIDE_MAC32[name] == ((bench.EC_WIDE_MUL[name] - bench.EC_WIDE_SQR[name]) * bench.EC_MAC_PER_MUL_P[name]
                                             + bench.EC_WIDE_SQR[name] * bench.EC_MAC_PER_SQR_P[name])
        # the full schedule is the common count; a lane whose H passes ec9.h's zero filter (false
        # positives ~2^-24 per addition) recomputes 4 products on the exact path
        assert int(np.median(lad)) == bench.EC_WIDE_MUL[name] and max(lad) <= bench.EC_WIDE_MUL[name] + 8, (name, lad)
        assert np.mean(lad) > 0.97 * bench.EC_WIDE_MUL[name], (name, lad)


@pytest.mark.parametrize("curve", [0, 1])
def test_ec_madd_w_matches_madd(curve):
    """The wide ladder's mixed addition (semi-reduced operands, infinity flag, Z3 = Z1 * 2H) gives
    the same points as the exception-complete jac_madd, including Q = acc (doubling), Q = -acc
    (infinity) and acc = infinity, under the host build's limb and Montgomery-output bound checks."""
    lib = hostk.lib()
    lib.t_ec_madd_w_cmp.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int]
    assert lib.t_ec_madd_w_cmp(curve, 12345 + curve, 400) == 0


def test_sha_over_splice_matches_materialised():
    """The hash kernels read SignableData = prefix || id || suffix straight from the template image
    and the id (no message is written): SHA-512 (challenge form) and SHA-256 resumed from the prefix
    midstate equal the hashes of the materialised bytes for every prefix length 0..299."""
    lib = hostk.lib()
    lib.t_sha_splice_cmp.argtypes = [ctypes.c_uint64, ctypes.c_int]
    assert lib.t_sha_splice_cmp(99, 3000) == 0


@pytest.mark.parametrize("curve", [0, 1])
def test_ec_wide_row_build_matches_three_pass(curve):
    """k_ec_wide_rows (co-Z additions, one lane per row, one inversion) builds the same affine
    entries as the three-pass build it replaced, for rows 0 and 32 (multiples 129..256) of several
    bases, every product's bound asserted."""
    import ctypes
    lib = hostk.lib()
    lib.t_ec_wide_row_cmp.argtypes = [ctypes.c_int, ctypes.c_uint32]
    for m in (1, 2, 3, 7, 255, 256, 65537, 0x7fffffff):
        assert lib.t_ec_wide_row_cmp(curve, m) == 0, m


def test_ed_wide_row_build_matches_three_pass():
    """k_ed_wide_rows (one lane per row, one inversion) builds the same half-scaled niels entries as
    the three-pass build it replaced, for the row bases m B of several m, limb bounds asserted."""
    import ctypes
    lib = hostk.lib()
    lib.t_ed_wide_row_cmp.argtypes = [ctypes.c_uint32]
    for m in (1, 2, 3, 8, 255, 4096, 65537, 0x7fffffff):
        assert lib.t_ed_wide_row_cmp(m) == 0, m


# ---------------------------------------------------------------- radix-2^29 products (fe9.h)
R29 = [29 * i for i in range(9)]


def _fe9_int(v, signed=False):
    return sum((int(np.int32(x)) if signed else int(x)) << o for x, o in zip(np.asarray(v, np.uint32), R29))


def _fe9_class(rng, cls):
    """Random limbs of one operand class of fe9.h, biased to the class's extremes."""
    M = 1 << 29
    hi = {"T": M, "A2": 2 * M + (1 << 18), "V": 3 * M + (1 << 17)}
    out = []
    for i in range(9):
        if cls == "S":
            b = M + (1 << 17) - 1
            x = rng.choice([b, -b, rng.randrange(-b, b + 1)])
            out.append(x & 0xffffffff)
            continue
        top = hi[cls] - 1 if not (cls == "T" and i != 1) else M - 1
        if cls == "T" and i == 1:
            top = M + (1 << 17) - 1
        lo = (1 << 28) if cls == "V" else 0
        out.append(rng.choice([top, lo, rng.randrange(lo, top + 1)]))
    return np.array(out, np.uint32)


@pytest.mark.parametrize("ca,cb,sgn", [("T", "T", 0), ("A2", "T", 0), ("A2", "A2", 0), ("A2", "V", 0), ("V", "A2", 0),
                                       ("S", "T", 1), ("S", "A2", 1), ("S", "V", 1), ("S", "S", 1), ("T", "T", 1)])
def test_fe9_mul_operand_classes(ca, cb, sgn):
    """Every product the wide ladder forms (fe9.h operand classes) is exact with tight output;
    the host build asserts each 64-bit column (FE_BOUNDS_CHECK) on extreme and random limbs."""
    lib = hostk.lib()
    rng = random.Random(hash((ca, cb, sgn)) & 0xffff)
    out = np.zeros(9, np.uint32)
    for _ in range(400):
        a, b = _fe9_class(rng, ca), _fe9_class(rng, cb)
        lib.t_fe9_mul(sgn, ptr(a), ptr(b), ptr(out))
        assert (_fe9_int(out) - _fe9_int(a, sgn) * _fe9_int(b, sgn)) % P == 0
        assert all(int(x) < (1 << 29) for i, x in enumerate(out) if i != 1) and int(out[1]) < (1 << 29) + (1 << 17)


def test_fe9_conversions():
    lib = hostk.lib()
    rng = random.Random(9)
    w = np.zeros(8, np.uint32)
    f9 = np.zeros(9, np.uint32)
    for _ in range(300):
        x = rng.choice([rng.randrange(P), P - 1, 0, 1, 2 ** 255 - 20])
        lib.t_fe9_from_fe(ptr(hostk.int_to_limbs(x)), ptr(f9))
        assert _fe9_int(f9) == x and all(int(v) < (1 << 29) for v in f9)
        big = _fe9_class(rng, rng.choice(["T", "A2", "V"]))  # any non-negative limbs
        lib.t_fe9_to_words(ptr(big), ptr(w))
        y = sum(int(v) << (32 * i) for i, v in enumerate(w))
        assert y < 2 ** 255 and (y - _fe9_int(big)) % P == 0


@pytest.mark.parametrize("curve", [0, 1])
def test_ec_madd9_matches_madd(curve):
    """The wide ladder's signed-limb addition (ec9.h: no carry chains, fused X3 and Y3) follows the
    exception-complete jac_madd over 60-addition chains of random multiples of G, including Q = +-R
    (doubling / infinity through the exact path), every product column asserted < 2^63."""
    lib = hostk.lib()
    lib.t_ec_madd9_cmp.argtypes = [ctypes.c_int, ctypes.c_uint64, ctypes.c_int, ctypes.c_int]
    assert lib.t_ec_madd9_cmp(curve, 777 + curve, 60, 60) == 0


@pytest.mark.parametrize("family", [0, 1, 2])  # secp256k1, secp256r1, Ed25519
def test_row_build_parked_matches_row_build(family):
    """k_ed_keyprep_tab / k_ec_keyprep_tab's row build (the walk parked lane-interleaved in a shared
    column, keyws.h tab_park_lanes) writes byte-identical entries to the in-row scratch build, for
    several row bases, every product's bound asserted."""
    import ctypes
    lib = hostk.lib()
    lib.t_row_parked_cmp.argtypes = [ctypes.c_int, ctypes.c_uint32]
    for m in (1, 2, 3, 7, 255, 65537, 0x7fffffff):
        assert lib.t_row_parked_cmp(family, m) == 0, m


@pytest.mark.parametrize("curve", [0, 1])
def test_ec9_product_forms_vs_big_integers(curve):
    """ec9.h's five product forms (a b, a b + e, a b + c d, and round 6's squares a^2 and a^2 + e over
    a doubled copy) against Python integers, on the operand classes jac_madd9 feeds them: tight
    values T (digits 0..7 in [0, 2^29), the rest in the top limb; up to 6p, digits all 2^29 - 1 at the
    extreme), differences S = T - T limb by limb, and e = -T - 2T (X3's E); every column bound
    asserted (FE_BOUNDS_CHECK). secp256r1 is Montgomery (R = 2^261: the product carries R^-1),
    secp256k1 plain."""
    lib = hostk.lib()
    u32p = ctypes.POINTER(ctypes.c_uint32)
    lib.t_ec9_mul.argtypes = [ctypes.c_int, ctypes.c_int, u32p, u32p, u32p, u32p, u32p]
    p = 2 ** 256 - 2 ** 32 - 977 if curve == 0 else 2 ** 256 - 2 ** 224 + 2 ** 192 + 2 ** 96 - 1
    rinv = pow(2 ** 261, -1, p) if curve == 1 else 1
    rng = random.Random(90 + curve)
    M = (1 << 29) - 1

    def tight(v):
        return [(v >> (29 * i)) & M for i in range(8)] + [v >> 232]

    def t_val(kind):
        if kind == "max":  # every digit 2^29 - 1, the top at the class bound
            return tight(((6 * p) >> 232 << 232) | ((1 << 232) - 1))
        return tight(rng.randrange(6 * p))

    def operand(kind):
        t = t_val(kind)
        if rng.random() < 0.5:
            return t
        u = t_val("rand" if kind == "max" else kind)
        return [x - y for x, y in zip(t if kind != "max" else [0] * 9, u if kind != "max" else t)]

    def arr(v):
        return (ctypes.c_uint32 * 9)(*[x & 0xFFFFFFFF for x in v])

    def val(v):
        return sum(x << (29 * i) for i, x in enumerate(v))

    out = (ctypes.c_uint32 * 9)()
    for it in range(60):
        kind = "max" if it < 6 else "rand"
        a, b, c, d = operand(kind), operand(kind), operand(kind), operand(kind)
        h, w = t_val(kind), t_val(kind)
        e = [-x - 2 * y for x, y in zip(h, w)]
        A, B, C, D, E = val(a), val(b), val(c), val(d), val(e)
        for form, want in ((0, A * B * rinv), (1, A * B * rinv + E), (2, (A * B + C * D) * rinv),
                           (3, A * A * rinv), (4, A * A * rinv + E)):
            lib.t_ec9_mul(curve, form, arr(a), arr(b), arr(e if form in (1, 4) else c), arr(d), out)
            got = val([ctypes.c_int32(x).value for x in out])
            assert (got - want) % p == 0, (curve, form, it)
