"""The Kotlin binding (jvm/.../CryptoBatch.kt; not compiled here: no JDK in the image) against the C
header and the Python mirror it must agree with:

- raiseForStatus fails closed: every non-VALID status arm ends in a throw, or (UNSUPPORTED only) in
  the JVM's own Crypto.doVerify, which throws or returns as the serial call does (Crypto.kt:474-484);
  KEY_INVALID throws even when the JVM decoder accepts the key;
- the status codes, the 16-bit length surrogates and the cg_stats size are the C ABI's and
  corda_amd/batch.py's;
- the handles are cleared by close() and checked by every entry point (no use after free);
- the node.conf block INTEGRATION.md shows has exactly the keys GpuVerifierConfig.fromConfig reads.
"""
import ctypes
import os
import re

import pytest

from corda_amd import _lib
from corda_amd import batch as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KT = os.path.join(ROOT, "jvm/src/main/kotlin/net/corda/core/crypto/CryptoBatch.kt")


@pytest.fixture(scope="module")
def kt():
    return open(KT).read()


def _header_enum():
    src = open(_lib.HEADER_PATH).read()
    return {m.group(1): int(m.group(2)) for m in re.finditer(r"\b(CG_[A-Z_]+)\s*=\s*(\d+)", src)}


def _when_arms(kt):
    """The arms of raiseForStatus's `when`: {label: body text}."""
    body = kt[kt.index("fun raiseForStatus("):]
    body = body[body.index("when (status.toInt() and 0xff) {") + len("when (status.toInt() and 0xff) {"):]
    depth, end = 1, 0
    for i, ch in enumerate(body):
        depth += ch == "{"
        depth -= ch == "}"
        if depth == 0:
            end = i
            break
    arms, cur = {}, None
    for line in body[:end].splitlines():
        m = re.match(r"\s*(CG_[A-Z_]+|else)\s*->\s*(.*)$", line)
        if m:
            cur = m.group(1)
            arms[cur] = m.group(2)
        elif cur:
            arms[cur] += "\n" + line
    return arms


def test_status_constants_match_header(kt):
    hdr = _header_enum()
    kconst = {m.group(1): int(m.group(2)) for m in re.finditer(r"const val (CG_[A-Z_]+) = (\d+)", kt)}
    for name in ("CG_VALID", "CG_INVALID", "CG_SIG_MALFORMED", "CG_KEY_INVALID", "CG_UNSUPPORTED", "CG_EMPTY",
                 "CG_NOT_RUN"):
        assert kconst[name] == hdr[name], name


def test_raise_for_status_fails_closed(kt):
    arms = _when_arms(kt)
    assert set(arms) == {"CG_VALID", "CG_INVALID", "CG_SIG_MALFORMED", "CG_KEY_INVALID", "CG_UNSUPPORTED",
                         "CG_EMPTY", "else"}
    assert arms["CG_VALID"].strip() == "return"
    for lab, body in arms.items():
        if lab in ("CG_VALID", "CG_UNSUPPORTED"):
            continue
        # the arm ends in a throw: one is present, and no `return` anywhere in the arm
        assert "throw " in body and "return" not in body, (lab, body)
    # KEY_INVALID: the JVM decoder first (its own exception), then an unconditional throw
    ki = arms["CG_KEY_INVALID"]
    assert ki.index("Crypto.decodePublicKey") < ki.index("throw InvalidKeyException")
    # UNSUPPORTED: the serial call itself, then return (Crypto.doVerify throws on failure)
    assert re.search(r"Crypto\.doVerify\(item\.publicKey, item\.signatureData, item\.clearData\);\s*return", arms["CG_UNSUPPORTED"])
    assert "IllegalStateException" in arms["else"]  # NOT_RUN: re-queue, never accepted


def test_surrogates_match_python_mirror(kt):
    def kbytes(name):
        m = re.search(name + r" = byteArrayOf\(([^)]*)\)", kt)
        return bytes(int(x.strip(), 0) for x in m.group(1).split(","))
    assert kbytes("SIG_SURROGATE_MALFORMED") == B.SIG_SURROGATE_MALFORMED
    assert kbytes("SIG_SURROGATE_INVALID") == B.SIG_SURROGATE_INVALID
    assert int(re.search(r"const val SIG_LEN_MAX = (0x[0-9A-Fa-f]+)", kt).group(1), 16) == B.SIG_LEN_MAX
    # every signature the binding packs goes through sigField (no raw `.size.toShort()` of a signature)
    assert "signatureData.size.toShort()" not in kt and "sig.bytes.size.toShort()" not in kt
    assert kt.count("sigField(keys.schemes[ki]") == 2


def test_stats_buffer_is_cg_stats(kt):
    assert int(re.search(r"STATS_BYTES = (\d+)", kt).group(1)) == ctypes.sizeof(_lib.cg_stats)


def test_handles_cleared_on_close(kt):
    close = kt[kt.index("fun close()"):kt.index("private inline fun <T> timed")]
    assert "ctx = 0" in close and "pool = 0" in close and "synchronized(lock)" in close
    assert "@Volatile private var ctx: Long = 0" in kt
    # no lazy delegate holding a freed pointer
    assert "lazy {" not in kt
    # every native verify call goes through handles() (opened under the lock, checked non-zero)
    for fn in ("verifyBatch", "verifyPacked", "verifyTransactionsPacked"):
        body = kt[kt.index(f"fun {fn}("):]
        body = body[:body.index("\n    }\n") if "\n    }\n" in body else len(body)]
        assert "handles()" in body and "check(c != 0L)" in body, fn


def test_node_conf_block_documented(kt):
    keys = set(re.findall(r'opt\("(\w+)"', kt))
    assert keys == {"devices", "minBatch", "chunkItems", "hostThreads"}
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = doc[doc.index("gpuVerifier {"):]
    block = block[:block.index("}") + 1]
    for k in keys:
        assert re.search(rf"\b{k}\s*=", block), k
    # the metric names follow the reference's verifier service (Verification.Duration / Success / Failure)
    for name in ("Verification.Duration", "Verification.Success", "Verification.Failure", "VerificationsInFlight"):
        assert f'"{name}"' in kt, name
