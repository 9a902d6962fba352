"""The Kotlin binding (jvm/.../CryptoBatch.kt; not compiled here: no JDK in the image) against the C
header and the Python mirror it must agree with:

- raiseForStatus fails closed: every non-VALID status arm ends in a throw, or (UNSUPPORTED only) in
  the JVM's own Crypto.doVerify, which throws or returns as the serial call does (Crypto.kt:474-484);
  KEY_INVALID throws even when the JVM decoder accepts the key;
- the status codes, the 16-bit length surrogates and the cg_stats size are the C ABI's and
  corda_amd/batch.py's;
- the handles are cleared by close(), which waits for the native calls in flight (no
  use after free), and every entry point runs on a context or a pool, re-queueing
  only the NOT_RUN items on a device fault;
- the JNI shim type-checks against include/cordagpu.h;
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
                         "CG_EMPTY", "CG_NOT_RUN", "else"}
    assert arms["CG_VALID"].strip() == "return"
    for lab, body in arms.items():
        if lab in ("CG_VALID", "CG_UNSUPPORTED", "CG_NOT_RUN"):
            continue
        # the arm ends in a throw: one is present, and no `return` anywhere in the arm
        assert "throw " in body and "return" not in body, (lab, body)
    # KEY_INVALID: the JVM decoder first (its own exception), then an unconditional throw
    ki = arms["CG_KEY_INVALID"]
    assert ki.index("Crypto.decodePublicKey") < ki.index("throw InvalidKeyException")
    # UNSUPPORTED: the serial call itself, then return (Crypto.doVerify throws on failure)
    assert re.search(r"Crypto\.doVerify\(item\.publicKey, item\.signatureData, item\.clearData\);\s*return", arms["CG_UNSUPPORTED"])
    # NOT_RUN (no device ran it, even after the re-queue): the JVM's own serial call, never accepted
    assert re.search(r"Crypto\.doVerify\(item\.publicKey, item\.signatureData, item\.clearData\);\s*return", arms["CG_NOT_RUN"])
    assert "IllegalStateException" in arms["else"]  # not a status the engine writes


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


def _fun_body(kt, name):
    """The text of `fun name(` up to the next member at the object's indentation."""
    at = re.search(rf"fun (?:<[^>]*> )?{name}\(", kt).start()
    nxt = re.search(r"\n    (?:private |internal )?(?:fun|val|var|class|object|/\*\*|@)", kt[at + 1:])
    return kt[at:at + 1 + nxt.start()] if nxt else kt[at:]


def test_handles_cleared_on_close(kt):
    """close() must not free a handle under a native call in flight: every native call
    runs inside withHandles (read lock across the call), close() and the open take the write lock."""
    close = _fun_body(kt, "close")
    assert "rw.write" in close and "ctx = 0" in close and "pool = 0" in close
    assert "private val rw = ReentrantReadWriteLock()" in kt
    wh = _fun_body(kt, "withHandles")
    assert "rw.read {" in wh and "return call(ctx, pool)" in wh and "rw.write {" in wh
    assert "lazy {" not in kt and "synchronized(" not in kt
    # the handles are read nowhere else, and every native verify call sits inside withHandles
    for m in re.finditer(r"\bnative(Verify\w*)\(", kt):
        line_start = kt.rfind("\n", 0, m.start())
        if "external fun" in kt[line_start:m.start()]:
            continue
        before = kt[:m.start()]
        assert before.rfind("withHandles {") > before.rfind("\n    fun ") and \
            before.rfind("withHandles {") > before.rfind("\n    private fun "), m.group(0)


def test_every_entry_point_takes_the_pool(kt):
    """with gpuVerifier.devices of several ordinals only a pool is open; no public
    entry point may then refuse to run (round 5: `check(c != 0L)` made verifyBatch, doVerifyAll above
    minBatch and verifyPacked throw on every call)."""
    assert "check(c != 0L)" not in kt and "handles()" not in kt
    for ext in ("nativeVerify", "nativeVerifyTxSignaturesPacked", "nativeVerifyTransactions"):
        decl = re.search(rf"external fun {ext}\((.*?)\): Int", kt, re.S).group(1)
        assert decl.replace(" ", "").startswith("ctx:Long,pool:Long,"), ext
        for call in re.finditer(rf"\b{ext}\(c, p,", kt):
            pass
        assert re.search(rf"\b{ext}\(c, p,", kt), f"{ext} is not called with both handles"
    for fn in ("verifyBatch", "verifyPacked", "verifyTxSignatures", "verifyTransactionsPacked", "doVerifyAll"):
        assert f"fun {fn}(" in kt, fn


def test_device_faults_requeue_by_status(kt):
    """on CG_ERR_DEVICE re-queue exactly the NOT_RUN items (once), never throw for
    the whole batch; anything still NOT_RUN is verified by Crypto.doVerify in raiseForStatus."""
    rq = _fun_body(kt, "requeueNotRun")
    assert "check(rc == CG_ERR_DEVICE)" in rq and "CG_NOT_RUN" in rq and "rerun(todo)" in rq
    assert "const val CG_ERR_DEVICE = -2" in kt.replace("private ", "")
    # each per-item native call is followed by requeueNotRun with a re-run of the NOT_RUN subset
    for fn, native in (("verifyItems", "nativeVerify"), ("verifySigs", "nativeVerifyTxSignaturesPacked"),
                       ("verifyPackedItems", "nativeVerify")):
        body = _fun_body(kt, fn)
        assert native + "(c, p," in body, fn
        assert "requeueNotRun(rc," in body and "requeue = false" in body.replace(", false)", ", requeue = false)"), fn
        assert "check(rc == 0)" not in body, fn
    # the public entry points run through those helpers
    assert "verifyItems(items, mode, requeue = true)" in _fun_body(kt, "verifyBatch")
    assert "verifySigs(txs, mode, requeue = true)" in _fun_body(kt, "verifyTxSignatures")
    assert "verifyPackedItems(" in _fun_body(kt, "verifyPacked")


def test_jni_shim_type_checks_against_the_header():
    """The shim compiles against include/cordagpu.h (a minimal jni.h stand-in supplies the JDK types):
    every cg_* call has the header's argument count and types."""
    import shutil
    import subprocess
    gcc = shutil.which("gcc")
    if not gcc:
        pytest.skip("no gcc")
    r = subprocess.run([gcc, "-fsyntax-only", "-Wall", "-Werror", "-Wno-unused-parameter",
                        "-I" + os.path.join(ROOT, "tests/native/jni_stub"), "-I" + os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "jvm/jni/cordagpu_jni.c")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    # parameter counts: Kotlin external (+ env, self) == the C export's
    c = open(os.path.join(ROOT, "jvm/jni/cordagpu_jni.c")).read()
    kt_src = open(KT).read()
    for m in re.finditer(r"external fun (\w+)\(([^)]*)\)", kt_src):
        name, params = m.group(1), m.group(2)
        nk = len([p for p in params.split(",") if p.strip()])
        cm = re.search(rf"Java_net_corda_core_crypto_CryptoBatch_{name}\((.*?)\)\s*{{", c, re.S)
        assert cm, name
        nc = len([p for p in cm.group(1).split(",") if p.strip()])
        assert nc == nk + 2, (name, nk, nc)


def test_node_conf_block_documented(kt):
    keys = set(re.findall(r'opt\("(\w+)"', kt))
    assert keys == {"devices", "minBatch", "chunkItems", "hostThreads", "tableBytesMax"}
    doc = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    block = doc[doc.index("gpuVerifier {"):]
    block = block[:block.index("}") + 1]
    for k in keys:
        assert re.search(rf"\b{k}\s*=", block), k
    # the metric names follow the reference's verifier service (Verification.Duration / Success / Failure)
    for name in ("Verification.Duration", "Verification.Success", "Verification.Failure", "VerificationsInFlight"):
        assert f'"{name}"' in kt, name
