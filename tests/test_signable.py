"""SignableData templates and the transaction-pipeline packing (host logic, CPU only).

The template bytes are a restatement of Kryo 4's wire format (PARITY UNPINNED: no JVM here,
corda_amd/signable.py); what is pinned here is the splice invariant the GPU relies on:
serialize(id) == prefix + id + suffix for every id and metadata value."""
import numpy as np
import pytest

from corda_amd import batch as B
from corda_amd import signable
from corda_amd import transactions as T
from corda_amd.crypto import PublicKey


@pytest.mark.parametrize("pv,sid", [(1, 4), (1, 3), (1, 2), (2, 4), (300, 1), (-1, 4)])
def test_template_splice_invariant(pv, sid):
    pre, suf = signable.template(pv, sid)
    assert pre.startswith(signable.KRYO_HEADER_V0_1)
    rng = np.random.default_rng(abs(pv) * 7 + sid)
    for _ in range(50):
        tx_id = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        assert signable.serialize(tx_id, pv, sid) == pre + tx_id + suf


def test_template_depends_on_metadata():
    assert signable.template(1, 4) != signable.template(1, 3)
    assert signable.template(1, 4) != signable.template(2, 4)
    pre, suf = signable.template(1, 4)
    assert 200 < len(pre) + 32 + len(suf) < 300  # ~270-byte SignableData


def test_pack_signed_transactions_layout():
    rng = np.random.default_rng(1)
    stxs = []
    for t in range(5):
        comps = [rng.integers(0, 256, int(rng.integers(0, 50)), dtype=np.uint8).tobytes() for _ in range(t)]
        w = T.WireTransactionData(comps, rng.integers(0, 256, 32, dtype=np.uint8).tobytes(), b"salt" * 3)
        sigs = [T.TransactionSignature(bytes([t, i]) * 32, PublicKey(4, bytes([i]) * 32), 1, 4 if i else 3)
                for i in range(3)]
        stxs.append(T.SignedWireTransaction(w, sigs))
    txs, comps, keys, sigs, tmpls, arena = T.pack_signed_transactions(stxs)
    assert len(txs) == 5 and len(sigs) == 15 and len(keys) == 3 and len(tmpls) == 2
    a = arena.tobytes()
    for t, stx in enumerate(stxs):
        r = txs[t]
        assert r["n"] == len(stx.wtx.components) + 1
        cs = comps[r["first"]:r["first"] + r["n"]]
        got = [a[c["off"]:c["off"] + c["len"]] for c in cs]
        assert got == stx.wtx.components + [stx.wtx.salt_blob]
        assert list(cs["flags"]) == [0] * len(stx.wtx.components) + [1]
        assert a[r["salt_off"]:r["salt_off"] + 32] == stx.wtx.salt
    for j, s in enumerate(sigs):
        src = stxs[s["tx_idx"]].sigs[j % 3]
        assert a[s["sig_off"]:s["sig_off"] + s["sig_len"]] == src.bytes
        k = keys[s["key_idx"]]
        assert a[k["off"]:k["off"] + k["len"]] == src.by.encoded
        tm = tmpls[s["tmpl"]]
        pre, suf = signable.template(src.platform_version, src.scheme_number_id)
        assert a[tm["prefix_off"]:tm["prefix_off"] + tm["prefix_len"]] == pre
        assert a[tm["suffix_off"]:tm["suffix_off"] + tm["suffix_len"]] == suf
    assert sigs.dtype == B.TXSIG_DTYPE and tmpls.dtype == B.TMPL_DTYPE
