"""GPU parity tests: the HIP path through the C ABI against the oracle.

Every verdict / digest is compared bit-for-bit with the CPU restatement of the reference
(oracle/, C and Python) on the same inputs:
  * the committed golden fixtures (tests/golden/*.json; RFC 8032, OpenSSL-cross-checked
    valid signatures, every Appendix A corruption class), in doVerify and isValid modes;
  * seeded synthetic batches at the BASELINE configs' shape, checked item by item against
    the C oracle (liboracle.so) and against the corruption labels;
  * SHA-256 / SHA-512 / Merkle / tx-id fixtures.
"""
import numpy as np
import pytest

import golden_io
from corda_amd import batch as B
from oracle import c_oracle, corda as ocorda

pytestmark = pytest.mark.gpu


def _check(engine, items_json, mode):
    b, exp, exp_iv = golden_io.sig_batch(items_json)
    st = engine.verify(b, mode)
    want = exp if mode == B.MODE_DOVERIFY else exp_iv
    bad = np.nonzero(st != want)[0]
    msgs = [f"{items_json[i]['class']} {items_json[i]['note']}: want {B.STATUS_NAMES[int(want[i])]} "
            f"got {B.STATUS_NAMES.get(int(st[i]), st[i])}" for i in bad[:20]]
    assert len(bad) == 0, "\n".join(msgs)


@pytest.mark.parametrize("mode", [B.MODE_DOVERIFY, B.MODE_ISVALID])
def test_ed25519_golden(engine, mode):
    _check(engine, golden_io.load("ed25519.json"), mode)


@pytest.mark.parametrize("mode", [B.MODE_DOVERIFY, B.MODE_ISVALID])
def test_ecdsa_golden(engine, mode):
    _check(engine, golden_io.load("ecdsa.json"), mode)


@pytest.mark.parametrize("mode", [B.MODE_DOVERIFY, B.MODE_ISVALID])
def test_reference_certificate_signatures(engine, mode):
    """BouncyCastle-made ECDSA signatures from the reference's own keystores
    (tests/golden/ref_certs.json, tools/gen/ref_vectors.py): issuer SPKI, DER signature,
    TBSCertificate; plus corruptions. The engine gives the JVM's verdict on each."""
    _check(engine, golden_io.load("ref_certs.json"), mode)


def test_reference_certificates_in_a_large_batch(engine):
    """The same reference items scattered through a 40k-item mixed batch (so they run on the wide
    and full-table ladders beside synthetic keys), bit-exact against the C oracle."""
    from tools.workload import wl
    ref_items = golden_io.load("ref_certs.json")
    rb, exp, _ = golden_io.sig_batch(ref_items)
    parts = [wl.ecdsa_batch(0, 20000, n_keys=8, msg_len=270, corrupt_permille=100, seed=71, nthreads=16)[0],
             wl.ecdsa_batch(1, 20000, n_keys=8, msg_len=270, corrupt_permille=100, seed=72, nthreads=16)[0]]
    parts += [rb] * 3
    b, _ = wl.concat(parts, shuffle_seed=73)
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    assert (st == B.VALID).sum() > 30000


@pytest.mark.parametrize("mode", [B.MODE_DOVERIFY, B.MODE_ISVALID])
def test_spki_golden(engine, mode):
    """Every SubjectPublicKeyInfo form of tests/golden/spki.json (accepted variants and malformed
    encodings, all three schemes; Crypto.kt:321-325) gets the oracle's verdict."""
    _check(engine, golden_io.load("spki.json"), mode)


def test_all_spki_mixed_batch_vs_c_oracle(engine):
    """A 70/20/10 mixed batch whose keys are all SPKI (what the Kotlin binding sends: canonical
    forms plus the NULL-parameter / compressed / hybrid variants), bit-exact against the C oracle
    and equal to the same batch with raw keys."""
    from tools.workload import wl
    parts = [wl.ed25519_batch(21000, n_keys=700, msg_len=270, corrupt_permille=120, seed=51, bad_key_every=61,
                              nthreads=16)[0],
             wl.ecdsa_batch(0, 6000, n_keys=300, msg_len=270, corrupt_permille=120, seed=52, nthreads=16)[0],
             wl.ecdsa_batch(1, 3000, n_keys=150, msg_len=270, corrupt_permille=120, seed=53, nthreads=16)[0]]
    raw, _ = wl.concat(parts, shuffle_seed=54)
    b = golden_io.spki_rekey(raw)
    assert np.all(b.keys["fmt"] == B.KEY_SPKI)
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    assert np.array_equal(st, engine.verify(raw, B.MODE_DOVERIFY))
    assert (st == B.VALID).sum() > 20000 and (st == B.KEY_INVALID).any()


def test_mixed_golden_shuffled(engine):
    """Ed25519 and ECDSA items interleaved in one batch, shuffled, keys shared."""
    items = golden_io.load("ed25519.json") + golden_io.load("ecdsa.json")
    rng = np.random.default_rng(3)
    perm = rng.permutation(len(items))
    items = [items[i] for i in perm]
    b, exp, _ = golden_io.sig_batch(items)
    st = engine.verify(b, B.MODE_DOVERIFY)
    assert np.array_equal(st, exp)


def test_synthetic_ed25519_vs_c_oracle(engine):
    from tools.workload import wl
    b, labels = wl.ed25519_batch(60000, n_keys=512, msg_len=270, corrupt_permille=150, seed=11, bad_key_every=64,
                                 nthreads=16)
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    # labels: A1/A2/A3/A6 invalid, A4 valid, A7 malformed (where the key decodes)
    kok = ref != B.KEY_INVALID
    assert np.all(st[(labels == 0) & kok] == B.VALID)
    assert np.all(st[np.isin(labels, [1, 2, 3, 6]) & kok] == B.INVALID)
    assert np.all(st[(labels == 4) & kok] == B.VALID)
    assert np.all(st[(labels == 7) & kok] == B.SIG_MALFORMED)


def test_key_use_modes_vs_c_oracle(engine):
    """Keys get full row tables, row 0 only, or no rows by how many items use them in the batch
    (keyws.h ED_DIRECT_MAX_USES): keys around the threshold (30000 items over 512 / 1000 keys), keys with one or two items,
    hot keys and unused keys in one shuffled batch, all bit-exact against the C oracle."""
    from tools.workload import wl
    parts = []
    for n_items, n_keys, seed in ((30000, 512, 21), (24000, 8000, 22), (30000, 1000, 23), (3000, 3000, 24)):
        b, _ = wl.ed25519_batch(n_items, n_keys=n_keys, msg_len=200, corrupt_permille=150, seed=seed,
                                bad_key_every=97, nthreads=16)
        parts.append(b)
    b, _ = wl.concat(parts, shuffle_seed=25)
    uses = np.bincount(b.items["key_idx"], minlength=len(b.keys))
    assert (uses == 0).any() and (uses == 1).any() and (uses >= 32).any() and ((uses > 1) & (uses < 32)).any()
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"


def test_key_use_modes_ecdsa_vs_c_oracle(engine):
    """The same table sizing for secp256r1 / secp256k1 keys (row 0 + 252-doubling ladder for keys
    with few items), mixed with Ed25519 keys in one batch, bit-exact against the C oracle."""
    from tools.workload import wl
    parts = []
    for curve in (0, 1):
        for n_items, n_keys, seed in ((6000, 64, 31), (5000, 2500, 32), (6000, 200, 33)):
            b, _ = wl.ecdsa_batch(curve, n_items, n_keys=n_keys, msg_len=150, corrupt_permille=120,
                                  seed=seed + 10 * curve, nthreads=16)
            parts.append(b)
    e, _ = wl.ed25519_batch(5000, n_keys=2000, msg_len=150, corrupt_permille=120, seed=39, nthreads=16)
    b, _ = wl.concat(parts + [e], shuffle_seed=40)
    uses = np.bincount(b.items["key_idx"], minlength=len(b.keys))
    assert (uses == 1).any() and (uses >= 32).any()
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"


def test_wide_tables_vs_c_oracle(engine):
    """Keys with >= KEY_WIDE_MIN_USES items get wide tables (keyws.h: one row per radix-2^8 digit,
    the radix-2^12 base-point tables, no doublings) next to full-table, row-0 and invalid keys of
    all three schemes in one shuffled batch; bit-exact against the C oracle through the host-buffer
    and the device-resident entry points."""
    from tools.workload import wl
    parts = [wl.ed25519_batch(40000, n_keys=16, msg_len=270, corrupt_permille=120, seed=61, bad_key_every=7,
                              nthreads=16)[0],
             wl.ed25519_batch(16000, n_keys=40, msg_len=200, corrupt_permille=120, seed=62, nthreads=16)[0],
             wl.ed25519_batch(3000, n_keys=2000, msg_len=100, corrupt_permille=120, seed=63, nthreads=16)[0],
             wl.ecdsa_batch(0, 14000, n_keys=14, msg_len=270, corrupt_permille=120, seed=64, nthreads=16)[0],
             wl.ecdsa_batch(1, 9000, n_keys=9, msg_len=270, corrupt_permille=120, seed=65, nthreads=16)[0],
             wl.ecdsa_batch(0, 4000, n_keys=100, msg_len=100, corrupt_permille=120, seed=66, nthreads=16)[0]]
    b, _ = wl.concat(parts, shuffle_seed=67)
    uses = np.bincount(b.items["key_idx"], minlength=len(b.keys))
    ed = b.keys["scheme"] == 4
    assert (uses[ed] >= 2400).sum() >= 14 and (uses[~ed] >= 900).sum() >= 20   # wide (keyws.h thresholds)
    assert ((uses >= 32) & (uses < 512)).any() and (uses == 1).any()
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    assert (st == B.VALID).sum() > 60000 and (st == B.KEY_INVALID).any()
    import torch  # the device-resident entry point (HBM buffers, the bench's form)
    dev = torch.device("cuda", 0)
    kd = torch.from_numpy(b.keys.view(np.uint8)).to(dev)
    idd = torch.from_numpy(b.items.view(np.uint8)).to(dev)
    ad = torch.from_numpy(b.arena).to(dev)
    sd = torch.full((b.n,), 255, dtype=torch.uint8, device=dev)
    engine.verify_device(kd.data_ptr(), len(b.keys), idd.data_ptr(), b.n, ad.data_ptr(), b.arena.size, sd.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(sd.cpu().numpy(), ref)


def test_long_messages_vs_c_oracle(engine):
    """Clear data longer than ITEM_LONG_MIN (1 KB) is hashed in waves of its own (plan_sort.hip:
    the long bit sorts those items after the short ones of their class and table mode), up to
    1 MB (CryptoUtilsTest.kt exercises 1 MB messages); every verdict equals the C oracle's, in one
    shuffled batch with short items of all three schemes."""
    from tools.workload import wl
    parts = [wl.ed25519_batch(30000, n_keys=300, msg_len=270, corrupt_permille=120, seed=71, nthreads=16)[0],
             wl.ed25519_batch(200, n_keys=50, msg_len=65536, corrupt_permille=120, seed=72, nthreads=16)[0],
             wl.ed25519_batch(300, n_keys=300, msg_len=1500, corrupt_permille=120, seed=73, nthreads=16)[0],
             wl.ed25519_batch(2, n_keys=2, msg_len=1 << 20, corrupt_permille=0, seed=74, nthreads=2)[0],
             wl.ecdsa_batch(1, 6000, n_keys=60, msg_len=270, corrupt_permille=120, seed=75, nthreads=16)[0],
             wl.ecdsa_batch(1, 150, n_keys=30, msg_len=20000, corrupt_permille=120, seed=76, nthreads=16)[0],
             wl.ecdsa_batch(0, 100, n_keys=100, msg_len=4096, corrupt_permille=120, seed=77, nthreads=16)[0],
             wl.ecdsa_batch(0, 2, n_keys=2, msg_len=1 << 20, corrupt_permille=0, seed=78, nthreads=2)[0]]
    b, _ = wl.concat(parts, shuffle_seed=79)
    assert (b.items["msg_len"] >= (1 << 20)).sum() == 4 and (b.items["msg_len"] > 1024).sum() > 700
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    assert (st[b.items["msg_len"] >= (1 << 20)] == B.VALID).all()


def test_host_buffer_chunked_path(engine):
    """cg_verify_batch on a batch large enough for the chunked H2D / verify pipeline: verdicts
    equal the C oracle's, including items whose offsets point outside the arena (CG_NOT_RUN) in a
    late chunk, and equal the single-copy fallback taken when the keys sit at the arena's end."""
    from corda_amd.batch import Batch
    from tools.workload import wl
    b, _ = wl.ed25519_batch(200000, n_keys=4096, msg_len=120, corrupt_permille=100, seed=51, nthreads=16)
    items = b.items.copy()
    items[190000]["msg_off"] = b.arena.size + 7
    items[199999]["sig_off"] = b.arena.size - 10
    b = Batch(b.keys, items, b.arena)
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    assert st[190000] == B.NOT_RUN and st[199999] == B.NOT_RUN
    # keys moved behind the items: one copy, same verdicts
    kb = np.concatenate([b.arena, np.zeros((-b.arena.size) % 4, np.uint8)])
    keys = b.keys.copy()
    parts = [kb]
    off = kb.size
    for j in range(len(keys)):
        o, n = int(keys[j]["off"]), int(keys[j]["len"])
        parts.append(b.arena[o:o + n])
        keys[j]["off"] = off
        off += n
    b2 = Batch(keys, items, np.concatenate(parts + [np.zeros(64, np.uint8)]))
    st2 = engine.verify(b2, B.MODE_DOVERIFY)
    assert np.array_equal(st2[:190000], st[:190000]) and np.array_equal(st2[190001:199999], st[190001:199999])


def test_edge_batches(engine):
    from corda_amd.batch import BatchBuilder
    items = golden_io.load("ed25519.json")
    # empty batch
    eb = BatchBuilder().build()
    assert engine.verify(eb).size == 0
    # unsupported scheme, bad key index, item outside the arena
    bb = BatchBuilder()
    it = items[5]
    k = bb.key(4, 0, bytes.fromhex(it["key"]))
    bb.add(k, bytes.fromhex(it["sig"]), bytes.fromhex(it["msg"]))
    k1 = bb.key(1, 1, b"\x30" * 300)  # RSA key: unsupported
    bb.add(k1, b"\x01" * 256, b"m")
    b = bb.build()
    items_arr = b.items.copy()
    extra = np.zeros(2, dtype=B.ITEM_DTYPE)
    extra[0] = items_arr[0]
    extra[0]["key_idx"] = 99  # out of range
    extra[1] = items_arr[0]
    extra[1]["msg_off"] = b.arena.size + 100  # outside arena
    b.items = np.concatenate([items_arr, extra])
    st = engine.verify(b)
    assert st.tolist() == [B.STATUS_BY_NAME[it["expect"]], B.UNSUPPORTED, B.NOT_RUN, B.NOT_RUN]


def test_sha_fixtures(engine):
    fx = golden_io.load("sha.json")
    msgs = [bytes.fromhex(x["msg"]) for x in fx]
    assert [d.hex() for d in engine.sha256(msgs)] == [x["sha256"] for x in fx]
    assert [d.hex() for d in engine.sha512(msgs)] == [x["sha512"] for x in fx]


def test_merkle_fixtures(engine):
    from corda_amd import merkle
    fx = golden_io.load("merkle.json")
    roots = [x for x in fx if x["kind"] == "root"]
    got, st = engine.merkle_roots([[bytes.fromhex(l) for l in x["leaves"]] for x in roots] + [[]])
    assert [g.hex() for g in got[:-1]] == [x["root"] for x in roots]
    assert st.tolist() == [0] * len(roots) + [1]
    txs = [x for x in fx if x["kind"] == "txid"]
    ids, st = merkle.tx_ids([([bytes.fromhex(c) for c in x["components"]], bytes.fromhex(x["salt"]),
                              bytes.fromhex(x["salt_blob"])) for x in txs], engine)
    assert [i.hex() for i in ids] == [x["id"] for x in txs]


def test_tx_ids_random_vs_oracle(engine):
    from corda_amd import merkle
    rng = np.random.default_rng(5)
    txs = []
    for t in range(3000):
        n = int(rng.integers(0, 20))
        blobs = [rng.integers(0, 256, int(rng.integers(0, 700)), dtype=np.uint8).tobytes() for _ in range(n)]
        salt = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        txs.append((blobs, salt, b"\x01" + salt))
    ids, st = merkle.tx_ids(txs, engine)
    for (blobs, salt, sb), got in zip(txs, ids):
        assert got == ocorda.tx_id(blobs, salt, sb)
    assert np.all(st == 0)


def test_tx_ids_of_kryo_encoded_components(engine):
    """WireTransaction ids over components encoded by the Kryo writer (corda_amd/kryo.py, pinned by
    the tutorial capture, tests/test_kryo.py): the GPU ids equal the oracle's MerkleTransaction.kt
    rule over the same encoded bytes, for transactions of every component type."""
    import hashlib
    from corda_amd import kryo as K, merkle
    rng = np.random.default_rng(6)
    txs = []
    for t in range(500):
        key = K.PublicKeyRef(4, rng.integers(0, 256, 32, dtype=np.uint8).tobytes())
        notary = K.Party(K.x500_der(f"CN=Notary{t % 7},O=R3,L=London,C=GB"), key)
        h = lambda: K.SecureHash(rng.integers(0, 256, 32, dtype=np.uint8).tobytes())  # noqa: E731
        iou = lambda: K.CordaObject("com.example.state.IOUState", (  # noqa: E731
            ("iou", "object", K.CordaObject("com.example.state.IOU", (("value", "int", int(rng.integers(0, 1 << 30))),))),
            ("recipient", "party", notary), ("sender", "party", notary)))
        wtx = K.WireTransaction(
            inputs=[K.StateRef(h(), int(i)) for i in range(int(rng.integers(0, 4)))],
            attachments=[h() for _ in range(int(rng.integers(0, 2)))],
            outputs=[K.TransactionState(iou(), notary) for _ in range(int(rng.integers(1, 4)))],
            commands=[K.Command(K.CordaObject("com.example.contract.IOUContract$Commands$Create"), (key,))],
            notary=notary, time_window=K.TimeWindow((1_700_000_000 + t, 0), None) if t % 2 else None,
            privacy_salt=K.PrivacySalt(hashlib.sha256(bytes([t % 256, t // 256])).digest()))
        d = wtx.data()
        txs.append((d.components, d.salt, d.salt_blob))
    ids, st = merkle.tx_ids(txs, engine)
    assert np.all(st == 0)
    for (blobs, salt, sb), got in zip(txs, ids):
        assert got == ocorda.tx_id(blobs, salt, sb)


def test_tutorial_transaction_end_to_end(engine):
    """The reference's captured transaction (docs/source/tutorial-cordapp.rst) through the engine:
    SHA-256 of its six Kryo components (rebuilt by the writer) and their Merkle root give the
    printed id; the two printed Ed25519 signatures over that id verify (and the swapped pairs do
    not), with raw and SPKI keys."""
    from kryo_fixtures import _captures, tutorial_components
    t = _captures()["tutorial"]
    leaves = engine.sha256(tutorial_components())
    roots, st = engine.merkle_roots([leaves])
    assert st[0] == 0 and roots[0].hex().upper() == t["id"]
    tx_id = roots[0]
    keys = [bytes.fromhex(k)[-32:] for k in t["signers"]]
    sigs = [bytes.fromhex(s) for s in t["sigs"]]
    b = B.BatchBuilder()
    for i, k in enumerate(keys):
        for j, s in enumerate(sigs):
            b.add_with_key(4, B.KEY_RAW, k, s, tx_id)
            b.add_with_key(4, B.KEY_SPKI, ocorda.ED25519_SPKI_PREFIX + k, s, tx_id)
    got = engine.verify(b.build(), B.MODE_DOVERIFY)
    assert list(got) == [B.VALID, B.VALID, B.INVALID, B.INVALID, B.INVALID, B.INVALID, B.VALID, B.VALID]


@pytest.mark.parametrize("mode", [B.MODE_DOVERIFY, B.MODE_ISVALID])
def test_reference_ed25519_signatures(engine, mode):
    """The tutorial's i2p-made signatures and builder-made corruptions of them
    (tests/golden/ref_ed25519.json)."""
    _check(engine, golden_io.load("ref_ed25519.json"), mode)


def test_crypto_api_behaviour():
    """The reference's own behavioural tests (CryptoUtilsTest.kt:233-286,
    TransactionSignatureTest.kt:33-40) through the host mirror."""
    from corda_amd.crypto import (Crypto, IllegalArgumentException, PublicKey, SignatureException)
    from oracle import ed25519_i2p as ed
    seed = ed.entropy_seed(70)
    pub = PublicKey(4, ed.public_from_seed(seed))
    data = b"Hello World"
    sig = ed.sign(seed, data)
    assert Crypto.do_verify(pub, sig, data) is True
    assert Crypto.is_valid(pub, sig, data) is True
    with pytest.raises(IllegalArgumentException):
        Crypto.do_verify(pub, sig, b"")
    with pytest.raises(IllegalArgumentException):
        Crypto.do_verify(pub, b"", data)
    zeros = bytes(100)
    assert Crypto.do_verify(pub, ed.sign(seed, zeros), zeros)
    big = np.random.default_rng(1).integers(0, 256, 1000000, dtype=np.uint8).tobytes()
    assert Crypto.do_verify(pub, ed.sign(seed, big), big)
    bad = bytearray(sig)
    bad[0] = (bad[0] + 1) & 0xFF
    with pytest.raises(SignatureException):
        Crypto.do_verify(pub, bytes(bad), data)
    assert Crypto.is_valid(pub, bytes(bad), data) is False
    with pytest.raises(SignatureException):
        Crypto.is_valid(pub, sig[:63], data)


@pytest.mark.parametrize("curve", [0, 1])
def test_synthetic_ecdsa_vs_c_oracle(engine, curve):
    from tools.workload import wl
    b, labels = wl.ecdsa_batch(curve, 20000, n_keys=256, msg_len=270, corrupt_permille=150, seed=21 + curve,
                               nthreads=16)
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"
    assert np.all(st[labels == 0] == B.VALID) and np.all(st[labels == 2] == B.VALID)
    assert np.all(st[np.isin(labels, [1, 3])] == B.INVALID)
    assert np.all(st[np.isin(labels, [6, 7])] == B.SIG_MALFORMED)


def test_mixed_notary_batch_vs_c_oracle(engine):
    """Config 5 shape in miniature: 70% Ed25519 / 20% P-256 / 10% k1, shuffled."""
    from tools.workload import wl
    e, _ = wl.ed25519_batch(14000, n_keys=256, corrupt_permille=120, seed=31, nthreads=16)
    r1, _ = wl.ecdsa_batch(1, 4000, n_keys=128, corrupt_permille=100, seed=32, nthreads=16)
    k1, _ = wl.ecdsa_batch(0, 2000, n_keys=128, corrupt_permille=100, seed=33, nthreads=16)
    b, _ = wl.concat([e, r1, k1], shuffle_seed=34)
    st = engine.verify(b, B.MODE_DOVERIFY)
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    assert np.array_equal(st, ref), f"{np.count_nonzero(st != ref)} mismatches"


def test_tx_pipeline_vs_generator_and_oracle(engine):
    """Config 4 in miniature through cg_verify_transactions: ids computed on the GPU equal
    the generator's and the oracle's WireTransaction.id; every signature over the spliced
    SignableData(id) gets the verdict of its label, and a sample matches the oracle."""
    from corda_amd import signable
    from tools.workload import wl
    w = wl.tx_pipeline(3000, n_keys=97, seed=41, corrupt_permille=60, nthreads=16)
    ids, txst, sst = engine.verify_transactions(w.txs, w.comps, w.keys, w.sigs, w.tmpls, w.arena)
    assert np.all(txst == 0)
    assert np.array_equal(ids, w.ids)
    a = w.arena.tobytes()
    for t in range(0, len(w.txs), 97):
        r = w.txs[t]
        cs = w.comps[r["first"]:r["first"] + r["n"]]
        blobs = [a[c["off"]:c["off"] + c["len"]] for c in cs]
        assert ocorda.tx_id(blobs[:-1], a[r["salt_off"]:r["salt_off"] + 32], blobs[-1]) == ids[t].tobytes()
    assert np.all(sst[w.labels == 0] == B.VALID)
    assert np.all(sst[w.labels == 1] == B.INVALID)
    assert np.count_nonzero(w.labels) > 0
    for j in range(0, len(w.sigs), 53):
        s = w.sigs[j]
        k = w.keys[s["key_idx"]]
        msg = signable.serialize(ids[s["tx_idx"]].tobytes(), 1, 4)
        want = ocorda.verify_item(4, 0, a[k["off"]:k["off"] + 32], a[s["sig_off"]:s["sig_off"] + 64], msg)
        assert sst[j] == want


def test_tx_pipeline_edges(engine):
    """Empty transaction (MerkleTreeException), signature rows pointing at a missing tx or
    template: CG_NOT_RUN; mixed-scheme signers (Ed25519 + secp256r1) through the host mirror
    with the serial loop's first-failure semantics (TransactionWithSignatures.kt:58-61)."""
    from corda_amd import signable
    from corda_amd import transactions as T
    from corda_amd.crypto import PublicKey, SignatureException
    from oracle import ecdsa_bc as ec, ed25519_i2p as ed
    rng = np.random.default_rng(9)
    seeds = [ed.entropy_seed(20 + i) for i in range(3)]
    ed_keys = [PublicKey(4, ed.public_from_seed(s)) for s in seeds]
    d = 0x1234567890abcdef1234567890abcdef1234567890abcdef1234567890abcdef
    r1_key = PublicKey(3, ec.raw_key(ec.public_point(3, d)))
    stxs, expect = [], []
    for t in range(12):
        comps = [rng.integers(0, 256, int(rng.integers(1, 300)), dtype=np.uint8).tobytes()
                 for _ in range(0 if t == 5 else int(rng.integers(1, 9)))]
        salt = rng.integers(0, 256, 32, dtype=np.uint8).tobytes()
        wtx = T.WireTransactionData(comps, salt, b"\x01" + salt)
        tid = ocorda.tx_id(comps, salt, b"\x01" + salt)
        sigs = []
        for i, s in enumerate(seeds):
            sigs.append(T.TransactionSignature(ed.sign(s, signable.serialize(tid, 1, 4)), ed_keys[i], 1, 4))
        rr, ss = ec.sign(3, d, signable.serialize(tid, 1, 3), 1000 + t)
        sigs.append(T.TransactionSignature(ec.der_encode_sig(rr, ss), r1_key, 1, 3))
        bad = None
        if t % 3 == 1:  # corrupt signature 2 and 3: the first failure (index 2) must be reported
            for i in (2, 3):
                b = bytearray(sigs[i].bytes)
                b[4] ^= 1
                sigs[i] = T.TransactionSignature(bytes(b), sigs[i].by, 1, sigs[i].scheme_number_id)
            bad = 2
        if t % 4 == 2:  # metadata mismatch: signed for schemeNumberID 4, claims 3 -> invalid
            sigs[0] = T.TransactionSignature(sigs[0].bytes, sigs[0].by, 1, 3)
            bad = 0
        stxs.append(T.SignedWireTransaction(wtx, sigs))
        expect.append((bad, tid))
    ids, results = T.verify_wire_transactions(stxs)
    for (bad, tid), got_id, res in zip(expect, ids, results):
        assert got_id == tid  # t = 5: no components, the salt leaf alone
        if bad is None:
            assert res is None
        else:
            assert res[0] == bad and isinstance(res[1], SignatureException)
    # raw ABI: rows pointing at a missing tx / template, and a transaction with no leaves at
    # all (MerkleTree.getMerkleTree on an empty list -> MerkleTreeException): CG_NOT_RUN
    txs, comps, keys, sigs, tmpls, arena = T.pack_signed_transactions(stxs[:3])
    sigs = sigs.copy()
    sigs[0]["tx_idx"] = 99
    sigs[1]["tmpl"] = 7
    txs = txs.copy()
    txs[2]["n"] = 0
    _, txst, sst = engine.verify_transactions(txs, comps, keys, sigs, tmpls, arena)
    assert sst[0] == B.NOT_RUN and sst[1] == B.NOT_RUN
    assert txst.tolist() == [0, 0, 1]
    assert np.all(sst[sigs["tx_idx"] == 2] == B.NOT_RUN)
    assert sst[2:8].tolist() == [B.VALID, B.VALID, B.VALID, B.VALID, B.INVALID, B.INVALID]  # tx 1: sigs 2, 3 bad
