"""Kryo encoding (corda_amd/kryo.py), pinned by the reference's own captures.

tests/golden/kryo_captures.json (tools/gen/kryo_captures.py) holds what the reference prints:
  * docs/source/tutorial-cordapp.rst: a SignedTransaction's ``txBits`` (1 310 bytes of Kryo),
    its two Ed25519 signatures, its id and the signers' ``toBase58String()`` keys;
  * samples/irs-demo/.../trade.json: two keys this snapshot parses at run time.
The writer rebuilds every captured byte from the values the tutorial prints (the Kryo mechanics:
chunk cascade, EXTENDED field order across the class hierarchy, reference markers, X500Name
framing), and 0.15's EdDSAPublicKey registration (45) from trade.json. The tutorial's version
differs from 0.15 in its WireTransaction serializer (it still had mustSign / TransactionType) and
in one registration id (EdDSAPublicKey 44); the rebuild uses that version's shape for the outer
object only, through the same writer."""
import hashlib

import pytest

from corda_amd import kryo as K
from kryo_fixtures import _captures, tutorial_components, tutorial_notary_key, tutorial_tx_bits
from oracle import corda as ocorda


def test_tutorial_tx_bits_rebuilt_byte_for_byte():
    cap = bytes.fromhex(_captures()["tutorial"]["tx_bits"])
    got = tutorial_tx_bits()
    if got != cap:
        j = next(j for j in range(min(len(got), len(cap))) if got[j] != cap[j]) if got[:len(cap)] != cap[:len(got)] \
            else min(len(got), len(cap))
        pytest.fail(f"first difference at byte {j}: got {got[j:j + 24].hex()} want {cap[j:j + 24].hex()}")


def test_tutorial_tx_id_reproduced():
    """The printed id is the Merkle root (zero-padded to 8 leaves, MerkleTree.kt:27-66) of
    SHA-256 over each component serialised alone without references (that version's
    availableComponents: outputs, commands, notary, mustSign keys, type; no nonces yet):
    reference-held bytes pin the component encoding and the Merkle rules end to end."""
    t = _captures()["tutorial"]
    leaves = [hashlib.sha256(c).digest() for c in tutorial_components()]
    assert len(leaves) == 6
    assert ocorda.merkle_root(leaves).hex().upper() == t["id"]


def test_tutorial_signatures_verify_over_the_id():
    """The tutorial's two signatures are i2p Ed25519 signatures by the two signer keys over the
    32-byte id: the reference's only Ed25519 vectors (also in tests/golden/ref_ed25519.json)."""
    t = _captures()["tutorial"]
    tx_id = bytes.fromhex(t["id"])
    keys = [bytes.fromhex(k)[-32:] for k in t["signers"]]
    sigs = [bytes.fromhex(s) for s in t["sigs"]]
    for i, k in enumerate(keys):
        for j, s in enumerate(sigs):
            st = ocorda.verify_item(4, 0, k, s, tx_id)
            assert st == (ocorda.VALID if i == j else ocorda.INVALID)


def test_base58_keys():
    """PublicKey.toBase58String() = Base58(serialize(key)) with references on: header, class id,
    NOT_NULL, writeBytesWithLength(A). The tutorial's version has EdDSAPublicKey = 44; this
    snapshot (trade.json, parsed at run time) has 45."""
    c = _captures()
    for k in c["tutorial"]["signers"]:
        raw = bytes.fromhex(k)
        assert K.public_key_base58_bytes(K.PublicKeyRef(4, raw[-32:]), reg=K.TUTORIAL) == raw
    for k in c["trade_json"]["keys"]:
        raw = bytes.fromhex(k)
        assert K.public_key_base58_bytes(K.PublicKeyRef(4, raw[-32:]), reg=K.V015) == raw
        assert K.V015.ed_key.reg == 45


def test_component_framing_0_15():
    """The Merkle-leaf form (references off, MerkleTransaction.kt:25,30) of each 0.15 component."""
    h = K.SecureHash(hashlib.sha256(b"prev").digest())
    b = K.serialize(h)
    assert b == K.HEADER + b"\x01\x00" + K.kryo_string("net.corda.core.crypto.SecureHash$SHA256") + \
        b"\x01" + K.kryo_string("OpaqueBytes.bytes") + b"\x21\x21" + h.bytes_ + b"\x00"
    name, names, f = K.decode(K.serialize(K.StateRef(h, 3)))
    assert name == "net.corda.core.contracts.StateRef" and names == ["StateRef.index", "StateRef.txhash"]
    assert f["StateRef.index"] == K.zigzag32(3)
    p = K.Party(K.x500_der("CN=Notary,O=R3,L=London,C=GB"), K.PublicKeyRef(4, bytes(range(32))))
    name, names, f = K.decode(K.serialize(p))
    assert names == ["AbstractParty.owningKey", "Party.name"]      # sorted by the EXTENDED name
    assert f["AbstractParty.owningKey"] == bytes([45 + 2, 32]) + bytes(range(32))
    assert f["Party.name"] == bytes([55 + 2]) + p.name_der        # X500NameSerializer: raw DER
    salt = K.PrivacySalt(bytes(range(1, 33)))
    assert K.serialize(salt).endswith(b"\x21\x21" + salt.bytes_ + b"\x00")


def test_signable_data_template_0_15():
    """SignableData(txId, SignatureMetadata(1, 4)) with references on: class names for the
    unregistered data classes, NOT_NULL markers, the byte[] marker, chunk framing."""
    tid = bytes(range(32))
    b = K.signable_data(tid, 1, 4)
    assert b.startswith(K.HEADER + b"\x01\x00" + K.kryo_string("net.corda.core.crypto.SignableData") + b"\x01\x02" +
                        K.kryo_string("SignableData.signatureMetadata") + K.kryo_string("SignableData.txId"))
    assert b.count(tid) == 1 and b.index(tid) == len(b) - len(tid) - 3
    assert K.signable_data(tid, 1, 3) != b and K.signable_data(tid, 2, 4) != b


def test_chunk_cascade_splits_large_fields():
    """A field larger than OutputChunked's 1024-byte buffer is split into several chunks and
    still reads back as its payload."""
    big = K.CordaObject("com.example.Blob", (("data", "bytes", bytes(range(256)) * 9),))
    ts = K.TransactionState(big, K.Party(K.x500_der("CN=N,C=GB"), K.PublicKeyRef(4, bytes(32))))
    blob = K.serialize(ts)
    name, names, f = K.decode(blob)
    assert names == ["TransactionState.data", "TransactionState.encumbrance", "TransactionState.notary"]
    assert f["TransactionState.encumbrance"] == b"\x00"
    assert bytes(range(256)) * 9 in f["TransactionState.data"] or len(f["TransactionState.data"]) > 2304


def test_wire_transaction_id_from_encoded_components():
    """WireTransaction.id = Merkle root over SHA256(kryo(c_i) || nonce_i) and SHA256(kryo(salt))
    (MerkleTransaction.kt:16-33, 74-93) over the encoded components."""
    h = K.SecureHash(hashlib.sha256(b"prev").digest())
    notary = K.Party(K.x500_der("CN=Notary,O=R3,L=London,C=GB"), K.PublicKeyRef(4, bytes(range(32))))
    iou = K.CordaObject("com.example.state.IOUState", (("iou", "object", K.CordaObject("com.example.state.IOU", (
        ("value", "int", 7),))), ("sender", "party", notary)))
    wtx = K.WireTransaction(inputs=[K.StateRef(h, 0), K.StateRef(h, 1)], attachments=[h],
                            outputs=[K.TransactionState(iou, notary)],
                            commands=[K.Command(K.CordaObject("com.example.Cmd$Create"), (notary.owning_key,))],
                            notary=notary, time_window=K.TimeWindow((1_700_000_000, 5), None),
                            privacy_salt=K.PrivacySalt(bytes(range(1, 33))))
    d = wtx.data()
    assert len(d.components) == 7
    leaves = [hashlib.sha256(c + ocorda.compute_nonce(d.salt, i)).digest() for i, c in enumerate(d.components)]
    leaves.append(hashlib.sha256(d.salt_blob).digest())
    assert ocorda.tx_id(d.components, d.salt, d.salt_blob) == ocorda.merkle_root(leaves)


def test_secure_hash_length_checked():
    with pytest.raises(ValueError):
        K.SecureHash(b"\x00" * 31)
