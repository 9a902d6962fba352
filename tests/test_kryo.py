"""Kryo encoding of WireTransaction components (corda_amd/kryo.py).

PARITY UNPINNED: no JVM capture exists (module docstring lists the assumptions). These tests pin
the structure the restatement commits to: Kryo P2P header, class framing, CompatibleFieldSerializer
schemas (EXTENDED names, field-name order, one chunk per field), determinism, and that the
encoded components feed WireTransaction.id exactly as MerkleTransaction.kt:16-33 prescribes."""
import hashlib

import pytest

from corda_amd import kryo as K
from oracle import corda as ocorda

ED = K.PublicKeyRef(4, bytes(range(32)))
EC = K.PublicKeyRef(3, bytes.fromhex("3059301306072a8648ce3d020106082a8648ce3d030107034200") + b"\x04" + bytes(64))
NOTARY = K.Party(bytes.fromhex("3031310b300906035504061302474231"), ED)   # an X500Name DER stand-in
H = K.SecureHash(hashlib.sha256(b"prev").digest())


def comps():
    return [K.StateRef(H, 0), K.StateRef(H, 7), H,
            K.TransactionState("net.corda.finance.contracts.asset.Cash$State", (("amount", 100), ("owner", b"o" * 44)),
                               "net.corda.finance.contracts.asset.Cash", NOTARY),
            K.TransactionState("com.example.IOUState", (("value", 5),), "com.example.IOUContract", NOTARY, encumbrance=1),
            K.Command("net.corda.finance.contracts.asset.Cash$Commands$Move", (), (ED, EC)),
            NOTARY, K.TimeWindow((1_700_000_000, 5), (1_700_000_060, 0)), K.TimeWindow(None, (1_700_000_060, 1))]


def test_header_class_and_schema_framing():
    for c in comps():
        b = K.serialize(c)
        assert b[:8] == b"corda\x00\x00\x01"
        name, fields = K.decode(b)
        assert name.startswith("net.corda.") or name.startswith("com.example.")
        assert fields and all(isinstance(v, bytes) for v in fields.values())
    name, f = K.decode(K.serialize(K.StateRef(H, 3)))
    assert name == "net.corda.core.contracts.StateRef" and sorted(f) == ["index", "txhash"]
    assert f["index"] == K.zigzag32(3)
    name, f = K.decode(K.serialize(K.TimeWindow((10, 0), None)))
    assert name == "net.corda.core.contracts.TimeWindow$From" and sorted(f) == ["fromTime"]
    name, f = K.decode(K.serialize(K.TimeWindow((10, 0), (20, 0))))
    assert name.endswith("TimeWindow$Between") and sorted(f) == ["fromTime", "untilTime"]


def test_extended_field_names_sorted_by_field():
    b = K.serialize(NOTARY)
    # Party: "name" declared in Party, "owningKey" in AbstractParty (EXTENDED names), sorted by field
    i = b.index(b"Party.nam")
    j = b.index(b"AbstractParty.owningKe")
    assert i < j


def test_deterministic_and_injective():
    cs = comps()
    blobs = [K.serialize(c) for c in cs]
    assert blobs == [K.serialize(c) for c in comps()]
    assert len(set(blobs)) == len(blobs)
    assert K.serialize(K.StateRef(H, 1)) != K.serialize(K.StateRef(H, 2))
    assert K.serialize(K.PrivacySalt(b"\x01" * 32)) != K.serialize(K.PrivacySalt(b"\x02" * 32))


def test_ed25519_key_as_abyte_ec_as_spki():
    b = K.serialize(K.Command("x.Cmd", (), (ED,)))
    assert K.varint(32) + ED.encoded in b  # Ed25519PublicKeySerializer: writeBytesWithLength(A)
    b = K.serialize(K.Command("x.Cmd", (), (EC,)))
    assert K.varint(len(EC.encoded)) + EC.encoded in b  # PublicKeySerializer: writeBytesWithLength(SPKI)


def test_wire_transaction_id_from_encoded_components():
    """WireTransaction.id = Merkle root over SHA256(kryo(c_i) || nonce_i) and SHA256(kryo(salt))
    (MerkleTransaction.kt:16-33, 74-93): the encoded components through the oracle's tx-id rule."""
    wtx = K.WireTransaction(inputs=comps()[:2], attachments=[H], outputs=comps()[3:5], commands=[comps()[5]],
                            notary=NOTARY, time_window=comps()[7], privacy_salt=K.PrivacySalt(bytes(range(32))))
    d = wtx.data()
    assert len(d.components) == 8
    leaves = [hashlib.sha256(c + ocorda.compute_nonce(d.salt, i)).digest() for i, c in enumerate(d.components)]
    leaves.append(hashlib.sha256(d.salt_blob).digest())
    assert ocorda.tx_id(d.components, d.salt, d.salt_blob) == ocorda.merkle_root(leaves)


def test_secure_hash_length_checked():
    with pytest.raises(ValueError):
        K.SecureHash(b"\x00" * 31)
