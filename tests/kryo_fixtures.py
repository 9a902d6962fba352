"""Objects rebuilt from the reference's Kryo captures (tests/golden/kryo_captures.json), shared by
tests/test_kryo.py and the GPU tests."""
import json
import os
import uuid as uuidlib

from corda_amd import kryo as K

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _captures():
    with open(os.path.join(GOLDEN, "kryo_captures.json")) as f:
        return json.load(f)


def _signed_long(v):
    return v - (1 << 64) if v >= 1 << 63 else v


def tutorial_notary_key():
    """The notary's Ed25519 key: the one value the tutorial does not print, read off the capture
    (the chunk after the notary Party's class name: 22 | 2e 20 | A)."""
    cap = bytes.fromhex(_captures()["tutorial"]["tx_bits"])
    i = cap.index(b"net.corda.core.identity.Part\xf9") + 29
    assert cap[i:i + 3] == b"\x22\x2e\x20"
    return cap[i + 3:i + 35]


def tutorial_objects():
    """The tutorial transaction's objects, rebuilt from the values it prints."""
    t = _captures()["tutorial"]
    key_b, key_a = [K.PublicKeyRef(4, bytes.fromhex(k)[-32:]) for k in t["signers"]]
    node_a = K.Party(K.x500_der(t["recipient"]), key_a)
    node_b = K.Party(K.x500_der(t["sender"]), key_b)
    notary = K.Party(K.x500_der(t["notary"]), K.PublicKeyRef(4, tutorial_notary_key()))
    u = uuidlib.UUID(t["uuid"])
    state = K.CordaObject("com.example.state.IOUState", (
        ("iou", "object", K.CordaObject("com.example.state.IOU", (("value", "int", t["iou_value"]),))),
        ("linearId", "object", K.CordaObject("net.corda.core.contracts.UniqueIdentifier", (
            ("externalId", "string", None),
            ("id", "object", K.CordaObject("java.util.UUID", (
                ("leastSigBits", "long", _signed_long(u.int & ((1 << 64) - 1))),
                ("mostSigBits", "long", _signed_long(u.int >> 64)))))))),
        ("recipient", "party", node_a), ("sender", "party", node_b)))
    return {"output": K.TransactionState(state, notary),
            "command": K.Command(K.CordaObject(t["command_class"]), (key_b, key_a)),
            "notary": notary, "must_sign": [key_b, key_a],
            "type": K.CordaObject("net.corda.core.contracts.TransactionType$General", kotlin_object=True)}


def tutorial_tx_bits():
    """The tutorial's WireTransaction through the writer. Outer shape = that version's
    WireTransactionSerializer (inputs, attachments, outputs, commands, notary, mustSign, type,
    timeWindow, each writeClassAndObject, registered as WireTransaction = 12 and written under
    noReferencesWithin<WireTransaction>, DefaultKryoCustomizer.kt:80); everything inside is the
    generic machinery."""
    reg, o = K.TUTORIAL, tutorial_objects()
    k = K.Kryo(references=True)
    out = K.Output()
    out.write_bytes(K.HEADER)
    out.write_atomic(K.varint(reg.wire_transaction + 2))
    out.write_atomic(K.varint(K.NOT_NULL))       # references on at the top: a new object
    k.references = False                         # NoReferencesSerializer (Kryo.kt:474-496)
    lst = lambda items: (reg.array_list, [K.to_java(reg, x) for x in items])  # noqa: E731
    for jc, v in (lst([]), lst([]), lst([o["output"]]), lst([o["command"]]), K.to_java(reg, o["notary"]),
                  lst(o["must_sign"]), K.to_java(reg, o["type"])):
        k.write_class_and_object(out, jc, v)
    k.write_class_and_object(out, None, None)    # timeWindow = null
    return out.getvalue()


def tutorial_components():
    """That version's availableComponents (outputs, commands, notary, mustSign keys, type), each
    serialised alone without references: the Merkle leaves' preimages."""
    o = tutorial_objects()
    return [K.serialize(x, references=False, reg=K.TUTORIAL)
            for x in [o["output"], o["command"], o["notary"]] + o["must_sign"] + [o["type"]]]
