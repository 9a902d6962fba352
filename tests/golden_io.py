"""Loads tests/golden/*.json fixtures into packed batches (test helper)."""
import json
import os

from corda_amd.batch import STATUS_BY_NAME, BatchBuilder

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)["items"]


def sig_batch(items):
    """Packs fixture items; returns (batch, expected_doverify, expected_isvalid) arrays."""
    import numpy as np
    b = BatchBuilder()
    for it in items:
        b.add_with_key(it["scheme"], it["key_fmt"], bytes.fromhex(it["key"]), bytes.fromhex(it["sig"]),
                       bytes.fromhex(it["msg"]))
    exp = np.array([STATUS_BY_NAME[i["expect"]] for i in items], dtype=np.uint8)
    exp_iv = np.array([STATUS_BY_NAME[i["expect_isvalid"]] for i in items], dtype=np.uint8)
    return b.build(), exp, exp_iv


def spki_rekey(b, seed=0):
    """The same batch with every key re-encoded as an X.509 SubjectPublicKeyInfo (CG_KEY_SPKI), the
    form the Kotlin binding sends: keys are appended to the arena and the key table rewritten.
    Ed25519 keys get the canonical 44-byte form, or the 46-byte NULL-parameter form for every
    fifth key; EC keys get the uncompressed form, or for every third key the compressed one, for
    every fifth the hybrid one (raw keys that are not on the curve stay uncompressed)."""
    import numpy as np
    from corda_amd import keys as K
    from corda_amd.batch import Batch
    from oracle import corda as ocorda, ecdsa_bc
    rng = np.random.default_rng(seed)
    arena = bytes(b.arena)
    extra = bytearray()
    base = (len(arena) + 3) & ~3
    keys = b.keys.copy()
    for i, k in enumerate(b.keys):
        raw = arena[int(k["off"]):int(k["off"]) + int(k["len"])]
        scheme, fmt = int(k["scheme"]), int(k["fmt"])
        spki = None
        if fmt == K.KEY_RAW and scheme == 4 and len(raw) == 32:
            spki = (ocorda.ED25519_SPKI_PREFIX_NULL if i % 5 == 4 else ocorda.ED25519_SPKI_PREFIX) + raw
        elif fmt == K.KEY_RAW and scheme in (2, 3) and len(raw) == 64:
            x, y = int.from_bytes(raw[:32], "big"), int.from_bytes(raw[32:], "big")
            on = x < ecdsa_bc.CURVES[scheme].p and y < ecdsa_bc.CURVES[scheme].p and \
                ecdsa_bc.CURVES[scheme].on_curve((x, y))
            if on and i % 3 == 2:
                spki = ecdsa_bc.spki_prefix(scheme, 33) + bytes([2 | (y & 1)]) + raw[:32]
            elif on and i % 5 == 4:
                spki = ecdsa_bc.spki_prefix(scheme, 65) + bytes([6 | (y & 1)]) + raw
            else:
                spki = ecdsa_bc.spki_prefix(scheme, 65) + b"\x04" + raw
        if spki is None:
            continue
        pad = (-len(extra)) % 4
        extra += bytes(pad)
        keys[i]["off"] = base + len(extra)
        keys[i]["len"] = len(spki)
        keys[i]["fmt"] = K.KEY_SPKI
        extra += spki
    new_arena = np.frombuffer(arena + bytes(base - len(arena)) + bytes(extra) + bytes(16), dtype=np.uint8).copy()
    return Batch(keys, b.items.copy(), new_arena)
