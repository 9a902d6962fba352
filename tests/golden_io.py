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
