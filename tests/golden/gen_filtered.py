#!/usr/bin/env python3
"""Generates tests/golden/filtered.json: tear-off fixtures for cg_verify_filtered
(FilteredTransaction.verify, MerkleTransaction.kt:173-178; PartialMerkleTree.build / verify,
PartialMerkleTree.kt:66-156). Expected statuses come from the oracle restatement
(oracle/corda.py). The reference's own PartialMerkleTreeTest.kt cases are restated first
(six leaves "abcdef", hashed here as SHA256(char) because the Kryo bytes of a serialised Char
are not pinned without a JVM), then seeded random tear-offs of transactions with the
corruption classes a notary can receive.

Usage:  python tests/golden/gen_filtered.py      (rewrites tests/golden/filtered.json)
"""
import hashlib
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import corda  # noqa: E402

RNG = random.Random(0xF17E)


def rbytes(n):
    return bytes(RNG.getrandbits(8) for _ in range(n))


def case(cls, root, leaves, ptree, filtered, note=""):
    st = corda.filtered_status(root, leaves, ptree, filtered)
    enc = ([{"blob": b.hex(), "nonce": n.hex()} for b, n in leaves] if filtered else [h.hex() for h in leaves])
    return {"cls": cls, "note": note, "filtered": filtered, "root": root.hex(), "leaves": enc,
            "pmt": [[k, h.hex() if h is not None else None] for k, h in corda.partial_tree_postorder(ptree)],
            "expect": st}


def reference_cases():
    """PartialMerkleTreeTest.kt:160-230 restated (bare PartialMerkleTree.verify)."""
    hashed = [hashlib.sha256(c.encode()).digest() for c in "abcdef"]
    mt = corda.merkle_tree(hashed)
    out = []
    # only left nodes branch (:160-165), include zero leaves (:167-171), include all leaves (:173-177)
    for incl, note in (([hashed[3], hashed[5]], "only left nodes branch"), ([], "include zero leaves"),
                       (hashed, "include all leaves")):
        pt = corda.partial_tree_build(mt, incl)
        out.append(case("ref_ok", mt[1], incl, pt, False, note))
    # too many leaves (:193-199)
    pt = corda.partial_tree_build(mt, [hashed[3], hashed[5]])
    out.append(case("ref_too_many", mt[1], [hashed[3], hashed[5], hashed[0]], pt, False, "too many leaves"))
    # too little leaves (:201-207)
    pt3 = corda.partial_tree_build(mt, [hashed[3], hashed[5], hashed[0]])
    out.append(case("ref_too_few", mt[1], [hashed[3], hashed[5]], pt3, False, "too little leaves"))
    # duplicate leaves (:209-216): five leaves, one included twice
    mt5 = corda.merkle_tree(hashed[:5])
    pt5 = corda.partial_tree_build(mt5, [hashed[3], hashed[4]])
    out.append(case("ref_duplicate", mt5[1], [hashed[3], hashed[4], hashed[4]], pt5, False, "duplicate leaves"))
    # different leaves (:218-223), wrong root (:225-231)
    out.append(case("ref_different", mt[1], [hashed[2], hashed[4]], pt, False, "different leaves"))
    out.append(case("ref_wrong_root", corda.hash_concat(hashed[3], hashed[5]), [hashed[3], hashed[5]], pt, False,
                    "wrong root"))
    # a one-leaf tree is its own root (:69-74, :95)
    pt1 = corda.partial_tree_build(corda.merkle_tree([hashed[0]]), [hashed[0]])
    out.append(case("ref_ok", hashed[0], [hashed[0]], pt1, False, "just a leaf"))
    assert [c["expect"] for c in out] == [0, 0, 0, 1, 1, 1, 1, 1, 0]
    return out


def random_tx():
    n = RNG.randrange(1, 20)
    blobs = [rbytes(RNG.randrange(1, 400)) for _ in range(n)]
    salt = rbytes(32)
    nonces = [corda.compute_nonce(salt, i) for i in range(n)]
    hashes = [corda.sha256(b + nn) for b, nn in zip(blobs, nonces)]
    hashes.append(corda.sha256(b"\x01" + salt))   # the salt leaf (never visible in FilteredLeaves)
    return blobs, nonces, hashes, corda.merkle_tree(hashes)


def filtered_cases(count):
    out = []
    classes = ["ok", "ok", "ok", "tampered_blob", "tampered_nonce", "wrong_root", "missing_leaf", "extra_leaf",
               "shuffled", "empty"]
    for k in range(count):
        cls = classes[k % len(classes)]
        blobs, nonces, hashes, mt = random_tx()
        n = len(blobs)
        vis = sorted(RNG.sample(range(n), RNG.randrange(1, n + 1))) if cls != "empty" else []
        pt = corda.partial_tree_build(mt, [hashes[i] for i in vis])
        leaves = [(blobs[i], nonces[i]) for i in vis]
        root = mt[1]
        if cls == "tampered_blob":
            j = RNG.randrange(len(leaves))
            b = bytearray(leaves[j][0])
            b[RNG.randrange(len(b))] ^= 1 << RNG.randrange(8)
            leaves[j] = (bytes(b), leaves[j][1])
        elif cls == "tampered_nonce":
            j = RNG.randrange(len(leaves))
            leaves[j] = (leaves[j][0], corda.sha256(leaves[j][1]))
        elif cls == "wrong_root":
            root = corda.sha256(root)
        elif cls == "missing_leaf":
            leaves.pop(RNG.randrange(len(leaves)))
        elif cls == "extra_leaf":
            leaves.append(leaves[RNG.randrange(len(leaves))])
        elif cls == "shuffled":   # multiset compare: the order of the visible leaves does not matter
            RNG.shuffle(leaves)
        out.append(case(cls, root, leaves, pt, True))
    return out


def main():
    items = reference_cases() + filtered_cases(120)
    meta = {"generator": "tests/golden/gen_filtered.py", "rng_seed": "0xF17E", "oracle": "oracle/corda.py",
            "status": "0 verify()==true, 1 false, 2 MerkleTreeException (no leaves)"}
    with open(os.path.join(HERE, "filtered.json"), "w") as f:
        json.dump({"meta": meta, "items": items}, f, indent=0)
    from collections import Counter
    print(len(items), "items", dict(Counter((c["cls"], c["expect"]) for c in items)))


if __name__ == "__main__":
    main()
