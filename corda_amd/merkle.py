"""Host mirror of SecureHash / MerkleTree / WireTransaction.id over the GPU hashing kernels.

Reference:
  * SecureHash.sha256 / hashConcat / zeroHash — core/.../crypto/SecureHash.kt:25,37,42
  * MerkleTree.getMerkleTree(leaves).hash — core/.../crypto/MerkleTree.kt:27-66 (empty list
    -> MerkleTreeException; zero-hash padding to 2^k; single leaf is its own root)
  * computeNonce / serializedHash / availableComponentHashes / WireTransaction.id —
    core/.../transactions/MerkleTransaction.kt:16-33,74-93, WireTransaction.kt:39,104

Component bytes are the Kryo serialisations produced by the host; this
module only packs them.
"""
import numpy as np

from .batch import COMPONENT_DTYPE, TX_DTYPE
from .crypto import Crypto


class MerkleTreeException(ValueError):
    pass


def sha256_batch(msgs, engine=None):
    return (engine or Crypto.engine()).sha256(msgs)


def merkle_roots(leaf_lists, engine=None):
    roots, st = (engine or Crypto.engine()).merkle_roots(leaf_lists)
    return roots, st


def merkle_root(leaves, engine=None):
    roots, st = merkle_roots([leaves], engine)
    if st[0]:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    return roots[0]


def pack_transactions(txs):
    """txs: list of (component_blobs, salt32, salt_blob). Returns (tx array, component array,
    arena) in the cg_tx / cg_component layout; the salt leaf is appended last."""
    chunks, off = [], 0
    comps, tx_rows = [], []

    def put(b):
        nonlocal off
        pad = (-off) % 4
        if pad:
            chunks.append(bytes(pad))
            off += pad
        o = off
        chunks.append(bytes(b))
        off += len(b)
        return o

    for blobs, salt, salt_blob in txs:
        first = len(comps)
        for b in blobs:
            comps.append((put(b), len(b), 0))
        comps.append((put(salt_blob), len(salt_blob), 1))
        salt_off = put(salt)
        tx_rows.append((first, len(blobs) + 1, 0, salt_off))
    arena = np.frombuffer(b"".join(chunks) + bytes(8), dtype=np.uint8).copy()
    c = np.zeros(len(comps), dtype=COMPONENT_DTYPE)
    for i, row in enumerate(comps):
        c[i] = row
    t = np.zeros(len(tx_rows), dtype=TX_DTYPE)
    for i, row in enumerate(tx_rows):
        t[i] = row
    return t, c, arena


def tx_ids(txs, engine=None):
    t, c, arena = pack_transactions(txs)
    ids, st = (engine or Crypto.engine()).tx_ids(t, c, arena)
    return [bytes(x) for x in ids], st
