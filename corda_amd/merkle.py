"""Host mirror of SecureHash / MerkleTree / WireTransaction.id over the GPU hashing kernels.

Reference:
  * SecureHash.sha256 / hashConcat / zeroHash — core/.../crypto/SecureHash.kt:25,37,42
  * MerkleTree.getMerkleTree(leaves).hash — core/.../crypto/MerkleTree.kt:27-66 (empty list
    -> MerkleTreeException; zero-hash padding to 2^k; single leaf is its own root)
  * computeNonce / serializedHash / availableComponentHashes / WireTransaction.id —
    core/.../transactions/MerkleTransaction.kt:16-33,74-93, WireTransaction.kt:39,104
  * PartialMerkleTree.build / verify — core/.../crypto/PartialMerkleTree.kt:45-157;
    FilteredTransaction.verify — MerkleTransaction.kt:146-179 (tear-offs)

Component bytes are the Kryo serialisations produced by the host; this
module only packs them.
"""
import numpy as np

from .batch import (COMPONENT_DTYPE, FLEAF_DTYPE, FLEAF_HASH, FTX_DTYPE, FTX_FILTERED, PMT_INCLUDED, PMT_LEAF,
                    PMT_NODE, PMT_NODE_DTYPE, TX_DTYPE)
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


# ---------------------------------------------------------------- tear-offs
# PartialTree nodes mirror PartialMerkleTree.PartialTree (PartialMerkleTree.kt:53-58).
class IncludedLeaf:
    __slots__ = ("hash",)

    def __init__(self, h):
        self.hash = bytes(h)


class Leaf:
    __slots__ = ("hash",)

    def __init__(self, h):
        self.hash = bytes(h)


class Node:
    __slots__ = ("left", "right")

    def __init__(self, left, right):
        self.left, self.right = left, right


class _FullNode:
    __slots__ = ("hash", "left", "right")

    def __init__(self, h, left=None, right=None):
        self.hash, self.left, self.right = h, left, right


def merkle_tree(leaves, engine=None):
    """MerkleTree.getMerkleTree (MerkleTree.kt:27-66) keeping every node: each level's
    hashConcat pairs are one SHA-256 batch on the GPU."""
    if len(leaves) == 0:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    eng = engine or Crypto.engine()
    lv = [_FullNode(bytes(x)) for x in leaves]
    while len(lv) & (len(lv) - 1):
        lv.append(_FullNode(bytes(32)))
    while len(lv) > 1:
        hs = eng.sha256([lv[i].hash + lv[i + 1].hash for i in range(0, len(lv), 2)])
        lv = [_FullNode(hs[j], lv[2 * j], lv[2 * j + 1]) for j in range(len(hs))]
    return lv[0]


class PartialMerkleTree:
    """PartialMerkleTree (PartialMerkleTree.kt:45-157). ``build`` is host logic over a full tree
    whose node hashes come from the GPU; ``verify`` runs on the GPU (cg_verify_filtered)."""

    def __init__(self, root):
        self.root = root

    @staticmethod
    def build(merkle_root, include_hashes):
        """PartialMerkleTree.build (:66-76): ``merkle_root`` from merkle_tree()."""
        include = [bytes(h) for h in include_hashes]
        if bytes(32) in include:
            raise ValueError("Zero hashes shouldn't be included in partial tree.")

        def check_full(t, level=0):
            if t.left is None:
                return level
            a, b = check_full(t.left, level + 1), check_full(t.right, level + 1)
            if a != b:
                raise MerkleTreeException("Got not full binary tree.")
            return a

        check_full(merkle_root)
        used = []

        def build(t):  # buildPartialTree (:98-123)
            if t.left is None:
                if t.hash in include:
                    used.append(t.hash)
                    return True, IncludedLeaf(t.hash)
                return False, Leaf(t.hash)
            lf, lt = build(t.left)
            rf, rt = build(t.right)
            if lf or rf:
                return True, Node(lt, rt)
            return False, Leaf(t.hash)

        tree = build(merkle_root)[1]
        if len(include) != len(used):
            raise MerkleTreeException("Some of the provided hashes are not in the tree.")
        return PartialMerkleTree(tree)

    def postorder(self):
        """[(kind, hash | None)] in cg_pmt_node post-order (iterative: no recursion limit)."""
        out, stack = [], [(self.root, False)]
        while stack:
            t, expanded = stack.pop()
            if isinstance(t, Node):
                if expanded:
                    out.append((PMT_NODE, None))
                else:
                    stack.append((t, True))
                    stack.append((t.right, False))
                    stack.append((t.left, False))
            else:
                out.append((PMT_INCLUDED if isinstance(t, IncludedLeaf) else PMT_LEAF, t.hash))
        return out

    def verify(self, merkle_root_hash, hashes_to_check, engine=None):
        """PartialMerkleTree.verify (:130-137) on the GPU."""
        st = verify_filtered_batch([(bytes(merkle_root_hash), [bytes(h) for h in hashes_to_check], None, self)],
                                   engine, filtered=False)[0]
        if st == 3:
            raise MerkleTreeException("malformed partial tree")
        return bool(st == 0)


class FilteredTransaction:
    """FilteredTransaction (MerkleTransaction.kt:146-179): rootHash, the visible components'
    serialised bytes with their nonces (FilteredLeaves, :101-138) and the partial tree."""

    def __init__(self, root_hash, component_blobs, nonces, partial_merkle_tree):
        if len(component_blobs) != len(nonces):
            raise ValueError("Each visible component should be accompanied by a nonce.")
        self.root_hash = bytes(root_hash)
        self.component_blobs = [bytes(b) for b in component_blobs]
        self.nonces = [bytes(n) for n in nonces]
        self.partial_merkle_tree = partial_merkle_tree

    def verify(self, engine=None):
        """FilteredTransaction.verify (:173-178): MerkleTreeException without leaves."""
        st = verify_filtered_batch([self], engine)[0]
        return raise_for_filtered_status(st)


def raise_for_filtered_status(st):
    if st == 2:
        raise MerkleTreeException("Transaction without included leaves.")
    if st == 3:
        raise MerkleTreeException("malformed partial tree")
    if st not in (0, 1):
        raise RuntimeError(f"filtered transaction not verified (status {st})")
    return bool(st == 0)


def pack_filtered(ftxs, filtered=True):
    """Pack FilteredTransactions (or (root, leaf_hashes, None, pmt) tuples for bare
    PartialMerkleTree.verify) into the cg_filtered_tx / cg_pmt_node / cg_filtered_leaf tables
    and one arena."""
    chunks, off = [], 0

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

    rows_t, rows_n, rows_l = [], [], []
    for f in ftxs:
        if isinstance(f, FilteredTransaction):
            root, pmt = f.root_hash, f.partial_merkle_tree
            leaves = [(put(b), put(n), len(b), 0) for b, n in zip(f.component_blobs, f.nonces)]
            flags = FTX_FILTERED if filtered else 0
        else:
            root, hashes, _, pmt = f
            leaves = [(put(h), 0, len(h), FLEAF_HASH) for h in hashes]
            flags = 0
        first_node, first_leaf = len(rows_n), len(rows_l)
        for kind, h in pmt.postorder():
            rows_n.append((put(h) if h is not None else 0, kind, 0))
        rows_l.extend(leaves)
        rows_t.append((first_node, first_leaf, put(root), len(rows_n) - first_node, len(leaves), flags, 0))
    arena = np.frombuffer(b"".join(chunks) + bytes(8), dtype=np.uint8).copy()
    t = np.array(rows_t, dtype=FTX_DTYPE) if rows_t else np.zeros(0, FTX_DTYPE)
    n = np.array(rows_n, dtype=PMT_NODE_DTYPE) if rows_n else np.zeros(0, PMT_NODE_DTYPE)
    lv = np.array(rows_l, dtype=FLEAF_DTYPE) if rows_l else np.zeros(0, FLEAF_DTYPE)
    return t, n, lv, arena


def verify_filtered_batch(ftxs, engine=None, filtered=True):
    """Status byte per tear-off (0 true, 1 false, 2 no leaves, 3 malformed), one GPU call: the
    batch form of NonValidatingNotaryFlow.receiveAndVerifyTx's ``it.verify()``
    (NonValidatingNotaryFlow.kt:22-27)."""
    if not ftxs:
        return np.zeros(0, np.uint8)
    t, n, lv, arena = pack_filtered(ftxs, filtered)
    return (engine or Crypto.engine()).verify_filtered(t, n, lv, arena)
