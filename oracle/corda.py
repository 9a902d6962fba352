"""Corda-level control flow restated on top of the arithmetic oracles.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

* ``verify_item``  = Crypto.doVerify(scheme, pub, sig, clear) / Crypto.isValid(...)
  (core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:474-484 and :553-559), mapped
  onto the batch status codes of include/cordagpu.h.
* ``merkle_root``  = MerkleTree.getMerkleTree (MerkleTree.kt:27-66).
* ``compute_nonce`` / ``component_hash`` / ``tx_id`` = MerkleTransaction.kt:16-33,93 and
  WireTransaction.id (WireTransaction.kt:39,104).
* ``check_signatures_are_valid`` = TransactionWithSignatures.checkSignaturesAreValid
  (TransactionWithSignatures.kt:58-62): serial, fail-fast on the first bad signature.
"""
import hashlib
import struct

from . import ecdsa_bc, ed25519_i2p

# ---- status codes (must match include/cordagpu.h) ----
VALID = 0          # isValid == true
INVALID = 1        # isValid == false  (doVerify: SignatureException("Signature Verification failed!"))
SIG_MALFORMED = 2  # engine SignatureException (length / DER decode)
KEY_INVALID = 3    # key decode IllegalArgumentException / InvalidKeyException
UNSUPPORTED = 4    # IllegalArgumentException("Unsupported key/algorithm ...")
EMPTY = 5          # doVerify IllegalArgumentException("Signature data is empty!" / "Clear data is empty ...")
NOT_RUN = 255

STATUS_NAMES = {VALID: "VALID", INVALID: "INVALID", SIG_MALFORMED: "SIG_MALFORMED",
                KEY_INVALID: "KEY_INVALID", UNSUPPORTED: "UNSUPPORTED", EMPTY: "EMPTY", NOT_RUN: "NOT_RUN"}

ECDSA_SECP256K1_SHA256 = 2
ECDSA_SECP256R1_SHA256 = 3
EDDSA_ED25519_SHA512 = 4

KEY_RAW = 0    # Ed25519: 32-byte A (as Kryo writes it, Kryo.kt:333); ECDSA: 64-byte X||Y big-endian
KEY_SPKI = 1   # X.509 SubjectPublicKeyInfo DER (PublicKey.encoded)
KEY_SEC1 = 2   # ECDSA only: 04||X||Y or 02/03||X

MODE_DOVERIFY = 0   # Crypto.doVerify semantics: empty sig / clear -> EMPTY
MODE_ISVALID = 1    # Crypto.isValid semantics: no empty checks

ED25519_SPKI_PREFIX = bytes.fromhex("302a300506032b6570032100")
# AlgorithmIdentifier with an explicit NULL parameter: Crypto.findSignatureScheme normalises DERNull
# to absent (Crypto.kt:219-228) and i2p 0.2.0 EdDSAPublicKey.decode accepts this 46-byte form
# (it reads Java keystore output). The old draft OID 1.3.101.100 form i2p also reads is not in
# Corda's algorithmMap (Crypto.kt:190-193), so Crypto.decodePublicKey rejects it.
ED25519_SPKI_PREFIX_NULL = bytes.fromhex("302c300706032b65700500032100")


def ed25519_spki_a(key):
    """The 32-byte A of an Ed25519 SPKI Crypto.decodePublicKey (Crypto.kt:321-325) accepts."""
    if len(key) == 44 and key[:12] == ED25519_SPKI_PREFIX:
        return key[12:]
    if len(key) == 46 and key[:14] == ED25519_SPKI_PREFIX_NULL:
        return key[14:]
    raise ed25519_i2p.KeyDecodeError("bad SubjectPublicKeyInfo")


def decode_key(scheme, key_fmt, key):
    """Returns a decoded key object or raises KeyDecodeError / ValueError."""
    key = bytes(key)
    if scheme == EDDSA_ED25519_SHA512:
        if key_fmt == KEY_SPKI:
            key = ed25519_spki_a(key)
        elif key_fmt != KEY_RAW:
            raise ed25519_i2p.KeyDecodeError("bad key format")
        return ed25519_i2p.PublicKey(key)
    if key_fmt == KEY_SPKI:
        return ecdsa_bc.decode_spki(scheme, key)
    if key_fmt == KEY_RAW and len(key) != 64:
        raise ecdsa_bc.KeyDecodeError("bad raw key length")
    if key_fmt not in (KEY_RAW, KEY_SEC1):
        raise ecdsa_bc.KeyDecodeError("bad key format")
    return ecdsa_bc.decode_point(ecdsa_bc.CURVES[scheme], key)


def verify_item(scheme, key_fmt, key, sig, msg, mode=MODE_DOVERIFY, decoded=None):
    """One batch item -> status byte. Precedence: UNSUPPORTED, KEY_INVALID, EMPTY,
    SIG_MALFORMED, INVALID/VALID (key decode happens before doVerify on the JVM)."""
    if scheme not in (ECDSA_SECP256K1_SHA256, ECDSA_SECP256R1_SHA256, EDDSA_ED25519_SHA512):
        return UNSUPPORTED
    try:
        k = decoded if decoded is not None else decode_key(scheme, key_fmt, key)
    except (ed25519_i2p.KeyDecodeError, ecdsa_bc.KeyDecodeError):
        return KEY_INVALID
    if mode == MODE_DOVERIFY and (len(sig) == 0 or len(msg) == 0):
        return EMPTY
    try:
        if scheme == EDDSA_ED25519_SHA512:
            ok = ed25519_i2p.verify(k, msg, sig)
        else:
            ok = ecdsa_bc.verify(scheme, k, msg, sig)
    except (ed25519_i2p.SignatureLengthError, ecdsa_bc.MalformedSignature):
        return SIG_MALFORMED
    return VALID if ok else INVALID


# ---------------- hashing / Merkle ----------------
ZERO_HASH = bytes(32)


def sha256(b):
    return hashlib.sha256(bytes(b)).digest()


def hash_concat(a, b):
    """SecureHash.hashConcat (SecureHash.kt:25)."""
    return sha256(bytes(a) + bytes(b))


class MerkleTreeException(ValueError):
    pass


def merkle_root(leaves):
    """MerkleTree.getMerkleTree(...).hash (MerkleTree.kt:27-66): empty -> exception,
    zero-hash padding to the next power of two, pairwise SHA256(L||R) per level,
    a single leaf is its own root."""
    if len(leaves) == 0:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    lv = [bytes(x) for x in leaves]
    n = len(lv)
    while n & (n - 1):
        lv.append(ZERO_HASH)
        n += 1
    while len(lv) > 1:
        lv = [hash_concat(lv[i], lv[i + 1]) for i in range(0, len(lv), 2)]
    return lv[0]


def compute_nonce(salt32, index):
    """computeNonce (MerkleTransaction.kt:33): SHA256(salt || BE32(index))."""
    return sha256(bytes(salt32) + struct.pack(">i", index))


def component_hash(blob, salt32, index, is_salt=False):
    """serializedHash(x, privacySalt, index) (MerkleTransaction.kt:16-25)."""
    if is_salt:
        return sha256(blob)
    return sha256(bytes(blob) + compute_nonce(salt32, index))


def tx_id(component_blobs, salt32, salt_blob):
    """WireTransaction.id: Merkle root over availableComponentHashes, the salt's own
    serialised blob appended last (MerkleTransaction.kt:74-93)."""
    hashes = [component_hash(b, salt32, i) for i, b in enumerate(component_blobs)]
    hashes.append(component_hash(salt_blob, salt32, len(component_blobs), is_salt=True))
    return merkle_root(hashes)


class SignatureException(Exception):
    pass


def check_signatures_are_valid(tx_id_bytes, sigs, message_of):
    """TransactionWithSignatures.checkSignaturesAreValid (TransactionWithSignatures.kt:58-62)
    restated over status codes: returns the index of the first non-VALID signature and its
    status (fail-fast order), or (None, VALID)."""
    for i, (scheme, key_fmt, key, sig, meta) in enumerate(sigs):
        st = verify_item(scheme, key_fmt, key, sig, message_of(tx_id_bytes, meta))
        if st != VALID:
            return i, st
    return None, VALID


# ---------------- tear-offs: PartialMerkleTree / FilteredTransaction ----------------
# A MerkleTree / PartialTree is a nested tuple: ("L", hash) leaf, ("I", hash) included leaf
# (partial trees only), ("N", hash_or_None, left, right) node (full trees carry the node hash).

def merkle_tree(leaves):
    """MerkleTree.getMerkleTree (MerkleTree.kt:27-66) keeping the whole tree: zero-hash padding
    to 2^k, then pairwise levels of Node(hashConcat(l, r), l, r)."""
    if len(leaves) == 0:
        raise MerkleTreeException("Cannot calculate Merkle root on empty hash list.")
    lv = [("L", bytes(x)) for x in leaves]
    while len(lv) & (len(lv) - 1):
        lv.append(("L", ZERO_HASH))
    while len(lv) > 1:
        lv = [("N", hash_concat(_thash(lv[i]), _thash(lv[i + 1])), lv[i], lv[i + 1]) for i in range(0, len(lv), 2)]
    return lv[0]


def _thash(t):
    return t[1]


def partial_tree_build(tree, include_hashes):
    """PartialMerkleTree.build (PartialMerkleTree.kt:66-123): zero hash not includable
    (IllegalArgumentException -> ValueError), full-tree check, every leaf whose hash is in
    include_hashes becomes an IncludedLeaf, subtrees without one are cut to a Leaf of their hash,
    and the used count must equal len(include_hashes)."""
    include = [bytes(h) for h in include_hashes]
    if ZERO_HASH in include:
        raise ValueError("Zero hashes shouldn't be included in partial tree.")

    def check_full(t, level=0):
        if t[0] == "L":
            return level
        a, b = check_full(t[2], level + 1), check_full(t[3], level + 1)
        if a != b:
            raise MerkleTreeException("Got not full binary tree.")
        return a

    check_full(tree)
    used = []

    def build(t):
        if t[0] == "L":
            if t[1] in include:
                used.append(t[1])
                return True, ("I", t[1])
            return False, ("L", t[1])
        lf, lt = build(t[2])
        rf, rt = build(t[3])
        if lf or rf:
            return True, ("N", None, lt, rt)
        return False, ("L", t[1])

    pt = build(tree)[1]
    if len(include) != len(used):
        raise MerkleTreeException("Some of the provided hashes are not in the tree.")
    return pt


def partial_tree_verify(ptree, root_hash, hashes_to_check):
    """PartialMerkleTree.verify (PartialMerkleTree.kt:130-156): recursive root, used hashes in
    tree order; groupBy equality (multiset) first, then the root."""
    used = []

    def root(t):
        if t[0] == "I":
            used.append(t[1])
            return t[1]
        if t[0] == "L":
            return t[1]
        return hash_concat(root(t[2]), root(t[3]))

    r = root(ptree)
    a, b = sorted(bytes(h) for h in hashes_to_check), sorted(used)
    if a != b:
        return False
    return r == bytes(root_hash)


def filtered_leaf_hash(blob, nonce):
    """serializedHash(x, nonce) (MerkleTransaction.kt:23-28): SHA256(kryo(x) || nonce)."""
    return sha256(bytes(blob) + bytes(nonce))


def filtered_tx_verify(root_hash, blobs, nonces, ptree):
    """FilteredTransaction.verify (MerkleTransaction.kt:173-178) with FilteredLeaves'
    availableComponentHashes (:137). Raises MerkleTreeException on no leaves."""
    if len(blobs) != len(nonces):
        raise ValueError("Each visible component should be accompanied by a nonce.")
    hashes = [filtered_leaf_hash(b, n) for b, n in zip(blobs, nonces)]
    if not hashes:
        raise MerkleTreeException("Transaction without included leaves.")
    return partial_tree_verify(ptree, root_hash, hashes)


def partial_tree_postorder(ptree):
    """The post-order stream of cg_pmt_node kinds (include/cordagpu.h): [(kind, hash|None)],
    kind 0 node / 1 leaf / 2 included leaf."""
    out = []

    def walk(t):
        if t[0] == "N":
            walk(t[2])
            walk(t[3])
            out.append((0, None))
        else:
            out.append((2 if t[0] == "I" else 1, t[1]))

    walk(ptree)
    return out


def partial_tree_from_postorder(stream):
    """Inverse of partial_tree_postorder: rebuilds the nested PartialTree (raises ValueError on a
    stream that does not reduce to one tree)."""
    stk = []
    for kind, h in stream:
        if kind == 0:
            if len(stk) < 2:
                raise ValueError("node without two children")
            r, l_ = stk.pop(), stk.pop()
            stk.append(("N", None, l_, r))
        elif kind in (1, 2):
            stk.append(("I" if kind == 2 else "L", bytes(h)))
        else:
            raise ValueError("unknown node kind")
    if len(stk) != 1:
        raise ValueError("stream does not reduce to one root")
    return stk[0]


def filtered_status(root_hash, leaves, ptree, filtered=True):
    """Status byte of include/cordagpu.h cg_verify_filtered for one tear-off. ``leaves``:
    [(blob, nonce)] (FilteredTransaction) or [hash] with filtered=False (PartialMerkleTree.verify)."""
    if filtered:
        try:
            ok = filtered_tx_verify(root_hash, [b for b, _ in leaves], [n for _, n in leaves], ptree)
        except MerkleTreeException:
            return 2
    else:
        ok = partial_tree_verify(ptree, root_hash, leaves)
    return 0 if ok else 1
