"""Host mirror of TransactionWithSignatures' signature checks, batched onto the GPU.

Reference: core/src/main/kotlin/net/corda/core/transactions/TransactionWithSignatures.kt
  * checkSignaturesAreValid (:58-62) — serial ``for (sig in sigs) sig.verify(id)``; the
    first failing signature's exception escapes.
  * verifySignaturesExcept(vararg allowedToBeMissing) (:41-47) — the check above, then
    SignaturesMissingException for required keys without a signature (:45-46, :72-78).

Here every signature of every transaction goes into ONE engine batch; the per-tx verdict
is then rebuilt in list order so the exception type, message and the index it refers to are
exactly those of the serial loop.

The signed clear data of a TransactionSignature is ``SignableData(txId, metadata)``
serialised with Kryo (Crypto.kt:499-502). ``check_signatures_are_valid_batch`` takes it from
the caller (``signable_data(tx_id, sig) -> bytes``). ``verify_wire_transactions`` is the
whole-pipeline form: it takes WireTransaction components, computes every id on the GPU and
splices the ids into per-metadata SignableData templates (corda_amd/signable.py) on the GPU
too, so the host never serialises per signature. ``verify_chain`` is
ResolveTransactionsFlow's whole dependency chain as one such call (SURVEY §8(f2),
ResolveTransactionsFlow.kt:36-96).
"""
from dataclasses import dataclass, field

import numpy as np

from . import batch as B
from . import signable
from .composite import is_fulfilled_by
from .crypto import (BatchItem, Crypto, HOST_EXCEPTION, IllegalArgumentException, PublicKey,  # noqa: F401
                     SCHEME_CODE_NAMES, GPU_SCHEMES, SignatureException, TransactionSignature)


class SignaturesMissingException(SignatureException):
    """SignedTransaction.SignaturesMissingException (SignedTransaction.kt:171-172): a
    SignatureException carrying the missing keys, their descriptions and the transaction id."""

    def __init__(self, missing, descriptions, tx_id):
        super().__init__(f"Missing signatures for {list(descriptions)} on transaction {bytes(tx_id).hex().upper()[:6]} "
                         f"for {', '.join(repr(k) for k in missing)}")
        self.missing = set(missing)
        self.descriptions = list(descriptions)
        self.id = tx_id

    @property
    def tx_id(self):
        return self.id


@dataclass(frozen=True)
class Command:
    """A command's value (its toString) and signers (Structures.kt Command(value, signers))."""
    value: str
    signers: tuple


@dataclass
class SignedTransaction:
    id: bytes
    sigs: list
    required_signing_keys: set = field(default_factory=set)
    commands: list = field(default_factory=list)   # Command, for getKeyDescriptions
    notary: object = None                          # the notary's owning key


def get_key_descriptions(stx, keys):
    """SignedTransaction.getKeyDescriptions (SignedTransaction.kt:65-75)."""
    out = [c.value for c in getattr(stx, "commands", []) if any(k in keys for k in c.signers)]
    if getattr(stx, "notary", None) is not None and stx.notary in keys:
        out.append("notary")
    return out


def get_missing_signatures(stx):
    """TransactionWithSignatures.getMissingSignatures (TransactionWithSignatures.kt:72-78): the
    required keys not fulfilled by the signatures' keys (composite-aware, CryptoUtils.kt:88-92)."""
    sig_keys = {s.by for s in stx.sigs}
    return {k for k in stx.required_signing_keys if not is_fulfilled_by(k, sig_keys)}


def _items(stxs, signable_data):
    items, owner = [], []
    for t, stx in enumerate(stxs):
        for s in stx.sigs:
            items.append(BatchItem(s.by, s.bytes, signable_data(stx.id, s)))
            owner.append(t)
    return items, owner


def _first_failures(stxs, status, errors, crypto):
    result = [None] * len(stxs)
    pos = 0
    for t, stx in enumerate(stxs):
        for i, s in enumerate(stx.sigs):
            st = int(status[pos + i])
            if st != B.VALID and result[t] is None:
                try:
                    crypto.raise_for_status(st, SCHEME_CODE_NAMES.get(s.by.scheme, ""), do_verify=True,
                                            error=errors.get(pos + i), key=s.by)
                except Exception as e:  # noqa: BLE001 - mirrored JVM exception
                    result[t] = (i, e)
        pos += len(stx.sigs)
    return result


def check_signatures_are_valid_batch(stxs, signable_data, crypto=Crypto):
    """Verifies all signatures of all transactions in one GPU batch (host-verified schemes and
    composite leaves routed by Crypto.verify_batch_ex).

    Returns, per transaction, None if every signature verified, else (index, exception)
    for the FIRST failing signature in list order (the one the serial loop would throw)."""
    items, owner = _items(stxs, signable_data)
    status, errors = crypto.verify_batch_ex(items, B.MODE_DOVERIFY) if items else (np.zeros(0, np.uint8), {})
    return _first_failures(stxs, status, errors, crypto)


def check_signatures_are_valid(stx, signable_data, crypto=Crypto):
    r = check_signatures_are_valid_batch([stx], signable_data, crypto)[0]
    if r is not None:
        raise r[1]


def verify_signatures_except(stx, signable_data, allowed_to_be_missing=(), crypto=Crypto):
    """TransactionWithSignatures.verifySignaturesExcept (TransactionWithSignatures.kt:41-47):
    the signatures' check, then SignaturesMissingException for required keys the signatures do not
    fulfil (composite-aware), minus the keys allowed to be missing."""
    check_signatures_are_valid(stx, signable_data, crypto)
    needed = get_missing_signatures(stx) - set(allowed_to_be_missing)
    if needed:
        raise SignaturesMissingException(needed, get_key_descriptions(stx, needed), stx.id)


# ---------------------------------------------------------------------------------------------
# WireTransaction-level pipeline: ids on the GPU, then every signature over SignableData(id).

@dataclass
class WireTransactionData:
    """The bytes WireTransaction.id is computed from (MerkleTransaction.kt:74-93): the
    serialised components in availableComponents order (inputs, attachments, outputs,
    commands, notary?, timeWindow?), the 32-byte PrivacySalt and its serialisation (the last
    leaf, hashed without a nonce)."""
    components: list
    salt: bytes
    salt_blob: bytes


@dataclass
class SignedWireTransaction:
    wtx: WireTransactionData
    sigs: list                       # TransactionSignature
    required_signing_keys: set = field(default_factory=set)
    inputs: list = field(default_factory=list)   # StateRef.txhash of each input (32-byte ids)
    commands: list = field(default_factory=list)
    notary: object = None


def pack_signed_transactions(stxs):
    """One arena for components, salts, keys, signatures and SignableData templates; returns
    (txs, comps, keys, sigs, tmpls, arena) in the include/cordagpu.h layouts."""
    bb = B.BatchBuilder()
    comps, tx_rows, sig_rows, tmpl_rows, tmpl_index = [], [], [], [], {}

    def tmpl_for(pv, sid):
        k = (pv, sid)
        if k not in tmpl_index:
            pre, suf = signable.template(pv, sid)
            tmpl_index[k] = len(tmpl_rows)
            tmpl_rows.append((bb._append(pre, 4), bb._append(suf, 4), len(pre), len(suf)))
        return tmpl_index[k]

    for t, stx in enumerate(stxs):
        w = stx.wtx
        first = len(comps)
        for blob in w.components:
            comps.append((bb._append(blob, 4), len(blob), 0))
        comps.append((bb._append(w.salt_blob, 4), len(w.salt_blob), 1))
        tx_rows.append((first, len(w.components) + 1, 0, bb._append(w.salt, 4)))
        for s in stx.sigs:
            k = bb.key(s.by.scheme, s.by.fmt, s.by.encoded)
            # a scheme the GPU does not run gets CG_UNSUPPORTED whatever its bytes (the host
            # verifies it afterwards, verify_wire_transactions): pack a 1-byte placeholder
            sb = B.sig_field(s.by.scheme, s.bytes) if s.by.scheme in GPU_SCHEMES else b"\x00"
            sig_rows.append((bb._append(sb, 4), t, k, len(sb), tmpl_for(s.platform_version, s.scheme_number_id), 0))
    built = bb.build()
    txs = np.array(tx_rows, dtype=B.TX_DTYPE) if tx_rows else np.zeros(0, B.TX_DTYPE)
    c = np.array(comps, dtype=B.COMPONENT_DTYPE) if comps else np.zeros(0, B.COMPONENT_DTYPE)
    sg = np.array(sig_rows, dtype=B.TXSIG_DTYPE) if sig_rows else np.zeros(0, B.TXSIG_DTYPE)
    tm = np.array(tmpl_rows, dtype=B.TMPL_DTYPE) if tmpl_rows else np.zeros(0, B.TMPL_DTYPE)
    return txs, c, built.keys, sg, tm, built.arena


def verify_wire_transactions(stxs, crypto=Crypto):
    """For each SignedWireTransaction: its id (WireTransaction.id) and None if every
    signature verifies, else (index, exception) of the FIRST failing signature in list order
    -- what ``SignedTransaction.verifySignaturesExcept`` would throw first
    (TransactionWithSignatures.kt:58-61). Ids, SignableData messages and verdicts are all
    computed on the GPU in one cg_verify_transactions call."""
    from .merkle import MerkleTreeException
    txs, comps, keys, sigs, tmpls, arena = pack_signed_transactions(stxs)
    ids, txst, sst = crypto.engine().verify_transactions(txs, comps, keys, sigs, tmpls, arena, B.MODE_DOVERIFY)
    sst = sst.copy()
    # signatures the GPU returned CG_UNSUPPORTED for (RSA, SPHINCS, composite keys): the host
    # fallback over SignableData(id, metadata) with the GPU-computed id
    errors, fb, pos = {}, [], 0
    for t, stx in enumerate(stxs):
        for i, s in enumerate(stx.sigs):
            if s.by.scheme not in GPU_SCHEMES and txst[t] == 0:
                pre, suf = signable.template(s.platform_version, s.scheme_number_id)
                fb.append((pos + i, BatchItem(s.by, s.bytes, pre + bytes(ids[t]) + suf)))
        pos += len(stx.sigs)
    if fb:
        st2, err2 = crypto.verify_batch_ex([b for _, b in fb], B.MODE_DOVERIFY)
        for j, (p, _) in enumerate(fb):
            sst[p] = st2[j]
            if j in err2:
                errors[p] = err2[j]
    out_ids, results, pos = [], [], 0
    for t, stx in enumerate(stxs):
        if txst[t] != 0:
            out_ids.append(None)
            results.append((0, MerkleTreeException("Cannot calculate Merkle root on empty hash list.")))
            pos += len(stx.sigs)
            continue
        out_ids.append(bytes(ids[t]))
        res = None
        for i, s in enumerate(stx.sigs):
            st = int(sst[pos + i])
            if st != B.VALID and res is None:
                try:
                    crypto.raise_for_status(st, SCHEME_CODE_NAMES.get(s.by.scheme, ""), do_verify=True,
                                            error=errors.get(pos + i), key=s.by)
                except Exception as e:  # noqa: BLE001 - mirrored JVM exception
                    res = (i, e)
        results.append(res)
        pos += len(stx.sigs)
    return out_ids, results


# ---------------------------------------------------------------------------------------------
# Whole-chain resolution: ResolveTransactionsFlow verifies every downloaded
# dependency in topological order, one SignedTransaction.verify at a time, and each verify
# checks the signatures twice (checkSignaturesAreValid, then verifyRequiredSignatures ->
# verifySignaturesExcept -> checkSignaturesAreValid again; SignedTransaction.kt:143-149,
# TransactionWithSignatures.kt:41-47). Here the whole chain -- every id and every signature --
# is one GPU call, each signature is verified once, and the ordered walk afterwards throws
# exactly what the serial loop would have thrown first.

class ExcessivelyLargeTransactionGraph(Exception):
    """ResolveTransactionsFlow.ExcessivelyLargeTransactionGraph (ResolveTransactionsFlow.kt:66)."""


def topological_sort(stxs, ids):
    """ResolveTransactionsFlow.topologicalSort (ResolveTransactionsFlow.kt:36-62) over
    transaction indices: dependencies before dependers, deterministic for a given list order
    (the forward graph keeps insertion order like the LinkedHashSet it restates). Iterative
    DFS, so chains deeper than Python's recursion limit sort too."""
    forward = {}
    for t, stx in enumerate(stxs):
        for h in stx.inputs:
            dep = forward.setdefault(bytes(h), {})
            dep.setdefault(t, None)
    visited, result = set(), []
    for root in range(len(stxs)):
        if ids[root] in visited:
            continue
        visited.add(ids[root])
        stack = [(root, iter(forward.get(ids[root], ())))]
        while stack:
            t, it = stack[-1]
            nxt = None
            for d in it:
                if ids[d] not in visited:
                    nxt = d
                    break
            if nxt is None:
                stack.pop()
                result.append(t)
            else:
                visited.add(ids[nxt])
                stack.append((nxt, iter(forward.get(ids[nxt], ()))))
    result.reverse()
    if len(result) != len(stxs):
        raise IllegalArgumentException("Failed requirement.")
    return result


def verify_chain(stxs, crypto=Crypto, check_sufficient_signatures=True, on_verified=None, limit=5000):
    """The signature half of ResolveTransactionsFlow.call's loop (ResolveTransactionsFlow.kt:88-96)
    for a downloaded set of SignedWireTransactions. Returns the transactions' indices in
    topological order, all verified. On the first transaction (in that order) whose check fails,
    raises what its SignedTransaction.verify would have raised first: MerkleTreeException (no
    id), the first failing signature's exception (SignatureException / InvalidKeyException /
    IllegalArgumentException, TransactionWithSignatures.kt:58-61) or SignaturesMissingException
    (:41-47). ``on_verified(index, id)`` runs for each transaction before the next is checked --
    where the flow records it and runs contract verification (out of scope here)."""
    if len(stxs) > limit:
        raise ExcessivelyLargeTransactionGraph()
    ids, results = verify_wire_transactions(stxs, crypto)
    if any(i is None for i in ids):
        # an id-less transaction cannot be placed in the graph: the serial flow fails on it when
        # it deserialises / hashes it, before any verification
        t = next(k for k, i in enumerate(ids) if i is None)
        raise results[t][1]
    order = topological_sort(stxs, ids)
    for t in order:
        stx = stxs[t]
        if results[t] is not None:
            raise results[t][1]
        if check_sufficient_signatures:
            missing = get_missing_signatures(stx)
            if missing:
                raise SignaturesMissingException(missing, get_key_descriptions(stx, missing), ids[t])
        if on_verified is not None:
            on_verified(t, ids[t])
    return order
