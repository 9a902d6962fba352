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
serialised with Kryo (Crypto.kt:499-502). That serialiser is not part of this engine
(SURVEY §8(f1)); callers pass ``signable_data(tx_id, metadata) -> bytes``.
"""
from dataclasses import dataclass, field

import numpy as np

from . import batch as B
from .crypto import BatchItem, Crypto, PublicKey, SCHEME_CODE_NAMES


class SignaturesMissingException(Exception):
    def __init__(self, missing, tx_id):
        super().__init__(f"Missing signatures for {sorted(k.encoded.hex() for k in missing)} on transaction "
                         f"{tx_id.hex()}")
        self.missing = missing
        self.tx_id = tx_id


@dataclass(frozen=True)
class TransactionSignature:
    bytes: bytes
    by: PublicKey
    platform_version: int = 1
    scheme_number_id: int = 4


@dataclass
class SignedTransaction:
    id: bytes
    sigs: list
    required_signing_keys: set = field(default_factory=set)


def _items(stxs, signable_data):
    items, owner = [], []
    for t, stx in enumerate(stxs):
        for s in stx.sigs:
            items.append(BatchItem(s.by, s.bytes, signable_data(stx.id, s)))
            owner.append(t)
    return items, owner


def check_signatures_are_valid_batch(stxs, signable_data, crypto=Crypto):
    """Verifies all signatures of all transactions in one GPU batch.

    Returns, per transaction, None if every signature verified, else (index, exception)
    for the FIRST failing signature in list order (the one the serial loop would throw)."""
    items, owner = _items(stxs, signable_data)
    status = crypto.verify_batch(items, B.MODE_DOVERIFY) if items else np.zeros(0, np.uint8)
    result = [None] * len(stxs)
    pos = 0
    for t, stx in enumerate(stxs):
        for i, s in enumerate(stx.sigs):
            st = int(status[pos + i])
            if st != B.VALID and result[t] is None:
                try:
                    crypto.raise_for_status(st, SCHEME_CODE_NAMES.get(s.by.scheme, ""), do_verify=True)
                except Exception as e:  # noqa: BLE001 - mirrored JVM exception
                    result[t] = (i, e)
        pos += len(stx.sigs)
    return result


def check_signatures_are_valid(stx, signable_data, crypto=Crypto):
    r = check_signatures_are_valid_batch([stx], signable_data, crypto)[0]
    if r is not None:
        raise r[1]


def verify_signatures_except(stx, signable_data, allowed_to_be_missing=(), crypto=Crypto):
    """TransactionWithSignatures.verifySignaturesExcept (TransactionWithSignatures.kt:41-47).
    Composite-key fulfilment (isFulfilledBy) is host logic and out of scope: required keys
    are matched by identity."""
    check_signatures_are_valid(stx, signable_data, crypto)
    sig_keys = {s.by for s in stx.sigs}
    needed = {k for k in stx.required_signing_keys if k not in sig_keys} - set(allowed_to_be_missing)
    if needed:
        raise SignaturesMissingException(needed, stx.id)
