"""SignableData message templates: the clear data a TransactionSignature signs.

Reference: ``Crypto.doVerify(txId, transactionSignature)`` verifies the signature over
``SignableData(txId, transactionSignature.signatureMetadata).serialize().bytes``
(core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:499-502; SignableData.kt:13,
SignatureMetadata.kt:15). The node serialises with the Kryo P2P context, references on
(node-api/.../serialization/SerializationScheme.kt:183-203,219-224), through
DefaultKryoCustomizer (CompatibleFieldSerializer, EXTENDED cached field names).

For a fixed (platformVersion, schemeNumberID) those bytes are ``prefix || txId || suffix``: the
txId is the only per-transaction part. The engine therefore takes one template per metadata
value and splices the ids in on the device (``cg_verify_tx_signatures*``,
``cg_verify_transactions*``) instead of the host serialising one object per signature.

The bytes come from corda_amd/kryo.py's Kryo 4 writer, whose mechanics (chunk cascade, field
order, reference markers, byte[] framing) reproduce a whole captured transaction from the
reference byte for byte (tests/test_kryo.py). SignableData, SignatureMetadata and
SecureHash$SHA256 are unregistered classes (written by name), so no registration id enters
these bytes. No JVM capture of a SignableData object itself exists in the reference.
"""
from . import kryo

KRYO_HEADER_V0_1 = kryo.HEADER  # SerializationScheme.kt:191,216
TXID_MARK = b"\x00" * 32


def serialize(tx_id, platform_version=1, scheme_number_id=4):
    """SignableData(txId, SignatureMetadata(platformVersion, schemeNumberID)) bytes."""
    assert len(tx_id) == 32
    return kryo.signable_data(bytes(tx_id), platform_version, scheme_number_id)


_TEMPLATES = {}


def template(platform_version=1, scheme_number_id=4):
    """(prefix, suffix) with serialize(id, ...) == prefix + id + suffix for every 32-byte id."""
    key = (platform_version, scheme_number_id)
    if key not in _TEMPLATES:
        a = serialize(TXID_MARK, platform_version, scheme_number_id)
        b = serialize(b"\xff" * 32, platform_version, scheme_number_id)
        pos = next(i for i in range(len(a)) if a[i] != b[i])
        prefix, suffix = a[:pos], a[pos + 32:]
        assert a[pos:pos + 32] == TXID_MARK and b[:pos] == prefix and b[pos + 32:] == suffix
        _TEMPLATES[key] = (prefix, suffix)
    return _TEMPLATES[key]
