"""Extracts the Kryo byte captures the reference holds into tests/golden/kryo_captures.json.

Runs in the build container only; reads two reference files as text (nothing is executed):

  docs/source/tutorial-cordapp.rst (``run verifiedTransactions`` output, lines ~466-510): one
      SignedTransaction as the node printed it: ``txBits`` (base64 of the serialised
      WireTransaction), two ``sigs`` (base64, 64-byte Ed25519 signatures), the ``id`` and the
      ``mustSign`` / command ``signers`` keys as ``PublicKey.toBase58String()``
      (EncodingUtils.kt:67 = Base58(key.serialize().bytes)), plus the decoded field values
      (IOU value, UUID, X.500 names) the tests rebuild the bytes from.
  samples/irs-demo/src/main/resources/net/corda/irs/simulation/trade.json: the fixed- and
      floating-rate payers' keys, Base58 strings this snapshot parses at run time
      (IRSSimulation.kt:116 -> JacksonSupport PartyDeserializer -> parsePublicKeyBase58).

The two signatures verify under i2p-EdDSA semantics (oracle/ed25519_i2p.py) over the 32-byte id
with the two signer keys: the version that printed the tutorial signed ``id.bytes`` directly
(DigitalSignature.WithKey). They are the reference's only Ed25519 signatures.
"""
import base64
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
REF = "/root/reference"
TUTORIAL = "docs/source/tutorial-cordapp.rst"
TRADE = "samples/irs-demo/src/main/resources/net/corda/irs/simulation/trade.json"
B58 = "123456789ABCDEFGHJKLMNPQRSTUVWXYZabcdefghijkmnopqrstuvwxyz"


def b58decode(s):
    n = 0
    for c in s:
        n = n * 58 + B58.index(c)
    b = n.to_bytes((n.bit_length() + 7) // 8, "big")
    return b"\x00" * (len(s) - len(s.lstrip("1"))) + b


def ed25519_items(tx_id, keys, sigs):
    """tests/golden/ref_ed25519.json: the two genuine signatures (origin "reference") and
    builder-made corruptions of them (Appendix A classes), verdicts from the i2p restatement."""
    sys.path.insert(0, ROOT)
    from oracle import corda as ocorda, ed25519_i2p as ed

    def item(key, sig, msg, cls, origin, note):
        st = ocorda.STATUS_NAMES[ocorda.verify_item(4, 0, key, sig, msg)]
        st_iv = ocorda.STATUS_NAMES[ocorda.verify_item(4, 0, key, sig, msg, ocorda.MODE_ISVALID)]
        return {"scheme": 4, "key_fmt": 0, "key": key.hex(), "sig": sig.hex(), "msg": msg.hex(), "expect": st,
                "expect_isvalid": st_iv, "class": cls, "origin": origin, "note": note}

    out = []
    for k, s in zip(keys, sigs):
        out.append(item(k, s, tx_id, "A0", "reference", "tutorial-cordapp.rst SignedTransaction sig over id.bytes"))
        r, sc = s[:32], int.from_bytes(s[32:], "little")
        m = bytearray(tx_id)
        m[5] ^= 0x10
        out.append(item(k, s, bytes(m), "A1", "builder-made", "one bit of the id flipped"))
        rr = bytearray(r)
        rr[3] ^= 0x01
        out.append(item(k, bytes(rr) + s[32:], tx_id, "A2", "builder-made", "one bit of R flipped"))
        out.append(item(k, r + (sc ^ (1 << 17)).to_bytes(32, "little"), tx_id, "A3", "builder-made",
                        "one bit of S flipped"))
        out.append(item(k, r + (sc + ed.L).to_bytes(32, "little"), tx_id, "A4", "builder-made",
                        "S + L: i2p 0.2.0 has no S < L check"))
        out.append(item(k, r + (sc | (0xF0 << 248)).to_bytes(32, "little"), tx_id, "A5", "builder-made",
                        "top bits of S set (slide carry past bit 255)"))
        out.append(item(k, s[:63], tx_id, "A7", "builder-made", "63-byte signature"))
        out.append(item(k, s + b"\x00", tx_id, "A7", "builder-made", "65-byte signature"))
        out.append(item(k, s, b"", "A7", "builder-made", "empty clear data"))
    out.append(item(keys[0], sigs[1], tx_id, "E9", "builder-made", "signature checked under the other signer's key"))
    out.append(item(keys[1], sigs[0], tx_id, "E9", "builder-made", "signature checked under the other signer's key"))
    return out


def main():
    text = open(os.path.join(REF, TUTORIAL)).read()
    start = text.index("- txBits:")
    block = text[start:start + 6000]
    tx_bits = base64.b64decode(re.search(r'txBits: "([^"]+)"', block).group(1))
    sigs_block = block[block.index("sigs:"):block.index("id:")]
    sigs = [base64.b64decode(s) for s in re.findall(r'- "([A-Za-z0-9+/=]+)"', sigs_block)]
    tx_id = re.search(r'\n\s+id: "([0-9A-F]{64})"', block).group(1)
    signers = re.findall(r'signers:\s*\n\s*- "(\w+)"\s*\n\s*- "(\w+)"', block)[0]
    must_sign = re.findall(r'mustSign:\s*\n\s*- "(\w+)"\s*\n\s*- "(\w+)"', block)[0]
    uuid = re.search(r'id: "([0-9a-f-]{36})"', block).group(1)
    iou_value = int(re.search(r'iou:\s*\n\s*value: (\d+)', block).group(1))
    sender = re.search(r'sender: "([^"]+)"', block).group(1)
    recipient = re.search(r'recipient: "([^"]+)"', block).group(1)
    notary = re.search(r'notary: "([^"]+)"', block).group(1)
    command_class = "com.example.contract.IOUContract$Commands$Create"  # printed as `value: {}`; named in txBits
    trade = json.load(open(os.path.join(REF, TRADE)))
    trade_keys = [trade["fixedLeg"]["fixedRatePayer"], trade["floatingLeg"]["floatingRatePayer"]]
    out = {
        "meta": {"generator": "tools/gen/kryo_captures.py", "sources": [TUTORIAL, TRADE]},
        "tutorial": {
            "tx_bits": tx_bits.hex(), "sigs": [s.hex() for s in sigs], "id": tx_id,
            "signers_base58": list(signers), "signers": [b58decode(k).hex() for k in signers],
            "must_sign_base58": list(must_sign),
            "uuid": uuid, "iou_value": iou_value, "sender": sender, "recipient": recipient, "notary": notary,
            "command_class": command_class,
        },
        "trade_json": {"keys_base58": trade_keys, "keys": [b58decode(k).hex() for k in trade_keys]},
    }
    dst = os.path.join(ROOT, "tests", "golden", "kryo_captures.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    items = ed25519_items(bytes.fromhex(tx_id), [b58decode(k)[-32:] for k in signers], sigs)
    with open(os.path.join(ROOT, "tests", "golden", "ref_ed25519.json"), "w") as f:
        json.dump({"meta": {"generator": "tools/gen/kryo_captures.py", "source": TUTORIAL,
                            "expect": "genuine items VALID (i2p-made, signer key over id.bytes); builder-made items: "
                                      "oracle/ed25519_i2p.py verdicts"}, "items": items}, f, indent=1)
    print(f"txBits {len(tx_bits)} B, {len(sigs)} sigs, id {tx_id[:16]}..., trade keys {len(trade_keys)} -> {dst}")


if __name__ == "__main__":
    main()
