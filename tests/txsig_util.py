"""Test helper: the message form of a cg_verify_tx_signatures batch (every signature's clear data
materialised as prefix || id || suffix), for checking the engine's device splice against the C
oracle, which verifies (key, sig, clear) items."""
import numpy as np

from corda_amd.batch import ITEM_DTYPE, Batch


def to_message_batch(tb):
    """Batch with item j = (keys[sigs[j].key_idx], sig bytes, SignableData bytes); a signature
    whose id / template index is out of range gets an out-of-range key index (NOT_RUN)."""
    n = len(tb.sigs)
    ids = tb.ids.reshape(-1, 32)
    chunks, items = [tb.arena], np.zeros(n, ITEM_DTYPE)
    off = (tb.arena.size + 15) & ~15
    chunks.append(np.zeros(off - tb.arena.size, np.uint8))
    for j, s in enumerate(tb.sigs):
        items[j]["sig_off"] = s["sig_off"]
        items[j]["sig_len"] = s["sig_len"]
        ok = s["tx_idx"] < len(ids) and s["tmpl"] < len(tb.tmpls)
        if not ok:
            items[j]["key_idx"] = 0xFFFFFFFF
            continue
        t = tb.tmpls[s["tmpl"]]
        pre = tb.arena[int(t["prefix_off"]):int(t["prefix_off"]) + int(t["prefix_len"])]
        suf = tb.arena[int(t["suffix_off"]):int(t["suffix_off"]) + int(t["suffix_len"])]
        msg = np.concatenate([pre, ids[s["tx_idx"]], suf])
        items[j]["msg_off"] = off
        items[j]["msg_len"] = msg.size
        items[j]["key_idx"] = s["key_idx"]
        pad = (-msg.size) % 4
        chunks.append(msg)
        chunks.append(np.zeros(pad, np.uint8))
        off += msg.size + pad
    chunks.append(np.zeros(64, np.uint8))
    return Batch(tb.keys, items, np.concatenate(chunks))
