"""One MI355X verification context (``cg_ctx``) per device, over the C ABI.

``Engine.verify(batch)`` is the batch form of Crypto.isValid / Crypto.doVerify
(core/src/main/kotlin/net/corda/core/crypto/Crypto.kt:474-484,553-559): one status byte
per item, codes as in include/cordagpu.h. ``Engine.verify_device`` is the same on
buffers already resident in HBM (raw device pointers, e.g. ``torch.Tensor.data_ptr()``).
"""
import ctypes

import numpy as np

from . import _lib
from .batch import COMPONENT_DTYPE, FLEAF_DTYPE, FTX_DTYPE, KEY_DTYPE, PMT_NODE_DTYPE, MODE_DOVERIFY, SPAN_DTYPE, TMPL_DTYPE, TX_DTYPE, TXSIG_DTYPE


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None and a.size else None


class Engine:
    def __init__(self, device=0, chunk_items=0, stage_timing=False, host_threads=0, table_bytes_max=0):
        """host_threads: cg_config.host_threads (0: CG_HOST_THREADS, else the CPU quota divided by the
        contexts open in this process); table_bytes_max: HBM the constant fixed-base tables may take
        (0: automatic; include/cordagpu.h, corda_amd/csrc/table_budget.h)."""
        L = _lib.lib()
        cfg = _lib.cg_config(device, _lib.FLAG_STAGE_TIMING if stage_timing else 0, 0, 0, chunk_items, host_threads,
                             0, table_bytes_max)
        h = ctypes.c_void_p()
        _lib.check(L.cg_open(ctypes.byref(h), ctypes.byref(cfg)), f"cg_open(device={device})")
        self._h = h
        self.device = device
        self.last_stats = None

    def info(self):
        """cg_context_info: device, fixed_base_bits (26 / 24 / 22), table_bytes, host_threads, chunk_items."""
        inf = _lib.cg_info()
        _lib.check(_lib.lib().cg_context_info(self._h, ctypes.byref(inf)), "cg_context_info")
        return {k: getattr(inf, k) for k, _ in _lib.cg_info._fields_ if k != "reserved"}

    def close(self):
        if self._h:
            _lib.lib().cg_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stage_times(self):
        """{stage: (ms, launches)} since the last read (Engine(stage_timing=True)); waits for the work."""
        n = len(_lib.STAGE_NAMES)
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_uint32 * n)()
        rc = _lib.lib().cg_stage_times(self._h, ms, cnt, n)
        if rc < 0:
            _lib.check(rc, "cg_stage_times")
        return {name: (ms[k], cnt[k]) for k, name in enumerate(_lib.STAGE_NAMES)}

    # ------------------------------------------------------------------ signatures
    def verify(self, batch, mode=MODE_DOVERIFY):
        st = np.full(batch.n, 255, dtype=np.uint8)
        stats = _lib.cg_stats()
        rc = _lib.lib().cg_verify_batch(self._h, _p(batch.keys), len(batch.keys), _p(batch.items), batch.n,
                                        _p(batch.arena), batch.arena.size, mode, _p(st), ctypes.byref(stats))
        _lib.check(rc, "cg_verify_batch")
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_stats._fields_}
        return st

    def reserve(self, max_keys, max_items):
        _lib.check(_lib.lib().cg_reserve(self._h, max_keys, max_items), "cg_reserve")

    def verify_device(self, d_keys, n_keys, d_items, n_items, d_arena, arena_len, d_status, mode=MODE_DOVERIFY,
                      stream=0):
        """Asynchronous: enqueues on `stream` (a hipStream_t as int; 0 = the context's stream)."""
        rc = _lib.lib().cg_verify_batch_device(self._h, d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode,
                                               d_status, stream or None)
        _lib.check(rc, "cg_verify_batch_device")

    def prepare_keys_device(self, d_keys, n_keys, d_arena, arena_len, stream=0):
        _lib.check(_lib.lib().cg_prepare_keys_device(self._h, d_keys, n_keys, d_arena, arena_len, stream or None),
                   "cg_prepare_keys_device")

    def verify_items_device(self, d_keys, n_keys, d_items, n_items, d_arena, arena_len, d_status,
                            mode=MODE_DOVERIFY, stream=0):
        rc = _lib.lib().cg_verify_items_device(self._h, d_keys, n_keys, d_items, n_items, d_arena, arena_len, mode,
                                               d_status, stream or None)
        _lib.check(rc, "cg_verify_items_device")

    # ------------------------------------------------------------------ hashing
    @staticmethod
    def _spans(msgs):
        chunks, spans, off = [], np.zeros(len(msgs), dtype=SPAN_DTYPE), 0
        for i, m in enumerate(msgs):
            pad = (-off) % 4
            if pad:
                chunks.append(bytes(pad))
                off += pad
            spans[i] = (off, len(m))
            chunks.append(bytes(m))
            off += len(m)
        arena = np.frombuffer(b"".join(chunks) + bytes(8), dtype=np.uint8).copy()
        return spans, arena

    def sha256(self, msgs):
        spans, arena = self._spans(msgs)
        out = np.zeros(32 * len(msgs), dtype=np.uint8)
        _lib.check(_lib.lib().cg_sha256_batch(self._h, _p(spans), len(msgs), _p(arena), arena.size - 8, _p(out)),
                   "cg_sha256_batch")
        return [out[32 * i:32 * i + 32].tobytes() for i in range(len(msgs))]

    def sha512(self, msgs):
        spans, arena = self._spans(msgs)
        out = np.zeros(64 * len(msgs), dtype=np.uint8)
        _lib.check(_lib.lib().cg_sha512_batch(self._h, _p(spans), len(msgs), _p(arena), arena.size - 8, _p(out)),
                   "cg_sha512_batch")
        return [out[64 * i:64 * i + 64].tobytes() for i in range(len(msgs))]

    def merkle_roots(self, leaf_lists):
        """MerkleTree.getMerkleTree(leaves).hash for each list; returns (roots, status)."""
        n = len(leaf_lists)
        first = np.zeros(n, dtype=np.uint64)
        count = np.zeros(n, dtype=np.uint32)
        flat, pos = [], 0
        for j, lv in enumerate(leaf_lists):
            first[j] = pos
            count[j] = len(lv)
            flat.extend(bytes(x) for x in lv)
            pos += len(lv)
        leaves = np.frombuffer(b"".join(flat) + bytes(32), dtype=np.uint8).copy()
        roots = np.zeros(32 * n, dtype=np.uint8)
        st = np.zeros(n, dtype=np.uint8)
        _lib.check(_lib.lib().cg_merkle_roots(self._h, _p(leaves), _p(first), _p(count), n, _p(roots), _p(st)),
                   "cg_merkle_roots")
        return [roots[32 * j:32 * j + 32].tobytes() for j in range(n)], st

    def tx_ids(self, txs, comps, arena):
        """WireTransaction.id for packed transactions (TX_DTYPE / COMPONENT_DTYPE / arena)."""
        assert txs.dtype == TX_DTYPE and comps.dtype == COMPONENT_DTYPE
        ids = np.zeros(32 * len(txs), dtype=np.uint8)
        st = np.zeros(len(txs), dtype=np.uint8)
        _lib.check(_lib.lib().cg_tx_ids(self._h, _p(txs), len(txs), _p(comps), len(comps), _p(arena), arena.size,
                                        _p(ids), _p(st)), "cg_tx_ids")
        return ids.reshape(-1, 32), st

    def verify_filtered(self, ftxs, nodes, leaves, arena):
        """FilteredTransaction.verify / PartialMerkleTree.verify for packed tear-offs
        (FTX_DTYPE / PMT_NODE_DTYPE / FLEAF_DTYPE / arena, cg_verify_filtered). Returns the
        per-transaction status bytes (0 true, 1 false, 2 MerkleTreeException, 3 malformed)."""
        assert ftxs.dtype == FTX_DTYPE and nodes.dtype == PMT_NODE_DTYPE and leaves.dtype == FLEAF_DTYPE
        st = np.full(len(ftxs), 255, dtype=np.uint8)
        _lib.check(_lib.lib().cg_verify_filtered(self._h, _p(ftxs), len(ftxs), _p(nodes), len(nodes), _p(leaves),
                                                 len(leaves), _p(arena), arena.size, _p(st)), "cg_verify_filtered")
        return st

    def verify_filtered_device(self, d_ftxs, n_ftx, d_nodes, n_nodes, d_leaves, n_leaves, d_arena, arena_len,
                               d_status, stream=0):
        """Asynchronous device form of verify_filtered (every table already in HBM)."""
        _lib.check(_lib.lib().cg_verify_filtered_device(self._h, d_ftxs, n_ftx, d_nodes, n_nodes, d_leaves, n_leaves,
                                                        d_arena, arena_len, d_status, stream or None),
                   "cg_verify_filtered_device")

    # ------------------------------------------------------------------ transactions
    def verify_transactions(self, txs, comps, keys, sigs, tmpls, arena, mode=MODE_DOVERIFY):
        """Tx ids + every signature over SignableData(id, metadata) in one call
        (cg_verify_transactions). Returns (ids [n_tx, 32], tx_status, sig_status)."""
        assert txs.dtype == TX_DTYPE and comps.dtype == COMPONENT_DTYPE and keys.dtype == KEY_DTYPE
        assert sigs.dtype == TXSIG_DTYPE and tmpls.dtype == TMPL_DTYPE
        ids = np.zeros(32 * len(txs), dtype=np.uint8)
        txst = np.zeros(len(txs), dtype=np.uint8)
        sst = np.full(len(sigs), 255, dtype=np.uint8)
        rc = _lib.lib().cg_verify_transactions(self._h, _p(txs), len(txs), _p(comps), len(comps), _p(keys), len(keys),
                                               _p(sigs), len(sigs), _p(tmpls), len(tmpls), _p(arena), arena.size,
                                               mode, _p(ids), _p(txst), _p(sst))
        _lib.check(rc, "cg_verify_transactions")
        return ids.reshape(-1, 32), txst, sst

    def verify_transactions_device(self, d_txs, n_tx, d_comps, n_comps, d_keys, n_keys, d_sigs, n_sigs, tmpls,
                                   d_arena, arena_len, d_ids, d_tx_status, d_sig_status, mode=MODE_DOVERIFY,
                                   stream=0):
        """Asynchronous device form; `tmpls` is a host TMPL_DTYPE array (template bytes in the arena)."""
        assert tmpls.dtype == TMPL_DTYPE
        rc = _lib.lib().cg_verify_transactions_device(self._h, d_txs, n_tx, d_comps, n_comps, d_keys, n_keys, d_sigs,
                                                      n_sigs, _p(tmpls), len(tmpls), d_arena, arena_len, mode, d_ids,
                                                      d_tx_status, d_sig_status, stream or None)
        _lib.check(rc, "cg_verify_transactions_device")

    # ------------------------------------------------------------------ signatures over tx ids
    def verify_tx_signatures(self, tb, mode=MODE_DOVERIFY):
        """Batch Crypto.doVerify(txId, TransactionSignature) (cg_verify_tx_signatures, Crypto.kt:499-502):
        ``tb`` is a batch.TxSigBatch; each signature's clear data is SignableData(id, metadata),
        spliced on the device. Returns one status byte per signature; cg_stats in last_stats."""
        st = np.full(len(tb.sigs), 255, dtype=np.uint8)
        stats = _lib.cg_stats()
        rc = _lib.lib().cg_verify_tx_signatures(self._h, _p(tb.keys), len(tb.keys), _p(tb.ids), tb.n_ids, _p(tb.sigs),
                                                len(tb.sigs), _p(tb.tmpls), len(tb.tmpls), _p(tb.arena), tb.arena.size,
                                                mode, _p(st), ctypes.byref(stats))
        _lib.check(rc, "cg_verify_tx_signatures")
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_stats._fields_}
        return st

    def verify_tx_signatures_packed(self, pb, mode=MODE_DOVERIFY):
        """cg_verify_tx_signatures_packed: ``pb`` a batch.PackedTxSigBatch (the 12-byte table and the
        dense signature stream). One status byte per signature; cg_stats in last_stats."""
        st = np.full(pb.n, 255, dtype=np.uint8)
        stats = _lib.cg_stats()
        rc = _lib.lib().cg_verify_tx_signatures_packed(self._h, _p(pb.keys), len(pb.keys), _p(pb.ids), pb.n_ids,
                                                       _p(pb.sigs), pb.n, _p(pb.stream), pb.stream.size, _p(pb.tmpls),
                                                       len(pb.tmpls), _p(pb.arena), pb.arena.size, mode, _p(st),
                                                       ctypes.byref(stats))
        _lib.check(rc, "cg_verify_tx_signatures_packed")
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_stats._fields_}
        return st

    def verify_tx_signatures_packed_device(self, d_keys, n_keys, d_ids, n_ids, d_sigs, n_sigs, sig_bytes_off,
                                           sig_bytes_len, tmpls, d_arena, arena_len, d_status, mode=MODE_DOVERIFY,
                                           stream=0):
        """Asynchronous device form: the signature stream at d_arena[sig_bytes_off, + sig_bytes_len)."""
        assert tmpls.dtype == TMPL_DTYPE
        rc = _lib.lib().cg_verify_tx_signatures_packed_device(self._h, d_keys, n_keys, d_ids, n_ids, d_sigs, n_sigs,
                                                              sig_bytes_off, sig_bytes_len, _p(tmpls), len(tmpls),
                                                              d_arena, arena_len, mode, d_status, stream or None)
        _lib.check(rc, "cg_verify_tx_signatures_packed_device")

    def verify_tx_signatures_device(self, d_keys, n_keys, d_ids, n_ids, d_sigs, n_sigs, tmpls, d_arena, arena_len,
                                    d_status, mode=MODE_DOVERIFY, stream=0):
        """Asynchronous device form; `tmpls` is a host TMPL_DTYPE array (template bytes in the arena)."""
        assert tmpls.dtype == TMPL_DTYPE
        rc = _lib.lib().cg_verify_tx_signatures_device(self._h, d_keys, n_keys, d_ids, n_ids, d_sigs, n_sigs,
                                                       _p(tmpls), len(tmpls), d_arena, arena_len, mode, d_status,
                                                       stream or None)
        _lib.check(rc, "cg_verify_tx_signatures_device")


class EnginePool:
    """One process, several devices (cg_pool): ``verify(batch)`` shards the items over the healthy
    slots, re-runs a failed slot's shard elsewhere, and returns one status byte per item (items
    no slot could run stay NOT_RUN and raise ``EngineUnavailable`` unless ``allow_partial``)."""

    def __init__(self, devices, chunk_items=0, host_threads=0, table_bytes_max=0):
        L = _lib.lib()
        cfg = _lib.cg_config(0, 0, 0, 0, chunk_items, host_threads, 0, table_bytes_max)
        devs = (ctypes.c_int32 * len(devices))(*devices)
        h = ctypes.c_void_p()
        _lib.check(L.cg_pool_open(ctypes.byref(h), devs, len(devices), ctypes.byref(cfg)), "cg_pool_open")
        self._h = h
        self.devices = list(devices)
        self.last_stats = None

    def close(self):
        if self._h:
            _lib.lib().cg_pool_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def healthy(self):
        L = _lib.lib()
        return [L.cg_pool_slot_healthy(self._h, k) == 1 for k in range(L.cg_pool_slots(self._h))]

    def inject_fault(self, slot, fail=True):
        _lib.check(_lib.lib().cg_pool_inject_fault(self._h, slot, 1 if fail else 0), "cg_pool_inject_fault")

    def verify(self, batch, mode=MODE_DOVERIFY, allow_partial=False):
        st = np.full(batch.n, 255, dtype=np.uint8)
        stats = _lib.cg_pool_stats()
        rc = _lib.lib().cg_pool_verify_batch(self._h, _p(batch.keys), len(batch.keys), _p(batch.items), batch.n,
                                             _p(batch.arena), batch.arena.size, mode, _p(st), ctypes.byref(stats))
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_pool_stats._fields_ if k != "reserved"}
        if rc != 0 and not allow_partial:
            _lib.check(rc, "cg_pool_verify_batch")
        return st

    def verify_tx_signatures(self, tb, mode=MODE_DOVERIFY, allow_partial=False):
        """cg_pool_verify_tx_signatures: the signature table sharded over the healthy slots."""
        st = np.full(len(tb.sigs), 255, dtype=np.uint8)
        stats = _lib.cg_pool_stats()
        rc = _lib.lib().cg_pool_verify_tx_signatures(self._h, _p(tb.keys), len(tb.keys), _p(tb.ids), tb.n_ids,
                                                     _p(tb.sigs), len(tb.sigs), _p(tb.tmpls), len(tb.tmpls),
                                                     _p(tb.arena), tb.arena.size, mode, _p(st), ctypes.byref(stats))
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_pool_stats._fields_ if k != "reserved"}
        if rc != 0 and not allow_partial:
            _lib.check(rc, "cg_pool_verify_tx_signatures")
        return st

    def verify_tx_signatures_packed(self, pb, mode=MODE_DOVERIFY, allow_partial=False):
        """cg_pool_verify_tx_signatures_packed: the 12-byte table sharded over the healthy slots."""
        st = np.full(pb.n, 255, dtype=np.uint8)
        stats = _lib.cg_pool_stats()
        rc = _lib.lib().cg_pool_verify_tx_signatures_packed(self._h, _p(pb.keys), len(pb.keys), _p(pb.ids), pb.n_ids,
                                                            _p(pb.sigs), pb.n, _p(pb.stream), pb.stream.size,
                                                            _p(pb.tmpls), len(pb.tmpls), _p(pb.arena), pb.arena.size,
                                                            mode, _p(st), ctypes.byref(stats))
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_pool_stats._fields_ if k != "reserved"}
        if rc != 0 and not allow_partial:
            _lib.check(rc, "cg_pool_verify_tx_signatures_packed")
        return st

    def verify_transactions(self, txs, comps, keys, sigs, tmpls, arena, mode=MODE_DOVERIFY, allow_partial=False):
        """cg_pool_verify_transactions: the whole call on one healthy slot, the next one on a device
        fault. Returns (ids [n_tx, 32], tx_status, sig_status) as Engine.verify_transactions."""
        ids = np.zeros(32 * len(txs), dtype=np.uint8)
        txst = np.zeros(len(txs), dtype=np.uint8)
        sst = np.full(len(sigs), 255, dtype=np.uint8)
        stats = _lib.cg_pool_stats()
        rc = _lib.lib().cg_pool_verify_transactions(self._h, _p(txs), len(txs), _p(comps), len(comps), _p(keys),
                                                    len(keys), _p(sigs), len(sigs), _p(tmpls), len(tmpls), _p(arena),
                                                    arena.size, mode, _p(ids), _p(txst), _p(sst), ctypes.byref(stats))
        self.last_stats = {k: getattr(stats, k) for k, _ in _lib.cg_pool_stats._fields_ if k != "reserved"}
        if rc != 0 and not allow_partial:
            _lib.check(rc, "cg_pool_verify_transactions")
        return ids.reshape(-1, 32), txst, sst

    def verify_requeue(self, batch, mode=MODE_DOVERIFY, between=None):
        """The JVM binding's re-queue (CryptoBatch.kt verifyBatch): on CG_ERR_DEVICE only the items left
        NOT_RUN go to the pool once more, as a sub-batch over the same keys and arena; what still stays
        NOT_RUN is returned as NOT_RUN (the binding hands those to Crypto.doVerify one by one).
        ``between()`` runs before the re-queue (tests clear a drill fault there)."""
        st = self.verify(batch, mode, allow_partial=True)
        rc_first = self.last_stats
        todo = np.flatnonzero(st == 255)
        if todo.size:
            if between:
                between()
            sub = batch.subset(todo)
            st2 = self.verify(sub, mode, allow_partial=True)
            st[todo] = st2
        self.first_stats = rc_first
        return st
