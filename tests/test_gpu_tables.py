"""GPU tests of round 6's multi-process / multi-device behaviour:

  * the constant fixed-base tables under a budget (cg_config.table_bytes_max): a context forced to
    the radix-2^24 and radix-2^22 builds reports that radix (cg_context_info) and returns the C
    oracle's verdicts on the golden sets and on a wide-table batch (hot keys of every scheme, the
    ladders that read the fixed-base tables), through the host and tx-signature entry points;
  * the JVM binding's re-queue (CryptoBatch.kt requeueNotRun) in its Python mirror
    EnginePool.verify_requeue: every slot faulted, then one cleared, and only the NOT_RUN items
    re-run;
  * cg_pool_verify_transactions: the whole call on one slot, failing over on a drill fault.
"""
import numpy as np
import pytest

import golden_io
from corda_amd import batch as B
from oracle import c_oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide_batch():
    from tools.workload import wl
    parts = [wl.ed25519_batch(24000, n_keys=8, msg_len=270, corrupt_permille=120, seed=161, bad_key_every=5,
                              nthreads=16)[0],
             wl.ed25519_batch(3000, n_keys=600, msg_len=120, corrupt_permille=120, seed=162, nthreads=16)[0],
             wl.ecdsa_batch(0, 9000, n_keys=6, msg_len=270, corrupt_permille=120, seed=163, nthreads=16)[0],
             wl.ecdsa_batch(1, 6000, n_keys=5, msg_len=270, corrupt_permille=120, seed=164, nthreads=16)[0],
             wl.ecdsa_batch(0, 2000, n_keys=90, msg_len=90, corrupt_permille=120, seed=165, nthreads=16)[0]]
    b, _ = wl.concat(parts, shuffle_seed=166)
    uses = np.bincount(b.items["key_idx"], minlength=len(b.keys))
    ed = b.keys["scheme"] == 4
    assert (uses[ed] >= 2400).sum() >= 6 and (uses[~ed] >= 900).sum() >= 8  # wide keys in every family
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    return b, ref


def test_default_context_takes_the_largest_tables(engine):
    from corda_amd import _lib
    inf = engine.info()
    L = _lib.lib()
    assert inf["fixed_base_bits"] in (26, 24, 22)
    assert inf["table_bytes"] == L.cg_table_bytes(inf["fixed_base_bits"])
    # a fresh MI355X (288 GB) holds the 91-GB set with the headroom to spare
    assert inf["fixed_base_bits"] == 26, inf


@pytest.mark.parametrize("bits", [24, 22])
def test_budgeted_tables_match_the_oracle(bits, wide_batch):
    from corda_amd import _lib
    from corda_amd.engine import Engine
    L = _lib.lib()
    budget = L.cg_table_bytes(bits)
    assert budget > 0
    with Engine(0, table_bytes_max=budget) as eng:
        inf = eng.info()
        assert inf["fixed_base_bits"] == bits and inf["table_bytes"] == budget, inf
        for name in ("ed25519.json", "ecdsa.json"):
            items = golden_io.load(name)
            gb, exp, exp_iv = golden_io.sig_batch(items)
            assert np.array_equal(eng.verify(gb, B.MODE_DOVERIFY), exp), name
            assert np.array_equal(eng.verify(gb, B.MODE_ISVALID), exp_iv), name
        b, ref = wide_batch
        st = eng.verify(b)
        assert np.array_equal(st, ref), f"radix 2^{bits}: {np.count_nonzero(st != ref)} mismatches"
        assert (st == B.VALID).sum() > 30000


def test_budgeted_tables_tx_signatures(engine):
    """The headline call shape (cg_verify_tx_signatures, hot keys on wide tables) at radix 2^22:
    the same verdicts as the default context's."""
    from corda_amd import _lib, signable
    from corda_amd.engine import Engine
    from tools.workload import wl
    pool, _, schemes = wl.notary_pool(1 << 14, ed_keys=24, ec_keys=12, seed=606, nthreads=16, sig_group=4)
    pre, _ = signable.template(1, 4)
    ids, id_idx = wl.pool_ids(pool, len(pre))
    idx = np.random.default_rng(607).integers(0, pool.n, 60000)
    tb = wl.tx_sig_stream(pool, schemes, idx, ids, id_idx, nthreads=16)
    ref = c_oracle.verify_batch(pool, B.MODE_DOVERIFY, 16)
    want = engine.verify_tx_signatures(tb)
    assert np.array_equal(want, ref[idx])
    with Engine(0, table_bytes_max=_lib.lib().cg_table_bytes(22)) as eng:
        assert eng.info()["fixed_base_bits"] == 22
        got = eng.verify_tx_signatures(tb)
    assert np.array_equal(got, want)
    assert (want == B.VALID).sum() > 30000 and (want == B.NOT_RUN).sum() == 0


def test_budget_below_every_table_set_is_an_argument_error():
    from corda_amd._lib import EngineUnavailable
    from corda_amd.engine import Engine
    with pytest.raises(EngineUnavailable, match="below the smallest"):
        Engine(0, table_bytes_max=1 << 30)


def test_pool_requeues_only_not_run_items(wide_batch):
    """CryptoBatch.requeueNotRun's mirror: every slot faulted -> CG_ERR_DEVICE, all NOT_RUN; the
    re-queue (after one slot's fault clears) runs exactly those items and ends at the oracle."""
    from corda_amd.engine import EnginePool
    b, ref = wide_batch
    with EnginePool([0, 0], chunk_items=20000) as ep:
        ep.inject_fault(0)
        ep.inject_fault(1)
        st = ep.verify_requeue(b, between=lambda: ep.inject_fault(1, False))
        assert ep.first_stats["not_run"] == b.n
        assert np.array_equal(st, ref)
        # a partial failure: slot 0 faulted, slot 1 healthy -> the pool re-runs slot 0's shard itself
        st = ep.verify_requeue(b)
        assert np.array_equal(st, ref) and ep.first_stats["not_run"] == 0
        # nothing comes back: the NOT_RUN items stay NOT_RUN (the JVM verifies them serially)
        ep.inject_fault(1)
        st = ep.verify_requeue(b)
        assert np.all(st == B.NOT_RUN)


def test_pool_verify_transactions_fails_over():
    from corda_amd.engine import Engine, EnginePool
    from tools.workload import wl
    w = wl.tx_pipeline(2000, n_keys=61, seed=661, corrupt_permille=60, nthreads=16)
    with Engine(0) as eng:
        ids0, txst0, sst0 = eng.verify_transactions(w.txs, w.comps, w.keys, w.sigs, w.tmpls, w.arena)
    assert np.array_equal(ids0, w.ids) and np.all(txst0 == 0)
    with EnginePool([0, 0]) as ep:
        ids, txst, sst = ep.verify_transactions(w.txs, w.comps, w.keys, w.sigs, w.tmpls, w.arena)
        assert np.array_equal(ids, ids0) and np.array_equal(sst, sst0) and ep.last_stats["reruns"] == 0
        ep.inject_fault(0)
        ids, txst, sst = ep.verify_transactions(w.txs, w.comps, w.keys, w.sigs, w.tmpls, w.arena)
        assert np.array_equal(ids, ids0) and np.array_equal(sst, sst0)
        assert ep.last_stats["reruns"] == 1 and ep.healthy() == [False, True]
        ep.inject_fault(1)
        _, _, sst = ep.verify_transactions(w.txs, w.comps, w.keys, w.sigs, w.tmpls, w.arena, allow_partial=True)
        assert np.all(sst == B.NOT_RUN) and ep.last_stats["not_run"] == len(w.sigs)
