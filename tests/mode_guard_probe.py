"""Child process of tests/test_gpu_txsig.py::test_skipped_modes_are_reported_not_run (run with
CG_TEST_SKIP_FAMILIES set, which the library reads once per process): keys of every table mode in
one host tx-signature call, the library told to skip the row-0 / quarter / full work of the
families in the mask. Prints one JSON line: per mode, how many items came back as the oracle's
verdict, as CG_NOT_RUN, or as anything else."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from corda_amd import batch as B  # noqa: E402
from corda_amd import signable  # noqa: E402
from corda_amd.engine import Engine  # noqa: E402
from oracle import c_oracle  # noqa: E402
from tools.workload import wl  # noqa: E402


def main():
    b, labels, schemes = wl.notary_pool(1 << 15, ed_keys=256, ec_keys=64, seed=93, nthreads=16, sig_group=4)
    pre, _ = signable.template(1, 4)
    ids, id_idx = wl.pool_ids(b, len(pre))
    ref = c_oracle.verify_batch(b, B.MODE_DOVERIFY, 16)
    rng = np.random.default_rng(78)
    per_key = [1, 3, 12, 40, 1900]
    key_of = b.items["key_idx"]
    order = np.argsort(key_of, kind="stable")
    starts = np.searchsorted(key_of[order], np.arange(len(b.keys) + 1))
    draws, uses = [], np.zeros(len(b.keys), np.int64)
    for k in range(len(b.keys)):
        mine = order[starts[k]:starts[k + 1]]
        if mine.size:
            n = per_key[k % len(per_key)]
            draws.append(rng.choice(mine, n))
            uses[k] = n
    idx = np.concatenate(draws)
    rng.shuffle(idx)
    tb = wl.tx_sig_stream(b, schemes, idx, ids, id_idx, nthreads=16)
    with Engine(0) as eng:
        st = eng.verify_tx_signatures(tb)
    hot = uses[key_of[idx]] == 1900  # wide tables (1900 >= both wide thresholds)
    out = {}
    for name, sel in (("wide", hot), ("other", ~hot)):
        out[name] = {"n": int(sel.sum()), "oracle": int((st[sel] == ref[idx][sel]).sum()),
                     "not_run": int((st[sel] == 255).sum()),
                     "other": int(((st[sel] != ref[idx][sel]) & (st[sel] != 255)).sum()),
                     # VALID verdicts returned (a verdict only a ladder can give)
                     "valid": int((st[sel] == 0).sum()), "valid_oracle": int((ref[idx][sel] == 0).sum())}
    detail = {}
    sch = schemes[idx]
    u = uses[key_of[idx]]
    for n in per_key:
        for sc in (2, 3, 4):
            sel = (u == n) & (sch == sc)
            if sel.any():
                detail[f"{n}x_s{sc}"] = {"n": int(sel.sum()), "valid": int((st[sel] == 0).sum()),
                                         "not_run": int((st[sel] == 255).sum()),
                                         "valid_oracle": int((ref[idx][sel] == 0).sum())}
    out["detail"] = detail
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
