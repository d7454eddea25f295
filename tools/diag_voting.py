"""Diagnostic: voting-parallel device learner on Criteo-shaped data (EFB bundles of sparse count
features) under its growth modes, 2 thread ranks on one GPU: held-out AUC per mode and whether
the models equal the host voting loop's (LGBM_AMD_HOST_ASSIST=1).

  python tools/diag_voting.py [rows_per_rank] [num_leaves]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import lightgbmv1_amd as lgb  # noqa: E402
from lightgbmv1_amd.models.workloads import make_criteo  # noqa: E402
from lightgbmv1_amd.parallel.inproc import ThreadRanks  # noqa: E402


def auc(y, p):
    from scipy.stats import rankdata
    r = rankdata(p)
    pos = y > 0.5
    npos, nneg = int(pos.sum()), int((~pos).sum())
    return float((r[pos].sum() - npos * (npos + 1) / 2.0) / max(1, npos * nneg))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    world = 2
    X, y, _ = make_criteo(world * n, 5)
    Xt, yt, _ = make_criteo(200000, 77)
    leaves = int(sys.argv[2]) if len(sys.argv) > 2 else 63
    base = {"objective": "binary", "num_leaves": leaves, "learning_rate": 0.1, "min_data_in_leaf": 20, "verbose": -1,
            "device_type": "gpu", "seed": 3, "max_bin": 255}
    full = lgb.Dataset(X, y, params=base, free_raw_data=False).construct()

    def run(env, learner="voting", rounds=6):
        old = {k: os.environ.get(k) for k in env}
        os.environ.update(env)
        try:
            def rank_fn(r):
                params = dict(base, tree_learner=learner, num_machines=world, pre_partition=True, top_k=20)
                bst = lgb.train(params, full.subset(np.arange(r, world * n, world)), rounds)
                return bst.model_to_string(), bst.predict(Xt)
            with ThreadRanks(world, timeout_s=300, device_comm=True) as tr:
                res = tr.run(rank_fn)
            assert all(x.ok for x in res), [str(x.error) for x in res]
            return res[0].value
        finally:
            for k, v in old.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    serial = lgb.train(base, full.subset(np.arange(world * n)), 6)
    print("serial AUC %.5f" % auc(yt, serial.predict(Xt)), flush=True)
    out = {}
    for name, env in [("rounds", {}), ("steps", {"LGBM_AMD_ROUND_K": "1"}),
                      ("host", {"LGBM_AMD_HOST_ASSIST": "1"}),
                      ("steps_dense", {"LGBM_AMD_ROUND_K": "1", "LGBM_AMD_SPARSE_ROWS": "0"}),
                      ("rounds_dense", {"LGBM_AMD_SPARSE_ROWS": "0"}),
                      ("steps_nodirect", {"LGBM_AMD_ROUND_K": "1", "LGBM_AMD_DIRECT_FROM_SPLIT": "100000"})]:
        m, p = run(env)
        out[name] = m
        print("%-12s AUC %.5f  equals host %s" % (name, auc(yt, p), "?" if "host" not in out else m == out["host"]),
              flush=True)

    def trees(m):
        return m[m.index("Tree=0"):m.index("end of trees")]
    for a_ in out:
        for b_ in out:
            if a_ < b_:
                print("%s == %s: %s" % (a_, b_, trees(out[a_]) == trees(out[b_])))
    # first differing tree line between steps and rounds
    ta, tb = trees(out["steps"]).splitlines(), trees(out["rounds"]).splitlines()
    for i, (la, lb) in enumerate(zip(ta, tb)):
        if la != lb:
            print("first difference steps vs rounds at line %d:\n  steps : %s\n  rounds: %s" % (i, la[:200], lb[:200]))
            break


if __name__ == "__main__":
    main()
