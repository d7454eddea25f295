"""Diagnostic: the distributed device learners (data / feature / voting, 2 thread ranks on one
GPU, device communicator) at 255 leaves under the leaf-scaled round width (16) and width 8:
the models must be equal.

  python tools/diag_width_dist.py [rows_per_rank] [num_leaves]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import lightgbmv1_amd as lgb  # noqa: E402
from lightgbmv1_amd.parallel.inproc import ThreadRanks  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200000
    world = 2
    rng = np.random.default_rng(5)
    X = rng.standard_normal((world * n, 28)).astype(np.float32)
    y = (X[:, :6].sum(axis=1) + 0.5 * rng.standard_normal(world * n) > 0).astype(np.float64)
    base = {"objective": "binary", "num_leaves": int(sys.argv[2]) if len(sys.argv) > 2 else 255, "learning_rate": 0.1, "min_data_in_leaf": 20, "verbose": -1,
            "device_type": "gpu", "seed": 3, "max_bin": 255}
    full = lgb.Dataset(X, y, params=base, free_raw_data=False).construct()
    ok = True
    for learner in ("data", "feature", "voting"):
        models = {}
        for k in ("16", "8", "1"):
            os.environ["LGBM_AMD_ROUND_K"] = k

            def rank_fn(r):
                params = dict(base, tree_learner=learner, num_machines=world, pre_partition=learner != "feature",
                              top_k=20)
                ds = full.subset(np.arange(r, world * n, world)) if learner != "feature" else full.subset(
                    np.arange(world * n))
                return lgb.train(params, ds, 6).model_to_string()

            with ThreadRanks(world, timeout_s=300, device_comm=True) as tr:
                res = tr.run(rank_fn)
            assert all(x.ok for x in res), [str(x.error) for x in res]
            assert res[0].value == res[1].value, (learner, k, "ranks differ")
            models[k] = res[0].value
        same = models["16"] == models["8"]
        ok = ok and same
        print("%-8s width 16 == width 8: %s, width 8 == one split per step: %s" % (
            learner, same, models["8"] == models["1"]), flush=True)
        for a_, b_ in (("16", "8"), ("8", "1")):
            la, lb = models[a_].splitlines(), models[b_].splitlines()
            d = [(x, z) for x, z in zip(la, lb) if x != z]
            if d:
                print("  %s vs %s: %d lines differ; first: %s | %s" % (a_, b_, len(d), d[0][0][:150], d[0][1][:150]))
    os.environ.pop("LGBM_AMD_ROUND_K", None)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
