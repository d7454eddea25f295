"""Which learner disagrees on the categorical round-growth case: host (cpu), one split per step,
rounds -- first tree's leaves and gains."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lightgbmv1_amd as lgb  # noqa: E402
from tests.test_gpu_rounds import _data  # noqa: E402

X, y = _data()
for name, dev, k in [("cpu", "cpu", None), ("steps", "gpu", "1"), ("rounds", "gpu", "8")]:
    if k is not None:
        os.environ["LGBM_AMD_ROUND_K"] = k
    p = {"verbose": -1, "device_type": dev, "seed": 11, "num_leaves": 31, "max_bin": 63, "objective": "binary"}
    ds = lgb.Dataset(X, y, params=p, categorical_feature=[9])
    bst = lgb.train(p, ds, 1)
    t = bst.dump_model()["tree_info"][0]
    gains = []

    def walk(n):
        if "split_gain" in n:
            gains.append(round(n["split_gain"], 2))
            walk(n["left_child"])
            walk(n["right_child"])
    walk(t["tree_structure"])
    print(name, t["num_leaves"], sorted(gains, reverse=True)[:8], flush=True)
