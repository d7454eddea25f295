"""debug: first tree of round growth (K=8) vs one split per step for a test_gpu_rounds case"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import lightgbmv1_amd as lgb
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
from test_gpu_rounds import _data, CASES
case = sys.argv[1]
X, y = _data()
params = dict(CASES[case])
p = {"verbose": -1, "device_type": "gpu", "seed": 11, "num_leaves": 31, "max_bin": 63}
p.update(params)
out = {}
for k in (1, 8):
    os.environ["LGBM_AMD_ROUND_K"] = str(k)
    bst = lgb.train(p, lgb.Dataset(X, y, params=p), 1)
    t = bst.dump_model()["tree_info"][0]["tree_structure"]
    seq = []
    def walk(n, d):
        if "leaf_index" in n:
            seq.append(("L", n["leaf_index"], n["leaf_count"], round(n["leaf_value"], 9)))
            return
        seq.append(("S", n["split_index"], n["split_feature"], n["threshold"], round(n["split_gain"], 6), n["internal_count"]))
        walk(n["left_child"], d + 1); walk(n["right_child"], d + 1)
    walk(t, 0)
    out[k] = seq
for a, b in zip(out[1], out[8]):
    print(("   " if a == b else "!! ") + str(a) + "  |  " + str(b))
