"""Print the first trees' leaf values with device vs host percentile renewal (debug aid)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import lightgbmv1_amd as lgb  # noqa: E402

rng = np.random.RandomState(11)
n = 20000
X = rng.randn(n, 6)
y = X[:, 0] * 2 + np.abs(X[:, 1]) + rng.standard_t(3, n)
params = {"verbose": -1, "device_type": "gpu", "num_leaves": 15, "seed": 2, "objective": "quantile", "alpha": 0.8}
out = {}
for mode in ("dev", "host"):
    os.environ["LGBM_AMD_HOST_RENEW"] = "1" if mode == "host" else "0"
    b = lgb.train(params, lgb.Dataset(X, y), 8)
    out[mode] = b.dump_model()["tree_info"]
for t in range(8):
    def leaves(node, acc):
        if "leaf_index" in node:
            acc[node["leaf_index"]] = (node["leaf_value"], node.get("leaf_count"))
        else:
            leaves(node["left_child"], acc)
            leaves(node["right_child"], acc)
        return acc
    a = leaves(out["dev"][t]["tree_structure"], {})
    b = leaves(out["host"][t]["tree_structure"], {})
    for k in sorted(a):
        if a[k] != b.get(k):
            print("tree", t, "leaf", k, "dev", repr(a[k]), "host", repr(b.get(k)))
print("done")
# recompute leaf 8 of tree 7 from the rows the model routes there
os.environ["LGBM_AMD_HOST_RENEW"] = "0"
b = lgb.train(params, lgb.Dataset(X, y), 8)
leaf = b.predict(X, pred_leaf=True)[:, 7]
prev = b.predict(X, num_iteration=7, raw_score=True)
r = (y.astype(np.float32).astype(np.float64) - prev)[leaf == 8]
n = len(r)
alpha = 0.8
fpos = (1.0 - alpha) * n
pos = int(fpos)
s = np.sort(r)[::-1]
v1, v2 = s[pos - 1], s[pos]
bias = fpos - pos
print("n", n, "pos", pos, "bias", repr(bias), "v1", repr(v1), "v2", repr(v2))
print("host formula", repr((v1 - (v1 - v2) * bias) * 0.1), "fma", repr(np.float64(v1 - np.float64((v1 - v2) * bias)) * 0.1))
