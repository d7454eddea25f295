"""Debug probe: first differing node between the CPU and device learners' first tree."""
import os, sys
import numpy as np
sys.path.insert(0, ".")
import lightgbmv1_amd as lgb

rng = np.random.RandomState(12)
n = 40000
X = rng.randn(n, 6).astype(np.float32)
X[:, 0] = rng.randint(0, 24, size=n)
X[:, 1] = rng.randint(0, 3, size=n)
eff = np.sin(np.arange(24) * 1.7)
y = ((1.5 * eff[X[:, 0].astype(int)] + 0.8 * (X[:, 1] == 2) + X[:, 2] + 0.3 * rng.randn(n)) > 0.2).astype(np.float32)
cat = [0, 1] if os.environ.get("NOCAT") is None else []
trees = {}
for device in ("cpu", "gpu"):
    params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "device_type": device,
              "max_cat_to_onehot": 4, "min_data_per_group": 50, "cat_smooth": 5, "deterministic": True}
    ds = lgb.Dataset(X, y, params=params, categorical_feature=cat or "auto", free_raw_data=False)
    b = lgb.train(params, ds, 1, verbose_eval=False)
    trees[device] = b.dump_model()["tree_info"][0]["tree_structure"]

def walk(a, b, path):
    ka = {k: a.get(k) for k in ("split_feature", "threshold", "internal_count", "leaf_value", "leaf_count", "split_gain")}
    kb = {k: b.get(k) for k in ka}
    same = ka["split_feature"] == kb["split_feature"] and str(ka["threshold"]) == str(kb["threshold"]) and \
        ka["internal_count"] == kb["internal_count"] and ka["leaf_count"] == kb["leaf_count"]
    print(path or "root", "OK" if same else "DIFF", ka, "|", kb)
    if not same:
        return
    for c in ("left_child", "right_child"):
        if c in a and c in b:
            walk(a[c], b[c], path + "/" + c[0])

walk(trees["cpu"], trees["gpu"], "")
