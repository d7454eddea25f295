"""Debug probe: categorical device training vs CPU (per-tree structure + device split self-check)."""
import json, sys, ctypes
import numpy as np
sys.path.insert(0, ".")
import lightgbmv1_amd as lgb
from lightgbmv1_amd import _native as nat

rng = np.random.RandomState(12)
n = 40000
X = rng.randn(n, 6).astype(np.float32)
X[:, 0] = rng.randint(0, 24, size=n)
X[:, 1] = rng.randint(0, 3, size=n)
eff = np.sin(np.arange(24) * 1.7)
y = ((1.5 * eff[X[:, 0].astype(int)] + 0.8 * (X[:, 1] == 2) + X[:, 2] + 0.3 * rng.randn(n)) > 0.2).astype(np.float32)
for rounds in (1, 2, 3, 5):
    out = {}
    for device in ("cpu", "gpu"):
        params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "device_type": device,
                  "max_cat_to_onehot": 4, "min_data_per_group": 50, "cat_smooth": 5, "deterministic": True, "max_bin": int(__import__("os").environ.get("MAXBIN", "255"))}
        ds = lgb.Dataset(X, y, params=params, categorical_feature=[0, 1], free_raw_data=False)
        b = lgb.train(params, ds, rounds, verbose_eval=False, keep_training_booster=True)
        t = b.dump_model()["tree_info"][-1]
        out[device] = (t["num_leaves"], t["tree_structure"].get("split_feature"), t["tree_structure"].get("threshold"))
        if device == "gpu":
            text = nat.read_string(lambda size, need, buf: nat.call("LGBM_AMD_BoosterDeviceCheckSplits", b.handle, size, need, buf), 1 << 16)
            rep = json.loads(text)
            print("rounds", rounds, "check:", {k: rep.get(k) for k in ("checked", "mismatched", "gain_mismatch", "layout")}, rep["details"][:3])
            p = b.predict(X)
            from scipy.stats import rankdata
            r = rankdata(p); pos = y > 0.5
            print("  gpu auc", (r[pos].sum() - pos.sum() * (pos.sum() + 1) / 2) / (pos.sum() * (~pos).sum()))
    print("rounds", rounds, out)
