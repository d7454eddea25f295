"""extra_trees on the headline shape (Higgs-like 10Mx28, 255 bins, 63 leaves): device-resident
growth vs the host-assisted learner (LGBM_AMD_HOST_ASSIST=1, run as a separate process).
Prints one JSON line per mode: ms per boosting iteration and held-out AUC."""
import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run(rows, steps, warmup):
    import lightgbmv1_amd as lgb
    rng = np.random.RandomState(0)
    X = rng.randn(rows + 200_000, 28).astype(np.float32)
    logit = X[:, 0] + 0.7 * X[:, 1] * X[:, 2] - 0.5 * np.abs(X[:, 3]) + 0.3 * X[:, 4]
    y = (logit + 0.5 * rng.randn(len(X)) > 0).astype(np.float32)
    params = {"objective": "binary", "device_type": "gpu", "num_leaves": 63, "max_bin": 255,
              "learning_rate": 0.1, "extra_trees": True, "verbose": -1}
    bst = lgb.Booster(params=params, train_set=lgb.Dataset(X[:rows], y[:rows], params=params))
    for _ in range(warmup):
        bst.update()
    t0 = time.perf_counter()
    for _ in range(steps):
        bst.update()
    dt = (time.perf_counter() - t0) / steps
    from scipy.stats import rankdata
    p = bst.predict(X[rows:])
    r = rankdata(p)
    pos = y[rows:] > 0.5
    auc = (r[pos].sum() - pos.sum() * (pos.sum() + 1) / 2) / (pos.sum() * (~pos).sum())
    mode = "host-assisted" if os.environ.get("LGBM_AMD_HOST_ASSIST") == "1" else "device-resident"
    print(json.dumps({"bench": "extra_trees", "mode": mode, "rows": rows, "ms_per_iter": round(dt * 1e3, 3),
                      "steps": steps, "auc_heldout": round(float(auc), 6)}), flush=True)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--child", action="store_true")
    a = ap.parse_args()
    if a.child:
        run(a.rows, a.steps, a.warmup)
    else:
        for host in ("0", "1"):
            env = dict(os.environ, LGBM_AMD_HOST_ASSIST=host)
            rc = subprocess.call([sys.executable, __file__, "--child", "--rows", str(a.rows), "--steps",
                                  str(a.steps), "--warmup", str(a.warmup)], env=env)
            if rc != 0:
                sys.exit(rc)
