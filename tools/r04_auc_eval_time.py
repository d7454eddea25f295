"""Latency of one training-set AUC evaluation (booster.eval_train) at the headline size."""
import os
import sys
import time

sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
import numpy as np  # noqa: E402

import bench  # noqa: E402
import lightgbmv1_amd as lgb  # noqa: E402

X, y = bench.make_rows(0, 10_000_000, 28)
params = {"objective": "binary", "metric": "auc", "max_bin": 255, "num_leaves": 63, "learning_rate": 0.1,
          "min_data_in_leaf": 1, "min_sum_hessian_in_leaf": 100, "device_type": "gpu", "verbose": int(sys.argv[1]) if len(sys.argv) > 1 else -1}
b = lgb.Booster(params=params, train_set=lgb.Dataset(X, y, params=params))
for _ in range(10):
    b.update()
b.eval_train()
ts = []
for _ in range(20):
    t = time.perf_counter()
    v = b.eval_train()[0][2]
    ts.append(time.perf_counter() - t)
print("eval_train ms: median %.3f min %.3f  auc %.10f" % (1e3 * np.median(ts), 1e3 * min(ts), v))
