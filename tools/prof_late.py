#!/usr/bin/env python3
"""Late-tree profiling helper: `train N` trains N headline iterations (untraced) and saves the
model; `cont K` continues K iterations from it (run under rocprofv3: the trace then holds
late trees only, after the init-score prediction).
  python tools/prof_late.py train 150 /tmp/m.txt ; rocprofv3 ... -- python tools/prof_late.py cont 3 /tmp/m.txt"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import lightgbmv1_amd as lgb  # noqa: E402
from bench import make_rows  # noqa: E402

mode, n, path = sys.argv[1], int(sys.argv[2]), sys.argv[3]
X, y = make_rows(0, 10_000_000, 28)
params = {"objective": "binary", "max_bin": 255, "num_leaves": 63, "learning_rate": 0.1, "min_data_in_leaf": 1,
          "min_sum_hessian_in_leaf": 100, "device_type": "gpu", "verbose": -1}
ds = lgb.Dataset(X, y, params=params, free_raw_data=False)
if mode == "train":
    lgb.train(params, ds, n).save_model(path)
else:
    lgb.train(params, ds, n, init_model=path)
print("done", mode, n)
