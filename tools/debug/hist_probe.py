"""Print device vs expected histogram bins of one leaf (debug aid for tests/test_gpu_kernels.py)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
import lightgbmv1_amd as lgb  # noqa: E402
import test_gpu_kernels as T  # noqa: E402

n = 20000
X, y = T._data(n)
params = dict(T.BASE)
ds = lgb.Dataset(X, y, params=params, free_raw_data=False)
bst = lgb.train(params, ds, int(sys.argv[1]) if len(sys.argv) > 1 else 4, verbose_eval=False,
                keep_training_booster=True)
bins, bounds = T._group_bins(ds)
g, h, scales = T._gradients(bst, n)
print("scales", scales, "g[:4]", g[:4], "h[:4]", h[:4], "bounds", bounds[:6])
gq = T._quantise(g, scales[0])
hq = T._quantise(h, scales[1])
for leaf in (0, 1):
    rows, hist, valid, sums = T._leaf_state(bst, leaf)
    print("leaf", leaf, "rows", len(rows), "sums", sums, "sum gq/scale", gq[rows].sum() / scales[0],
          "sum hq/scale", hq[rows].sum() / scales[1])
    gi = bins[rows, 0] + bounds[0]
    exp = np.bincount(gi[bins[rows, 0] != 0], weights=gq[rows][bins[rows, 0] != 0], minlength=bounds[-1])
    exph = np.bincount(gi[bins[rows, 0] != 0], weights=hq[rows][bins[rows, 0] != 0], minlength=bounds[-1])
    for b in range(1, 8):
        print("  bin", b, "dev", hist[b], "exp", exp[b], exph[b], "valid", valid[b])
    print("  dev total g over group0", hist[1:bounds[1], 0].sum(), "exp", exp[1:bounds[1]].sum())
