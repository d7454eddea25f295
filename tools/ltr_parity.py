"""Tree-by-tree parity of the MI355X learner against this framework's CPU learner on a
LambdaRank task (MS-LTR-shaped synthetic data, smaller): the first tree whose split
features / thresholds differ, and held-out NDCG@10 of both models.

    python tools/ltr_parity.py [--rows 300000] [--features 100] [--trees 30] [--params JSON]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import lightgbmv1_amd as lgb  # noqa: E402
from lightgbmv1_amd.models.workloads import make_ltr  # noqa: E402


def ndcg_at(y, p, group, k=10):
    out, start = [], 0
    for g in group:
        yy, pp = y[start:start + g], p[start:start + g]
        start += g
        order = np.argsort(-pp, kind="stable")
        disc = 1.0 / np.log2(np.arange(2, min(g, k) + 2))
        gain = 2.0 ** yy - 1
        dcg = float(np.sum(gain[order][:k] * disc))
        idcg = float(np.sum(np.sort(gain)[::-1][:k] * disc))
        out.append(dcg / idcg if idcg > 0 else 1.0)
    return float(np.mean(out))


def splits(model, t):
    block = model.split("Tree=%d\n" % t)[1].split("\n\n")[0]
    rows = dict(line.split("=", 1) for line in block.splitlines() if "=" in line)
    return rows.get("split_feature"), rows.get("threshold"), rows.get("leaf_value")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=300000)
    ap.add_argument("--features", type=int, default=100)
    ap.add_argument("--trees", type=int, default=30)
    ap.add_argument("--params", default="{}")
    args = ap.parse_args()
    X, y, group = make_ltr(args.rows, 7, num_features=args.features)
    Xt, yt, gt = make_ltr(60000, 8, num_features=args.features)
    base = {"objective": "lambdarank", "num_leaves": 255, "max_bin": 63, "learning_rate": 0.1,
            "min_data_in_leaf": 1, "min_sum_hessian_in_leaf": 100, "verbose": -1, "seed": 3,
            "num_threads": min(16, os.cpu_count() or 8)}
    base.update(json.loads(args.params))
    models, ndcg = {}, {}
    for dev in ("cpu", "gpu"):
        p = dict(base, device_type=dev)
        ds = lgb.Dataset(X, y, group=group, params=p)
        bst = lgb.train(p, ds, args.trees)
        models[dev] = bst.model_to_string()
        ndcg[dev] = ndcg_at(yt, bst.predict(Xt), gt)
    first_diff, detail = None, None
    for t in range(args.trees):
        a, b = splits(models["cpu"], t), splits(models["gpu"], t)
        if a[0] != b[0] or a[1] != b[1]:
            first_diff = t
            fa, fb = a[0].split(), b[0].split()
            ta, tb = a[1].split(), b[1].split()
            k = next((i for i in range(min(len(fa), len(fb))) if fa[i] != fb[i] or ta[i] != tb[i]), None)
            detail = {"node": k, "nodes": [len(fa), len(fb)],
                      "cpu": None if k is None else [fa[k], ta[k]], "gpu": None if k is None else [fb[k], tb[k]]}
            break
    print(json.dumps({"params": base, "trees": args.trees, "first_tree_with_different_splits": first_diff,
                      "first_difference": detail, "ndcg10_cpu": round(ndcg["cpu"], 6),
                      "ndcg10_gpu": round(ndcg["gpu"], 6)}), flush=True)


if __name__ == "__main__":
    main()
