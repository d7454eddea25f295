"""BASELINE.json config #4: MS-LTR-shaped 3M x 700 LambdaRank with GOSS on one MI355X.

Synthetic learning-to-rank data of the MS-LTR shape (queries of 20-220 documents, ~120 on
average; 5 relevance grades with MS-LTR-like proportions; 40 informative dense features,
dense noise and sparse count-like features), objective=lambdarank, boosting=goss,
num_leaves=255, max_bin=63 (the reference's GPU comparison settings for MS-LTR,
docs/GPU-Performance.rst:108-125).  A step is one boosting iteration; warmup covers the
first 1 / learning_rate iterations, so every timed iteration samples with GOSS.  NDCG@10
is reported on held-out queries.

  python tools/bench_ltr.py --steps 50 --warmup 12
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

# reference MS-LTR (2.27M x 137), 255 leaves, 63 bins, GTX 1080: 111 s / 500 iterations
BASELINE_SEC_PER_ITER = 111.0 / 500


def make_ltr(num_rows, num_features, seed):
    from lightgbmv1_amd.models.workloads import make_ltr as _make
    return _make(num_rows, seed, num_features=num_features)


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=12)
    ap.add_argument("--rows", type=int, default=3_000_000)
    ap.add_argument("--features", type=int, default=700)
    ap.add_argument("--leaves", type=int, default=255)
    ap.add_argument("--max-bin", type=int, default=63)
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--test-rows", type=int, default=200_000)
    ap.add_argument("--params", default="{}", help="extra training parameters (JSON)")
    args = ap.parse_args()
    import threading
    t_start = time.time()

    def heartbeat():  # long data generation: progress lines for job monitors
        while True:
            time.sleep(30.0)
            print("[bench] %.0f s elapsed" % (time.time() - t_start), file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    import lightgbmv1_amd as lgb

    t0 = time.time()
    X, y, group = make_ltr(args.rows, args.features, 7)
    params = {"objective": "lambdarank", "boosting": "goss", "num_leaves": args.leaves, "max_bin": args.max_bin,
              "learning_rate": 0.1, "min_data_in_leaf": 1, "min_sum_hessian_in_leaf": 100,
              "device_type": args.device, "verbose": -1, "num_threads": min(16, os.cpu_count() or 8)}
    params.update(json.loads(args.params))
    train = lgb.Dataset(X, y, group=group, params=params, free_raw_data=True)
    booster = lgb.Booster(params=params, train_set=train)
    del X
    setup_s = time.time() - t0
    for _ in range(args.warmup):
        booster.update()
    lgb.device_synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        booster.update()
    lgb.device_synchronize()
    sec = (time.perf_counter() - t1) / max(1, args.steps)
    Xt, yt, gt = make_ltr(args.test_rows, args.features, 8)
    ndcg = ndcg_at(yt, booster.predict(Xt), gt)
    # the histograms' precision (gpu_hist_precision=auto: wide int64 sums for listwise objectives)
    prec = params.get("gpu_hist_precision", "auto")
    if params.get("gpu_use_dp") or (prec == "auto" and params["objective"] in ("lambdarank", "rank_xendcg")):
        prec = "fx64"
    elif prec == "auto":
        prec = "fx32"
    hist = "fp64" if args.device == "cpu" else prec
    print(json.dumps({
        "metric": "sec/iteration lambdarank + GOSS on MS-LTR-shaped 3Mx700 (255 leaves, 63 bins); NDCG@10",
        "value": round(sec, 6), "unit": "s/iter", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(1000 * sec, 4), "higher_is_better": False,
        "vs_baseline": round(sec / BASELINE_SEC_PER_ITER, 6), "dtype": "fp32-grad/%s-hist/fp64-scan" % hist,
        "data": "synthetic", "device": args.device,
        "config": {"model": "gbdt lambdarank {}, num_leaves={}, max_bin={}".format(params["boosting"], args.leaves,
                                                                                  args.max_bin),
                   "rows": args.rows, "features": args.features, "queries": int(len(group))},
        "ndcg10_heldout": round(ndcg, 6), "trees": booster.num_trees(), "setup_s": round(setup_s, 1)}), flush=True)


if __name__ == "__main__":
    main()
