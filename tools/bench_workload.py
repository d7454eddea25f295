"""Training speed and quality on any of the reference's benchmark workloads
(lightgbmv1_amd/models/workloads.py: higgs, epsilon, bosch, ms_ltr, expo, yahoo_ltr,
criteo) with the reference's GPU-comparison configuration (num_leaves=255,
min_data_in_leaf=1, min_sum_hessian_in_leaf=100; docs/GPU-Performance.rst:108-125).

  python tools/bench_workload.py --name epsilon --max-bin 63 --steps 50
  python tools/bench_workload.py --name ms_ltr --rows 500000 --steps 20

Prints one JSON line: sec/iteration over the timed steps, the reference's published
GTX 1080 sec/iteration at this max_bin (its 500-iteration wall time / 500) and the
held-out AUC / NDCG@10 after the trained iterations.  --rows scales the dataset down
(the reference number is then not directly comparable; the line says so).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def auc(y, p):
    from scipy.stats import rankdata
    r = rankdata(p)
    pos = y > 0.5
    npos, nneg = int(pos.sum()), int((~pos).sum())
    return float((r[pos].sum() - npos * (npos + 1) / 2.0) / max(1, npos * nneg))


def ndcg10(y, p, group):
    out, s = [], 0
    for g in group:
        yy, pp = y[s:s + g], p[s:s + g]
        s += g
        gain = 2.0 ** yy - 1
        disc = 1.0 / np.log2(np.arange(2, min(10, g) + 2))
        ideal = np.sort(gain)[::-1][:10] @ disc
        if ideal > 0:
            out.append(gain[np.argsort(-pp, kind="stable")][:10] @ disc / ideal)
    return float(np.mean(out)) if out else 1.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--name", default="higgs")
    ap.add_argument("--rows", type=int, default=0, help="0: the real dataset's size")
    ap.add_argument("--test-rows", type=int, default=200_000)
    ap.add_argument("--max-bin", type=int, default=63)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--verbose", type=int, default=-1)
    args = ap.parse_args()
    import threading
    t_start = time.time()
    stop = threading.Event()

    def heartbeat():  # long setups (11M x 700) print progress for job monitors
        while not stop.wait(30.0):
            print("[bench_workload] %.0f s elapsed" % (time.time() - t_start), file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    import lightgbmv1_amd as lgb
    from lightgbmv1_amd import models

    w = models.get(args.name)
    rows = args.rows or w.rows
    t0 = time.time()
    X, y, group = w.make(rows)
    params = w.params(args.max_bin, args.device)
    params["num_threads"] = min(16, os.cpu_count() or 8)
    params["verbose"] = args.verbose
    ds = lgb.Dataset(X, y, group=group, params=params, categorical_feature=w.categorical or "auto",
                     free_raw_data=True)
    booster = lgb.Booster(params=params, train_set=ds)
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
    Xt, yt, gt = w.make(args.test_rows, seed=987)
    pred = booster.predict(Xt)
    quality = {"auc": auc(yt, pred)} if w.task == "binary" else {"ndcg@10": ndcg10(yt, pred, gt)}
    ref = w.reference.get("gtx1080_s_500it", {}).get(args.max_bin)
    print(json.dumps({
        "workload": args.name, "rows": rows, "features": w.features, "max_bin": args.max_bin,
        "num_leaves": params["num_leaves"], "device": args.device, "steps": args.steps,
        "sec_per_iter": round(sec, 6),
        "ref_gtx1080_sec_per_iter": None if ref is None else ref / 500.0,
        "speedup_vs_ref": None if ref is None else round(ref / 500.0 / sec, 2),
        "rows_scaled": rows != w.rows, "trees": args.warmup + args.steps, **quality,
        "setup_s": round(setup_s, 1), "data": "synthetic",
        "env": {k: v for k, v in os.environ.items() if k.startswith("LGBM_AMD_")},
    }))
    stop.set()


if __name__ == "__main__":
    main()
