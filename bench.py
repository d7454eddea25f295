"""Headline benchmark: sec/iteration of GBDT training on a Higgs-shaped 10M x 28 binary task.

Config (BASELINE.json / docs GPU-Performance): objective=binary, max_bin=255,
num_leaves=63, learning_rate=0.1, min_data_in_leaf=1, min_sum_hessian_in_leaf=100,
device_type=gpu.  A "step" is one boosting iteration (gradients + one tree + score
update).  Synthetic data: 10M rows x 28 float32 features with a non-linear label
(21 "low-level" + 7 "high-level" derived features, Higgs-like layout); AUC on a
held-out synthetic set is reported for parity checks.

  python bench.py --gpus 1 --steps 50 --warmup 5
  python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
      --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 5

With N>1 ranks the 10M rows are sharded row-wise (rank r owns rows r*10M/N ...), one
process per GPU, tree_learner=data: each round reduce-scatters its expansions' histograms to
the feature owners and all-gathers the owners' results over the peer communicator (one kernel
per collective reading the peers' HBM over xGMI; RCCL with LGBM_AMD_DEVICE_COMM=rccl).  Strong
scaling: the total work is fixed, and the trees equal the 1-GPU trees.

AUC parity: `auc_ref` is the held-out AUC of the same run (rows, generator seeds, tree count)
trained by this framework's CPU learner, which grows the reference CLI's trees byte for byte
(tests/test_golden.py); the values are pinned in tools/bench_auc_ref.json.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_SEC_PER_ITER = 0.232  # GTX 1080, Higgs 10.5M x 28, 255 bins
AUC_REF_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tools", "bench_auc_ref.json")


def auc_reference(rows, features, leaves, max_bin, test_rows, trees, params):
    """The pinned CPU-learner AUC of this exact run, or None when the fixture has none."""
    if params or not os.path.exists(AUC_REF_FILE):
        return None
    key = dict(rows=rows, features=features, leaves=leaves, max_bin=max_bin, test_rows=test_rows, trees=trees)
    for e in json.load(open(AUC_REF_FILE))["entries"]:
        if all(e.get(k) == v for k, v in key.items()):
            return e
    return None


def make_rows(start, count, num_features=28, seed=20240601):
    """Deterministic synthetic Higgs-like rows [start, start+count) (models/workloads.py)."""
    from lightgbmv1_amd.models.workloads import make_higgs
    X, y, _ = make_higgs(count, seed=seed, start=start, num_features=num_features)
    return X, y


def roc_auc(y, p):
    from scipy.stats import rankdata
    ranks = rankdata(p)
    pos = y > 0.5
    npos, nneg = int(pos.sum()), int((~pos).sum())
    return float((ranks[pos].sum() - npos * (npos + 1) / 2.0) / max(1, npos * nneg))


def growth_stats(booster):
    """[trees, device-resident, rounds, expansions, splits, collective bytes, trees launched
    speculatively] so far (LGBM_AMD_BoosterGrowthStats: counters, no device synchronisation)"""
    import ctypes
    from lightgbmv1_amd import _native as nat
    out = (ctypes.c_double * 7)()
    nat.call("LGBM_AMD_BoosterGrowthStats", booster.handle, out, ctypes.c_int(7))
    return list(out)


def _device_sync(lgb):
    """Drain the device queue around the timed region (the learner's own HIP runtime;
    torch.cuda.synchronize() as well when torch already drives a GPU in this process)."""
    lgb.device_synchronize()
    torch = sys.modules.get("torch")
    if torch is not None and torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=500)  # the metric's 500 trees
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--features", type=int, default=28)
    ap.add_argument("--leaves", type=int, default=63)
    ap.add_argument("--max-bin", type=int, default=255)
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--test-rows", type=int, default=500_000)
    ap.add_argument("--hist-precision", choices=["fx32", "fx64"], default="fx32",
                    help="fx32: 32-bit fixed-point (g, h) per row, packed in one 64-bit histogram word; "
                         "fx64 (gpu_use_dp): 2x 64-bit words, 31-bit row resolution")
    ap.add_argument("--params", default="{}", help="extra training parameters (JSON)")
    ap.add_argument("--eval-train", action="store_true",
                    help="evaluate the training AUC after every iteration inside the timed loop "
                         "(valid_sets=[dtrain] cost; device-resident metric)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import lightgbmv1_amd as lgb
    from lightgbmv1_amd.parallel import torch_dist

    if world > 1:
        torch_dist.init_network(use_rccl=args.device == "gpu")
    n_total = args.rows
    lo = n_total * rank // world
    hi = n_total * (rank + 1) // world
    t0 = time.time()
    X, y = make_rows(lo, hi - lo, args.features)
    params = {
        "objective": "binary",
        "metric": "auc",
        "max_bin": args.max_bin,
        "num_leaves": args.leaves,
        "learning_rate": 0.1,
        "min_data_in_leaf": 1,
        "min_sum_hessian_in_leaf": 100,
        "device_type": args.device,
        "tree_learner": "data" if world > 1 else "serial",
        "num_machines": world,
        "pre_partition": True,
        "verbose": -1,
        "num_threads": min(16, os.cpu_count() or 8),
        "gpu_use_dp": args.hist_precision == "fx64",
    }
    params.update(json.loads(args.params))
    train = lgb.Dataset(X, y, params=params, free_raw_data=True)
    booster = lgb.Booster(params=params, train_set=train)
    del X
    setup_s = time.time() - t0
    for _ in range(args.warmup):
        booster.update()
    torch_dist.barrier()
    # (with speculation -- LGBM_AMD_SPECULATE=1, one process -- the last warm-up update launched
    # the first timed tree, and this synchronisation lets it finish before the clock starts; the
    # last timed update launches one more tree, which the closing synchronisation waits for: the
    # timed region runs exactly `steps` trees' device work)
    _device_sync(lgb)
    stats0 = growth_stats(booster) if args.device == "gpu" else None
    t1 = time.perf_counter()
    train_auc = None
    for _ in range(args.steps):
        booster.update()
        if args.eval_train:
            train_auc = booster.eval_train()[0][2]
    _device_sync(lgb)
    torch_dist.barrier()
    elapsed = time.perf_counter() - t1
    elapsed = torch_dist.allreduce_max(elapsed)
    sec_per_iter = elapsed / max(1, args.steps)
    diag = {}
    if stats0 is not None and args.steps > 0:
        # the timed trees' growth counters (no synchronisation inside the timed loop)
        d = [b - a for a, b in zip(stats0, growth_stats(booster))]
        diag = {"rounds_per_tree": round(d[2] / max(1.0, d[0]), 2),
                "collective_bytes_per_iter": round(d[5] / args.steps),
                "speculated_trees": int(d[6])}
    auc = None
    if rank == 0 and args.test_rows > 0:
        Xt, yt = make_rows(n_total + 12345678, args.test_rows, args.features)
        auc = roc_auc(yt, booster.predict(Xt))
    ref = auc_reference(n_total, args.features, args.leaves, args.max_bin, args.test_rows, booster.num_trees(),
                        json.loads(args.params)) if args.device == "gpu" else None
    auc_fields = {"auc_ref": ref["auc"] if ref else None,
                  "auc_delta": float("%.3g" % (auc - ref["auc"])) if ref and auc is not None else None}
    if rank == 0:
        print(json.dumps({
            "metric": "sec/iteration (500 trees, 255 bins, 63 leaves) on Higgs-shaped 10Mx28; AUC parity",
            "value": round(sec_per_iter, 6),
            "unit": "s/iter",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * sec_per_iter, 4),
            "higher_is_better": False,
            "scaling": "strong",
            "vs_baseline": round(sec_per_iter / BASELINE_SEC_PER_ITER, 6),
            # (g, h) are fp32; histogram inputs are fixed-point at a per-tree power-of-two scale
            # (fx32: 2^30 / (16384 * max|g|), i.e. ~16 bits below max|g| per row; fx64: 2^31 /
            # max|g|), summed exactly in int64, independent of the row count; scans in fp64
            "dtype": "fp32-grad/{}-hist/fp64-scan".format(args.hist_precision),
            "data": "synthetic",
            "config": {"model": "gbdt binary, num_leaves={}, max_bin={}".format(args.leaves, args.max_bin),
                       "global_batch": n_total, "seq_len": args.features,
                       "parallelism": "dp{}".format(world) if world > 1 else "single"},
            "auc_heldout": auc,
            **auc_fields,
            "trees": booster.num_trees(),
            "device_comm": torch_dist.device_comm_kind() if world > 1 else None,
            **({"device_topology": torch_dist.device_topology()} if world > 1 else {}),
            **diag,
            **({"train_auc": train_auc} if args.eval_train else {}),
            "setup_s": round(setup_s, 2),
        }), flush=True)
    if world > 1:
        torch_dist.shutdown()


if __name__ == "__main__":
    main()
