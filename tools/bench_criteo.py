"""BASELINE.json config #5 proxy: Criteo-shaped sparse CTR data (67 count-encoded features,
most of them sparse, bundled by EFB) at 100M rows per GPU, 255 leaves.

The reference's distributed experiment (docs/Experiments.rst:188-242) trains Criteo
1.7B x 67 with 255 leaves: 627.8 s per tree on one machine, 80 s on 8, 42 s on 16.  A
1B-row job on 8 MI355X is 125M rows per GPU; this script measures the per-tree time of
one GPU on a 100M-row shard of that shape (the multi-GPU run adds one histogram
all-reduce per split on top).  Synthetic data: 13 dense heavy-tailed counts + 54 sparse
count features (97-99.5% zeros), ~3.4% positives.

  python tools/bench_criteo.py --rows 100000000 --steps 10 --warmup 2
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/bench_criteo.py \
      --rows R --learner voting      # config #5's learner: R rows per rank, one process per GPU
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

REF_SEC_PER_TREE_1_MACHINE = 627.8   # 1.7B rows, 1 machine (docs/Experiments.rst:231)
REF_SEC_PER_TREE_8_MACHINES = 80.0   # 1.7B rows, 8 machines (:237)


def make_ctr(num_rows, seed):
    from lightgbmv1_amd.models.workloads import make_criteo
    X, y, _ = make_criteo(num_rows, seed)
    return X, y


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=100_000_000)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--leaves", type=int, default=255)
    ap.add_argument("--device", default="gpu")
    ap.add_argument("--learner", default="serial", choices=["serial", "data", "voting"],
                    help="under torchrun: the distributed learner (rows are per rank)")
    ap.add_argument("--top-k", type=int, default=20)
    args = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    import threading
    t_start = time.time()

    def heartbeat():  # long data generation: progress lines for job monitors
        while True:
            time.sleep(30.0)
            print("[bench] %.0f s elapsed" % (time.time() - t_start), file=sys.stderr, flush=True)

    threading.Thread(target=heartbeat, daemon=True).start()
    import lightgbmv1_amd as lgb
    from lightgbmv1_amd.parallel import torch_dist

    if world > 1:
        torch_dist.init_network(use_rccl=args.device == "gpu")
    t0 = time.time()
    X, y = make_ctr(args.rows, 5 + rank)  # (each rank its own shard)
    t_gen = time.time() - t0
    params = {"objective": "binary", "num_leaves": args.leaves, "learning_rate": 0.1, "max_bin": 255,
              "min_data_in_leaf": 20, "device_type": args.device, "verbose": -1,
              "num_threads": min(16 // max(1, world) if world > 1 else 16, os.cpu_count() or 8)}
    if world > 1:
        params.update(tree_learner=args.learner, num_machines=world, pre_partition=True, top_k=args.top_k)
    train = lgb.Dataset(X, y, params=params, free_raw_data=True)
    booster = lgb.Booster(params=params, train_set=train)
    del X
    setup_s = time.time() - t0
    for _ in range(args.warmup):
        booster.update()
    torch_dist.barrier()
    lgb.device_synchronize()
    t1 = time.perf_counter()
    for _ in range(args.steps):
        booster.update()
    lgb.device_synchronize()
    torch_dist.barrier()
    sec = torch_dist.allreduce_max((time.perf_counter() - t1) / max(1, args.steps))
    # the reference's single-machine time scaled to this shard's rows (linear in rows)
    ref_scaled = REF_SEC_PER_TREE_1_MACHINE * args.rows * world / 1.7e9
    if rank != 0:
        torch_dist.shutdown() if world > 1 else None
        return
    print(json.dumps({
        "metric": "sec/tree, Criteo-shaped 67 sparse count features (EFB), 255 leaves, one GPU shard",
        "value": round(sec, 6), "unit": "s/tree", "ranks": world, "learner": args.learner if world > 1 else "serial",
        "steps": args.steps, "warmup": args.warmup,
        "higher_is_better": False, "rows_per_rank": args.rows, "dtype": "fp32-grad/fx32-hist/fp64-scan", "data": "synthetic",
        "reference_1_machine_scaled_to_rows_s": round(ref_scaled, 3),
        "reference_8_machines_1p7B_s": REF_SEC_PER_TREE_8_MACHINES,
        "data_gen_s": round(t_gen, 1), "setup_s": round(setup_s, 1), "trees": booster.num_trees()}), flush=True)
    if world > 1:
        torch_dist.shutdown()


if __name__ == "__main__":
    main()
