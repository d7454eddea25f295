"""One rank of a multi-process run over the built-in TCP mesh (``machines=`` list).

  python net_worker.py MODE RANK MACHINES OUT_DIR
MODE "collectives": runs allgather / reduce-scatter / all-reduce checks and writes
OUT_DIR/coll_<rank>.json; "train": trains a data-parallel model and writes
OUT_DIR/model_<rank>.txt; "die": joins the mesh and exits at once (peer failure);
"survive": joins, then trains -- it must fail with an error, not hang or abort;
"train_mpi": like "train" over the MPI transport (LGBM_AMD_NETWORK=mpi in the environment,
MACHINES only gives the world size).
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))

import lightgbmv1_amd as lgb  # noqa: E402
from lightgbmv1_amd import _native as nat  # noqa: E402
from lightgbmv1_amd.parallel import host  # noqa: E402


def rank_vector(rank, n, salt=0):
    # integer-valued doubles: sums are exact whatever the reduction order
    return (np.arange(n, dtype=np.float64) % 97) * (rank + 1) + salt


def collectives(rank, world, out_dir):
    res = {}
    # variable-size allgather (rank r sends r*3+1 items; one empty block when world > 2)
    blocks = host.allgather(rank_vector(rank, 0 if rank == 1 and world > 2 else rank * 3 + 1))
    res["allgather"] = [b.tolist() for b in blocks]
    counts = [(i * 7) % 5 + 2 for i in range(world)]
    mine = host.reduce_scatter_sum(rank_vector(rank, sum(counts)), counts)
    res["reduce_scatter"] = mine.tolist()
    for size in (5, 100000):  # small: allgather + local sum; large: reduce-scatter + allgather
        res["allreduce_%d" % size] = host.allreduce_sum(rank_vector(rank, size, salt=1)).sum()
    with open(os.path.join(out_dir, "coll_%d.json" % rank), "w") as f:
        json.dump(res, f)


def make_data(n=3000, f=8, seed=11):
    rng = np.random.RandomState(seed)
    X = rng.rand(n, f)
    y = (X[:, 0] + 0.5 * X[:, 1] + 0.2 * rng.rand(n) > 0.9).astype(np.float64)
    return X, y


def train(rank, world, machines, port, out_dir):
    X, y = make_data()
    idx = np.arange(rank, X.shape[0], world)
    params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "tree_learner": "data",
              "num_machines": world, "machines": machines, "local_listen_port": port, "pre_partition": True,
              "min_data_in_leaf": 20, "seed": 3, "deterministic": True, "num_threads": 2, "time_out": 1}
    bst = lgb.train(params, lgb.Dataset(X[idx], y[idx], params=params), 8)
    with open(os.path.join(out_dir, "model_%d.txt" % rank), "w") as f:
        f.write(bst.model_to_string())


def train_mpi(rank, world, out_dir):
    nat.call("LGBM_NetworkInit", nat.cstr(""), nat.c_int(0), nat.c_int(1), nat.c_int(world))
    assert host.world() == (rank, world), host.world()
    X, y = make_data()
    idx = np.arange(rank, X.shape[0], world)
    params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "tree_learner": "data",
              "num_machines": world, "pre_partition": True, "min_data_in_leaf": 20, "seed": 3,
              "deterministic": True, "num_threads": 2}
    bst = lgb.train(params, lgb.Dataset(X[idx], y[idx], params=params), 8)
    with open(os.path.join(out_dir, "model_mpi_%d.txt" % rank), "w") as f:
        f.write(bst.model_to_string())
    nat.call("LGBM_NetworkFree")


def main():
    mode, rank, machines, out_dir = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4]
    ports = [int(m.split(":")[1]) for m in machines.split(",")]
    world = len(ports)
    if mode == "train_mpi":
        train_mpi(rank, world, out_dir)
        return
    if mode == "train":
        train(rank, world, machines, ports[rank], out_dir)
        return
    nat.call("LGBM_NetworkInit", nat.cstr(machines), nat.c_int(ports[rank]), nat.c_int(1), nat.c_int(world))
    if mode == "collectives":
        collectives(rank, world, out_dir)
    elif mode == "die":
        os._exit(0)
    elif mode == "survive":
        try:
            for _ in range(50):
                host.allreduce_sum(np.ones(1000))
            result = "no error"
        except lgb.LightGBMError as e:
            result = "error: %s" % e
        with open(os.path.join(out_dir, "survivor_%d.txt" % rank), "w") as f:
            f.write(result)
    nat.call("LGBM_NetworkFree")


if __name__ == "__main__":
    main()
