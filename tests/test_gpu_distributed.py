"""Distributed device learners on one MI355X: ranks are threads of this process, each with
its own stream, joined by the capture-safe peer communicator (one kernel per collective that
reads the peer ranks' windows; src/network/peer_comm.cpp, src/device/peer_kernels.hip) -- the
same kernels and the same captured round graphs as one process per GPU over xGMI, only the
windows are mapped by pointer instead of hipIpc handles.  The collective sequence:
  * data-parallel: per split the histogrammed child's int64 histogram is reduce-scattered
    to the feature owners, owners scan their features, the per-feature split records are
    all-gathered and every rank picks the same split (reference
    src/treelearner/data_parallel_tree_learner.cpp:61-123, 154-247);
  * feature-parallel: every rank holds all rows, builds and scans only its features, then
    the records are gathered (feature_parallel_tree_learner.cpp:37-77);
  * voting-parallel: every rank scans its local histograms, proposes its top_k features per
    leaf, the proposals are all-gathered and every rank runs the same election; only the
    elected features' histograms are all-reduced and scanned globally
    (voting_parallel_tree_learner.cpp:151-343).
Checks: identical models on every rank; the same splits as the serial device learner (bin
mappers shared through Dataset.subset); feature-parallel equal to serial to rounding."""
import ctypes
import os
import sys

import numpy as np
import pytest

import lightgbmv1_amd as lgb
from lightgbmv1_amd.basic import _load_lib, _safe_call
from lightgbmv1_amd.parallel.inproc import ThreadRanks

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "helpers"))
from dist_worker import make_data  # noqa: E402

pytestmark = pytest.mark.gpu

N = 20000
# boost_from_average off: distributed training starts from the mean of the ranks' initial
# scores (reference gbdt.cpp BoostFromAverage, Network::GlobalSyncUpByMean), which differs from
# the serial learner's in the 5th digit -- the trees are compared with the serial ones exactly
BASE = {"objective": "binary", "num_leaves": 31, "verbose": -1, "device_type": "gpu", "min_data_in_leaf": 20,
        "seed": 3, "deterministic": True, "max_bin": 63, "learning_rate": 0.1, "boost_from_average": False}


def _trees(m):
    return m[m.index("Tree=0"):m.index("end of trees")]


def _tree_fields(model_str):
    """per tree: {key: value string} of the tree sections"""
    out, cur = [], None
    for line in model_str.splitlines():
        if line.startswith("Tree="):
            cur = {}
            out.append(cur)
        elif line.startswith("end of trees"):
            break
        elif cur is not None and "=" in line:
            k, v = line.split("=", 1)
            cur[k] = v
    return out


def _same_trees_but_counts(a, b):
    """Every tree of two models grows the same splits and leaf values; only the counts may
    differ.  The reference's data-parallel learner keeps the split's *estimated* global counts
    for the new leaves (data_parallel_tree_learner.cpp:249-256, SplitInner(update_cnt=false),
    estimates RoundInt(hess * num_data / sum_hess), feature_histogram.hpp:866,885-886) where the
    serial learner counts the partition (serial_tree_learner.cpp:567-571): leaf_count and
    internal_count are estimates there."""
    ta, tb = _tree_fields(a), _tree_fields(b)
    assert len(ta) == len(tb)
    for i, (x, y) in enumerate(zip(ta, tb)):
        for k in ("num_leaves", "split_feature", "threshold", "decision_type", "left_child", "right_child",
                  "leaf_value", "split_gain", "internal_value"):
            assert x.get(k) == y.get(k), "tree %d: %s" % (i, k)


def _splits(model_str, tree=0):
    """(split_feature, threshold) lines of one tree of a text model."""
    block = model_str.split("Tree=%d\n" % tree)[1].split("\n\n")[0]
    rows = dict(line.split("=", 1) for line in block.splitlines() if "=" in line)
    return rows.get("split_feature"), rows.get("threshold")


def _run(learner, world, rounds=8, comm=True, **extra):
    X, y = make_data(N, 10)
    full = lgb.Dataset(X, y, params=BASE, free_raw_data=False).construct()
    serial = lgb.train(BASE, full.subset(np.arange(N)), rounds)

    def rank_fn(r):
        params = dict(BASE, tree_learner=learner, num_machines=world, **extra)
        if learner in ("data", "voting"):
            params["pre_partition"] = True
            ds = full.subset(np.arange(r, N, world))  # this rank's rows, the shared bin mappers
        else:
            ds = full.subset(np.arange(N))
        bst = lgb.train(params, ds, rounds)
        return bst.model_to_string(), bst.predict(X)

    with ThreadRanks(world, timeout_s=120, device_comm=comm) as tr:
        res = tr.run(rank_fn)
    assert all(r.ok for r in res), [str(r.error) for r in res]
    return X, y, serial, [r.value for r in res]


@pytest.mark.parametrize("comm,world", [("peer", 3), ("peer", 8), ("host", 3)])
def test_device_comm_self_test_threads(comm, world, gpu_available):
    """Every device collective of the in-process communicators (all-reduce sum / max,
    int64 reduce-scatter, allgather) on thread ranks; the peer comm also replays its
    collectives from a captured graph."""
    lib = _load_lib()

    def rank_fn(r):
        ok = ctypes.c_int(0)
        _safe_call(lib.LGBM_AMD_RcclSelfTest(ctypes.byref(ok)))
        if comm == "peer":
            ok2 = ctypes.c_int(0)
            _safe_call(lib.LGBM_AMD_RcclGraphSelfTest(ctypes.byref(ok2)))
            return ok.value * ok2.value
        return ok.value

    with ThreadRanks(world, timeout_s=60, device_comm=comm) as tr:
        res = tr.run(rank_fn)
    assert all(r.ok for r in res), [str(r.error) for r in res]
    assert [r.value for r in res] == [1] * world


@pytest.mark.parametrize("world", [2, 4])
def test_device_data_parallel_reduce_scatter(world, gpu_available):
    X, y, serial, out = _run("data", world)
    for m, _ in out[1:]:
        assert _trees(m) == _trees(out[0][0])
    # histograms are exact integer sums at the same fixed-point scale (all-reduced max |g|) on
    # every rank, so the global histograms equal the serial learner's: every tree grows the
    # same splits and leaf values (counts are the reference data-parallel learner's estimates)
    _same_trees_but_counts(out[0][0], serial.model_to_string())
    np.testing.assert_array_equal(out[0][1], serial.predict(X))


@pytest.mark.parametrize("world", [2, 3])
def test_device_feature_parallel(world, gpu_available):
    X, y, serial, out = _run("feature", world)
    for m, _ in out[1:]:
        assert _trees(m) == _trees(out[0][0])
    # every rank has every row and the histograms are exact integer sums: the whole model of the
    # serial device learner (splits, counts, leaf values), and its predictions bit for bit
    assert _trees(out[0][0]) == _trees(serial.model_to_string())
    np.testing.assert_array_equal(out[0][1], serial.predict(X))


@pytest.mark.parametrize("world", [2, 4])
def test_device_voting_parallel(world, gpu_available, capfd, monkeypatch):
    capfd.readouterr()
    X, y, serial, out = _run("voting", world, top_k=4, verbose=2)
    log = capfd.readouterr().out
    assert "voting-parallel device learner" in log and "device-resident growth" in log
    assert "host-assisted growth" not in log
    for m, _ in out[1:]:
        assert _trees(m) == _trees(out[0][0])
    from sklearn.metrics import roc_auc_score
    assert abs(roc_auc_score(y, out[0][1]) - roc_auc_score(y, serial.predict(X))) < 0.01
    # the host voting loop (host-assisted growth, same election rules) grows the same model
    monkeypatch.setenv("LGBM_AMD_HOST_ASSIST", "1")
    _, _, _, host = _run("voting", world, top_k=4)
    assert _trees(out[0][0]) == _trees(host[0][0])


@pytest.mark.parametrize("world", [2, 3])
def test_data_parallel_per_tree_ownership(world, gpu_available, monkeypatch, capfd):
    """feature_fraction < 1: the tree's used feature groups are re-assigned to the least-loaded
    rank by bins every tree (reference DataParallelTreeLearner::BeforeTrain); ownership only
    decides which rank scans which feature, so the models equal the static-owner layout's
    (LGBM_AMD_STATIC_OWNERS=1) on every rank."""
    capfd.readouterr()
    _, _, _, dyn = _run("data", world, rounds=6, feature_fraction=0.6, verbose=2)
    log = capfd.readouterr().out
    assert "re-assigned per tree over the used features" in log
    monkeypatch.setenv("LGBM_AMD_STATIC_OWNERS", "1")
    _, _, _, stat = _run("data", world, rounds=6, feature_fraction=0.6)
    for (md, _), (ms, _) in zip(dyn, stat):
        assert _trees(md) == _trees(ms)
    for m, _ in dyn[1:]:
        assert _trees(m) == _trees(dyn[0][0])


@pytest.mark.parametrize("learner", ["data", "voting"])
def test_device_distributed_with_efb_bundles(learner, gpu_available):
    """Sparse mutually exclusive columns bundled by EFB (rank 0's bundles shared by every rank)
    under the device data- / voting-parallel learners: identical models on every rank."""
    rng = np.random.RandomState(17)
    n, world = 24000, 2
    X = np.zeros((n, 14))
    owner = rng.randint(0, 10, n)
    for j in range(10):
        X[owner == j, j] = rng.rand((owner == j).sum()) + 0.5
    X[:, 10:] = rng.randn(n, 4)
    y = (X[:, 0] + X[:, 4] - X[:, 7] + X[:, 10] + 0.3 * rng.randn(n) > 0.6).astype(np.float64)

    def rank_fn(r):
        params = dict(BASE, tree_learner=learner, num_machines=world, pre_partition=True, top_k=6)
        idx = np.arange(r, n, world)
        bst = lgb.train(params, lgb.Dataset(X[idx], y[idx], params=params), 6)
        return bst.model_to_string()

    with ThreadRanks(world, timeout_s=120, device_comm=True) as tr:
        res = tr.run(rank_fn)
    assert all(r.ok for r in res), [str(r.error) for r in res]
    assert _trees(res[0].value) == _trees(res[1].value)


@pytest.mark.parametrize("learner,world,k,mode", [("data", 2, 8, ""), ("data", 4, 8, ""), ("feature", 3, 8, ""),
                                                  ("voting", 2, 6, ""), ("voting", 4, 6, ""),
                                                  ("data", 2, 8, "bynode"), ("data", 3, 8, "bynode"),
                                                  ("feature", 2, 8, "bynode"), ("data", 2, 8, "cegb"),
                                                  ("data", 3, 8, "cegb"), ("feature", 3, 8, "cegb")])
def test_distributed_round_growth_equals_one_split_per_step(learner, world, k, mode, gpu_available, monkeypatch,
                                                            tmp_path):
    """Distributed round growth (round_kernels.hip: up to k leaves expanded per round, the
    histograms reduce-scattered and the per-feature records gathered once per round instead of
    once per split; voting: one proposal allgather and one elected-histogram all-reduce per
    round for all of the round's children) grows the same trees as one split per step
    (LGBM_AMD_ROUND_K=1), on every rank; the iteration log shows the rounds (fewer than the
    splits).  Per-node sampling and CEGB coupled penalties too: their folds are deferred to the
    plan's replay, which every rank runs on the gathered per-feature results and flags."""
    extra = {"top_k": 4} if learner == "voting" else {}
    if mode == "bynode":
        extra["feature_fraction_bynode"] = 0.6
    elif mode == "cegb":
        extra.update(cegb_penalty_split=0.5, cegb_penalty_feature_coupled=[5, 1, 3, 0, 2, 1, 4, 0, 1, 2],
                     cegb_tradeoff=0.8)
    monkeypatch.setenv("LGBM_AMD_ROUND_K", "1")
    _, _, _, base = _run(learner, world, rounds=6, **extra)
    monkeypatch.setenv("LGBM_AMD_ROUND_K", str(k))
    log = tmp_path / "iters.jsonl"
    monkeypatch.setenv("LGBM_AMD_ITER_LOG", str(log))
    _, _, _, spec = _run(learner, world, rounds=6, **extra)
    monkeypatch.delenv("LGBM_AMD_ITER_LOG")
    for (mb, _), (ms, _) in zip(base, spec):
        assert _trees(mb) == _trees(ms)
    import glob
    import json
    rows = [json.loads(line) for f in glob.glob(str(log) + "*") for line in open(f)]
    assert rows and all(row["rounds"][0] > 0 for row in rows)
    # the peer comm is capture-safe: the rounds and their collectives ran from hipGraphs
    assert all(row["graph"][0] for row in rows)
    assert sum(row["rounds"][0] for row in rows) < sum(row["leaves"][0] - 1 for row in rows)


@pytest.mark.parametrize("learner", ["voting", "data"])
def test_one_split_per_step_past_direct_partials(learner, gpu_available, monkeypatch):
    """Trees of more than 100 splits grown one split per step: from split direct_from_split
    (100) the serial learner's split scans sum the row blocks' partial histograms themselves and
    no reduce kernel is launched; the learners with global counts (data- and voting-parallel)
    never do, so their steps keep the reduce kernel.  Round 6 found voting's steps without it
    past split 100 (stale histograms: held-out AUC 0.68 instead of 0.81 on Criteo-shaped data,
    tools/diag_voting.py).  The one-split-per-step model equals round growth's, on every rank."""
    extra = {"num_leaves": 160, "min_data_in_leaf": 5}
    if learner == "voting":
        extra["top_k"] = 4
    monkeypatch.setenv("LGBM_AMD_ROUND_K", "1")
    _, _, _, steps = _run(learner, 2, rounds=3, **extra)
    monkeypatch.delenv("LGBM_AMD_ROUND_K")
    _, _, _, rounds = _run(learner, 2, rounds=3, **extra)
    for (ms, _), (mr, _) in zip(steps, rounds):
        assert _trees(ms) == _trees(mr)
    assert max(int(x["num_leaves"]) for x in _tree_fields(steps[0][0])) > 101


@pytest.mark.parametrize("comm", ["peer", "host"])
def test_device_collective_fault_mid_tree_raises_on_every_rank(comm, gpu_available):
    """A rank fails inside a device collective in the middle of a data-parallel tree (fault
    injected into its 30th device collective, within the second tree's rounds): the failing
    rank raises; its peer raises instead of waiting forever -- at its next host rendezvous
    (host comm), or when its device-side wait hits the timeout inside the captured round graph
    (peer comm) -- and the GPU stays usable (a serial model trains afterwards)."""
    import time
    X, y = make_data(N, 10)
    full = lgb.Dataset(X, y, params=BASE, free_raw_data=False).construct()
    world = 2

    def rank_fn(r):
        params = dict(BASE, tree_learner="data", num_machines=world, pre_partition=True)
        return lgb.train(params, full.subset(np.arange(r, N, world)), 8).model_to_string()

    t0 = time.time()
    with ThreadRanks(world, timeout_s=8 if comm == "peer" else 60, fail_rank=1, device_comm=comm,
                     device_fail_at_call=30) as tr:
        res = tr.run(rank_fn)
    assert time.time() - t0 < 45
    if comm == "peer":
        assert not res[1].ok and "injected fault (rank 1, collective 30)" in str(res[1].error), str(res[1].error)
        assert not res[0].ok and "timed out waiting for a peer rank (rank 0, collective 30)" in str(res[0].error), \
            str(res[0].error)
    else:
        assert not res[1].ok and "injected fault in rank 1 at device collective call 30" in str(res[1].error)
        assert not res[0].ok and "injected fault" in str(res[0].error), str(res[0].error)
    # the device is left usable
    bst = lgb.train(BASE, full.subset(np.arange(N)), 2)
    assert bst.num_trees() == 2


@pytest.mark.parametrize("learner", ["data", "voting", "feature"])
def test_multiprocess_peer_comm(learner, gpu_available, tmp_path):
    """One process per rank (2 processes sharing the box's one GPU): the production path of a
    multi-GPU node -- torch.distributed (gloo) for the host collectives, the peer comm's windows
    exported with hipIpcGetMemHandle and mapped by the other process, the round collectives
    captured in the round graphs (ITER_LOG "graph": true) -- for the data-, voting- and
    feature-parallel learners.  Identical models and predictions on both ranks, a useful model,
    and each rank's topology record: the peer identified by PCI bus id (here the same device)."""
    import json
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    world = 2
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2", LGBM_TEST_DEVICE="gpu", LGBM_TEST_RCCL="1",
                   LGBM_AMD_DEVICE_COMM="peer", LGBM_TEST_REQUIRE_COMM="peer",
                   LGBM_AMD_ITER_LOG=str(tmp_path / ("iters_%d.jsonl" % r)),
                   LGBM_TEST_PARAMS=json.dumps({"max_bin": 63}))
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "helpers", "dist_worker.py"), learner,
                                       str(tmp_path)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=150)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out.decode())
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out
    models = [(tmp_path / ("model_%d.txt" % r)).read_text() for r in range(world)]
    assert _trees(models[0]) == _trees(models[1])
    import glob
    rows = [json.loads(line) for f in glob.glob(str(tmp_path / "iters_*")) for line in open(f)]
    assert rows and all(row["graph"][0] for row in rows), rows[:2]
    preds = [np.load(str(tmp_path / ("pred_%d.npy" % r))) for r in range(world)]
    np.testing.assert_array_equal(preds[0], preds[1])
    from sklearn.metrics import roc_auc_score
    X, y = make_data()
    assert roc_auc_score(y, preds[0]) > 0.8
    for r in range(world):
        topo = json.loads((tmp_path / ("topo_%d.json" % r)).read_text())
        assert topo["device_comm"] == "peer" and topo["self_test"] == {"eager": True, "graph": True}
        assert topo["rank"] == r and topo["bus_id"]
        (peer,) = topo["peers"]
        assert peer["rank"] == 1 - r and peer["bus_id"] == topo["bus_id"] and peer["same_device"]


@pytest.mark.parametrize("learner,world,mode", [("data", 2, "bynode"), ("data", 3, "bynode"), ("data", 2, "cegb"),
                                                ("feature", 2, "bynode"), ("feature", 3, "cegb"),
                                                ("data", 2, "bynode_ic"), ("feature", 3, "bynode_ic")])
def test_distributed_modes_device_resident(learner, world, mode, gpu_available, capfd, tmp_path):
    """Per-node column sampling and CEGB split / coupled penalties under the distributed device
    learners grow device-resident (every rank draws the same node samples and holds the same CEGB
    state; the owners' scans apply them): identical trees on every rank, and the serial device
    learner's first tree (exact integer histograms: the global histograms of the shards are the
    serial ones)."""
    if mode == "bynode":
        extra = {"feature_fraction_bynode": 0.6}
    elif mode == "bynode_ic":  # (per-node masks drawn on the device from the branch-allowed pool)
        extra = {"feature_fraction_bynode": 0.6, "interaction_constraints": [[0, 1, 2], [3, 4, 5, 6], [1, 7, 8, 9]]}
    else:
        extra = {"cegb_penalty_split": 0.5, "cegb_penalty_feature_coupled": [5, 1, 3, 0, 2, 1, 4, 0, 1, 2],
                 "cegb_tradeoff": 0.8}
    capfd.readouterr()
    X, y, _, dev = _run(learner, world, rounds=5, verbose=2, **extra)
    log = capfd.readouterr().out
    assert "device-resident growth" in log and "host-assisted growth" not in log
    for md, _ in dev:
        assert _trees(md) == _trees(dev[0][0])
    full = lgb.Dataset(X, y, params=BASE, free_raw_data=False).construct()
    serial = lgb.train(dict(BASE, **extra), full.subset(np.arange(N)), 5)
    # the same trees as the serial device learner (the shards' global histograms are its exact
    # integer histograms); data-parallel leaf counts are the reference's estimates
    _same_trees_but_counts(dev[0][0], serial.model_to_string())


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("forced", [
    {"feature": 0, "threshold": 0.1, "left": {"feature": 7, "threshold": -0.2, "left": {"feature": 3, "threshold": 0.5}},
     "right": {"feature": 5, "threshold": 0.3}},
    # an invalid node (an unknown feature) ends the forced splits early
    {"feature": 6, "threshold": 0.0, "left": {"feature": 99, "threshold": 1.0}, "right": {"feature": 2, "threshold": 0.0}},
], ids=["valid", "invalid_node"])
def test_feature_parallel_forced_splits_device_resident(world, forced, gpu_available, capfd, tmp_path):
    """Forced splits under the feature-parallel learner grow device-resident: the owner of a
    forced node's feature computes its record in its split scan, the records are gathered with
    the per-feature results and every rank's pick applies the owner's.  Every rank has every
    row, so the trees equal the serial device learner's (itself equal to host-assisted growth,
    tests/test_gpu_learner.py::test_forced_splits_on_device) and the forced root is applied."""
    import json as _json
    path = tmp_path / "forced.json"
    path.write_text(_json.dumps(forced))
    extra = {"forcedsplits_filename": str(path)}
    capfd.readouterr()
    X, y, _, dev = _run("feature", world, rounds=5, verbose=2, **extra)
    log = capfd.readouterr().out
    assert "device-resident growth" in log and "host-assisted growth" not in log
    for md, _ in dev:
        assert _trees(md) == _trees(dev[0][0])
    full = lgb.Dataset(X, y, params=BASE, free_raw_data=False).construct()
    serial = lgb.train(dict(BASE, **extra), full.subset(np.arange(N)), 5)
    assert _trees(dev[0][0]) == _trees(serial.model_to_string())
    if forced["feature"] == 0:  # (the valid schedule: its root is applied)
        root = serial.dump_model()["tree_info"][0]["tree_structure"]
        assert root["split_feature"] == forced["feature"]


@pytest.mark.parametrize("world", [2, 3])
def test_voting_bynode_device_resident(world, gpu_available, capfd, monkeypatch):
    """Voting-parallel with per-node column sampling on the device: the local scans evaluate
    every feature, the global scans of the elected features apply the node's sample (drawn in
    the host voting loop's order); the trees equal the host voting loop's (host-assisted growth)
    on every rank."""
    extra = {"feature_fraction_bynode": 0.6, "top_k": 4}
    capfd.readouterr()
    _, _, _, dev = _run("voting", world, rounds=5, verbose=2, **extra)
    log = capfd.readouterr().out
    assert "device-resident growth" in log and "host-assisted growth" not in log
    for md, _ in dev:
        assert _trees(md) == _trees(dev[0][0])
    monkeypatch.setenv("LGBM_AMD_HOST_ASSIST", "1")
    _, _, _, host = _run("voting", world, rounds=5, **extra)
    assert _trees(host[0][0]) == _trees(dev[0][0])


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("extra", [{}, {"feature_fraction_bynode": 0.6}, {"top_k": 10}],
                         ids=["top4", "top4_bynode", "top10"])
def test_voting_extra_trees_device_resident(world, extra, gpu_available, capfd, monkeypatch):
    """Voting-parallel extra_trees grows device-resident: the local scans draw from the feature
    generators (only the features the parent's local scan could split), the global scans from a
    second generator set on the rank that owns each elected histogram (reference
    voting_parallel_tree_learner.cpp:61-90 and CopyLocalHistogram); every rank replays every
    owner's draws.  Every rank grows the same model, and the first tree splits exactly as the
    host voting loop's.  Later trees are compared by quality only: the device scan's random-
    threshold sums differ from the host's in the last digit (test_gpu_learner.py::
    test_extra_trees_device_resident), and through the next gradients voting's small local
    leaves can flip a later split (the draws themselves were checked equal, owner by owner,
    until such a flip: profiles/r06_voting_extra_trees.md)."""
    params = dict({"extra_trees": True, "extra_seed": 7, "top_k": 4}, **extra)
    capfd.readouterr()
    X, y, _, dev = _run("voting", world, rounds=6, verbose=2, **params)
    log = capfd.readouterr().out
    assert "device-resident growth" in log and "host-assisted growth" not in log
    for md, _ in dev:
        assert _trees(md) == _trees(dev[0][0])
    monkeypatch.setenv("LGBM_AMD_HOST_ASSIST", "1")
    _, _, _, host = _run("voting", world, rounds=6, **params)
    td, th = _tree_fields(dev[0][0]), _tree_fields(host[0][0])
    for k in ("num_leaves", "split_feature", "threshold", "left_child", "right_child", "leaf_count"):
        assert td[0].get(k) == th[0].get(k), k
    from sklearn.metrics import roc_auc_score
    # (six random-threshold trees of two forests that part after tree 0: measured gaps up to 0.026)
    assert abs(roc_auc_score(y, dev[0][1]) - roc_auc_score(y, host[0][1])) < 0.04


@pytest.mark.parametrize("growth", ["rounds", "steps"])
@pytest.mark.parametrize("world", [2, 3])
def test_voting_local_scan_interaction_constraints(world, growth, gpu_available, capfd, monkeypatch):
    """Voting's local scans evaluate the tree's sample: interaction constraints do not apply
    there, only to the global scans of the elected features through the node's feature set
    (VotingParallelTreeLearner::FindBestSplits / FindBestSplitsFromHistograms), so a feature a
    branch may not use can still be proposed and elected.  The models equal the host voting
    loop's on every rank, with round growth and with one split per step."""
    extra = {"top_k": 3, "min_data_in_leaf": 40,
             "interaction_constraints": [[0, 1, 2], [2, 3, 4, 5], [6, 7, 8, 9]]}
    if growth == "steps":
        monkeypatch.setenv("LGBM_AMD_ROUND_K", "1")
    capfd.readouterr()
    _, _, _, dev = _run("voting", world, rounds=6, verbose=2, **extra)
    log = capfd.readouterr().out
    assert "device-resident growth" in log and "host-assisted growth" not in log
    for md, _ in dev:
        assert _trees(md) == _trees(dev[0][0])
    monkeypatch.setenv("LGBM_AMD_HOST_ASSIST", "1")
    _, _, _, host = _run("voting", world, rounds=6, **extra)
    # the same splits; a leaf's value and weight may differ in the last bit (the host scan sums
    # the scaled bins as doubles, the device scan the integer bins first)
    td, th = _tree_fields(dev[0][0]), _tree_fields(host[0][0])
    assert len(td) == len(th)
    for i, (a, b) in enumerate(zip(td, th)):
        for k in a:
            if k in ("leaf_value", "leaf_weight"):
                np.testing.assert_allclose(np.array(a[k].split(), float), np.array(b[k].split(), float), rtol=1e-12,
                                           err_msg="tree %d: %s" % (i, k))
            else:
                assert a[k] == b.get(k), "tree %d: %s" % (i, k)


def test_bench_py_under_torchrun_two_processes(gpu_available, tmp_path):
    """The multi-GPU benchmark entry point as the driver launches it (torch.distributed.run,
    one process per rank, peer comm), here with 2 processes sharing the box's GPU and 1M rows:
    rank 0 prints one JSON line with n_gpus 2 and dp2 parallelism."""
    import json
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    root = os.path.dirname(HERE)
    env = dict(os.environ, OMP_NUM_THREADS="4")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                          "--gpus", "2", "--steps", "5", "--warmup", "2", "--rows", "1000000", "--test-rows", "50000"],
                         cwd=str(tmp_path), env=env, capture_output=True, text=True, timeout=180)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["config"]["parallelism"] == "dp2" and rec["ms_per_step"] > 0
    assert rec["auc_heldout"] > 0.7
    assert "peer device comm unavailable" not in out.stdout
