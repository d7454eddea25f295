"""Multi-process training on the CPU learner with world_size 2 (gloo host collectives over
127.0.0.1): data-parallel (reduce-scatter of histograms), voting-parallel (PV-Tree) and
feature-parallel learners (reference src/treelearner/{data,voting,feature}_parallel_tree_learner.cpp).
Every rank must end with the same model, of the expected quality."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
from sklearn.metrics import roc_auc_score

import lightgbmv1_amd as lgb

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "helpers"))
from dist_worker import make_data  # noqa: E402


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


_RENDEZVOUS_ERRORS = ("Address already in use", "EADDRINUSE", "Connection refused", "connect()", "Socket Timeout")


def _run(learner, tmp_path, world=2, device="cpu", extra=None):
    # the free port can be taken between the probe and the rendezvous: retry on that only
    for attempt in range(3):
        try:
            return _run_once(learner, tmp_path, world, device, extra)
        except AssertionError as e:
            if attempt == 2 or not any(m in str(e) for m in _RENDEZVOUS_ERRORS):
                raise


def _run_once(learner, tmp_path, world, device, extra=None):
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port), OMP_NUM_THREADS="2", LGBM_TEST_DEVICE=device,
                   LGBM_TEST_PARAMS=json.dumps(extra or {}))
        if device == "cpu":
            env["HIP_VISIBLE_DEVICES"] = ""
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "helpers", "dist_worker.py"), learner,
                                       str(tmp_path)], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    outs = []
    for p in procs:
        try:
            out, _ = p.communicate(timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            out, _ = p.communicate()
        outs.append(out.decode())
    for p, out in zip(procs, outs):
        assert p.returncode == 0, out
    models = [(tmp_path / ("model_%d.txt" % r)).read_text() for r in range(world)]
    preds = [np.load(str(tmp_path / ("pred_%d.npy" % r))) for r in range(world)]
    return models, preds


def _trees(m):
    return m[m.index("Tree=0"):m.index("end of trees")]


@pytest.mark.parametrize("learner", ["data", "voting", "feature"])
def test_parallel_learners_agree_across_ranks(learner, tmp_path):
    models, preds = _run(learner, tmp_path)
    assert _trees(models[0]) == _trees(models[1])
    np.testing.assert_array_equal(preds[0], preds[1])
    X, y = make_data()
    assert roc_auc_score(y, preds[0]) > 0.8


@pytest.mark.parametrize("learner", ["data", "voting"])
def test_row_wise_histograms_and_bounded_pool_across_ranks(learner, tmp_path):
    """The reference fork's headline setting (train.conf: data-parallel, force_row_wise=true)
    with a bounded histogram pool: ranks agree and the fit holds."""
    models, preds = _run(learner, tmp_path, extra={"force_row_wise": True, "histogram_pool_size": 0.01})
    assert _trees(models[0]) == _trees(models[1])
    X, y = make_data()
    assert roc_auc_score(y, preds[0]) > 0.8


def test_feature_parallel_matches_serial(tmp_path):
    models, preds = _run("feature", tmp_path)
    X, y = make_data()
    params = {"objective": "binary", "num_leaves": 15, "learning_rate": 0.1, "verbose": -1,
              "min_data_in_leaf": 20, "seed": 3, "deterministic": True}
    serial = lgb.train(params, lgb.Dataset(X, y), num_boost_round=20)
    np.testing.assert_allclose(preds[0], serial.predict(X), rtol=1e-9, atol=1e-12)


def test_data_parallel_close_to_serial(tmp_path):
    _, preds = _run("data", tmp_path)
    X, y = make_data()
    params = {"objective": "binary", "num_leaves": 15, "learning_rate": 0.1, "verbose": -1,
              "min_data_in_leaf": 20, "seed": 3}
    serial = lgb.train(params, lgb.Dataset(X, y), num_boost_round=20)
    # bins are found on shards, so splits can differ slightly; the fit must not
    assert abs(roc_auc_score(y, preds[0]) - roc_auc_score(y, serial.predict(X))) < 0.01


@pytest.mark.gpu
def test_device_data_parallel_two_ranks_one_gpu(tmp_path, gpu_available):
    """Data-parallel device learner, both ranks on one GPU (host collectives between them):
    ranks agree, and the fit matches the CPU data-parallel run's quality."""
    models, preds = _run("data", tmp_path, device="gpu")
    assert _trees(models[0]) == _trees(models[1])
    X, y = make_data()
    auc = roc_auc_score(y, preds[0])
    assert auc > 0.8
    cpu_dir = tmp_path / "cpu"
    cpu_dir.mkdir()
    _, cpu_preds = _run("data", cpu_dir, device="cpu")
    assert abs(auc - roc_auc_score(y, cpu_preds[0])) < 0.01


@pytest.mark.gpu
def test_device_voting_parallel_two_ranks_one_gpu(tmp_path, gpu_available):
    """Voting-parallel (PV-Tree) over the device learner: device histograms / partitions,
    host voting exchange; ranks agree and the fit matches the CPU voting learner's quality."""
    models, preds = _run("voting", tmp_path, device="gpu")
    assert _trees(models[0]) == _trees(models[1])
    X, y = make_data()
    auc = roc_auc_score(y, preds[0])
    assert auc > 0.8
    cpu_dir = tmp_path / "cpu"
    cpu_dir.mkdir()
    _, cpu_preds = _run("voting", cpu_dir, device="cpu")
    assert abs(auc - roc_auc_score(y, cpu_preds[0])) < 0.01


def _thread_rank_train(rank, world=2, learner="data", rounds=10):
    X, y = make_data()
    idx = np.arange(rank, X.shape[0], world)
    params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "tree_learner": learner,
              "num_machines": world, "pre_partition": True, "min_data_in_leaf": 20, "seed": 3,
              "deterministic": True, "num_threads": 2}
    if learner == "voting":
        params["top_k"] = 5
    ds = lgb.Dataset(X[idx], y[idx], params=params)
    return lgb.train(params, ds, rounds).model_to_string()


@pytest.mark.parametrize("learner", ["data", "voting"])
def test_thread_ranks_in_one_process(learner):
    """Ranks as threads of one process (in-process transport): ranks build identical models."""
    from lightgbmv1_amd.parallel.inproc import ThreadRanks
    with ThreadRanks(2, timeout_s=60) as tr:
        res = tr.run(lambda r: _thread_rank_train(r, learner=learner))
    assert all(r.ok for r in res), [str(r.error) for r in res]
    assert _trees(res[0].value) == _trees(res[1].value)


def test_injected_fault_fails_every_rank_promptly():
    """A fault injected into rank 1's 4th collective: rank 1 raises it, rank 0 raises
    'peer rank failed' instead of hanging."""
    import time
    from lightgbmv1_amd.parallel.inproc import ThreadRanks
    t0 = time.time()
    with ThreadRanks(2, timeout_s=60, fail_rank=1, fail_at_call=4) as tr:
        res = tr.run(lambda r: _thread_rank_train(r))
    assert time.time() - t0 < 30
    assert not res[1].ok and "injected fault" in str(res[1].error)
    assert not res[0].ok and "peer rank failed" in str(res[0].error)


def test_collective_timeout_when_a_rank_never_arrives():
    import time
    from lightgbmv1_amd.parallel.inproc import ThreadRanks
    t0 = time.time()
    with ThreadRanks(2, timeout_s=2.0) as tr:
        res = tr.run(lambda r: _thread_rank_train(r) if r == 0 else None)
    assert time.time() - t0 < 30
    assert not res[0].ok and "timed out" in str(res[0].error)
    assert res[1].ok


def _efb_rank_train(rank, world, learner):
    import ctypes
    from lightgbmv1_amd import _native as nat
    rng = np.random.RandomState(17)
    n = 6000
    X = np.zeros((n, 14))
    owner = rng.randint(0, 10, n)
    for j in range(10):  # ten mutually exclusive sparse columns: bundled by EFB
        X[owner == j, j] = rng.rand((owner == j).sum()) + 0.5
    X[:, 10:] = rng.randn(n, 4)
    y = (X[:, 0] + X[:, 4] - X[:, 7] + X[:, 10] + 0.3 * rng.randn(n) > 0.6).astype(np.float64)
    idx = np.arange(rank, n, world)
    params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "tree_learner": learner,
              "num_machines": world, "pre_partition": True, "min_data_in_leaf": 20, "seed": 3,
              "deterministic": True, "num_threads": 2, "top_k": 6}
    ds = lgb.Dataset(X[idx], y[idx], params=params).construct()
    ng = ctypes.c_int(0)
    nat.call("LGBM_AMD_DatasetGetGroupBins", ds.handle, None, None, ctypes.byref(ng))
    bst = lgb.train(params, ds, 8)
    return ng.value, bst.model_to_string()


@pytest.mark.parametrize("learner", ["data", "voting"])
def test_efb_bundles_under_distributed_training(learner):
    """EFB with several ranks: rank 0's bundles are used by every rank (their samples differ),
    so the feature layout is shared and every rank builds the same model."""
    from lightgbmv1_amd.parallel.inproc import ThreadRanks
    with ThreadRanks(3, timeout_s=60) as tr:
        res = tr.run(lambda r: _efb_rank_train(r, 3, learner))
    assert all(r.ok for r in res), [str(r.error) for r in res]
    groups = [r.value[0] for r in res]
    assert len(set(groups)) == 1 and groups[0] < 14, groups
    assert len({_trees(r.value[1]) for r in res}) == 1
