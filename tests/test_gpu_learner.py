"""MI355X learner vs the CPU serial learner (same binned data, same parameters).

Device histograms are exact int64 sums of fixed-point (g, h) (per-tree power-of-two
scales), the host's are fp64 sums, and the device scans evaluate thresholds with parallel
prefix sums, so trees are compared structurally (split features / thresholds of the
first tree) and by metric, not bit for bit.
"""
import numpy as np
import pytest

import lightgbmv1_amd as lgb

pytestmark = pytest.mark.gpu


def _data(n=60000, f=16, seed=1):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, f).astype(np.float32)
    X[:, 3] = np.abs(X[:, 3])  # skewed feature
    X[rng.rand(n) < 0.05, 5] = np.nan  # missing values
    X[:, 6] = np.where(rng.rand(n) < 0.6, 0.0, X[:, 6])  # zero-heavy feature (most frequent bin 0)
    X[:, 7] = np.where(rng.rand(n) < 0.7, 2.5, X[:, 7])  # most frequent bin not 0
    logit = X[:, 0] + 0.7 * X[:, 1] * X[:, 2] - 0.5 * X[:, 3] + 0.3 * np.nan_to_num(X[:, 5]) + 0.4 * X[:, 7]
    y = (logit + 0.3 * rng.randn(n) > 0).astype(np.float32)
    return X, y


def _auc(y, p):
    from scipy.stats import rankdata
    r = rankdata(p)
    pos = y > 0.5
    return (r[pos].sum() - pos.sum() * (pos.sum() + 1) / 2) / (pos.sum() * (~pos).sum())


def _train(X, y, device, rounds=20, **extra):
    params = {"objective": "binary", "num_leaves": 31, "max_bin": 63, "learning_rate": 0.1,
              "min_data_in_leaf": 20, "verbose": -1, "device_type": device, "seed": 7}
    params.update(extra)
    ds = lgb.Dataset(X, y, params=params)
    return lgb.train(params, ds, rounds, verbose_eval=False)


def test_first_tree_matches_cpu(gpu_available):
    X, y = _data()
    cpu = _train(X, y, "cpu", rounds=1).dump_model()["tree_info"][0]["tree_structure"]
    gpu = _train(X, y, "gpu", rounds=1).dump_model()["tree_info"][0]["tree_structure"]
    # root and its children split on the same features at the same thresholds
    for path in ([], ["left_child"], ["right_child"]):
        a, b = cpu, gpu
        for k in path:
            a, b = a[k], b[k]
        assert a["split_feature"] == b["split_feature"]
        assert a["threshold"] == pytest.approx(b["threshold"])
        assert a["split_gain"] == pytest.approx(b["split_gain"], rel=1e-3)
        assert a["internal_count"] == b["internal_count"]


def test_auc_parity_with_cpu(gpu_available):
    X, y = _data()
    Xt, yt = _data(20000, seed=2)
    p_cpu = _train(X, y, "cpu", rounds=30).predict(Xt)
    p_gpu = _train(X, y, "gpu", rounds=30).predict(Xt)
    assert abs(_auc(yt, p_cpu) - _auc(yt, p_gpu)) < 2e-3
    assert np.corrcoef(p_cpu, p_gpu)[0, 1] > 0.995


def test_regression_and_bagging_on_device(gpu_available):
    rng = np.random.RandomState(3)
    X = rng.randn(40000, 10).astype(np.float32)
    y = (2 * X[:, 0] + np.sin(3 * X[:, 1]) + 0.1 * rng.randn(40000)).astype(np.float32)
    params = dict(objective="regression", bagging_fraction=0.7, bagging_freq=1, feature_fraction=0.8)
    b_gpu = _train(X, y, "gpu", rounds=40, **params)
    b_cpu = _train(X, y, "cpu", rounds=40, **params)
    mse_gpu = np.mean((b_gpu.predict(X) - y) ** 2)
    mse_cpu = np.mean((b_cpu.predict(X) - y) ** 2)
    assert mse_gpu < 0.2 and abs(mse_gpu - mse_cpu) < 0.05


def test_host_assisted_mode_categorical(gpu_available):
    rng = np.random.RandomState(4)
    X = rng.randn(30000, 6).astype(np.float32)
    X[:, 0] = rng.randint(0, 12, size=30000)
    y = ((X[:, 0] % 3 == 0) * 1.5 + X[:, 1] + 0.2 * rng.randn(30000) > 0.7).astype(np.float32)
    params = {"objective": "binary", "num_leaves": 15, "verbose": -1, "device_type": "gpu"}
    ds = lgb.Dataset(X, y, params=params, categorical_feature=[0])
    b = lgb.train(params, ds, 20, verbose_eval=False)
    assert _auc(y, b.predict(X)) > 0.9
    model = b.dump_model()
    assert any("num_cat" in t and t["num_cat"] > 0 for t in model["tree_info"])


def test_multiclass_on_device(gpu_available):
    rng = np.random.RandomState(5)
    X = rng.randn(30000, 8).astype(np.float32)
    y = np.argmax(X[:, :3] + 0.3 * rng.randn(30000, 3), axis=1).astype(np.float32)
    b = _train(X, y, "gpu", rounds=20, objective="multiclass", num_class=3)
    acc = np.mean(np.argmax(b.predict(X), axis=1) == y)
    assert acc > 0.85


def test_rccl_comm_single_rank(gpu_available):
    """The RCCL device communicator (the multi-GPU histogram all-reduce path) on one rank."""
    import ctypes
    import numpy as np
    from lightgbmv1_amd.basic import _load_lib
    lib = _load_lib()
    size = ctypes.c_int(0)
    assert lib.LGBM_AMD_RcclUniqueIdSize(ctypes.byref(size)) == 0
    uid = np.zeros(size.value, dtype=np.uint8)
    assert lib.LGBM_AMD_RcclGetUniqueId(uid.ctypes.data_as(ctypes.c_char_p)) == 0
    assert lib.LGBM_AMD_RcclInit(ctypes.c_int(1), ctypes.c_int(0), ctypes.c_int(0),
                                 uid.ctypes.data_as(ctypes.c_char_p)) == 0
    ok = ctypes.c_int(0)
    try:
        assert lib.LGBM_AMD_RcclSelfTest(ctypes.byref(ok)) == 0
        assert ok.value == 1
    finally:
        lib.LGBM_AMD_RcclFree()
