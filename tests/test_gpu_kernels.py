"""Kernel-level checks of the device learner's hot path, on the state the last device-grown
tree leaves in HBM (read back through LGBM_AMD_BoosterDevice* in the C API):

* histograms (k_hist root pass, fused k_split partition + histogram, k_hist_reduce, and the
  parent - sibling subtraction in k_find): every leaf's raw fixed-point slot must EQUAL a
  torch fp64 scatter-add of the leaf's rows' quantised (g, h) at the kernel's own scale --
  exact integers, so any off-by-one in a bin, a row or a block boundary fails;
* partition (k_split): the leaves' row lists are disjoint, cover the bag, and every row sits
  in the leaf the CPU predictor routes its raw feature values to;
* split scan (k_find + pick): every leaf's device best split equals the CPU split finder's
  (src/treelearner/split_finder.cpp) on the same dequantised histogram -- NaN / zero missing
  values, most-frequent-bin offset, categorical (one-hot and sorted), monotone, L1 /
  max_delta_step / path smoothing, wide int64 histograms (gpu_use_dp), bagging, EFB bundles,
  and multi-block leaves (> 16k rows).
"""
import ctypes
import json

import numpy as np
import pytest

import lightgbmv1_amd as lgb
from lightgbmv1_amd import _native as nat

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _last_tree_on_device(monkeypatch):
    """the device-state hooks read the last tree: no next tree launched early (LGBM_AMD_SPECULATE)"""
    monkeypatch.setenv("LGBM_AMD_SPECULATE", "0")


def _data(n, seed=5, f=10):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, f)
    X[rng.rand(n) < 0.08, 1] = np.nan                          # NaN missing
    X[:, 2] = np.where(rng.rand(n) < 0.7, 0.0, X[:, 2])        # most frequent bin 0 (offset 1)
    X[:, 3] = np.where(rng.rand(n) < 0.6, 1.5, X[:, 3])        # most frequent bin not 0
    X[:, 4] = rng.randint(0, 24, n)                            # categorical, many categories
    X[:, 5] = rng.randint(0, 4, n)                             # categorical, one-hot sized
    X[:, 6] = np.round(X[:, 6], 1)                             # ties between thresholds
    logit = (X[:, 0] + 0.8 * np.nan_to_num(X[:, 1]) - 0.6 * X[:, 2] + 0.5 * (X[:, 3] > 1)
             + 0.3 * (X[:, 4] % 5 == 1) - 0.4 * (X[:, 5] == 2) + 0.3 * X[:, 6] * X[:, 7])
    y = (logit + 0.5 * rng.randn(n) > 0).astype(np.float64)
    return X, y


def _efb_data(n, seed=9):
    """Mutually exclusive sparse columns (bundled by EFB into shared groups) + dense ones."""
    rng = np.random.RandomState(seed)
    X = np.zeros((n, 12))
    owner = rng.randint(0, 8, n)
    for j in range(8):
        rows = owner == j
        X[rows, j] = rng.rand(rows.sum()) * (j + 1)
    X[:, 8:] = rng.randn(n, 4)
    y = (X[:, 0] + X[:, 3] - X[:, 5] + X[:, 8] + 0.3 * rng.randn(n) > 0.5).astype(np.float64)
    return X, y


def _sparse_data(n, seed=13, f=320, density=0.03):
    """Mostly-zero continuous columns (63 bins each: > 16384 histogram bins in all, two
    row-sparse bin tiles) and a few dense ones."""
    rng = np.random.RandomState(seed)
    X = np.where(rng.rand(n, f) < density, rng.randn(n, f), 0.0)
    X[:, :3] = rng.randn(n, 3)
    logit = X[:, 0] - X[:, 1] + 2.0 * X[:, 5:40].sum(1) - 1.5 * X[:, 200:240].sum(1)
    y = (logit + 0.3 * rng.randn(n) > 0).astype(np.float64)
    return X, y


BASE = {"objective": "binary", "num_leaves": 31, "max_bin": 63, "learning_rate": 0.1, "min_data_in_leaf": 20,
        "verbose": -1, "device_type": "gpu", "seed": 7, "deterministic": True}

CASES = {
    "numeric": ({}, 20000),
    "categorical": ({"categorical_feature": [4, 5]}, 20000),
    "zero_missing": ({"zero_as_missing": True}, 20000),
    "monotone": ({"monotone_constraints": [1, 0, -1, 0, 0, 0, 0, 0, 0, 0]}, 20000),
    "regularised": ({"lambda_l1": 0.5, "lambda_l2": 1.0, "max_delta_step": 0.7, "path_smooth": 2.0,
                     "min_gain_to_split": 0.01}, 20000),
    "wide_dp": ({"gpu_use_dp": True}, 20000),
    "bagging": ({"bagging_fraction": 0.7, "bagging_freq": 1, "bagging_seed": 3}, 20000),
    "multi_block": ({"num_leaves": 63}, 150000),
    "efb": ({"max_bin": 31}, 30000),
    # one 511-bin group among 63-bin ones: 16-bit words next to 8-bit words in each row
    "mixed_width": ({"max_bin_by_feature": [63] * 7 + [511] + [63] * 2}, 20000),
    "mixed_width_dp": ({"max_bin_by_feature": [511] + [63] * 9, "gpu_use_dp": True}, 20000),
    # the same data with every group widened to 16 bits (LGBM_AMD_UNIFORM_BINS=1)
    "uniform_wide": ({"max_bin_by_feature": [63] * 7 + [511] + [63] * 2, "_env": {"LGBM_AMD_UNIFORM_BINS": "1"}},
                     20000),
    # row-sparse storage (lists of each row's stored bins) forced on dense data, with EFB
    # bundles, wide histograms, a 16-bit group and bagging; chosen by itself on sparse data
    # with two bin tiles
    "sparse_rows": ({"_env": {"LGBM_AMD_SPARSE_ROWS": "1"}, "categorical_feature": [4, 5]}, 20000),
    "sparse_rows_efb": ({"max_bin": 31, "_env": {"LGBM_AMD_SPARSE_ROWS": "1"}}, 30000),
    "sparse_rows_dp_wide": ({"gpu_use_dp": True, "max_bin_by_feature": [511] + [63] * 9, "bagging_fraction": 0.7,
                             "bagging_freq": 1, "_env": {"LGBM_AMD_SPARSE_ROWS": "1"}}, 20000),
    "sparse_auto_tiles": ({"min_data_in_leaf": 5}, 20000),
    # 4-bit storage: every group <= 16 bins, eight groups to a word (max_bin 15), packed and
    # wide histograms, multi-block leaves with bagging; the row-major fallback of the split
    # column (no column copy) reads the half-bytes
    "nibble": ({"max_bin": 15, "_env": {"LGBM_AMD_NIBBLE_BINS": "1"}}, 20000),
    "nibble_dp": ({"max_bin": 15, "gpu_use_dp": True, "_env": {"LGBM_AMD_NIBBLE_BINS": "1"}}, 20000),
    "nibble_multi_block": ({"max_bin": 15, "num_leaves": 63, "bagging_fraction": 0.8, "bagging_freq": 1,
                            "_env": {"LGBM_AMD_NIBBLE_BINS": "1"}}, 150000),
    "nibble_no_column_copy": ({"max_bin": 15, "_env": {"LGBM_AMD_COLUMN_COPY": "0", "LGBM_AMD_NIBBLE_BINS": "1"}},
                              20000),
}


def _group_bins(ds):
    ng = ctypes.c_int(0)
    nat.call("LGBM_AMD_DatasetGetGroupBins", ds.handle, None, None, ctypes.byref(ng))
    bins = np.zeros((ds.num_data(), ng.value), dtype=np.int32)
    bounds = np.zeros(ng.value + 1, dtype=np.int64)
    nat.call("LGBM_AMD_DatasetGetGroupBins", ds.handle, bins.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
             bounds.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(ng))
    return bins, bounds


def _gradients(bst, n):
    g = np.zeros(n, dtype=np.float32)
    h = np.zeros(n, dtype=np.float32)
    scales = np.zeros(2, dtype=np.float64)
    nat.call("LGBM_AMD_BoosterDeviceGradients", bst.handle, g.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
             h.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), scales.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return g, h, scales


def _leaf_state(bst, leaf):
    cnt = ctypes.c_int(0)
    hlen = ctypes.c_int64(0)
    nat.call("LGBM_AMD_BoosterDeviceLeafState", bst.handle, ctypes.c_int(leaf), None, ctypes.byref(cnt), None,
             None, ctypes.byref(hlen), None)
    rows = np.zeros(cnt.value, dtype=np.int32)
    hist = np.zeros(hlen.value, dtype=np.int64)
    valid = np.zeros(hlen.value // 2, dtype=np.int8)
    sums = np.zeros(3, dtype=np.float64)
    nat.call("LGBM_AMD_BoosterDeviceLeafState", bst.handle, ctypes.c_int(leaf),
             rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.byref(cnt),
             hist.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), valid.ctypes.data_as(ctypes.POINTER(ctypes.c_int8)),
             ctypes.byref(hlen), sums.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return rows, hist.reshape(-1, 2), valid.astype(bool), sums


def _check_splits(bst):
    text = nat.read_string(lambda size, need, buf: nat.call("LGBM_AMD_BoosterDeviceCheckSplits", bst.handle, size,
                                                            need, buf), 1 << 16)
    return json.loads(text)


def _quantise(v, scale):
    # the kernels' __float2ll_rn(v * (float)scale): an fp32 product by a power of two, rounded
    # half to even
    return np.rint(v.astype(np.float32) * np.float32(scale)).astype(np.float64)


@pytest.mark.parametrize("case", list(CASES))
def test_device_tree_state(gpu_available, case, monkeypatch):
    import torch
    extra, n = CASES[case]
    make = _efb_data if case in ("efb", "sparse_rows_efb") else _sparse_data if case == "sparse_auto_tiles" else _data
    X, y = make(n)
    params = dict(BASE, **extra)
    cat = params.pop("categorical_feature", "auto")
    for k, v in params.pop("_env", {}).items():
        monkeypatch.setenv(k, v)
    # the last tree's gradients stay readable (the score walk would compute the next ones)
    monkeypatch.setenv("LGBM_AMD_FUSE_GRAD", "0")
    ds = lgb.Dataset(X, y, params=params, categorical_feature=cat, free_raw_data=False)
    bst = lgb.train(params, ds, 4, verbose_eval=False, keep_training_booster=True)
    # the device training scores (tree walks over the binned rows) equal the CPU predictor's
    got = ctypes.c_int64(0)
    train_pred = np.zeros(n, dtype=np.float64)
    nat.call("LGBM_BoosterGetPredict", bst.handle, ctypes.c_int(0), ctypes.byref(got),
             train_pred.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    assert got.value == n
    np.testing.assert_allclose(train_pred, bst.predict(X), rtol=1e-9, atol=1e-12)
    num_leaves = bst.dump_model()["tree_info"][-1]["num_leaves"]
    assert num_leaves > 4

    bins, bounds = _group_bins(ds)
    g, h, scales = _gradients(bst, n)
    gq = torch.from_numpy(_quantise(g, scales[0]))
    hq = torch.from_numpy(_quantise(h, scales[1]))
    nbins = int(bounds[-1])
    # hist index of every (row, group): the group's first bin + the row's group bin; group
    # bin 0 (every member feature at its most frequent bin) is never accumulated
    gidx = torch.from_numpy(bins.astype(np.int64) + bounds[:-1][None, :])
    stored = torch.from_numpy(bins != 0)

    leaf_of_row = bst.predict(X, pred_leaf=True)[:, -1]
    seen = np.zeros(n, dtype=np.int32)
    checked_bins = 0
    for leaf in range(num_leaves):
        rows, hist, valid, sums = _leaf_state(bst, leaf)
        checked_bins += int(valid.sum())
        assert len(rows) == int(sums[2])
        # partition: every row of the leaf is routed to it by the CPU predictor
        assert np.all(leaf_of_row[rows] == leaf), (case, leaf)
        seen[rows] += 1
        # histogram: torch fp64 scatter-add of the rows' quantised (g, h)
        r = torch.from_numpy(rows.astype(np.int64))
        idx = gidx[r][stored[r]]
        exp_g = torch.zeros(nbins, dtype=torch.float64).scatter_add_(
            0, idx, gq[r].unsqueeze(1).expand(-1, bins.shape[1])[stored[r]])
        exp_h = torch.zeros(nbins, dtype=torch.float64).scatter_add_(
            0, idx, hq[r].unsqueeze(1).expand(-1, bins.shape[1])[stored[r]])
        dev_g = hist[:, 0].astype(np.float64)
        dev_h = hist[:, 1].astype(np.float64)
        # only the slices of features evaluated for the leaf are materialised (group bin 0
        # belongs to no feature; a feature the parent could not split on is skipped)
        bad_g = np.flatnonzero((dev_g != exp_g.numpy()) & valid)
        bad_h = np.flatnonzero((dev_h != exp_h.numpy()) & valid)
        assert bad_g.size == 0 and bad_h.size == 0, (case, leaf, bad_g[:5], bad_h[:5])
    assert checked_bins > num_leaves * 10
    # the leaves partition the bag: no row twice; without bagging, every row once
    assert seen.max() <= 1
    if "bagging_fraction" not in extra:
        assert seen.min() == 1

    rep = _check_splits(bst)
    assert rep["device_mode"] and rep["checked"] > 0, rep
    assert rep["mismatched"] == 0, json.dumps(rep)
    expect_layout = {"mixed_width": "mixed", "mixed_width_dp": "mixed", "uniform_wide": "16", "numeric": "8",
                     "nibble": "4", "nibble_dp": "4", "nibble_multi_block": "4", "nibble_no_column_copy": "4",
                     "sparse_rows": "sparse", "sparse_rows_efb": "sparse", "sparse_rows_dp_wide": "sparse",
                     "sparse_auto_tiles": "sparse"}
    if case in expect_layout:
        assert rep["layout"] == expect_layout[case], rep["layout"]
    if case == "sparse_auto_tiles":
        assert rep["hist_tiles"] == 2


@pytest.mark.parametrize("dtype,order", [(np.float32, "C"), (np.float64, "F")])
def test_device_binning_matches_host(tmp_path, monkeypatch, dtype, order):
    """k_value_to_bin (src/device/bin_kernels.hip) writes the same group columns as the host's
    per-value ValueToBin push: NaN / zero missing, most-frequent-bin offsets, ties on bin
    bounds, EFB bundles of sparse columns; categorical groups stay on the host."""
    rng = np.random.RandomState(3)
    n = 70000
    X, y = _data(n, f=10)
    sp = np.zeros((n, 6))
    for j in range(6):                                   # mutually exclusive sparse columns: EFB
        rows = rng.rand(n) < 0.04
        sp[rows & (sp.sum(axis=1) == 0), j] = rng.randn(int((rows & (sp.sum(axis=1) == 0)).sum())) + 3
    X = np.hstack([X, sp])
    X[:50, 0] = np.linspace(-1, 1, 50)                   # values on and around bin bounds
    X = np.asarray(X, dtype=dtype, order=order)
    params = {"objective": "binary", "max_bin": 63, "verbose": -1, "device_type": "gpu"}
    files = []
    for mode in ("0", "1"):
        monkeypatch.setenv("LGBM_AMD_DEVICE_BINNING", mode)
        ds = lgb.Dataset(X, y, params=params, categorical_feature=[4, 5]).construct()
        f = tmp_path / ("bins_%s.bin" % mode)
        ds.save_binary(str(f))
        files.append(f.read_bytes())
    assert len(files[0]) > 100 and files[0] == files[1]
    # and a small bound check of one value: the validation set binned on the device against
    # the training set's mappers gives the same model predictions
    monkeypatch.setenv("LGBM_AMD_DEVICE_BINNING", "1")
    tr = lgb.Dataset(X, y, params=params, categorical_feature=[4, 5])
    va = lgb.Dataset(X[:20000], y[:20000], reference=tr, categorical_feature=[4, 5])
    bst = lgb.train(dict(params, num_leaves=15), tr, num_boost_round=3, valid_sets=[va])
    assert bst.num_trees() == 3
