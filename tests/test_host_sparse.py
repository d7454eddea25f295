"""Sparse host storage of feature groups (reference SparseBin, src/io/sparse_bin.hpp): a group
whose rows are mostly at their features' most frequent bins keeps only the rows that are not,
with their bins (include/lgbm_amd/dataset.h FeatureGroup).  Models must not depend on the
storage: CPU col-wise / row-wise histograms, subsets, binary files and validation sets give
the same trees with sparse groups (auto, or every group via LGBM_AMD_HOST_SPARSE=1) as with
dense ones (LGBM_AMD_HOST_SPARSE=0); the binary file of sparse data shrinks accordingly."""
import os

import numpy as np
import pytest

import lightgbmv1_amd as lgb


def _sparse_data(n=20000, f=30, density=0.05, seed=3):
    rng = np.random.RandomState(seed)
    X = np.where(rng.rand(n, f) < density, rng.randn(n, f), 0.0)
    X[:, :2] = rng.randn(n, 2)
    y = (X[:, 0] + X[:, 1] + 3 * X[:, 2:12].sum(1) - 2 * X[:, 12:20].sum(1) + 0.3 * rng.randn(n) > 0).astype(float)
    return X, y


def _trees(bst):
    m = bst.model_to_string()
    return m[m.index("Tree=0"):m.index("end of trees")]


@pytest.mark.parametrize("extra", [{}, {"force_row_wise": True}, {"bagging_fraction": 0.7, "bagging_freq": 1},
                                   {"enable_bundle": False}], ids=["colwise", "rowwise", "bagging", "no_efb"])
def test_sparse_groups_give_identical_models(extra, monkeypatch):
    X, y = _sparse_data()
    params = dict({"objective": "binary", "num_leaves": 31, "verbose": -1, "num_threads": 2, "seed": 1}, **extra)

    def run(mode):
        monkeypatch.setenv("LGBM_AMD_HOST_SPARSE", mode) if mode else monkeypatch.delenv("LGBM_AMD_HOST_SPARSE",
                                                                                         raising=False)
        ds = lgb.Dataset(X[:15000], y[:15000], params=params, free_raw_data=False)
        va = lgb.Dataset(X[15000:], y[15000:], reference=ds)
        ev = {}
        bst = lgb.train(params, ds, 10, valid_sets=[va], evals_result=ev, verbose_eval=False)
        sub = lgb.train(params, ds.construct().subset(np.arange(0, 15000, 2)), 5)
        return _trees(bst), ev["valid_0"]["binary_logloss"], _trees(sub)

    dense = run("0")
    assert run("") == dense   # auto: the sparse columns' groups are sparse
    assert run("1") == dense  # every group sparse


def test_sparse_binary_file_roundtrip_and_size(tmp_path, monkeypatch):
    X, y = _sparse_data(n=30000, f=40, density=0.02)
    params = {"objective": "binary", "verbose": -1, "num_threads": 2, "enable_bundle": False}
    sizes, models = {}, {}
    for mode in ("0", "1"):
        monkeypatch.setenv("LGBM_AMD_HOST_SPARSE", mode)
        path = str(tmp_path / ("d%s.bin" % mode))
        lgb.Dataset(X, y, params=params).construct().save_binary(path)
        sizes[mode] = os.path.getsize(path)
        monkeypatch.delenv("LGBM_AMD_HOST_SPARSE")
        models[mode] = _trees(lgb.train(params, lgb.Dataset(path, params=params), 5))
    assert models["0"] == models["1"]
    # 38 sparse columns at 2%: (row index + bin) per stored row instead of a byte per row
    assert sizes["1"] < 0.5 * sizes["0"], sizes
