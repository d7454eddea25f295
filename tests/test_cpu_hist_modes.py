"""CPU learner histogram machinery: col-wise / row-wise threading
(force_col_wise / force_row_wise / auto test, reference dataset.cpp:589-684) and the bounded
histogram pool (histogram_pool_size, LRU eviction, reference feature_histogram.hpp:1061-1301).
The modes sum the same values in different orders, so models agree to rounding."""
import numpy as np

import lightgbmv1_amd as lgb


def _data(n=6000, f=12, seed=7):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, f)
    X[:, 3] = rng.randint(0, 700, n)          # a 2-byte group (>256 bins with max_bin=1023)
    X[rng.rand(n) < 0.05, 1] = np.nan
    y = X[:, 0] + 0.5 * X[:, 1] ** 2 * (X[:, 2] > 0) + 0.002 * X[:, 3] + 0.1 * rng.randn(n)
    return X, np.nan_to_num(y)


def _train(extra, rounds=15, capsys=None):
    X, y = _data()
    params = {"objective": "regression", "num_leaves": 31, "learning_rate": 0.1, "max_bin": 1023,
              "min_data_in_leaf": 5, "verbose": 1, "num_threads": 4}
    params.update(extra)
    bst = lgb.train(params, lgb.Dataset(X, y, params={"max_bin": 1023, "verbose": -1}), num_boost_round=rounds)
    return bst, bst.predict(X)


def test_row_wise_matches_col_wise(capsys):
    _, p_col = _train({"force_col_wise": True})
    _, p_row = _train({"force_row_wise": True})
    _, p_auto = _train({})
    out = capsys.readouterr().out
    assert "Auto-choosing" in out and "multi-threading" in out
    np.testing.assert_allclose(p_row, p_col, rtol=1e-9, atol=1e-9)
    np.testing.assert_allclose(p_auto, p_col, rtol=1e-9, atol=1e-9)


def test_bounded_histogram_pool(capsys):
    # one leaf histogram is 2 x 8 B x ~3500 bins (56 KB): 0.05 MB leaves the minimum of 2 slots
    full, p_full = _train({"force_col_wise": True})
    small, p_small = _train({"force_col_wise": True, "histogram_pool_size": 0.05})
    out = capsys.readouterr().out
    assert "Histogram pool:" in out
    np.testing.assert_allclose(p_small, p_full, rtol=1e-7, atol=1e-7)
    assert small.num_trees() == full.num_trees()
