"""Round growth (speculative multi-leaf expansion, src/device/round_kernels.hip) grows the
trees of one-split-per-step growth, bit for bit.

Each round expands the current leaves of highest gain at once (partition + children's
histograms and split scans); the planner replays the reference's best-first order
(serial_tree_learner.cpp:152-202: argmax over the leaves' best splits, gain then real feature
then leaf id) and accepts expansions while the argmax leaf is expanded.  Histograms are exact
integer sums, so the trees -- and the whole model text -- must equal those of
LGBM_AMD_ROUND_K=1 (the one-split-per-step kernels) for every case below.
"""
import json

import numpy as np
import pytest

import lightgbmv1_amd as lgb

pytestmark = pytest.mark.gpu


def _data(n=40000, f=12, seed=3):
    rng = np.random.RandomState(seed)
    X = rng.randn(n, f).astype(np.float32)
    X[:, 3] = np.abs(X[:, 3])
    X[rng.rand(n) < 0.05, 5] = np.nan
    X[:, 6] = np.where(rng.rand(n) < 0.6, 0.0, X[:, 6])
    X[:, 7] = np.where(rng.rand(n) < 0.7, 2.5, X[:, 7])
    X[:, 9] = rng.randint(0, 12, size=n)  # categorical
    logit = (X[:, 0] + 0.7 * X[:, 1] * X[:, 2] - 0.5 * X[:, 3] + 0.3 * np.nan_to_num(X[:, 5]) + 0.4 * X[:, 7]
             + 0.6 * np.isin(X[:, 9], [1, 4, 7]))
    y = (logit + 0.3 * rng.randn(n) > 0).astype(np.float32)
    return X, y


def _model(monkeypatch, tmp_path, k, X, y, params, rounds=12, tag=""):
    monkeypatch.setenv("LGBM_AMD_ROUND_K", str(k))
    log = tmp_path / ("iters_%s_%d.jsonl" % (tag, k))
    monkeypatch.setenv("LGBM_AMD_ITER_LOG", str(log))
    p = {"verbose": -1, "device_type": "gpu", "seed": 11, "num_leaves": 31, "max_bin": 63}
    p.update(params)
    cat = p.pop("_cat", None)
    ds = lgb.Dataset(X, y, params=p, categorical_feature=cat if cat is not None else "auto")
    bst = lgb.train(p, ds, rounds)
    monkeypatch.delenv("LGBM_AMD_ITER_LOG")
    rows = [json.loads(line) for line in log.read_text().splitlines()]
    return bst.model_to_string(), rows


CASES = {
    "binary": {"objective": "binary"},
    "binary_63": {"objective": "binary", "num_leaves": 63, "max_bin": 255},
    "categorical": {"objective": "binary", "_cat": [9]},
    "bagging": {"objective": "binary", "bagging_fraction": 0.7, "bagging_freq": 1},
    "goss": {"objective": "binary", "boosting": "goss", "learning_rate": 0.3},
    "max_depth": {"objective": "binary", "num_leaves": 63, "max_depth": 5},
    "min_data": {"objective": "binary", "min_data_in_leaf": 1500},
    "monotone": {"objective": "binary", "monotone_constraints": [1, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 0]},
    "l1_reg": {"objective": "regression", "lambda_l1": 0.5, "max_delta_step": 2.0, "path_smooth": 1.0},
    "interaction": {"objective": "binary", "interaction_constraints": [[0, 1, 2], [3, 4, 5, 6, 7], [8, 9, 10, 11]]},
    "wide": {"objective": "binary", "gpu_use_dp": True},
    "multiclass": {"objective": "multiclass", "num_class": 3},
    "quantile": {"objective": "quantile", "alpha": 0.3},
    "ff_bytree": {"objective": "binary", "feature_fraction": 0.6},
    "leaves_511": {"objective": "binary", "num_leaves": 511, "min_data_in_leaf": 10},  # (plan LDS past 64 KiB)
}


@pytest.mark.parametrize("case", list(CASES))
def test_round_growth_equals_one_split_per_step(case, monkeypatch, tmp_path, gpu_available):
    X, y = _data()
    params = dict(CASES[case])
    if params["objective"] == "multiclass":
        y = np.digitize(X[:, 0] + 0.5 * X[:, 1], [-0.5, 0.5]).astype(np.float32)
    elif params["objective"] in ("regression", "quantile"):
        y = (X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + 0.2 * np.random.RandomState(4).randn(len(y))).astype(np.float32)
    base, base_rows = _model(monkeypatch, tmp_path, 1, X, y, params, tag=case)
    spec, spec_rows = _model(monkeypatch, tmp_path, 8, X, y, params, tag=case)
    assert all(r == 0 for row in base_rows for r in row["rounds"])
    # round growth ran (device-resident) and needed fewer rounds than splits
    rounds = [r for row in spec_rows for r in row["rounds"]]
    splits = [lv - 1 for row in spec_rows for lv in row["leaves"]]
    assert all(row["device_resident"][0] for row in spec_rows)
    assert all(r > 0 for r, s in zip(rounds, splits) if s > 0)
    if case in ("binary", "binary_63"):
        assert sum(rounds) < 0.7 * sum(splits), (rounds, splits)
    assert base == spec


@pytest.mark.parametrize("k", [2, 5, 16])
def test_round_width_does_not_change_trees(k, monkeypatch, tmp_path, gpu_available):
    X, y = _data(seed=8)
    params = {"objective": "binary", "num_leaves": 127, "min_data_in_leaf": 5}
    base, _ = _model(monkeypatch, tmp_path, 1, X, y, params, rounds=6, tag="w")
    spec, rows = _model(monkeypatch, tmp_path, k, X, y, params, rounds=6, tag="w")
    assert base == spec
    assert all(r > 0 for row in rows for r in row["rounds"])


def test_round_growth_many_row_blocks(monkeypatch, tmp_path, gpu_available):
    """Leaves of many row blocks: the round's reduce kernel (chunks combined with atomics into
    the parity buffers the previous round's scans zeroed) instead of direct partial sums."""
    X, y = _data(n=600000, seed=9)
    params = {"objective": "binary", "num_leaves": 63, "max_bin": 255, "bagging_fraction": 0.9, "bagging_freq": 1}
    base, _ = _model(monkeypatch, tmp_path, 1, X, y, params, rounds=5, tag="big")
    spec, rows = _model(monkeypatch, tmp_path, 8, X, y, params, rounds=5, tag="big")
    assert [lv for row in rows for lv in row["leaves"]] == [63] * 5
    assert base == spec


@pytest.mark.parametrize("vmax", ["0", "1", "3", "14"])
def test_round_speculation_depth_does_not_change_trees(vmax, monkeypatch, tmp_path, gpu_available):
    """Speculation below the leaves (expansions of the children of expanded, not yet accepted
    leaves, LGBM_AMD_ROUND_VMAX levels deep, one index buffer per level + 2): the replay
    accepts whole chains; the trees, and every leaf's rows (scores, quantile renewal), stay
    those of one split per step."""
    X, y = _data(n=200000, seed=12)
    y = (X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + 0.2 * np.random.RandomState(4).randn(len(y))).astype(np.float32)
    params = {"objective": "quantile", "alpha": 0.4, "num_leaves": 63, "max_bin": 255, "bagging_fraction": 0.8,
              "bagging_freq": 1}
    base, _ = _model(monkeypatch, tmp_path, 1, X, y, params, rounds=8, tag="vd" + vmax)
    monkeypatch.setenv("LGBM_AMD_ROUND_VMAX", vmax)
    spec, rows = _model(monkeypatch, tmp_path, 8, X, y, params, rounds=8, tag="vd" + vmax)
    assert base == spec
    rounds = [r for row in rows for r in row["rounds"]]
    splits = [lv - 1 for row in rows for lv in row["leaves"]]
    assert all(r > 0 for r, s in zip(rounds, splits) if s > 0)
    if vmax != "0":
        # chains are accepted in one replay
        assert sum(rounds) < 0.5 * sum(splits), (rounds, splits)


@pytest.mark.parametrize("fused", ["0", "1"])
def test_round_kernel_variants(fused, monkeypatch, tmp_path, gpu_available):
    """The fused partition + histogram kernel and the partition / per-child histogram pair."""
    X, y = _data(n=300000, seed=10)
    params = {"objective": "binary", "num_leaves": 63, "max_bin": 255}
    base, _ = _model(monkeypatch, tmp_path, 1, X, y, params, rounds=4, tag="v" + fused)
    monkeypatch.setenv("LGBM_AMD_ROUND_FUSED", fused)
    spec, _ = _model(monkeypatch, tmp_path, 8, X, y, params, rounds=4, tag="v" + fused)
    assert base == spec


def test_round_growth_sparse_rows(monkeypatch, tmp_path, gpu_available):
    """Row-sparse storage and EFB bundles through the round kernels."""
    rng = np.random.RandomState(21)
    n = 30000
    X = np.where(rng.rand(n, 40) < 0.1, rng.randn(n, 40), 0.0)
    X[:, :4] = rng.randn(n, 4)
    y = (X[:, 0] + X[:, 1] * X[:, 2] + X[:, 4:20].sum(1) + 0.3 * rng.randn(n) > 0).astype(np.float32)
    params = {"objective": "binary", "num_leaves": 63, "max_bin_by_feature": [511] + [63] * 39}
    monkeypatch.setenv("LGBM_AMD_SPARSE_ROWS", "1")
    base, _ = _model(monkeypatch, tmp_path, 1, X, y, params, rounds=8, tag="sp")
    spec, _ = _model(monkeypatch, tmp_path, 8, X, y, params, rounds=8, tag="sp")
    assert base == spec


def test_round_growth_self_check(monkeypatch, gpu_available):
    """Every leaf's device best split against the CPU split finder on the device histograms
    (pending expansions: the leaf's histogram is the sum of its children's slots)."""
    from lightgbmv1_amd import _native as nat
    monkeypatch.setenv("LGBM_AMD_ROUND_K", "8")
    monkeypatch.setenv("LGBM_AMD_SPECULATE", "0")  # (the device must hold the last tree, not the next)
    X, y = _data(seed=5)
    p = {"objective": "binary", "verbose": -1, "device_type": "gpu", "num_leaves": 63, "max_bin": 63, "seed": 3}
    bst = lgb.train(p, lgb.Dataset(X, y, params=p), 3, keep_training_booster=True)
    res = json.loads(nat.read_string(lambda size, need, buf: nat.call(
        "LGBM_AMD_BoosterDeviceCheckSplits", bst.handle, size, need, buf), 1 << 16))
    assert res["device_mode"] and res["checked"] > 0
    assert res["mismatched"] == 0, res


def test_timed_growth_mode_choice_keeps_the_trees(monkeypatch, tmp_path, capfd):
    """LGBM_AMD_ROUND_AUTO=1 (by default from 16M rows per rank): trees 1-2 are timed with
    round growth and tree 4 with one split per step, and the faster mode grows the rest.  The
    growth mode never changes a tree: the model equals pure round growth's, and the iteration
    log shows the probe trees without rounds."""
    X, y = _data()
    params = {"objective": "binary", "verbose": 1}
    monkeypatch.setenv("LGBM_AMD_ROUND_AUTO", "0")
    base, _ = _model(monkeypatch, tmp_path, 6, X, y, params, rounds=10, tag="fixed")
    capfd.readouterr()
    monkeypatch.setenv("LGBM_AMD_ROUND_AUTO", "1")
    auto, rows = _model(monkeypatch, tmp_path, 6, X, y, params, rounds=10, tag="auto")
    out = capfd.readouterr()
    assert "growth timed at" in out.out + out.err
    assert auto == base
    per_tree = [r["rounds"][0] for r in rows]
    assert per_tree[3] == 0 and per_tree[4] == 0 and per_tree[1] > 0


@pytest.mark.parametrize("params", [
    {"objective": "binary", "feature_fraction_bynode": 0.6},
    {"objective": "binary", "feature_fraction_bynode": 0.5, "feature_fraction": 0.8, "num_leaves": 63},
    {"objective": "binary", "feature_fraction_bynode": 0.4, "min_data_in_leaf": 1500},
    {"objective": "binary", "feature_fraction_bynode": 0.6, "max_depth": 5, "num_leaves": 63},
    {"objective": "regression", "feature_fraction_bynode": 0.7, "bagging_fraction": 0.7, "bagging_freq": 1},
    {"objective": "binary", "feature_fraction_bynode": 0.6, "num_leaves": 127},
], ids=["bynode", "bytree_bynode_63", "min_data", "max_depth", "regression_bagging", "leaves_127"])
def test_bynode_rounds_equal_one_split_per_step(params, monkeypatch, tmp_path, gpu_available):
    """Per-node feature sampling on round growth (KArgs::round_bynode): the scans evaluate every
    feature of a node, the replay folds each node's results with its draw once it knows the
    split that created it, and keeps the reference's splittable flags per leaf id (persisting
    across trees).  The models -- several trees, so the sampler's state and the flag rows carry
    over -- equal one split per step's, and round growth was used."""
    X, y = _data()
    X = X[:, [0, 1, 2, 3, 4, 5, 6, 7, 8, 10, 11]]  # (numerical features: the round path's scope)
    if params["objective"] == "regression":
        y = X[:, 0] + X[:, 1] * X[:, 2] + 0.1 * np.nan_to_num(X[:, 5])
    p = dict(params, feature_fraction_seed=7)
    rounds, rows = _model(monkeypatch, tmp_path, 8, X, y, p, rounds=15, tag="bynode")
    assert sum(sum(r["rounds"]) for r in rows) > 0  # (the trees grew in rounds)
    monkeypatch.setenv("LGBM_AMD_BYNODE_ROUNDS", "0")
    steps, _ = _model(monkeypatch, tmp_path, 8, X, y, p, rounds=15, tag="bynode_steps")
    assert rounds == steps


@pytest.mark.parametrize("params", [
    {"objective": "binary", "feature_fraction_bynode": 0.6, "_cat": [9]},
    {"objective": "binary", "feature_fraction_bynode": 0.5, "_cat": [9, 7], "num_leaves": 63, "max_cat_to_onehot": 8},
], ids=["cat", "two_cats_63"])
def test_bynode_rounds_categorical_equal_one_split_per_step(params, monkeypatch, tmp_path, gpu_available):
    """Per-node sampling on round growth with categorical features: each node keeps its
    categorical features' category sets (KArgs::node_fb_cat), and the replay copies the
    winner's set to the node's best.  The models equal one split per step's."""
    X, y = _data()
    if 7 in params["_cat"]:
        X = X.copy()
        X[:, 7] = np.random.RandomState(5).randint(0, 40, size=len(y))
    p = dict(params, feature_fraction_seed=7)
    rounds, rows = _model(monkeypatch, tmp_path, 8, X, y, dict(p), rounds=12, tag="bynode_cat")
    assert sum(sum(r["rounds"]) for r in rows) > 0  # (the trees grew in rounds)
    steps, _ = _model(monkeypatch, tmp_path, 1, X, y, dict(p), rounds=12, tag="bynode_cat_steps")
    assert rounds == steps


@pytest.mark.parametrize("params", [
    {"objective": "binary", "cegb_penalty_split": 1e-4},
    {"objective": "binary", "cegb_tradeoff": 0.5, "cegb_penalty_split": 4e-5, "num_leaves": 63, "max_bin": 255},
    {"objective": "binary", "cegb_penalty_split": 1e-5, "cegb_penalty_feature_coupled": [0.3] * 6},
    {"objective": "regression", "cegb_penalty_feature_coupled": [0.2, 0.0] * 3, "feature_fraction": 0.7},
    {"objective": "binary", "cegb_penalty_split": 2e-5, "feature_fraction_bynode": 0.6, "_cat": []},
    {"objective": "binary", "cegb_penalty_split": 1e-5, "cegb_penalty_feature_coupled": [5.0] * 6, "_first": True},
    {"objective": "binary", "cegb_tradeoff": 0.5, "cegb_penalty_feature_coupled": [40.0, 2.0, 0.0] * 2,
     "feature_fraction": 0.7, "num_leaves": 63, "_first": True},
    {"objective": "binary", "cegb_penalty_feature_coupled": [20.0] * 6, "feature_fraction_bynode": 0.6, "_first": True},
    {"objective": "binary", "cegb_penalty_feature_coupled": [10.0] * 6, "num_leaves": 127, "min_data_in_leaf": 40,
     "_first": True},
], ids=["split", "split_tradeoff_63", "coupled", "coupled_bytree", "split_bynode", "coupled_first_trees",
        "coupled_large_63", "coupled_bynode", "coupled_127"])
def test_cegb_rounds_equal_one_split_per_step(params, monkeypatch, tmp_path, gpu_available):
    """CEGB penalties on round growth (GPUTreeLearner::CegbRounds): the scans subtract the split
    penalty of the node's rows; with coupled penalties a tree grows in rounds once every feature
    of its sample is used (no refunds or coupled terms left in it), the earlier trees one split
    per step.  The models equal one split per step's, and rounds were used."""
    X, y = _data()
    X = X[:, [0, 1, 2, 3, 5, 7]]  # (informative features: every one is used within a few trees)
    p = dict(params, feature_fraction_seed=5)
    first = p.pop("_first", False)  # (coupled penalties from the first tree: refunds inside round trees)
    if p["objective"] == "regression":
        y = (X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + 0.2 * np.random.RandomState(4).randn(len(y))).astype(np.float32)
    rounds, rows = _model(monkeypatch, tmp_path, 8, X, y, dict(p), rounds=15, tag="cegb")
    assert sum(sum(r["rounds"]) for r in rows) > 0  # (some trees grew in rounds)
    if first:
        assert sum(rows[0]["rounds"]) > 0  # (the first tree, with every feature unused, too)
    steps, _ = _model(monkeypatch, tmp_path, 1, X, y, dict(p), rounds=15, tag="cegb_steps")
    assert rounds == steps


@pytest.mark.parametrize("params", [
    {"objective": "binary", "extra_trees": True},
    {"objective": "binary", "extra_trees": True, "num_leaves": 63, "max_bin": 255},
    {"objective": "regression", "extra_trees": True, "bagging_fraction": 0.7, "bagging_freq": 1},
    {"objective": "binary", "extra_trees": True, "min_data_in_leaf": 1500, "max_depth": 6},
    {"objective": "binary", "extra_trees": True, "monotone_constraints": [1, 0, 0, -1, 0, 0, 0, 1, 0, 0, 0, 0]},
    {"objective": "binary", "extra_trees": True, "zero_as_missing": True, "lambda_l1": 0.3},
    {"objective": "binary", "extra_trees": True, "feature_fraction_bynode": 0.6, "feature_fraction": 0.8},
    {"objective": "binary", "extra_trees": True, "num_leaves": 127, "min_data_in_leaf": 40},
], ids=["binary", "leaves_63", "regression_bagging", "min_data_depth", "monotone", "zero_missing_l1", "bynode",
        "leaves_127"])
def test_extra_trees_rounds_equal_one_split_per_step(params, monkeypatch, tmp_path, gpu_available):
    """extra_trees on round growth (KArgs::round_xt): the scans store every node's per-bin
    prefixes, the replay draws each child's thresholds in the sequential order and evaluates
    them exactly; the models -- several trees, so the generators' states carry over -- equal
    one split per step's (the step scans' draws), and round growth was used."""
    X, y = _data()
    p = dict(params, extra_seed=9, feature_fraction_seed=5)
    if p["objective"] == "regression":
        y = (X[:, 0] + 0.5 * X[:, 1] * X[:, 2] + 0.2 * np.random.RandomState(4).randn(len(y))).astype(np.float32)
    rounds, rows = _model(monkeypatch, tmp_path, 8, X, y, dict(p), rounds=12, tag="xt")
    assert sum(sum(r["rounds"]) for r in rows) > 0  # (the trees grew in rounds)
    steps, _ = _model(monkeypatch, tmp_path, 1, X, y, dict(p), rounds=12, tag="xt_steps")
    assert rounds == steps



def _growth_stats(bst):
    import ctypes
    from lightgbmv1_amd import _native as nat
    out = (ctypes.c_double * 7)()
    nat.call("LGBM_AMD_BoosterGrowthStats", bst.handle, out, ctypes.c_int(7))
    return list(out)


@pytest.mark.parametrize("case", ["plain", "feature_fraction", "valid_early_stop", "rollback", "reset_lr",
                                  "regression_l1", "bagging"])
def test_speculative_next_tree_equals_sequential(case, monkeypatch, gpu_available):
    """The next tree launched when a tree's last plan is seen (before the host returns through
    GBDT; LGBM_AMD_SPECULATE=1, opt-in) grows the model of launching it when GBDT asks for it,
    bit for bit: with a per-tree feature sample drawn at launch, with validation and early
    stopping between iterations, after a rollback or a learning-rate reset (the launched tree is
    drained and regrown from the same sample), and where GBDT forbids it (leaf renewal,
    bagging).  The growth counters show which trees were launched early."""
    X, y = _data(n=60000, seed=21)
    Xv, yv = _data(n=8000, seed=22)
    params = {"objective": "binary", "verbose": -1, "device_type": "gpu", "seed": 5, "num_leaves": 31,
              "max_bin": 63, "learning_rate": 0.1}
    if case == "feature_fraction":
        params["feature_fraction"] = 0.7
    if case == "regression_l1":
        params["objective"] = "regression_l1"
    if case == "bagging":
        params.update(bagging_fraction=0.7, bagging_freq=1)

    def run(spec):
        monkeypatch.setenv("LGBM_AMD_SPECULATE", "1" if spec else "0")
        ds = lgb.Dataset(X, y, params=params, free_raw_data=False)
        if case == "valid_early_stop":
            dv = lgb.Dataset(Xv, yv, reference=ds)
            bst = lgb.train(dict(params, metric="auc"), ds, 40, valid_sets=[dv], early_stopping_rounds=3,
                            verbose_eval=False, keep_training_booster=True)
        elif case in ("rollback", "reset_lr"):
            bst = lgb.Booster(params, ds)
            for _ in range(4):
                bst.update()
            if case == "rollback":
                bst.rollback_one_iter()
            else:
                bst.reset_parameter({"learning_rate": 0.05})
            for _ in range(4):
                bst.update()
        else:
            bst = lgb.train(params, ds, 12, keep_training_booster=True)
        stats = _growth_stats(bst)
        text = bst.model_to_string()
        del bst
        return text, stats

    seq, st0 = run(False)
    spec, st1 = run(True)
    assert spec == seq
    assert st0[6] == 0
    if case in ("regression_l1", "bagging"):
        assert st1[6] == 0  # (GBDT does not allow it)
    else:
        assert st1[6] >= 3, st1
