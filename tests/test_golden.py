"""Parity against the reference itself: the golden oracle of SURVEY.md §7.7-10 / §7.8.

The oracle is the reference's CPU command line program compiled from its own sources in a
scratch copy (``tools/build_golden.sh``: USE_GPU=OFF, nothing prebuilt is run); ``LGBM_GOLDEN_CLI``
points at it (default /tmp/refbuild/lightgbm).  The tests skip when it is absent.

* ``test_reference_models_predict_identically``: models the reference trains on its bundled
  examples (binary with weights, regression with init scores, multiclass, lambdarank) load here
  and predict bit-identically to the reference's own predictions (printed with 17 digits), from
  the Python package and from this framework's CLI.
* ``test_cpu_learner_trees_match_reference``: this framework's CPU learner, trained with the
  same configuration file, grows the same trees: split features, thresholds, decision types and
  tree shapes equal, leaf values equal to 1e-12 relative.
* ``test_headline_auc_matches_reference``: a 63-leaf, 255-bin Higgs-shaped run (bench.py's
  generator, 200k rows, 50 trees): the reference and this framework's CPU learner write the same
  tree sections byte for byte, hence the same held-out AUC.  (The device learner's AUC is pinned
  to the CPU learner's at the full headline size: profiles/r04_auc_parity_500trees.md.)
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

import lightgbmv1_amd as lgb

ORACLE = os.environ.get("LGBM_GOLDEN_CLI", "/tmp/refbuild/lightgbm")
OUR_CLI = os.path.join(os.path.dirname(lgb.__file__), "lib", "lightgbm")
HERE = os.path.dirname(os.path.abspath(__file__))
REF_EXAMPLES = os.environ.get("LGBM_AMD_REF_EXAMPLES", "/root/reference/examples")

pytestmark = pytest.mark.skipif(not os.access(ORACLE, os.X_OK),
                                reason="golden oracle not built (tools/build_golden.sh): " + ORACLE)

# (example directory, file prefix, test data file)
EXAMPLES = [("binary_classification", "binary", "binary.test"),
            ("regression", "regression", "regression.test"),
            ("multiclass_classification", "multiclass", "multiclass.test"),
            ("lambdarank", "rank", "rank.test")]


def _example(tmp_path, name):
    for root in (REF_EXAMPLES, os.path.join(HERE, "data", "examples")):
        src = os.path.join(root, name)
        if os.path.isdir(src):
            dst = tmp_path / name
            shutil.copytree(src, dst)
            for f in dst.iterdir():
                os.chmod(f, 0o644)
            return dst
    pytest.skip("example %s not available" % name)


def _run(cli, cwd, *args):
    r = subprocess.run([cli] + list(args), cwd=str(cwd), capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (cli, args, r.stdout[-2000:], r.stderr[-2000:])
    return r.stdout


def _train_args(trees):
    # no validation output during training (it only logs), a fixed thread count
    return ["config=train.conf", "num_trees=%d" % trees, "num_threads=4", "metric_freq=1000", "verbosity=-1"]


def _trees(model_text):
    """per tree: {key: value string} of the tree section"""
    out = []
    cur = None
    for line in model_text.splitlines():
        if line.startswith("Tree="):
            cur = {}
            out.append(cur)
        elif line.startswith("end of trees"):
            break
        elif cur is not None and "=" in line:
            k, v = line.split("=", 1)
            cur[k] = v
    return out


@pytest.mark.parametrize("name,prefix,test_file", EXAMPLES, ids=[e[0] for e in EXAMPLES])
def test_reference_models_predict_identically(tmp_path, name, prefix, test_file):
    d = _example(tmp_path, name)
    _run(ORACLE, d, *(_train_args(20) + ["output_model=ref_model.txt"]))
    _run(ORACLE, d, "task=predict", "data=" + test_file, "input_model=ref_model.txt", "output_result=ref_pred.txt",
         "verbosity=-1")
    ref = np.loadtxt(d / "ref_pred.txt")
    bst = lgb.Booster(model_file=str(d / "ref_model.txt"))
    assert bst.num_trees() == 20 * (5 if prefix == "multiclass" else 1)
    ours = bst.predict(str(d / test_file))
    np.testing.assert_array_equal(ours.reshape(ref.shape), ref)
    _run(OUR_CLI, d, "task=predict", "data=" + test_file, "input_model=ref_model.txt", "output_result=our_pred.txt",
         "verbosity=-1")
    np.testing.assert_array_equal(np.loadtxt(d / "our_pred.txt"), ref)
    # the model text written back from the loaded model keeps every tree field
    again = _trees(bst.model_to_string())
    for a, b in zip(_trees((d / "ref_model.txt").read_text()), again):
        for k in ("split_feature", "threshold", "decision_type", "left_child", "right_child", "leaf_value",
                  "leaf_count", "internal_count", "num_cat"):
            assert a.get(k) == b.get(k), k


@pytest.mark.parametrize("name,prefix,test_file", EXAMPLES, ids=[e[0] for e in EXAMPLES])
def test_cpu_learner_trees_match_reference(tmp_path, name, prefix, test_file):
    d = _example(tmp_path, name)
    _run(ORACLE, d, *(_train_args(10) + ["output_model=ref_model.txt"]))
    _run(OUR_CLI, d, *(_train_args(10) + ["output_model=our_model.txt", "device_type=cpu"]))
    ref = _trees((d / "ref_model.txt").read_text())
    ours = _trees((d / "our_model.txt").read_text())
    assert len(ref) == len(ours)
    for i, (a, b) in enumerate(zip(ref, ours)):
        for k in ("num_leaves", "split_feature", "threshold", "decision_type", "left_child", "right_child",
                  "leaf_count", "internal_count"):
            assert a[k] == b[k], "tree %d: %s" % (i, k)
        np.testing.assert_allclose(np.array(b["leaf_value"].split(), dtype=float),
                                   np.array(a["leaf_value"].split(), dtype=float), rtol=1e-12, atol=0,
                                   err_msg="tree %d leaf_value" % i)


def test_headline_auc_matches_reference(tmp_path):
    import sys
    sys.path.insert(0, os.path.dirname(HERE))
    from bench import make_rows, roc_auc
    X, y = make_rows(0, 200_000, 28)
    Xt, yt = make_rows(10_000_000 + 12345678, 50_000, 28)
    train = tmp_path / "higgs.train"
    np.savetxt(train, np.column_stack([y, X]), fmt="%.9g", delimiter="\t")
    test = tmp_path / "higgs.test"
    np.savetxt(test, np.column_stack([yt, Xt]), fmt="%.9g", delimiter="\t")
    conf = ["task=train", "objective=binary", "max_bin=255", "num_leaves=63", "learning_rate=0.1",
            "min_data_in_leaf=1", "min_sum_hessian_in_leaf=100", "num_trees=50", "num_threads=4", "verbosity=-1",
            "data=higgs.train"]
    _run(ORACLE, tmp_path, *(conf + ["output_model=ref.txt"]))
    _run(OUR_CLI, tmp_path, *(conf + ["output_model=ours.txt", "device_type=cpu"]))
    for model, out in (("ref.txt", "ref_pred.txt"), ("ours.txt", "our_pred.txt")):
        _run(ORACLE, tmp_path, "task=predict", "data=higgs.test", "input_model=" + model, "output_result=" + out,
             "verbosity=-1")
    sec = lambda t: t[t.index("Tree=0"):t.index("end of trees")]
    assert sec((tmp_path / "ours.txt").read_text()) == sec((tmp_path / "ref.txt").read_text())
    auc_ref = roc_auc(yt, np.loadtxt(tmp_path / "ref_pred.txt"))
    auc_ours = roc_auc(yt, np.loadtxt(tmp_path / "our_pred.txt"))
    assert auc_ref > 0.75
    assert auc_ours == auc_ref
