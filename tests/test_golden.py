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
  to the CPU learner's at the full headline size: profiles/r04_golden_headline.md and bench.py's
  auc_ref, pinned in tools/bench_auc_ref.json.)
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


def _sparse_multival_data(path, n=6000, seed=7):
    """20 random 10%-dense features (EFB leaves them to its second round: one multi-value group
    in the reference, reference dataset.cpp:188-231), 4 dense features and a label."""
    rng = np.random.RandomState(seed)
    dense = rng.randn(n, 4)
    sparse = np.where(rng.rand(n, 20) < 0.1, rng.randint(1, 30, size=(n, 20)), 0).astype(float)
    y = (dense[:, 0] + 0.3 * sparse[:, :5].sum(axis=1) / 10 + 0.3 * rng.randn(n) > 0.2).astype(float)
    np.savetxt(path, np.column_stack([y, dense, sparse]), fmt="%.9g", delimiter="\t")


BINARY_CASES = [("binary_classification", "binary.train", "binary.test"),
                ("lambdarank", "rank.train", "rank.test"),
                ("sparse_multival", "sparse.train", None),
                ("sparse_multival_host_sparse", "sparse.train", None)]


@pytest.mark.parametrize("name,train_file,test_file", BINARY_CASES, ids=[c[0] for c in BINARY_CASES])
def test_dataset_binary_files_interchange(tmp_path, monkeypatch, name, train_file, test_file):
    """Dataset binary files (reference dataset.cpp:890-992 / dataset_loader.cpp:273-525): the
    reference's save_binary output and this framework's are the same bytes; each side trains
    from the other's file the trees it trains from the text file.  With host-sparse storage
    (LGBM_AMD_HOST_SPARSE=1) the bundles are written as sparse groups -- other bytes, which the
    reference reads and trains the same trees from."""
    host_sparse = name.endswith("_host_sparse")
    if name.startswith("sparse_multival"):
        d = tmp_path / name
        d.mkdir()
        _sparse_multival_data(d / train_file)
        conf = ["task=train", "objective=binary", "data=" + train_file, "num_trees=8", "num_leaves=15",
                "num_threads=4", "verbosity=-1"]
    else:
        d = _example(tmp_path, name)
        conf = _train_args(8)
    ref_dir, our_dir = tmp_path / "ref_bin", tmp_path / "our_bin"
    shutil.copytree(d, ref_dir)
    shutil.copytree(d, our_dir)
    _run(ORACLE, ref_dir, *(conf + ["save_binary=true", "output_model=ref_model.txt"]))
    if host_sparse:
        monkeypatch.setenv("LGBM_AMD_HOST_SPARSE", "1")
    _run(OUR_CLI, our_dir, *(conf + ["save_binary=true", "output_model=our_model.txt", "device_type=cpu"]))
    monkeypatch.delenv("LGBM_AMD_HOST_SPARSE", raising=False)
    ref_bin = (ref_dir / (train_file + ".bin")).read_bytes()
    our_bin = (our_dir / (train_file + ".bin")).read_bytes()
    assert ref_bin.startswith(b"______LightGBM_Binary_File_Token______\n")
    if host_sparse:
        assert our_bin != ref_bin and our_bin[:200] == ref_bin[:200]
    else:
        assert our_bin == ref_bin
    if name.startswith("sparse_multival"):  # (the reference wrote a multi-value group: it is exercised)
        ds = lgb.Dataset(str(ref_dir / (train_file + ".bin"))).construct()
        assert ds.num_data() == 6000
    ref_trees = _trees((ref_dir / "ref_model.txt").read_text())
    # the reference's file trains the same trees here ...
    x_dir, y_dir = tmp_path / "x", tmp_path / "y"
    for dd in (x_dir, y_dir):
        dd.mkdir()
    (x_dir / "ref.bin").write_bytes(ref_bin)
    (y_dir / "our.bin").write_bytes(our_bin)
    conf_bin = [c for c in conf if not c.startswith("data=") and c != "config=train.conf"]
    if "config=train.conf" in conf:
        keep = [line for line in (d / "train.conf").read_text().splitlines()
                if line.strip() and not line.strip().startswith("#") and not line.strip().startswith(("data", "valid"))]
        (x_dir / "train.conf").write_text("\n".join(keep) + "\n")
        (y_dir / "train.conf").write_text("\n".join(keep) + "\n")
        conf_bin = ["config=train.conf"] + conf_bin
    _run(OUR_CLI, x_dir, *(conf_bin + ["data=ref.bin", "output_model=m.txt", "device_type=cpu"]))
    # ... and this framework's file trains the same trees in the reference
    _run(ORACLE, y_dir, *(conf_bin + ["data=our.bin", "output_model=m.txt"]))
    for other in (_trees((x_dir / "m.txt").read_text()), _trees((y_dir / "m.txt").read_text())):
        assert len(other) == len(ref_trees)
        for i, (a, b) in enumerate(zip(ref_trees, other)):
            for k in ("num_leaves", "split_feature", "threshold", "decision_type", "left_child", "right_child",
                      "leaf_count", "internal_count"):
                assert a[k] == b[k], "tree %d: %s" % (i, k)
            np.testing.assert_allclose(np.array(b["leaf_value"].split(), dtype=float),
                                       np.array(a["leaf_value"].split(), dtype=float), rtol=1e-12, atol=0)
