"""C API through ctypes (reference tests/c_api_test/test_.py exercises the same calls):
datasets from a file / dense matrix / CSR / CSC, binary save, booster training and
evaluation, model save + reload, prediction from a matrix and from a file, error reporting."""
import ctypes
import os

import numpy as np
import pytest
from scipy import sparse

from lightgbmv1_amd.libpath import find_lib_path

C_API_DTYPE_FLOAT32 = 0
C_API_DTYPE_FLOAT64 = 1
C_API_DTYPE_INT32 = 2
C_API_DTYPE_INT64 = 3
C_API_PREDICT_NORMAL = 0


@pytest.fixture(scope="module")
def lib():
    lib = ctypes.cdll.LoadLibrary(find_lib_path()[0])
    lib.LGBM_GetLastError.restype = ctypes.c_char_p
    return lib


def _c(s):
    return ctypes.c_char_p(s.encode())


def _check(lib, ret):
    if ret != 0:
        raise RuntimeError(lib.LGBM_GetLastError().decode())


def _data(n=600, f=6, seed=0):
    rng = np.random.RandomState(seed)
    X = rng.rand(n, f)
    X[rng.rand(n, f) < 0.3] = 0.0
    y = (X[:, 0] + X[:, 1] > 0.7).astype(np.float64)
    return X, y


def _set_label(lib, handle, y):
    lab = np.ascontiguousarray(y, dtype=np.float32)
    _check(lib, lib.LGBM_DatasetSetField(handle, _c("label"), lab.ctypes.data_as(ctypes.c_void_p),
                                         ctypes.c_int(len(lab)), ctypes.c_int(C_API_DTYPE_FLOAT32)))


def _from_mat(lib, X, y, ref=None):
    h = ctypes.c_void_p()
    data = np.ascontiguousarray(X, dtype=np.float64)
    _check(lib, lib.LGBM_DatasetCreateFromMat(data.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(C_API_DTYPE_FLOAT64),
                                              ctypes.c_int32(X.shape[0]), ctypes.c_int32(X.shape[1]), ctypes.c_int(1),
                                              _c("max_bin=15"), ref, ctypes.byref(h)))
    _set_label(lib, h, y)
    return h


def _from_csr(lib, X, y, ref=None):
    csr = sparse.csr_matrix(X)
    h = ctypes.c_void_p()
    indptr = csr.indptr.astype(np.int32)
    indices = csr.indices.astype(np.int32)
    vals = csr.data.astype(np.float64)
    _check(lib, lib.LGBM_DatasetCreateFromCSR(indptr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(C_API_DTYPE_INT32),
                                              indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                              vals.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(C_API_DTYPE_FLOAT64),
                                              ctypes.c_int64(len(indptr)), ctypes.c_int64(len(vals)),
                                              ctypes.c_int64(X.shape[1]), _c("max_bin=15"), ref, ctypes.byref(h)))
    _set_label(lib, h, y)
    return h


def _from_csc(lib, X, y, ref=None):
    csc = sparse.csc_matrix(X)
    h = ctypes.c_void_p()
    indptr = csc.indptr.astype(np.int32)
    indices = csc.indices.astype(np.int32)
    vals = csc.data.astype(np.float64)
    _check(lib, lib.LGBM_DatasetCreateFromCSC(indptr.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(C_API_DTYPE_INT32),
                                              indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                              vals.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(C_API_DTYPE_FLOAT64),
                                              ctypes.c_int64(len(indptr)), ctypes.c_int64(len(vals)),
                                              ctypes.c_int64(X.shape[0]), _c("max_bin=15"), ref, ctypes.byref(h)))
    _set_label(lib, h, y)
    return h


def _num_data(lib, h):
    n = ctypes.c_int()
    _check(lib, lib.LGBM_DatasetGetNumData(h, ctypes.byref(n)))
    return n.value


@pytest.mark.parametrize("maker", [_from_mat, _from_csr, _from_csc])
def test_dataset_creation(lib, maker, tmp_path):
    X, y = _data()
    h = maker(lib, X, y)
    assert _num_data(lib, h) == X.shape[0]
    nf = ctypes.c_int()
    _check(lib, lib.LGBM_DatasetGetNumFeature(h, ctypes.byref(nf)))
    assert nf.value == X.shape[1]
    path = str(tmp_path / "d.bin")
    _check(lib, lib.LGBM_DatasetSaveBinary(h, _c(path)))
    h2 = ctypes.c_void_p()
    _check(lib, lib.LGBM_DatasetCreateFromFile(_c(path), _c(""), None, ctypes.byref(h2)))
    assert _num_data(lib, h2) == X.shape[0]
    _check(lib, lib.LGBM_DatasetFree(h))
    _check(lib, lib.LGBM_DatasetFree(h2))


def test_booster_train_eval_save_predict(lib, tmp_path):
    X, y = _data()
    Xv, yv = _data(200, seed=1)
    train = _from_mat(lib, X, y)
    valid = _from_mat(lib, Xv, yv, ref=train)
    booster = ctypes.c_void_p()
    _check(lib, lib.LGBM_BoosterCreate(train, _c("objective=binary metric=auc,binary_logloss verbose=-1"),
                                       ctypes.byref(booster)))
    _check(lib, lib.LGBM_BoosterAddValidData(booster, valid))
    fin = ctypes.c_int()
    for _ in range(20):
        _check(lib, lib.LGBM_BoosterUpdateOneIter(booster, ctypes.byref(fin)))
    cnt = ctypes.c_int()
    _check(lib, lib.LGBM_BoosterGetEvalCounts(booster, ctypes.byref(cnt)))
    assert cnt.value == 2
    res = np.zeros(cnt.value)
    out_len = ctypes.c_int()
    _check(lib, lib.LGBM_BoosterGetEval(booster, ctypes.c_int(1), ctypes.byref(out_len),
                                        res.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
    assert res[0] > 0.9  # auc on the valid set
    it = ctypes.c_int()
    _check(lib, lib.LGBM_BoosterGetCurrentIteration(booster, ctypes.byref(it)))
    assert it.value == 20
    model = str(tmp_path / "model.txt")
    _check(lib, lib.LGBM_BoosterSaveModel(booster, ctypes.c_int(0), ctypes.c_int(-1), ctypes.c_int(0), _c(model)))
    # reload and predict from a matrix
    b2 = ctypes.c_void_p()
    n_it = ctypes.c_int()
    _check(lib, lib.LGBM_BoosterCreateFromModelfile(_c(model), ctypes.byref(n_it), ctypes.byref(b2)))
    assert n_it.value == 20
    mat = np.ascontiguousarray(Xv, dtype=np.float64)
    preds = np.zeros(Xv.shape[0])
    plen = ctypes.c_int64()
    for b in (booster, b2):
        _check(lib, lib.LGBM_BoosterPredictForMat(b, mat.ctypes.data_as(ctypes.c_void_p),
                                                  ctypes.c_int(C_API_DTYPE_FLOAT64), ctypes.c_int32(Xv.shape[0]),
                                                  ctypes.c_int32(Xv.shape[1]), ctypes.c_int(1),
                                                  ctypes.c_int(C_API_PREDICT_NORMAL), ctypes.c_int(0),
                                                  ctypes.c_int(-1), _c(""), ctypes.byref(plen),
                                                  preds.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        assert plen.value == Xv.shape[0]
        if b is booster:
            first = preds.copy()
    np.testing.assert_array_equal(first, preds)
    # predict from a text file
    data_file = str(tmp_path / "valid.tsv")
    np.savetxt(data_file, np.column_stack([yv, Xv]), delimiter="\t", fmt="%.17g")
    out_file = str(tmp_path / "preds.txt")
    _check(lib, lib.LGBM_BoosterPredictForFile(b2, _c(data_file), ctypes.c_int(0),
                                               ctypes.c_int(C_API_PREDICT_NORMAL), ctypes.c_int(0),
                                               ctypes.c_int(-1), _c(""), _c(out_file)))
    np.testing.assert_allclose(np.loadtxt(out_file), first, rtol=1e-12)
    for h in (booster, b2):
        _check(lib, lib.LGBM_BoosterFree(h))
    _check(lib, lib.LGBM_DatasetFree(train))
    _check(lib, lib.LGBM_DatasetFree(valid))


def test_error_reporting(lib):
    h = ctypes.c_void_p()
    ret = lib.LGBM_DatasetCreateFromFile(_c("/nonexistent/data.txt"), _c(""), None, ctypes.byref(h))
    assert ret != 0
    assert len(lib.LGBM_GetLastError()) > 0


def test_device_count_entry(lib):
    n = ctypes.c_int(-1)
    assert lib.LGBM_AMD_DeviceCount(ctypes.byref(n)) == 0
    assert n.value >= 0
    if os.environ.get("HIP_VISIBLE_DEVICES") == "":
        assert n.value == 0


def test_get_predict_without_training_data(lib):
    """LGBM_BoosterGetPredict(data 0) on a booster without training data (lgb.train's default:
    the returned booster is rebuilt from its model string) reports an error instead of reading
    a missing score buffer; with keep_training_booster it returns the training scores."""
    import lightgbmv1_amd as lgb
    rng = np.random.RandomState(0)
    X = rng.randn(2000, 5)
    y = (X[:, 0] > 0).astype(float)
    params = {"objective": "binary", "verbose": -1}
    got = ctypes.c_int64(0)
    buf = np.zeros(2000)
    out = buf.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
    b = lgb.train(params, lgb.Dataset(X, y), 3)
    assert lib.LGBM_BoosterGetPredict(b.handle, ctypes.c_int(0), ctypes.byref(got), out) != 0
    assert b"training data" in lib.LGBM_GetLastError()
    b = lgb.train(params, lgb.Dataset(X, y), 3, keep_training_booster=True)
    assert lib.LGBM_BoosterGetPredict(b.handle, ctypes.c_int(0), ctypes.byref(got), out) == 0
    assert got.value == 2000
    np.testing.assert_allclose(buf, b.predict(X), rtol=1e-12)
