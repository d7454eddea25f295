"""Core Python wrapper: Dataset, Booster and the ctypes bridge to the native library.

Public behaviour mirrors reference python-package/lightgbm/basic.py (lazy Dataset
construction, reference datasets for validation, pandas categorical handling, Booster
training / evaluation / prediction / model IO).  The native side is
``lib_lightgbmv1_amd.so`` (C API in include/lgbm_amd/c_api.h); with
``device_type='gpu'`` training runs on the MI355X learner.
"""
import copy
import ctypes
import json
import os
import warnings
from collections import OrderedDict
from tempfile import NamedTemporaryFile

import numpy as np
import scipy.sparse

from .compat import (PANDAS_INSTALLED, dt_DataTable, integer_types, numeric_types, pd_DataFrame, pd_Series,
                     string_type)
from .libpath import find_lib_path
from .utils.param_table import PARAMETERS as _PARAMETERS


def _log_callback(msg):
    """Redirect native logs to Python's stdout."""
    print("{0:s}".format(msg.decode("utf-8")), end="")


_LIB = None
_LOG_CALLBACK = None


def _load_lib():
    global _LIB, _LOG_CALLBACK
    if _LIB is not None:
        return _LIB
    lib_path = find_lib_path()
    lib = ctypes.cdll.LoadLibrary(lib_path[0])
    lib.LGBM_GetLastError.restype = ctypes.c_char_p
    _LOG_CALLBACK = ctypes.CFUNCTYPE(None, ctypes.c_char_p)(_log_callback)
    lib.callback = _LOG_CALLBACK
    if lib.LGBM_RegisterLogCallback(_LOG_CALLBACK) != 0:
        raise LightGBMError(lib.LGBM_GetLastError().decode("utf-8"))
    _LIB = lib
    return lib


class _LazyLib(object):
    def __getattr__(self, name):
        return getattr(_load_lib(), name)


_LIB_PROXY = _LazyLib()


class LightGBMError(Exception):
    """Error thrown by the native library."""


def _safe_call(ret):
    if ret != 0:
        raise LightGBMError(_load_lib().LGBM_GetLastError().decode("utf-8"))


def _from_tensor(data):
    """torch.Tensor (CPU or a HIP device) -> numpy; anything else unchanged.

    Device tensors are copied to the host once here; the library bins them and keeps its
    own device copy of the binned matrix (PyTorch-ROCm interop)."""
    mod = type(data).__module__
    if mod.startswith("torch") and hasattr(data, "detach"):
        return data.detach().cpu().numpy()
    return data


def is_numeric(obj):
    try:
        float(obj)
        return True
    except (TypeError, ValueError):
        return False


def is_numpy_1d_array(data):
    return isinstance(data, np.ndarray) and len(data.shape) == 1


def is_1d_list(data):
    return isinstance(data, list) and (not data or is_numeric(data[0]))


def list_to_1d_numpy(data, dtype=np.float32, name="list"):
    if is_numpy_1d_array(data):
        if data.dtype == dtype:
            return data
        return data.astype(dtype=dtype, copy=False)
    if is_1d_list(data):
        return np.asarray(data, dtype=dtype)
    if isinstance(data, pd_Series):
        if _get_bad_pandas_dtypes([data.dtypes]):
            raise ValueError("Series.dtypes must be int, float or bool")
        return np.asarray(data, dtype=dtype)
    raise TypeError("Wrong type({0}) for {1}.\nIt should be list, numpy 1-D array or pandas Series".format(
        type(data).__name__, name))


def cfloat32_array_to_numpy(cptr, length):
    if isinstance(cptr, ctypes.POINTER(ctypes.c_float)):
        return np.ctypeslib.as_array(cptr, shape=(length,)).copy()
    raise RuntimeError("Expected float pointer")


def cfloat64_array_to_numpy(cptr, length):
    if isinstance(cptr, ctypes.POINTER(ctypes.c_double)):
        return np.ctypeslib.as_array(cptr, shape=(length,)).copy()
    raise RuntimeError("Expected double pointer")


def cint32_array_to_numpy(cptr, length):
    if isinstance(cptr, ctypes.POINTER(ctypes.c_int32)):
        return np.ctypeslib.as_array(cptr, shape=(length,)).copy()
    raise RuntimeError("Expected int32 pointer")


def cint64_array_to_numpy(cptr, length):
    if isinstance(cptr, ctypes.POINTER(ctypes.c_int64)):
        return np.ctypeslib.as_array(cptr, shape=(length,)).copy()
    raise RuntimeError("Expected int64 pointer")


def c_str(string):
    return ctypes.c_char_p(string.encode("utf-8"))


def c_array(ctype, values):
    return (ctype * len(values))(*values)


def param_dict_to_str(data):
    """Convert a parameter dict to the native ``key=value`` string."""
    if data is None or not data:
        return ""
    pairs = []
    for key, val in data.items():
        if isinstance(val, (list, tuple, set)) or is_numpy_1d_array(val):
            def to_string(x):
                if isinstance(x, list):
                    return "[{}]".format(",".join(map(str, x)))
                return str(x)
            pairs.append(str(key) + "=" + ",".join(map(to_string, val)))
        elif isinstance(val, string_type) or isinstance(val, numeric_types) or is_numeric(val):
            pairs.append(str(key) + "=" + str(val))
        elif val is not None:
            raise TypeError("Unknown type of parameter:%s, got:%s" % (key, type(val).__name__))
    return " ".join(pairs)


class _TempFile(object):
    def __enter__(self):
        with NamedTemporaryFile(prefix="lightgbm_tmp_", delete=True) as f:
            self.name = f.name
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        if os.path.isfile(self.name):
            os.remove(self.name)

    def readlines(self):
        with open(self.name, "r+") as f:
            ret = f.readlines()
        return ret

    def writelines(self, lines):
        with open(self.name, "w+") as f:
            f.writelines(lines)


class _ConfigAliases(object):
    """Alias table generated from the single parameter specification (tools/param_spec.py)."""

    aliases = {name: {name} | set(spec["aliases"]) for name, spec in _PARAMETERS.items()}
    # keys handled specially by the Python layer
    aliases.setdefault("group_column", {"group_column", "group", "group_id", "query_column", "query", "query_id"})

    @classmethod
    def get(cls, *args):
        ret = set()
        for i in args:
            ret |= cls.aliases.get(i, {i})
        return ret


MAX_INT32 = (1 << 31) - 1

C_API_DTYPE_FLOAT32 = 0
C_API_DTYPE_FLOAT64 = 1
C_API_DTYPE_INT32 = 2
C_API_DTYPE_INT64 = 3

C_API_PREDICT_NORMAL = 0
C_API_PREDICT_RAW_SCORE = 1
C_API_PREDICT_LEAF_INDEX = 2
C_API_PREDICT_CONTRIB = 3

C_API_MATRIX_TYPE_CSR = 0
C_API_MATRIX_TYPE_CSC = 1

C_API_FEATURE_IMPORTANCE_SPLIT = 0
C_API_FEATURE_IMPORTANCE_GAIN = 1

FIELD_TYPE_MAPPER = {"label": C_API_DTYPE_FLOAT32,
                     "weight": C_API_DTYPE_FLOAT32,
                     "init_score": C_API_DTYPE_FLOAT64,
                     "group": C_API_DTYPE_INT32}

FEATURE_IMPORTANCE_TYPE_MAPPER = {"split": C_API_FEATURE_IMPORTANCE_SPLIT,
                                  "gain": C_API_FEATURE_IMPORTANCE_GAIN}


def convert_from_sliced_object(data):
    """Fix the memory of multi-dimensional sliced object."""
    if isinstance(data, np.ndarray) and isinstance(data.base, np.ndarray):
        if not data.flags.c_contiguous:
            warnings.warn("Usage of np.ndarray subset (sliced data) is not recommended "
                          "due to it will double the peak memory cost in LightGBM.")
            return np.copy(data)
    return data


def c_float_array(data):
    if is_1d_list(data):
        data = np.asarray(data)
    if is_numpy_1d_array(data):
        data = convert_from_sliced_object(data)
        assert data.flags.c_contiguous
        if data.dtype == np.float32:
            ptr_data = data.ctypes.data_as(ctypes.POINTER(ctypes.c_float))
            type_data = C_API_DTYPE_FLOAT32
        elif data.dtype == np.float64:
            ptr_data = data.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
            type_data = C_API_DTYPE_FLOAT64
        else:
            raise TypeError("Expected np.float32 or np.float64, met type({})".format(data.dtype))
    else:
        raise TypeError("Unknown type({})".format(type(data).__name__))
    return (ptr_data, type_data, data)


def c_int_array(data):
    if is_1d_list(data):
        data = np.asarray(data)
    if is_numpy_1d_array(data):
        data = convert_from_sliced_object(data)
        assert data.flags.c_contiguous
        if data.dtype == np.int32:
            ptr_data = data.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
            type_data = C_API_DTYPE_INT32
        elif data.dtype == np.int64:
            ptr_data = data.ctypes.data_as(ctypes.POINTER(ctypes.c_int64))
            type_data = C_API_DTYPE_INT64
        else:
            raise TypeError("Expected np.int32 or np.int64, met type({})".format(data.dtype))
    else:
        raise TypeError("Unknown type({})".format(type(data).__name__))
    return (ptr_data, type_data, data)


def _get_bad_pandas_dtypes(dtypes):
    pandas_dtype_mapper = {"int8", "int16", "int32", "int64", "uint8", "uint16", "uint32", "uint64",
                           "float16", "float32", "float64", "bool"}
    return [i for i, dtype in enumerate(dtypes) if str(getattr(dtype, "name", dtype)) not in pandas_dtype_mapper
            and not str(dtype).startswith("Sparse")]


def _data_from_pandas(data, feature_name, categorical_feature, pandas_categorical):
    if isinstance(data, pd_DataFrame):
        if len(data.shape) != 2 or data.shape[0] < 1:
            raise ValueError("Input data must be 2 dimensional and non empty.")
        if feature_name == "auto" or feature_name is None:
            data = data.rename(columns=str)
        cat_cols = [col for col, dtype in zip(data.columns, data.dtypes) if str(dtype) == "category"]
        cat_cols_not_ordered = [col for col in cat_cols if not data[col].cat.ordered]
        if pandas_categorical is None:  # train dataset
            pandas_categorical = [list(data[col].cat.categories) for col in cat_cols]
        else:
            if len(cat_cols) != len(pandas_categorical):
                raise ValueError("train and valid dataset categorical_feature do not match.")
            for col, category in zip(cat_cols, pandas_categorical):
                if list(data[col].cat.categories) != list(category):
                    data[col] = data[col].cat.set_categories(category)
        if len(cat_cols):  # cat_cols is list
            data = data.copy()  # not alter origin DataFrame
            data[cat_cols] = data[cat_cols].apply(lambda x: x.cat.codes).replace({-1: np.nan})
        if categorical_feature is not None:
            if feature_name is None:
                feature_name = list(data.columns)
            if categorical_feature == "auto":  # use cat cols from DataFrame
                categorical_feature = cat_cols_not_ordered
            else:  # use cat cols specified by user
                categorical_feature = list(categorical_feature)
        if feature_name == "auto":
            feature_name = list(data.columns)
        bad_indices = _get_bad_pandas_dtypes(data.dtypes)
        if bad_indices:
            raise ValueError("DataFrame.dtypes for data must be int, float or bool.\n"
                             "Did not expect the data types in the following fields: "
                             + ", ".join(data.columns[bad_indices]))
        data = data.values
        if data.dtype != np.float32 and data.dtype != np.float64:
            data = data.astype(np.float32)
    else:
        if feature_name == "auto":
            feature_name = None
        if categorical_feature == "auto":
            categorical_feature = None
    return data, feature_name, categorical_feature, pandas_categorical


def _label_from_pandas(label):
    if isinstance(label, pd_DataFrame):
        if len(label.columns) > 1:
            raise ValueError("DataFrame for label cannot have multiple columns")
        if _get_bad_pandas_dtypes(label.dtypes):
            raise ValueError("DataFrame.dtypes for label must be int, float or bool")
        label = np.ravel(label.values.astype(np.float32, copy=False))
    return label


def _dump_pandas_categorical(pandas_categorical, file_name=None):
    pandas_str = ("\npandas_categorical:" + json.dumps(pandas_categorical, default=_json_default_with_numpy) + "\n")
    if file_name is not None:
        with open(file_name, "a") as f:
            f.write(pandas_str)
    return pandas_str


def _load_pandas_categorical(file_name=None, model_str=None):
    pandas_key = "pandas_categorical:"
    offset = -len(pandas_key)
    if file_name is not None:
        max_offset = -os.path.getsize(file_name)
        with open(file_name, "rb") as f:
            while True:
                if offset < max_offset:
                    offset = max_offset
                f.seek(offset, os.SEEK_END)
                lines = f.readlines()
                if len(lines) >= 2:
                    break
                offset *= 2
        last_line = lines[-1].decode("utf-8").strip()
        if not last_line.startswith(pandas_key):
            last_line = lines[-2].decode("utf-8").strip()
    elif model_str is not None:
        idx = model_str.rfind("\n", 0, offset)
        last_line = model_str[idx:].strip()
    if last_line.startswith(pandas_key):
        return json.loads(last_line[len(pandas_key):])
    return None


def _json_default_with_numpy(obj):
    if isinstance(obj, (np.integer, np.floating, np.bool_)):
        return obj.item()
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    return obj


class _InnerPredictor(object):
    """Prediction-only handle (reference basic.py:455-905)."""

    def __init__(self, model_file=None, booster_handle=None, pred_parameter=None):
        self.handle = ctypes.c_void_p()
        self.__is_manage_handle = True
        if model_file is not None:
            out_num_iterations = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterCreateFromModelfile(c_str(model_file),
                                                                   ctypes.byref(out_num_iterations),
                                                                   ctypes.byref(self.handle)))
            out_num_class = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterGetNumClasses(self.handle, ctypes.byref(out_num_class)))
            self.num_class = out_num_class.value
            self.num_total_iteration = out_num_iterations.value
            self.pandas_categorical = _load_pandas_categorical(file_name=model_file)
        elif booster_handle is not None:
            self.__is_manage_handle = False
            self.handle = booster_handle
            out_num_class = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterGetNumClasses(self.handle, ctypes.byref(out_num_class)))
            self.num_class = out_num_class.value
            self.num_total_iteration = self.current_iteration()
            self.pandas_categorical = None
        else:
            raise TypeError("Need model_file or booster_handle to create a predictor")
        pred_parameter = {} if pred_parameter is None else pred_parameter
        self.pred_parameter = param_dict_to_str(pred_parameter)

    def __del__(self):
        try:
            if self.__is_manage_handle:
                _safe_call(_load_lib().LGBM_BoosterFree(self.handle))
        except AttributeError:
            pass

    def __getstate__(self):
        this = self.__dict__.copy()
        this.pop("handle", None)
        return this

    def predict(self, data, start_iteration=0, num_iteration=-1, raw_score=False, pred_leaf=False,
                pred_contrib=False, data_has_header=False, is_reshape=True):
        if isinstance(data, Dataset):
            raise TypeError("Cannot use Dataset instance for prediction, please use raw data instead")
        data = _data_from_pandas(data, None, None, self.pandas_categorical)[0]
        predict_type = C_API_PREDICT_NORMAL
        if raw_score:
            predict_type = C_API_PREDICT_RAW_SCORE
        if pred_leaf:
            predict_type = C_API_PREDICT_LEAF_INDEX
        if pred_contrib:
            predict_type = C_API_PREDICT_CONTRIB
        int_data_has_header = 1 if data_has_header else 0
        data = _from_tensor(data)
        if isinstance(data, string_type):
            with _TempFile() as f:
                _safe_call(_load_lib().LGBM_BoosterPredictForFile(
                    self.handle, c_str(data), ctypes.c_int(int_data_has_header), ctypes.c_int(predict_type),
                    ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), c_str(self.pred_parameter),
                    c_str(f.name)))
                lines = f.readlines()
                nrow = len(lines)
                preds = [float(token) for line in lines for token in line.split("\t")]
                preds = np.asarray(preds, dtype=np.float64)
        elif isinstance(data, scipy.sparse.csr_matrix):
            preds, nrow = self.__pred_for_csr(data, start_iteration, num_iteration, predict_type)
        elif isinstance(data, scipy.sparse.csc_matrix):
            preds, nrow = self.__pred_for_csc(data, start_iteration, num_iteration, predict_type)
        elif isinstance(data, np.ndarray):
            preds, nrow = self.__pred_for_np2d(data, start_iteration, num_iteration, predict_type)
        elif isinstance(data, list):
            try:
                data = np.array(data)
            except BaseException:
                raise ValueError("Cannot convert data list to numpy array.")
            preds, nrow = self.__pred_for_np2d(data, start_iteration, num_iteration, predict_type)
        elif isinstance(data, dt_DataTable):
            preds, nrow = self.__pred_for_np2d(data.to_numpy(), start_iteration, num_iteration, predict_type)
        else:
            try:
                warnings.warn("Converting data to scipy sparse matrix.")
                csr = scipy.sparse.csr_matrix(data)
            except BaseException:
                raise TypeError("Cannot predict data for type {}".format(type(data).__name__))
            preds, nrow = self.__pred_for_csr(csr, start_iteration, num_iteration, predict_type)
        if pred_leaf:
            preds = preds.astype(np.int32)
        is_sparse = scipy.sparse.issparse(preds) or isinstance(preds, list)
        if is_reshape and not is_sparse and preds.size != nrow:
            if preds.size % nrow == 0:
                preds = preds.reshape(nrow, -1)
            else:
                raise ValueError("Length of predict result (%d) cannot be divide nrow (%d)" % (preds.size, nrow))
        return preds

    def __get_num_preds(self, start_iteration, num_iteration, nrow, predict_type):
        if nrow > MAX_INT32:
            raise LightGBMError("LightGBM cannot perform prediction for data with number of rows greater than "
                                "MAX_INT32 (%d).\nYou can split your data into chunks and then concatenate "
                                "predictions for them" % MAX_INT32)
        n_preds = ctypes.c_int64(0)
        _safe_call(_load_lib().LGBM_BoosterCalcNumPredict(self.handle, ctypes.c_int(nrow), ctypes.c_int(predict_type),
                                                          ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                                                          ctypes.byref(n_preds)))
        return n_preds.value

    def __pred_for_np2d(self, mat, start_iteration, num_iteration, predict_type):
        if len(mat.shape) != 2:
            raise ValueError("Input numpy.ndarray or list must be 2 dimensional")

        def inner_predict(mat, start_iteration, num_iteration, predict_type, preds=None):
            if mat.dtype == np.float32 or mat.dtype == np.float64:
                data = np.asarray(mat.reshape(mat.size), dtype=mat.dtype)
            else:
                data = np.array(mat.reshape(mat.size), dtype=np.float32)
            ptr_data, type_ptr_data, _ = c_float_array(data)
            n_preds = self.__get_num_preds(start_iteration, num_iteration, mat.shape[0], predict_type)
            if preds is None:
                preds = np.zeros(n_preds, dtype=np.float64)
            elif len(preds.shape) != 1 or len(preds) != n_preds:
                raise ValueError("Wrong length of pre-allocated predict array")
            out_num_preds = ctypes.c_int64(0)
            _safe_call(_load_lib().LGBM_BoosterPredictForMat(
                self.handle, ptr_data, ctypes.c_int(type_ptr_data), ctypes.c_int32(mat.shape[0]),
                ctypes.c_int32(mat.shape[1]), ctypes.c_int(1), ctypes.c_int(predict_type),
                ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), c_str(self.pred_parameter),
                ctypes.byref(out_num_preds), preds.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            if n_preds != out_num_preds.value:
                raise ValueError("Wrong length for predict results")
            return preds, mat.shape[0]

        nrow = mat.shape[0]
        if nrow > MAX_INT32:
            sections = np.arange(start=MAX_INT32, stop=nrow, step=MAX_INT32)
            n_preds = [self.__get_num_preds(start_iteration, num_iteration, i, predict_type)
                       for i in np.diff([0] + list(sections) + [nrow])]
            n_preds_sections = np.array([0] + n_preds, dtype=np.intp).cumsum()
            preds = np.zeros(sum(n_preds), dtype=np.float64)
            for chunk, (start_idx_pred, end_idx_pred) in zip(np.array_split(mat, sections),
                                                             zip(n_preds_sections, n_preds_sections[1:])):
                inner_predict(chunk, start_iteration, num_iteration, predict_type, preds[start_idx_pred:end_idx_pred])
            return preds, nrow
        return inner_predict(mat, start_iteration, num_iteration, predict_type)

    def __create_sparse_native(self, cs, out_shape, out_ptr_indptr, out_ptr_indices, out_ptr_data, indptr_type,
                               data_type, is_csr=True):
        data_indices_len = out_shape[0]
        indptr_len = out_shape[1]
        if indptr_type == C_API_DTYPE_INT32:
            out_indptr = cint32_array_to_numpy(out_ptr_indptr, indptr_len)
        elif indptr_type == C_API_DTYPE_INT64:
            out_indptr = cint64_array_to_numpy(out_ptr_indptr, indptr_len)
        else:
            raise TypeError("Expected int32 or int64 type for indptr")
        if data_type == C_API_DTYPE_FLOAT32:
            out_data = cfloat32_array_to_numpy(out_ptr_data, data_indices_len)
        elif data_type == C_API_DTYPE_FLOAT64:
            out_data = cfloat64_array_to_numpy(out_ptr_data, data_indices_len)
        else:
            raise TypeError("Expected float32 or float64 type for data")
        out_indices = cint32_array_to_numpy(out_ptr_indices, data_indices_len)
        per_class_shape = [cs.shape[0], cs.shape[1] + 1]
        if self.num_class > 1:
            offset = 0
            cs_output_matrices = []
            step = per_class_shape[0] + 1 if is_csr else per_class_shape[1] + 1
            for _ in range(self.num_class):
                part_ptr = out_indptr[offset:offset + step]
                start, end = part_ptr[0], part_ptr[-1]
                part_ptr = part_ptr - start
                if is_csr:
                    m = scipy.sparse.csr_matrix((out_data[start:end], out_indices[start:end], part_ptr),
                                                per_class_shape)
                else:
                    m = scipy.sparse.csc_matrix((out_data[start:end], out_indices[start:end], part_ptr),
                                                per_class_shape)
                cs_output_matrices.append(m)
                offset += step
        else:
            if is_csr:
                cs_output_matrices = scipy.sparse.csr_matrix((out_data, out_indices, out_indptr), per_class_shape)
            else:
                cs_output_matrices = scipy.sparse.csc_matrix((out_data, out_indices, out_indptr), per_class_shape)
        _safe_call(_load_lib().LGBM_BoosterFreePredictSparse(out_ptr_indptr, out_ptr_indices, out_ptr_data,
                                                             ctypes.c_int(indptr_type), ctypes.c_int(data_type)))
        return cs_output_matrices

    def __pred_for_csr(self, csr, start_iteration, num_iteration, predict_type):
        nrow = len(csr.indptr) - 1

        def inner_predict(csr, start_iteration, num_iteration, predict_type, preds=None):
            ptr_indptr, type_ptr_indptr, __ = c_int_array(csr.indptr)
            ptr_data, type_ptr_data, _ = c_float_array(csr.data)
            csr_indices = csr.indices.astype(np.int32, copy=False)
            n_preds = self.__get_num_preds(start_iteration, num_iteration, nrow, predict_type)
            if preds is None:
                preds = np.zeros(n_preds, dtype=np.float64)
            out_num_preds = ctypes.c_int64(0)
            _safe_call(_load_lib().LGBM_BoosterPredictForCSR(
                self.handle, ptr_indptr, ctypes.c_int32(type_ptr_indptr),
                csr_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr_data, ctypes.c_int(type_ptr_data),
                ctypes.c_int64(len(csr.indptr)), ctypes.c_int64(len(csr.data)), ctypes.c_int64(csr.shape[1]),
                ctypes.c_int(predict_type), ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                c_str(self.pred_parameter), ctypes.byref(out_num_preds),
                preds.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            if n_preds != out_num_preds.value:
                raise ValueError("Wrong length for predict results")
            return preds, nrow

        def inner_predict_sparse(csr, start_iteration, num_iteration, predict_type):
            ptr_indptr, type_ptr_indptr, __ = c_int_array(csr.indptr)
            ptr_data, type_ptr_data, _ = c_float_array(csr.data)
            csr_indices = csr.indices.astype(np.int32, copy=False)
            matrix_type = C_API_MATRIX_TYPE_CSR
            if type_ptr_indptr == C_API_DTYPE_INT32:
                out_ptr_indptr = ctypes.POINTER(ctypes.c_int32)()
            else:
                out_ptr_indptr = ctypes.POINTER(ctypes.c_int64)()
            out_ptr_indices = ctypes.POINTER(ctypes.c_int32)()
            if type_ptr_data == C_API_DTYPE_FLOAT32:
                out_ptr_data = ctypes.POINTER(ctypes.c_float)()
            else:
                out_ptr_data = ctypes.POINTER(ctypes.c_double)()
            out_shape = np.zeros(2, dtype=np.int64)
            _safe_call(_load_lib().LGBM_BoosterPredictSparseOutput(
                self.handle, ptr_indptr, ctypes.c_int32(type_ptr_indptr),
                csr_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr_data, ctypes.c_int(type_ptr_data),
                ctypes.c_int64(len(csr.indptr)), ctypes.c_int64(len(csr.data)), ctypes.c_int64(csr.shape[1]),
                ctypes.c_int(predict_type), ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                c_str(self.pred_parameter), ctypes.c_int(matrix_type),
                out_shape.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(out_ptr_indptr),
                ctypes.byref(out_ptr_indices), ctypes.byref(out_ptr_data)))
            matrices = self.__create_sparse_native(csr, out_shape, out_ptr_indptr, out_ptr_indices, out_ptr_data,
                                                   type_ptr_indptr, type_ptr_data, is_csr=True)
            return matrices, nrow

        if predict_type == C_API_PREDICT_CONTRIB:
            return inner_predict_sparse(csr, start_iteration, num_iteration, predict_type)
        return inner_predict(csr, start_iteration, num_iteration, predict_type)

    def __pred_for_csc(self, csc, start_iteration, num_iteration, predict_type):
        nrow = csc.shape[0]
        if nrow > MAX_INT32:
            return self.__pred_for_csr(csc.tocsr(), start_iteration, num_iteration, predict_type)
        if predict_type == C_API_PREDICT_CONTRIB:
            ptr_indptr, type_ptr_indptr, __ = c_int_array(csc.indptr)
            ptr_data, type_ptr_data, _ = c_float_array(csc.data)
            csc_indices = csc.indices.astype(np.int32, copy=False)
            if type_ptr_indptr == C_API_DTYPE_INT32:
                out_ptr_indptr = ctypes.POINTER(ctypes.c_int32)()
            else:
                out_ptr_indptr = ctypes.POINTER(ctypes.c_int64)()
            out_ptr_indices = ctypes.POINTER(ctypes.c_int32)()
            if type_ptr_data == C_API_DTYPE_FLOAT32:
                out_ptr_data = ctypes.POINTER(ctypes.c_float)()
            else:
                out_ptr_data = ctypes.POINTER(ctypes.c_double)()
            out_shape = np.zeros(2, dtype=np.int64)
            _safe_call(_load_lib().LGBM_BoosterPredictSparseOutput(
                self.handle, ptr_indptr, ctypes.c_int32(type_ptr_indptr),
                csc_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr_data, ctypes.c_int(type_ptr_data),
                ctypes.c_int64(len(csc.indptr)), ctypes.c_int64(len(csc.data)), ctypes.c_int64(csc.shape[0]),
                ctypes.c_int(predict_type), ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                c_str(self.pred_parameter), ctypes.c_int(C_API_MATRIX_TYPE_CSC),
                out_shape.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(out_ptr_indptr),
                ctypes.byref(out_ptr_indices), ctypes.byref(out_ptr_data)))
            matrices = self.__create_sparse_native(csc, out_shape, out_ptr_indptr, out_ptr_indices, out_ptr_data,
                                                   type_ptr_indptr, type_ptr_data, is_csr=False)
            return matrices, nrow
        n_preds = self.__get_num_preds(start_iteration, num_iteration, nrow, predict_type)
        preds = np.zeros(n_preds, dtype=np.float64)
        out_num_preds = ctypes.c_int64(0)
        ptr_indptr, type_ptr_indptr, __ = c_int_array(csc.indptr)
        ptr_data, type_ptr_data, _ = c_float_array(csc.data)
        csc_indices = csc.indices.astype(np.int32, copy=False)
        _safe_call(_load_lib().LGBM_BoosterPredictForCSC(
            self.handle, ptr_indptr, ctypes.c_int32(type_ptr_indptr),
            csc_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ptr_data, ctypes.c_int(type_ptr_data),
            ctypes.c_int64(len(csc.indptr)), ctypes.c_int64(len(csc.data)), ctypes.c_int64(csc.shape[0]),
            ctypes.c_int(predict_type), ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
            c_str(self.pred_parameter), ctypes.byref(out_num_preds),
            preds.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        if n_preds != out_num_preds.value:
            raise ValueError("Wrong length for predict results")
        return preds, nrow

    def current_iteration(self):
        out_cur_iter = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterGetCurrentIteration(self.handle, ctypes.byref(out_cur_iter)))
        return out_cur_iter.value


class Dataset(object):
    """Dataset in LightGBM (lazily constructed on the native side)."""

    def __init__(self, data, label=None, reference=None, weight=None, group=None, init_score=None, silent=False,
                 feature_name="auto", categorical_feature="auto", params=None, free_raw_data=True):
        self.handle = None
        self.data = data
        self.label = label
        self.reference = reference
        self.weight = weight
        self.group = group
        self.init_score = init_score
        self.silent = silent
        self.feature_name = feature_name
        self.categorical_feature = categorical_feature
        self.params = copy.deepcopy(params)
        self.free_raw_data = free_raw_data
        self.used_indices = None
        self.need_slice = True
        self._predictor = None
        self.pandas_categorical = None
        self.params_back_up = None
        self.feature_penalty = None
        self.monotone_constraints = None
        self.version = 0

    def __del__(self):
        try:
            self._free_handle()
        except AttributeError:
            pass

    def get_params(self):
        """Get the used parameters in the Dataset."""
        if self.params is not None:
            dataset_params = _ConfigAliases.get(
                "bin_construct_sample_cnt", "categorical_feature", "data_random_seed", "enable_bundle",
                "feature_pre_filter", "forcedbins_filename", "group_column", "header", "ignore_column",
                "is_enable_sparse", "label_column", "max_bin", "max_bin_by_feature", "min_data_in_bin",
                "pre_partition", "two_round", "use_missing", "weight_column", "zero_as_missing")
            return {k: v for k, v in self.params.items() if k in dataset_params}
        return {}

    def _free_handle(self):
        if self.handle is not None:
            _safe_call(_load_lib().LGBM_DatasetFree(self.handle))
            self.handle = None
        self.need_slice = True
        if self.used_indices is not None:
            self.data = None
        return self

    def _set_init_score_by_predictor(self, predictor, data, used_indices=None):
        data_has_header = False
        if isinstance(data, string_type):
            data_has_header = any(self.params.get(alias, False) for alias in _ConfigAliases.get("header"))
        num_data = self.num_data()
        if predictor is not None:
            init_score = predictor.predict(data, raw_score=True, data_has_header=data_has_header, is_reshape=False)
            if used_indices is not None:
                assert not self.need_slice
                if isinstance(data, string_type):
                    sub_init_score = np.zeros(num_data * predictor.num_class, dtype=np.float32)
                    assert num_data == len(used_indices)
                    for i in range(len(used_indices)):
                        for j in range(predictor.num_class):
                            sub_init_score[i * predictor.num_class + j] = \
                                init_score[used_indices[i] * predictor.num_class + j]
                    init_score = sub_init_score
            if predictor.num_class > 1:
                # need to regroup init_score
                new_init_score = np.zeros(init_score.size, dtype=np.float32)
                for i in range(num_data):
                    for j in range(predictor.num_class):
                        new_init_score[j * num_data + i] = init_score[i * predictor.num_class + j]
                init_score = new_init_score
        elif self.init_score is not None:
            init_score = np.zeros(self.init_score.shape, dtype=np.float32)
        else:
            return self
        self.set_init_score(init_score)

    def _lazy_init(self, data, label=None, reference=None, weight=None, group=None, init_score=None,
                   predictor=None, silent=False, feature_name="auto", categorical_feature="auto", params=None):
        if data is None:
            self.handle = None
            return self
        data, label, weight, init_score = (_from_tensor(data), _from_tensor(label), _from_tensor(weight),
                                           _from_tensor(init_score))
        if reference is not None:
            self.pandas_categorical = reference.pandas_categorical
            categorical_feature = reference.categorical_feature
        data, feature_name, categorical_feature, self.pandas_categorical = _data_from_pandas(
            data, feature_name, categorical_feature, self.pandas_categorical)
        label = _label_from_pandas(label)

        # process for args
        params = {} if params is None else params
        args_names = (getattr(self.__class__, "_lazy_init").__code__.co_varnames[
            :getattr(self.__class__, "_lazy_init").__code__.co_argcount])
        for key, _ in params.items():
            if key in args_names:
                warnings.warn("{0} keyword has been found in `params` and will be ignored.\n"
                              "Please use {0} argument of the Dataset constructor to pass this parameter."
                              .format(key))
        # user can set verbose with params, it has higher priority
        if not any(verbose_alias in params for verbose_alias in _ConfigAliases.get("verbosity")) and silent:
            params["verbose"] = -1
        # get categorical features
        if categorical_feature is not None:
            categorical_indices = set()
            feature_dict = {}
            if feature_name is not None:
                feature_dict = {name: i for i, name in enumerate(feature_name)}
            for name in categorical_feature:
                if isinstance(name, string_type) and name in feature_dict:
                    categorical_indices.add(feature_dict[name])
                elif isinstance(name, integer_types):
                    categorical_indices.add(name)
                else:
                    raise TypeError("Wrong type({}) or unknown name({}) in categorical_feature"
                                    .format(type(name).__name__, name))
            if categorical_indices:
                for cat_alias in _ConfigAliases.get("categorical_feature"):
                    if cat_alias in params:
                        warnings.warn("{} in param dict is overridden.".format(cat_alias))
                        params.pop(cat_alias, None)
                params["categorical_column"] = sorted(categorical_indices)

        params_str = param_dict_to_str(params)
        self.params = params
        # process for reference dataset
        ref_dataset = None
        if isinstance(reference, Dataset):
            ref_dataset = reference.construct().handle
        elif reference is not None:
            raise TypeError("Reference dataset should be None or dataset instance")
        # start construct data
        if isinstance(data, string_type):
            self.handle = ctypes.c_void_p()
            _safe_call(_load_lib().LGBM_DatasetCreateFromFile(c_str(data), c_str(params_str), ref_dataset,
                                                              ctypes.byref(self.handle)))
        elif isinstance(data, scipy.sparse.csr_matrix):
            self.__init_from_csr(data, params_str, ref_dataset)
        elif isinstance(data, scipy.sparse.csc_matrix):
            self.__init_from_csc(data, params_str, ref_dataset)
        elif isinstance(data, np.ndarray):
            self.__init_from_np2d(data, params_str, ref_dataset)
        elif isinstance(data, list) and len(data) > 0 and all(isinstance(x, np.ndarray) for x in data):
            self.__init_from_list_np2d(data, params_str, ref_dataset)
        elif isinstance(data, dt_DataTable):
            self.__init_from_np2d(data.to_numpy(), params_str, ref_dataset)
        else:
            try:
                csr = scipy.sparse.csr_matrix(data)
                self.__init_from_csr(csr, params_str, ref_dataset)
            except BaseException:
                raise TypeError("Cannot initialize Dataset from {}".format(type(data).__name__))
        if label is not None:
            self.set_label(label)
        if self.get_label() is None:
            raise ValueError("Label should not be None")
        if weight is not None:
            self.set_weight(weight)
        if group is not None:
            self.set_group(group)
        if isinstance(predictor, _InnerPredictor):
            if self._predictor is None and init_score is not None:
                warnings.warn("The init_score will be overridden by the prediction of init_model.")
            self._set_init_score_by_predictor(predictor, data)
        elif init_score is not None:
            self.set_init_score(init_score)
        elif predictor is not None:
            raise TypeError("Wrong predictor type {}".format(type(predictor).__name__))
        # set feature names
        return self.set_feature_name(feature_name)

    def __init_from_np2d(self, mat, params_str, ref_dataset):
        if len(mat.shape) != 2:
            raise ValueError("Input numpy.ndarray must be 2 dimensional")
        self.handle = ctypes.c_void_p()
        if mat.dtype == np.float32 or mat.dtype == np.float64:
            data = np.asarray(mat.reshape(mat.size), dtype=mat.dtype)
        else:
            data = np.array(mat.reshape(mat.size), dtype=np.float32)
        ptr_data, type_ptr_data, _ = c_float_array(data)
        _safe_call(_load_lib().LGBM_DatasetCreateFromMat(
            ptr_data, ctypes.c_int(type_ptr_data), ctypes.c_int32(mat.shape[0]), ctypes.c_int32(mat.shape[1]),
            ctypes.c_int(1), c_str(params_str), ref_dataset, ctypes.byref(self.handle)))
        return self

    def __init_from_list_np2d(self, mats, params_str, ref_dataset):
        ncol = mats[0].shape[1]
        nrow = np.zeros((len(mats),), np.int32)
        if mats[0].dtype == np.float64:
            ptr_data = (ctypes.POINTER(ctypes.c_double) * len(mats))()
        else:
            ptr_data = (ctypes.POINTER(ctypes.c_float) * len(mats))()
        holders = []
        type_ptr_data = None
        for i, mat in enumerate(mats):
            if len(mat.shape) != 2:
                raise ValueError("Input numpy.ndarray must be 2 dimensional")
            if mat.shape[1] != ncol:
                raise ValueError("Input arrays must have same number of columns")
            nrow[i] = mat.shape[0]
            if mat.dtype == np.float32 or mat.dtype == np.float64:
                mats[i] = np.asarray(mat.reshape(mat.size), dtype=mat.dtype)
            else:
                mats[i] = np.array(mat.reshape(mat.size), dtype=np.float32)
            chunk_ptr_data, chunk_type_ptr_data, holder = c_float_array(mats[i])
            if type_ptr_data is not None and chunk_type_ptr_data != type_ptr_data:
                raise ValueError("Input chunks must have same type")
            ptr_data[i] = chunk_ptr_data
            type_ptr_data = chunk_type_ptr_data
            holders.append(holder)
        self.handle = ctypes.c_void_p()
        _safe_call(_load_lib().LGBM_DatasetCreateFromMats(
            ctypes.c_int32(len(mats)), ctypes.cast(ptr_data, ctypes.POINTER(ctypes.POINTER(ctypes.c_double))),
            ctypes.c_int(type_ptr_data), nrow.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.c_int32(ncol),
            ctypes.c_int(1), c_str(params_str), ref_dataset, ctypes.byref(self.handle)))
        return self

    def __init_from_csr(self, csr, params_str, ref_dataset):
        if len(csr.indices) != len(csr.data):
            raise ValueError("Length mismatch: {} vs {}".format(len(csr.indices), len(csr.data)))
        self.handle = ctypes.c_void_p()
        ptr_indptr, type_ptr_indptr, __ = c_int_array(csr.indptr)
        ptr_data, type_ptr_data, _ = c_float_array(csr.data)
        assert csr.shape[1] <= MAX_INT32
        csr_indices = csr.indices.astype(np.int32, copy=False)
        _safe_call(_load_lib().LGBM_DatasetCreateFromCSR(
            ptr_indptr, ctypes.c_int(type_ptr_indptr), csr_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            ptr_data, ctypes.c_int(type_ptr_data), ctypes.c_int64(len(csr.indptr)), ctypes.c_int64(len(csr.data)),
            ctypes.c_int64(csr.shape[1]), c_str(params_str), ref_dataset, ctypes.byref(self.handle)))
        return self

    def __init_from_csc(self, csc, params_str, ref_dataset):
        if len(csc.indices) != len(csc.data):
            raise ValueError("Length mismatch: {} vs {}".format(len(csc.indices), len(csc.data)))
        self.handle = ctypes.c_void_p()
        ptr_indptr, type_ptr_indptr, __ = c_int_array(csc.indptr)
        ptr_data, type_ptr_data, _ = c_float_array(csc.data)
        assert csc.shape[0] <= MAX_INT32
        csc_indices = csc.indices.astype(np.int32, copy=False)
        _safe_call(_load_lib().LGBM_DatasetCreateFromCSC(
            ptr_indptr, ctypes.c_int(type_ptr_indptr), csc_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
            ptr_data, ctypes.c_int(type_ptr_data), ctypes.c_int64(len(csc.indptr)), ctypes.c_int64(len(csc.data)),
            ctypes.c_int64(csc.shape[0]), c_str(params_str), ref_dataset, ctypes.byref(self.handle)))
        return self

    def construct(self):
        """Lazy init."""
        if self.handle is None:
            if self.reference is not None:
                reference_params = self.reference.get_params()
                if self.get_params() != reference_params:
                    warnings.warn("Overriding the parameters from Reference Dataset.")
                    self._update_params(reference_params)
                if self.used_indices is None:
                    # create valid
                    self._lazy_init(self.data, label=self.label, reference=self.reference, weight=self.weight,
                                    group=self.group, init_score=self.init_score, predictor=self._predictor,
                                    silent=self.silent, feature_name=self.feature_name, params=self.params)
                else:
                    # construct subset
                    used_indices = list_to_1d_numpy(self.used_indices, np.int32, name="used_indices")
                    assert used_indices.flags.c_contiguous
                    if self.reference.group is not None:
                        group_info = np.array(self.reference.group).astype(np.int32, copy=False)
                        _, self.group = np.unique(np.repeat(range(len(group_info)), repeats=group_info)[
                            self.used_indices], return_counts=True)
                    self.handle = ctypes.c_void_p()
                    params_str = param_dict_to_str(self.params)
                    _safe_call(_load_lib().LGBM_DatasetGetSubset(
                        self.reference.construct().handle,
                        used_indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                        ctypes.c_int32(used_indices.shape[0]), c_str(params_str), ctypes.byref(self.handle)))
                    if not self.free_raw_data:
                        self.get_data()
                    if self.group is not None:
                        self.set_group(self.group)
                    if self.get_label() is None:
                        raise ValueError("Label should not be None.")
                    if isinstance(self._predictor, _InnerPredictor) and self._predictor is not self.reference._predictor:
                        self.get_data()
                        self._set_init_score_by_predictor(self._predictor, self.data, used_indices)
            else:
                # create train
                self._lazy_init(self.data, label=self.label, weight=self.weight, group=self.group,
                                init_score=self.init_score, predictor=self._predictor, silent=self.silent,
                                feature_name=self.feature_name, categorical_feature=self.categorical_feature,
                                params=self.params)
            if self.free_raw_data:
                self.data = None
        return self

    def create_valid(self, data, label=None, weight=None, group=None, init_score=None, silent=False, params=None):
        """Create validation data aligned with the current Dataset."""
        ret = Dataset(data, label=label, reference=self, weight=weight, group=group, init_score=init_score,
                      silent=silent, params=params, free_raw_data=self.free_raw_data)
        ret._predictor = self._predictor
        ret.pandas_categorical = self.pandas_categorical
        return ret

    def subset(self, used_indices, params=None):
        """Get subset of current Dataset."""
        if params is None:
            params = self.params
        ret = Dataset(None, reference=self, feature_name=self.feature_name,
                      categorical_feature=self.categorical_feature, params=params, free_raw_data=self.free_raw_data)
        ret._predictor = self._predictor
        ret.pandas_categorical = self.pandas_categorical
        ret.used_indices = sorted(used_indices)
        return ret

    def save_binary(self, filename):
        """Save Dataset to a binary file."""
        _safe_call(_load_lib().LGBM_DatasetSaveBinary(self.construct().handle, c_str(filename)))
        return self

    def _update_params(self, params):
        if not params:
            return self
        params = copy.deepcopy(params)

        def update():
            if not self.params:
                self.params = params
            else:
                self.params_back_up = copy.deepcopy(self.params)
                self.params.update(params)

        if self.handle is None:
            update()
        elif params is not None:
            ret = _load_lib().LGBM_DatasetUpdateParamChecking(c_str(param_dict_to_str(self.params)),
                                                              c_str(param_dict_to_str(params)))
            if ret != 0:
                # could be updated if data is not freed
                if self.data is not None:
                    update()
                    self._free_handle()
                else:
                    raise LightGBMError(_load_lib().LGBM_GetLastError().decode("utf-8"))
        return self

    def _reverse_update_params(self):
        if self.handle is None:
            self.params = copy.deepcopy(self.params_back_up)
            self.params_back_up = None
        return self

    def set_field(self, field_name, data):
        """Set property into the Dataset."""
        if self.handle is None:
            raise Exception("Cannot set %s before construct dataset" % field_name)
        if data is None:
            # set to None
            _safe_call(_load_lib().LGBM_DatasetSetField(self.handle, c_str(field_name), None, ctypes.c_int(0),
                                                        ctypes.c_int(FIELD_TYPE_MAPPER[field_name])))
            return self
        dtype = np.float32
        if field_name == "group":
            dtype = np.int32
        elif field_name == "init_score":
            dtype = np.float64
        data = list_to_1d_numpy(data, dtype, name=field_name)
        if data.dtype == np.float32 or data.dtype == np.float64:
            ptr_data, type_data, _ = c_float_array(data)
        elif data.dtype == np.int32:
            ptr_data, type_data, _ = c_int_array(data)
        else:
            raise TypeError("Expected np.float32/64 or np.int32, met type({})".format(data.dtype))
        if type_data != FIELD_TYPE_MAPPER[field_name]:
            raise TypeError("Input type error for set_field")
        _safe_call(_load_lib().LGBM_DatasetSetField(self.handle, c_str(field_name), ptr_data,
                                                    ctypes.c_int(len(data)), ctypes.c_int(type_data)))
        self.version += 1
        return self

    def get_field(self, field_name):
        """Get property from the Dataset."""
        if self.handle is None:
            raise Exception("Cannot get %s before construct Dataset" % field_name)
        tmp_out_len = ctypes.c_int()
        out_type = ctypes.c_int()
        ret = ctypes.POINTER(ctypes.c_void_p)()
        _safe_call(_load_lib().LGBM_DatasetGetField(self.handle, c_str(field_name), ctypes.byref(tmp_out_len),
                                                    ctypes.byref(ret), ctypes.byref(out_type)))
        if out_type.value != FIELD_TYPE_MAPPER[field_name]:
            raise TypeError("Return type error for get_field")
        if tmp_out_len.value == 0:
            return None
        if out_type.value == C_API_DTYPE_INT32:
            return cint32_array_to_numpy(ctypes.cast(ret, ctypes.POINTER(ctypes.c_int32)), tmp_out_len.value)
        if out_type.value == C_API_DTYPE_FLOAT32:
            return cfloat32_array_to_numpy(ctypes.cast(ret, ctypes.POINTER(ctypes.c_float)), tmp_out_len.value)
        if out_type.value == C_API_DTYPE_FLOAT64:
            return cfloat64_array_to_numpy(ctypes.cast(ret, ctypes.POINTER(ctypes.c_double)), tmp_out_len.value)
        raise TypeError("Unknown type")

    def set_categorical_feature(self, categorical_feature):
        """Set categorical features."""
        if self.categorical_feature == categorical_feature:
            return self
        if self.data is not None:
            if self.categorical_feature is None:
                self.categorical_feature = categorical_feature
                return self._free_handle()
            if categorical_feature == "auto":
                warnings.warn("Using categorical_feature in Dataset.")
                return self
            warnings.warn("categorical_feature in Dataset is overridden.\n"
                          "New categorical_feature is {}".format(sorted(list(categorical_feature))))
            self.categorical_feature = categorical_feature
            return self._free_handle()
        raise LightGBMError("Cannot set categorical feature after freed raw data, "
                            "set free_raw_data=False when construct Dataset to avoid this.")

    def _set_predictor(self, predictor):
        if predictor is self._predictor and (predictor is None or predictor.current_iteration() ==
                                             self._predictor.current_iteration()):
            return self
        if self.handle is None:
            self._predictor = predictor
        elif self.data is not None:
            self._predictor = predictor
            self._set_init_score_by_predictor(self._predictor, self.data)
        elif self.used_indices is not None and self.reference is not None and self.reference.data is not None:
            self._predictor = predictor
            self._set_init_score_by_predictor(self._predictor, self.reference.data, self.used_indices)
        else:
            raise LightGBMError("Cannot set predictor after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        return self

    def set_reference(self, reference):
        """Set reference Dataset."""
        self.set_categorical_feature(reference.categorical_feature) \
            .set_feature_name(reference.feature_name) \
            ._set_predictor(reference._predictor)
        # we're done if self and reference share a common upstrem reference
        if self.get_ref_chain().intersection(reference.get_ref_chain()):
            return self
        if self.data is not None:
            self.reference = reference
            return self._free_handle()
        raise LightGBMError("Cannot set reference after freed raw data, "
                            "set free_raw_data=False when construct Dataset to avoid this.")

    def set_feature_name(self, feature_name):
        """Set feature name."""
        if feature_name != "auto":
            self.feature_name = feature_name
        if self.handle is not None and feature_name is not None and feature_name != "auto":
            if len(feature_name) != self.num_feature():
                raise ValueError("Length of feature_name({}) and num_feature({}) don't match"
                                 .format(len(feature_name), self.num_feature()))
            c_feature_name = [c_str(name) for name in feature_name]
            _safe_call(_load_lib().LGBM_DatasetSetFeatureNames(self.handle, c_array(ctypes.c_char_p, c_feature_name),
                                                               ctypes.c_int(len(feature_name))))
        return self

    def set_label(self, label):
        """Set label of Dataset."""
        self.label = label
        if self.handle is not None:
            label = list_to_1d_numpy(_label_from_pandas(label), name="label")
            self.set_field("label", label)
            self.label = self.get_field("label")  # original values can be modified at cpp side
        return self

    def set_weight(self, weight):
        """Set weight of each instance."""
        if weight is not None and np.all(weight == 1):
            weight = None
        self.weight = weight
        if self.handle is not None:
            if weight is None:
                self.set_field("weight", None)  # clears the native weights
                return self
            weight = list_to_1d_numpy(weight, name="weight")
            self.set_field("weight", weight)
            self.weight = self.get_field("weight")  # original values can be modified at cpp side
        return self

    def set_init_score(self, init_score):
        """Set init score of Booster to start from."""
        self.init_score = init_score
        if self.handle is not None and init_score is None:
            self.set_field("init_score", None)
        elif self.handle is not None:
            init_score = list_to_1d_numpy(init_score, np.float64, name="init_score")
            self.set_field("init_score", init_score)
            self.init_score = self.get_field("init_score")  # original values can be modified at cpp side
        return self

    def set_group(self, group):
        """Set group size of Dataset (used for ranking)."""
        self.group = group
        if self.handle is not None and group is not None:
            group = list_to_1d_numpy(group, np.int32, name="group")
            self.set_field("group", group)
        return self

    def get_feature_name(self):
        """Get the names of columns (features) in the Dataset."""
        if self.handle is None:
            raise LightGBMError("Cannot get feature_name before construct dataset")
        num_feature = self.num_feature()
        tmp_out_len = ctypes.c_int(0)
        reserved_string_buffer_size = 255
        required_string_buffer_size = ctypes.c_size_t(0)
        string_buffers = [ctypes.create_string_buffer(reserved_string_buffer_size) for _ in range(num_feature)]
        ptr_string_buffers = (ctypes.c_char_p * num_feature)(*map(ctypes.addressof, string_buffers))
        _safe_call(_load_lib().LGBM_DatasetGetFeatureNames(
            self.handle, ctypes.c_int(num_feature), ctypes.byref(tmp_out_len),
            ctypes.c_size_t(reserved_string_buffer_size), ctypes.byref(required_string_buffer_size),
            ptr_string_buffers))
        if num_feature != tmp_out_len.value:
            raise ValueError("Length of feature names doesn't equal with num_feature")
        if reserved_string_buffer_size < required_string_buffer_size.value:
            actual = required_string_buffer_size.value
            string_buffers = [ctypes.create_string_buffer(actual) for _ in range(num_feature)]
            ptr_string_buffers = (ctypes.c_char_p * num_feature)(*map(ctypes.addressof, string_buffers))
            _safe_call(_load_lib().LGBM_DatasetGetFeatureNames(
                self.handle, ctypes.c_int(num_feature), ctypes.byref(tmp_out_len), ctypes.c_size_t(actual),
                ctypes.byref(required_string_buffer_size), ptr_string_buffers))
        return [string_buffers[i].value.decode("utf-8") for i in range(num_feature)]

    def get_label(self):
        """Get the label of the Dataset."""
        if self.label is None:
            self.label = self.get_field("label")
        return self.label

    def get_weight(self):
        """Get the weight of the Dataset."""
        if self.weight is None:
            self.weight = self.get_field("weight")
        return self.weight

    def get_init_score(self):
        """Get the initial score of the Dataset."""
        if self.init_score is None:
            self.init_score = self.get_field("init_score")
        return self.init_score

    def get_data(self):
        """Get the raw data of the Dataset."""
        if self.handle is None:
            raise Exception("Cannot get data before construct Dataset")
        if self.need_slice and self.used_indices is not None and self.reference is not None:
            self.data = self.reference.data
            if self.data is not None:
                if isinstance(self.data, np.ndarray) or scipy.sparse.issparse(self.data):
                    self.data = self.data[self.used_indices, :]
                elif isinstance(self.data, pd_DataFrame):
                    self.data = self.data.iloc[self.used_indices].copy()
                elif isinstance(self.data, dt_DataTable):
                    self.data = self.data[self.used_indices, :]
                else:
                    warnings.warn("Cannot subset {} type of raw data.\nReturning original raw data"
                                  .format(type(self.data).__name__))
            self.need_slice = False
        if self.data is None:
            raise LightGBMError("Cannot call `get_data` after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        return self.data

    def get_group(self):
        """Get the group of the Dataset."""
        if self.group is None:
            self.group = self.get_field("group")
            if self.group is not None:
                # group data from LightGBM is boundaries data, need to convert to group size
                self.group = np.diff(self.group)
        return self.group

    def num_data(self):
        """Get the number of rows in the Dataset."""
        if self.handle is not None:
            ret = ctypes.c_int()
            _safe_call(_load_lib().LGBM_DatasetGetNumData(self.handle, ctypes.byref(ret)))
            return ret.value
        raise LightGBMError("Cannot get num_data before construct dataset")

    def num_feature(self):
        """Get the number of columns (features) in the Dataset."""
        if self.handle is not None:
            ret = ctypes.c_int()
            _safe_call(_load_lib().LGBM_DatasetGetNumFeature(self.handle, ctypes.byref(ret)))
            return ret.value
        raise LightGBMError("Cannot get num_feature before construct dataset")

    def get_ref_chain(self, ref_limit=100):
        """Get a chain of Dataset objects."""
        head = self
        ref_chain = set()
        while len(ref_chain) < ref_limit:
            if isinstance(head, Dataset):
                ref_chain.add(head)
                if (head.reference is not None) and (head.reference not in ref_chain):
                    head = head.reference
                else:
                    break
            else:
                break
        return ref_chain

    def add_features_from(self, other):
        """Add features from other Dataset to the current Dataset."""
        if self.handle is None or other.handle is None:
            raise ValueError("Both source and target Datasets must be constructed before adding features")
        _safe_call(_load_lib().LGBM_DatasetAddFeaturesFrom(self.handle, other.handle))
        return self

    def _dump_text(self, filename):
        """Save Dataset to a text file (for debugging)."""
        _safe_call(_load_lib().LGBM_DatasetDumpText(self.construct().handle, c_str(filename)))
        return self


class Booster(object):
    """Booster in LightGBM."""

    def __init__(self, params=None, train_set=None, model_file=None, model_str=None, silent=False):
        self.handle = None
        self.network = False
        self.__need_reload_eval_info = True
        self._train_data_name = "training"
        self.__attr = {}
        self.__set_objective_to_none = False
        self.best_iteration = -1
        self.best_score = {}
        params = {} if params is None else copy.deepcopy(params)
        # user can set verbose with params, it has higher priority
        if not any(verbose_alias in params for verbose_alias in _ConfigAliases.get("verbosity")) and silent:
            params["verbose"] = -1
        if train_set is not None:
            # Training task
            if not isinstance(train_set, Dataset):
                raise TypeError("Training data should be Dataset instance, met {}".format(type(train_set).__name__))
            params_str = param_dict_to_str(params)
            # set network if necessary
            for alias in _ConfigAliases.get("machines"):
                if alias in params:
                    machines = params[alias]
                    if isinstance(machines, string_type):
                        num_machines = len(machines.split(","))
                    elif isinstance(machines, (list, set)):
                        num_machines = len(machines)
                        machines = ",".join(machines)
                    else:
                        raise ValueError("Invalid machines in params.")
                    self.set_network(machines,
                                     local_listen_port=params.get("local_listen_port", 12400),
                                     listen_time_out=params.get("listen_time_out", 120),
                                     num_machines=params.setdefault("num_machines", num_machines))
                    break
            # construct booster object
            train_set.construct()
            # copy the parameters from train_set
            params.update(train_set.get_params())
            params_str = param_dict_to_str(params)
            self.handle = ctypes.c_void_p()
            _safe_call(_load_lib().LGBM_BoosterCreate(train_set.handle, c_str(params_str), ctypes.byref(self.handle)))
            # save reference to data
            self.train_set = train_set
            self.valid_sets = []
            self.name_valid_sets = []
            self.__num_dataset = 1
            self.__init_predictor = train_set._predictor
            if self.__init_predictor is not None:
                _safe_call(_load_lib().LGBM_BoosterMerge(self.handle, self.__init_predictor.handle))
            out_num_class = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterGetNumClasses(self.handle, ctypes.byref(out_num_class)))
            self.__num_class = out_num_class.value
            # buffer for inner predict
            self.__inner_predict_buffer = [None]
            self.__is_predicted_cur_iter = [False]
            self.__get_eval_info()
            self.pandas_categorical = train_set.pandas_categorical
            self.train_set_version = train_set.version
        elif model_file is not None:
            # Prediction task
            out_num_iterations = ctypes.c_int(0)
            self.handle = ctypes.c_void_p()
            _safe_call(_load_lib().LGBM_BoosterCreateFromModelfile(c_str(model_file), ctypes.byref(out_num_iterations),
                                                                   ctypes.byref(self.handle)))
            out_num_class = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterGetNumClasses(self.handle, ctypes.byref(out_num_class)))
            self.__num_class = out_num_class.value
            self.pandas_categorical = _load_pandas_categorical(file_name=model_file)
        elif model_str is not None:
            self.model_from_string(model_str, not silent)
        else:
            raise TypeError("Need at least one training dataset or model file or model string "
                            "to create Booster instance")
        self.params = params

    def __del__(self):
        try:
            if self.network:
                self.free_network()
        except AttributeError:
            pass
        try:
            if self.handle is not None:
                _safe_call(_load_lib().LGBM_BoosterFree(self.handle))
        except AttributeError:
            pass

    def __copy__(self):
        return self.__deepcopy__(None)

    def __deepcopy__(self, _):
        model_str = self.model_to_string(num_iteration=-1)
        booster = Booster(model_str=model_str)
        return booster

    def __getstate__(self):
        this = self.__dict__.copy()
        handle = this["handle"]
        this.pop("train_set", None)
        this.pop("valid_sets", None)
        if handle is not None:
            this["handle"] = self.model_to_string(num_iteration=-1)
        return this

    def __setstate__(self, state):
        model_str = state.get("handle", None)
        if model_str is not None:
            handle = ctypes.c_void_p()
            out_num_iterations = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterLoadModelFromString(c_str(model_str), ctypes.byref(out_num_iterations),
                                                                   ctypes.byref(handle)))
            state["handle"] = handle
        self.__dict__.update(state)

    def free_dataset(self):
        """Free Booster's Datasets."""
        self.__dict__.pop("train_set", None)
        self.__dict__.pop("valid_sets", None)
        self.__num_dataset = 0
        return self

    def _free_buffer(self):
        self.__inner_predict_buffer = []
        self.__is_predicted_cur_iter = []
        return self

    def set_network(self, machines, local_listen_port=12400, listen_time_out=120, num_machines=1):
        """Set the network configuration (TCP mesh)."""
        _safe_call(_load_lib().LGBM_NetworkInit(c_str(machines), ctypes.c_int(local_listen_port),
                                                ctypes.c_int(listen_time_out), ctypes.c_int(num_machines)))
        self.network = True
        return self

    def free_network(self):
        """Free Booster's network."""
        _safe_call(_load_lib().LGBM_NetworkFree())
        self.network = False
        return self

    def trees_to_dataframe(self):
        """Parse the fitted model and return in an easy-to-read pandas DataFrame."""
        if not PANDAS_INSTALLED:
            raise LightGBMError("This method cannot be run without pandas installed")
        from pandas import DataFrame

        if self.num_trees() == 0:
            raise LightGBMError("There are no trees in this Booster and thus nothing to parse")

        def _is_split_node(tree):
            return "split_index" in tree.keys()

        def create_node_record(tree, node_depth=1, tree_index=None, feature_names=None, parent_node=None):
            def _get_node_index(tree, tree_index):
                tree_num = str(tree_index) + "-" if tree_index is not None else ""
                is_split = _is_split_node(tree)
                node_type = "S" if is_split else "L"
                # if a single node tree it won't have `leaf_index` so return 0
                node_num = str(tree.get("split_index" if is_split else "leaf_index", 0))
                return tree_num + node_type + node_num

            def _get_split_feature(tree, feature_names):
                if _is_split_node(tree):
                    if feature_names is not None:
                        feature_name = feature_names[tree["split_feature"]]
                    else:
                        feature_name = tree["split_feature"]
                else:
                    feature_name = None
                return feature_name

            def _is_single_node_tree(tree):
                return set(tree.keys()) == {"leaf_value"}

            node = OrderedDict()
            node["tree_index"] = tree_index
            node["node_depth"] = node_depth
            node["node_index"] = _get_node_index(tree, tree_index)
            node["left_child"] = None
            node["right_child"] = None
            node["parent_index"] = parent_node
            node["split_feature"] = _get_split_feature(tree, feature_names)
            node["split_gain"] = None
            node["threshold"] = None
            node["decision_type"] = None
            node["missing_direction"] = None
            node["missing_type"] = None
            node["value"] = None
            node["weight"] = None
            node["count"] = None
            if _is_split_node(tree):
                node["left_child"] = _get_node_index(tree["left_child"], tree_index)
                node["right_child"] = _get_node_index(tree["right_child"], tree_index)
                node["split_gain"] = tree["split_gain"]
                node["threshold"] = tree["threshold"]
                node["decision_type"] = tree["decision_type"]
                node["missing_direction"] = "left" if tree["default_left"] else "right"
                node["missing_type"] = tree["missing_type"]
                node["value"] = tree["internal_value"]
                node["weight"] = tree["internal_weight"]
                node["count"] = tree["internal_count"]
            else:
                node["value"] = tree["leaf_value"]
                if not _is_single_node_tree(tree):
                    node["weight"] = tree["leaf_weight"]
                    node["count"] = tree["leaf_count"]
            return node

        def tree_dict_to_node_list(tree, node_depth=1, tree_index=None, feature_names=None, parent_node=None):
            node = create_node_record(tree, node_depth=node_depth, tree_index=tree_index,
                                      feature_names=feature_names, parent_node=parent_node)
            res = [node]
            if _is_split_node(tree):
                # traverse the next level of the tree
                children = ["left_child", "right_child"]
                for child in children:
                    subtree_list = tree_dict_to_node_list(tree[child], node_depth=node_depth + 1,
                                                          tree_index=tree_index, feature_names=feature_names,
                                                          parent_node=node["node_index"])
                    # In tree format, "subtree_list" is a list of node records (dicts),
                    # and we add node to the list.
                    res.extend(subtree_list)
            return res

        model_dict = self.dump_model()
        feature_names = model_dict["feature_names"]
        model_list = []
        for tree in model_dict["tree_info"]:
            model_list.extend(tree_dict_to_node_list(tree["tree_structure"], tree_index=tree["tree_index"],
                                                     feature_names=feature_names))
        return DataFrame(model_list, columns=model_list[0].keys())

    def set_train_data_name(self, name):
        """Set the name to the training Dataset."""
        self._train_data_name = name
        return self

    def add_valid(self, data, name):
        """Add validation data."""
        if not isinstance(data, Dataset):
            raise TypeError("Validation data should be Dataset instance, met {}".format(type(data).__name__))
        if data._predictor is not self.__init_predictor:
            raise LightGBMError("Add validation data failed, you should use same predictor for these data")
        _safe_call(_load_lib().LGBM_BoosterAddValidData(self.handle, data.construct().handle))
        self.valid_sets.append(data)
        self.name_valid_sets.append(name)
        self.__num_dataset += 1
        self.__inner_predict_buffer.append(None)
        self.__is_predicted_cur_iter.append(False)
        return self

    def reset_parameter(self, params):
        """Reset parameters of Booster."""
        params_str = param_dict_to_str(params)
        if params_str:
            _safe_call(_load_lib().LGBM_BoosterResetParameter(self.handle, c_str(params_str)))
        self.params.update(params)
        return self

    def update(self, train_set=None, fobj=None):
        """Update Booster for one iteration."""
        # need reset training data
        if train_set is None and self.train_set_version != self.train_set.version:
            train_set = self.train_set
            is_the_same_train_set = False
        else:
            is_the_same_train_set = train_set is self.train_set and self.train_set_version == train_set.version
        if train_set is not None and not is_the_same_train_set:
            if not isinstance(train_set, Dataset):
                raise TypeError("Training data should be Dataset instance, met {}".format(type(train_set).__name__))
            if train_set._predictor is not self.__init_predictor:
                raise LightGBMError("Replace training data failed, you should use same predictor for these data")
            self.train_set = train_set
            _safe_call(_load_lib().LGBM_BoosterResetTrainingData(self.handle, self.train_set.construct().handle))
            self.__inner_predict_buffer[0] = None
            self.train_set_version = self.train_set.version
        is_finished = ctypes.c_int(0)
        if fobj is None:
            if self.__set_objective_to_none:
                raise LightGBMError("Cannot update due to null objective function.")
            _safe_call(_load_lib().LGBM_BoosterUpdateOneIter(self.handle, ctypes.byref(is_finished)))
            self.__is_predicted_cur_iter = [False for _ in range(self.__num_dataset)]
            return is_finished.value == 1
        if not self.__set_objective_to_none:
            self.reset_parameter({"objective": "none"}).__set_objective_to_none = True
        grad, hess = fobj(self.__inner_predict(0), self.train_set)
        return self.__boost(grad, hess)

    def __boost(self, grad, hess):
        grad = list_to_1d_numpy(grad, name="gradient")
        hess = list_to_1d_numpy(hess, name="hessian")
        assert grad.flags.c_contiguous
        assert hess.flags.c_contiguous
        if len(grad) != len(hess):
            raise ValueError("Lengths of gradient({}) and hessian({}) don't match".format(len(grad), len(hess)))
        is_finished = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterUpdateOneIterCustom(
            self.handle, grad.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
            hess.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(is_finished)))
        self.__is_predicted_cur_iter = [False for _ in range(self.__num_dataset)]
        return is_finished.value == 1

    def rollback_one_iter(self):
        """Rollback one iteration."""
        _safe_call(_load_lib().LGBM_BoosterRollbackOneIter(self.handle))
        self.__is_predicted_cur_iter = [False for _ in range(self.__num_dataset)]
        return self

    def current_iteration(self):
        """Get the index of the current iteration."""
        out_cur_iter = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterGetCurrentIteration(self.handle, ctypes.byref(out_cur_iter)))
        return out_cur_iter.value

    def num_model_per_iteration(self):
        """Get number of models per iteration."""
        model_per_iter = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterNumModelPerIteration(self.handle, ctypes.byref(model_per_iter)))
        return model_per_iter.value

    def num_trees(self):
        """Get number of weak sub-models."""
        num_trees = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterNumberOfTotalModel(self.handle, ctypes.byref(num_trees)))
        return num_trees.value

    def upper_bound(self):
        """Get upper bound value of a model."""
        ret = ctypes.c_double(0)
        _safe_call(_load_lib().LGBM_BoosterGetUpperBoundValue(self.handle, ctypes.byref(ret)))
        return ret.value

    def lower_bound(self):
        """Get lower bound value of a model."""
        ret = ctypes.c_double(0)
        _safe_call(_load_lib().LGBM_BoosterGetLowerBoundValue(self.handle, ctypes.byref(ret)))
        return ret.value

    def eval(self, data, name, feval=None):
        """Evaluate for data."""
        if not isinstance(data, Dataset):
            raise TypeError("Can only eval for Dataset instance")
        data_idx = -1
        if data is self.train_set:
            data_idx = 0
        else:
            for i in range(len(self.valid_sets)):
                if data is self.valid_sets[i]:
                    data_idx = i + 1
                    break
        # need to push new valid data
        if data_idx == -1:
            self.add_valid(data, name)
            data_idx = self.__num_dataset - 1
        return self.__inner_eval(name, data_idx, feval)

    def eval_train(self, feval=None):
        """Evaluate for training data."""
        return self.__inner_eval(self._train_data_name, 0, feval)

    def eval_valid(self, feval=None):
        """Evaluate for validation data."""
        return [item for i in range(1, self.__num_dataset)
                for item in self.__inner_eval(self.name_valid_sets[i - 1], i, feval)]

    def save_model(self, filename, num_iteration=None, start_iteration=0, importance_type="split"):
        """Save Booster to file."""
        if num_iteration is None:
            num_iteration = self.best_iteration
        importance_type_int = FEATURE_IMPORTANCE_TYPE_MAPPER[importance_type]
        _safe_call(_load_lib().LGBM_BoosterSaveModel(self.handle, ctypes.c_int(start_iteration),
                                                     ctypes.c_int(num_iteration), ctypes.c_int(importance_type_int),
                                                     c_str(filename)))
        _dump_pandas_categorical(self.pandas_categorical, filename)
        return self

    def shuffle_models(self, start_iteration=0, end_iteration=-1):
        """Shuffle models."""
        _safe_call(_load_lib().LGBM_BoosterShuffleModels(self.handle, ctypes.c_int(start_iteration),
                                                         ctypes.c_int(end_iteration)))
        return self

    def model_from_string(self, model_str, verbose=True):
        """Load Booster from a string."""
        if self.handle is not None:
            _safe_call(_load_lib().LGBM_BoosterFree(self.handle))
        self._free_buffer()
        self.handle = ctypes.c_void_p()
        out_num_iterations = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterLoadModelFromString(c_str(model_str), ctypes.byref(out_num_iterations),
                                                               ctypes.byref(self.handle)))
        out_num_class = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterGetNumClasses(self.handle, ctypes.byref(out_num_class)))
        if verbose:
            print("Finished loading model, total used %d iterations" % int(out_num_iterations.value))
        self.__num_class = out_num_class.value
        self.pandas_categorical = _load_pandas_categorical(model_str=model_str)
        return self

    def model_to_if_else(self, num_iteration=None):
        """Standalone C++ source of the model (the CLI's convert_model task).

        The generated file defines ``extern "C"`` ``lgbm_predict_raw(const double* row,
        double* out)`` and ``lgbm_predict_leaf``; compile it into any program to score rows
        without this library.
        """
        if num_iteration is None:
            num_iteration = self.best_iteration
        with _TempFile() as f:
            _safe_call(_load_lib().LGBM_AMD_BoosterSaveModelToIfElse(self.handle, ctypes.c_int(num_iteration),
                                                                     c_str(f.name)))
            return "".join(f.readlines())

    def model_to_string(self, num_iteration=None, start_iteration=0, importance_type="split"):
        """Save Booster to string."""
        if num_iteration is None:
            num_iteration = self.best_iteration
        importance_type_int = FEATURE_IMPORTANCE_TYPE_MAPPER[importance_type]
        buffer_len = 1 << 20
        tmp_out_len = ctypes.c_int64(0)
        string_buffer = ctypes.create_string_buffer(buffer_len)
        ptr_string_buffer = ctypes.c_char_p(*[ctypes.addressof(string_buffer)])
        _safe_call(_load_lib().LGBM_BoosterSaveModelToString(
            self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), ctypes.c_int(importance_type_int),
            ctypes.c_int64(buffer_len), ctypes.byref(tmp_out_len), ptr_string_buffer))
        actual_len = tmp_out_len.value
        # if buffer length is not long enough, re-allocate a buffer
        if actual_len > buffer_len:
            string_buffer = ctypes.create_string_buffer(actual_len)
            ptr_string_buffer = ctypes.c_char_p(*[ctypes.addressof(string_buffer)])
            _safe_call(_load_lib().LGBM_BoosterSaveModelToString(
                self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                ctypes.c_int(importance_type_int), ctypes.c_int64(actual_len), ctypes.byref(tmp_out_len),
                ptr_string_buffer))
        ret = string_buffer.value.decode("utf-8")
        ret += _dump_pandas_categorical(self.pandas_categorical)
        return ret

    def dump_model(self, num_iteration=None, start_iteration=0, importance_type="split"):
        """Dump Booster to JSON format."""
        if num_iteration is None:
            num_iteration = self.best_iteration
        importance_type_int = FEATURE_IMPORTANCE_TYPE_MAPPER[importance_type]
        buffer_len = 1 << 20
        tmp_out_len = ctypes.c_int64(0)
        string_buffer = ctypes.create_string_buffer(buffer_len)
        ptr_string_buffer = ctypes.c_char_p(*[ctypes.addressof(string_buffer)])
        _safe_call(_load_lib().LGBM_BoosterDumpModel(
            self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration), ctypes.c_int(importance_type_int),
            ctypes.c_int64(buffer_len), ctypes.byref(tmp_out_len), ptr_string_buffer))
        actual_len = tmp_out_len.value
        if actual_len > buffer_len:
            string_buffer = ctypes.create_string_buffer(actual_len)
            ptr_string_buffer = ctypes.c_char_p(*[ctypes.addressof(string_buffer)])
            _safe_call(_load_lib().LGBM_BoosterDumpModel(
                self.handle, ctypes.c_int(start_iteration), ctypes.c_int(num_iteration),
                ctypes.c_int(importance_type_int), ctypes.c_int64(actual_len), ctypes.byref(tmp_out_len),
                ptr_string_buffer))
        ret = json.loads(string_buffer.value.decode("utf-8"))
        ret["pandas_categorical"] = json.loads(json.dumps(self.pandas_categorical, default=_json_default_with_numpy))
        return ret

    def predict(self, data, start_iteration=0, num_iteration=None, raw_score=False, pred_leaf=False,
                pred_contrib=False, data_has_header=False, is_reshape=True, **kwargs):
        """Make a prediction."""
        predictor = self._to_predictor(copy.deepcopy(kwargs))
        if num_iteration is None:
            if start_iteration <= 0:
                num_iteration = self.best_iteration
            else:
                num_iteration = -1
        return predictor.predict(data, start_iteration, num_iteration, raw_score, pred_leaf, pred_contrib,
                                 data_has_header, is_reshape)

    def refit(self, data, label, decay_rate=0.9, **kwargs):
        """Refit the existing Booster by new data."""
        if self.__set_objective_to_none:
            raise LightGBMError("Cannot refit due to null objective function.")
        predictor = self._to_predictor(copy.deepcopy(kwargs))
        leaf_preds = predictor.predict(data, -1, pred_leaf=True)
        nrow, ncol = leaf_preds.shape
        out_is_linear = False  # noqa: F841  (linear trees are not part of this model version)
        train_set = Dataset(data, label, silent=True)
        new_params = copy.deepcopy(self.params)
        new_params["refit_decay_rate"] = decay_rate
        new_booster = Booster(new_params, train_set)
        # Copy models
        _safe_call(_load_lib().LGBM_BoosterMerge(new_booster.handle, predictor.handle))
        leaf_preds = leaf_preds.reshape(-1)
        ptr_data, _, _ = c_int_array(leaf_preds)
        _safe_call(_load_lib().LGBM_BoosterRefit(new_booster.handle, ptr_data, ctypes.c_int32(nrow),
                                                 ctypes.c_int32(ncol)))
        new_booster.network = self.network
        new_booster.__attr = self.__attr.copy()
        return new_booster

    def get_leaf_output(self, tree_id, leaf_id):
        """Get the output of a leaf."""
        ret = ctypes.c_double(0)
        _safe_call(_load_lib().LGBM_BoosterGetLeafValue(self.handle, ctypes.c_int(tree_id), ctypes.c_int(leaf_id),
                                                        ctypes.byref(ret)))
        return ret.value

    def _to_predictor(self, pred_parameter=None):
        predictor = _InnerPredictor(booster_handle=self.handle, pred_parameter=pred_parameter)
        predictor.pandas_categorical = self.pandas_categorical
        return predictor

    def num_feature(self):
        """Get number of features."""
        out_num_feature = ctypes.c_int(0)
        _safe_call(_load_lib().LGBM_BoosterGetNumFeature(self.handle, ctypes.byref(out_num_feature)))
        return out_num_feature.value

    def feature_name(self):
        """Get names of features."""
        num_feature = self.num_feature()
        tmp_out_len = ctypes.c_int(0)
        reserved_string_buffer_size = 255
        required_string_buffer_size = ctypes.c_size_t(0)
        string_buffers = [ctypes.create_string_buffer(reserved_string_buffer_size) for _ in range(num_feature)]
        ptr_string_buffers = (ctypes.c_char_p * num_feature)(*map(ctypes.addressof, string_buffers))
        _safe_call(_load_lib().LGBM_BoosterGetFeatureNames(
            self.handle, ctypes.c_int(num_feature), ctypes.byref(tmp_out_len),
            ctypes.c_size_t(reserved_string_buffer_size), ctypes.byref(required_string_buffer_size),
            ptr_string_buffers))
        if num_feature != tmp_out_len.value:
            raise ValueError("Length of feature names doesn't equal with num_feature")
        if reserved_string_buffer_size < required_string_buffer_size.value:
            actual = required_string_buffer_size.value
            string_buffers = [ctypes.create_string_buffer(actual) for _ in range(num_feature)]
            ptr_string_buffers = (ctypes.c_char_p * num_feature)(*map(ctypes.addressof, string_buffers))
            _safe_call(_load_lib().LGBM_BoosterGetFeatureNames(
                self.handle, ctypes.c_int(num_feature), ctypes.byref(tmp_out_len), ctypes.c_size_t(actual),
                ctypes.byref(required_string_buffer_size), ptr_string_buffers))
        return [string_buffers[i].value.decode("utf-8") for i in range(num_feature)]

    def feature_importance(self, importance_type="split", iteration=None):
        """Get feature importances."""
        if iteration is None:
            iteration = self.best_iteration
        importance_type_int = FEATURE_IMPORTANCE_TYPE_MAPPER[importance_type]
        result = np.zeros(self.num_feature(), dtype=np.float64)
        _safe_call(_load_lib().LGBM_BoosterFeatureImportance(self.handle, ctypes.c_int(iteration),
                                                             ctypes.c_int(importance_type_int),
                                                             result.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
        if importance_type_int == 0:
            return result.astype(np.int32)
        return result

    def get_split_value_histogram(self, feature, bins=None, xgboost_style=False):
        """Get split value histogram for the specified feature."""
        def add(root):
            """Recursively add thresholds."""
            if "split_index" in root:  # non-leaf
                if feature_names is not None and isinstance(feature, string_type):
                    split_feature = feature_names[root["split_feature"]]
                else:
                    split_feature = root["split_feature"]
                if split_feature == feature:
                    if isinstance(root["threshold"], string_type):
                        raise LightGBMError("Cannot compute split value histogram for the categorical feature")
                    values.append(root["threshold"])
                add(root["left_child"])
                add(root["right_child"])

        model = self.dump_model()
        feature_names = model.get("feature_names")
        tree_infos = model["tree_info"]
        values = []
        for tree_info in tree_infos:
            add(tree_info["tree_structure"])

        if bins is None or isinstance(bins, integer_types) and xgboost_style:
            n_unique = len(np.unique(values))
            bins = max(min(n_unique, bins) if bins is not None else n_unique, 1)
        hist, bin_edges = np.histogram(values, bins=bins)
        if xgboost_style:
            ret = np.column_stack((bin_edges[1:], hist))
            ret = ret[ret[:, 1] > 0]
            if PANDAS_INSTALLED:
                from pandas import DataFrame
                return DataFrame(ret, columns=["SplitValue", "Count"])
            return ret
        return hist, bin_edges

    def __inner_eval(self, data_name, data_idx, feval=None):
        if data_idx >= self.__num_dataset:
            raise ValueError("Data_idx should be smaller than number of dataset")
        self.__get_eval_info()
        ret = []
        if self.__num_inner_eval > 0:
            result = np.zeros(self.__num_inner_eval, dtype=np.float64)
            tmp_out_len = ctypes.c_int(0)
            _safe_call(_load_lib().LGBM_BoosterGetEval(self.handle, ctypes.c_int(data_idx), ctypes.byref(tmp_out_len),
                                                       result.ctypes.data_as(ctypes.POINTER(ctypes.c_double))))
            if tmp_out_len.value != self.__num_inner_eval:
                raise ValueError("Wrong length of eval results")
            for i in range(self.__num_inner_eval):
                ret.append((data_name, self.__name_inner_eval[i], result[i], self.__higher_better_inner_eval[i]))
        if callable(feval):
            feval = [feval]
        if feval is not None:
            if data_idx == 0:
                cur_data = self.train_set
            else:
                cur_data = self.valid_sets[data_idx - 1]
            for eval_function in feval:
                if eval_function is None:
                    continue
                feval_ret = eval_function(self.__inner_predict(data_idx), cur_data)
                if isinstance(feval_ret, list):
                    for eval_name, val, is_higher_better in feval_ret:
                        ret.append((data_name, eval_name, val, is_higher_better))
                else:
                    eval_name, val, is_higher_better = feval_ret
                    ret.append((data_name, eval_name, val, is_higher_better))
        return ret

    def __inner_predict(self, data_idx):
        if data_idx >= self.__num_dataset:
            raise ValueError("Data_idx should be smaller than number of dataset")
        if self.__inner_predict_buffer[data_idx] is None:
            if data_idx == 0:
                n_preds = self.train_set.num_data() * self.__num_class
            else:
                n_preds = self.valid_sets[data_idx - 1].num_data() * self.__num_class
            self.__inner_predict_buffer[data_idx] = np.zeros(n_preds, dtype=np.float64)
        # avoid to predict many time in one iteration
        if not self.__is_predicted_cur_iter[data_idx]:
            tmp_out_len = ctypes.c_int64(0)
            data_ptr = self.__inner_predict_buffer[data_idx].ctypes.data_as(ctypes.POINTER(ctypes.c_double))
            _safe_call(_load_lib().LGBM_BoosterGetPredict(self.handle, ctypes.c_int(data_idx), ctypes.byref(tmp_out_len),
                                                          data_ptr))
            if tmp_out_len.value != len(self.__inner_predict_buffer[data_idx]):
                raise ValueError("Wrong length of predict results for data %d" % (data_idx))
            self.__is_predicted_cur_iter[data_idx] = True
        return self.__inner_predict_buffer[data_idx]

    def __get_eval_info(self):
        if self.__need_reload_eval_info:
            self.__need_reload_eval_info = False
            out_num_eval = ctypes.c_int(0)
            # Get num of inner evals
            _safe_call(_load_lib().LGBM_BoosterGetEvalCounts(self.handle, ctypes.byref(out_num_eval)))
            self.__num_inner_eval = out_num_eval.value
            if self.__num_inner_eval > 0:
                # Get name of evals
                tmp_out_len = ctypes.c_int(0)
                reserved_string_buffer_size = 255
                required_string_buffer_size = ctypes.c_size_t(0)
                string_buffers = [ctypes.create_string_buffer(reserved_string_buffer_size)
                                  for _ in range(self.__num_inner_eval)]
                ptr_string_buffers = (ctypes.c_char_p * self.__num_inner_eval)(*map(ctypes.addressof, string_buffers))
                _safe_call(_load_lib().LGBM_BoosterGetEvalNames(
                    self.handle, ctypes.c_int(self.__num_inner_eval), ctypes.byref(tmp_out_len),
                    ctypes.c_size_t(reserved_string_buffer_size), ctypes.byref(required_string_buffer_size),
                    ptr_string_buffers))
                if self.__num_inner_eval != tmp_out_len.value:
                    raise ValueError("Length of eval names doesn't equal with num_evals")
                self.__name_inner_eval = [string_buffers[i].value.decode("utf-8")
                                          for i in range(self.__num_inner_eval)]
                self.__higher_better_inner_eval = [name.startswith(("auc", "ndcg@", "map@", "average_precision"))
                                                   for name in self.__name_inner_eval]

    def attr(self, key):
        """Get attribute string from the Booster."""
        return self.__attr.get(key, None)

    def set_attr(self, **kwargs):
        """Set attributes to the Booster."""
        for key, value in kwargs.items():
            if value is not None:
                if not isinstance(value, string_type):
                    raise ValueError("Only string values are accepted")
                self.__attr[key] = value
            else:
                self.__attr.pop(key, None)
        return self


def get_timers():
    """Phase timers of the native library (enabled with LGBM_AMD_TIMETAG=1) as {name: seconds}."""
    buf = ctypes.create_string_buffer(1 << 16)
    out_len = ctypes.c_int64(0)
    _safe_call(_load_lib().LGBM_AMD_GetTimers(ctypes.c_int64(1 << 16), ctypes.byref(out_len), buf))
    ret = {}
    for item in buf.value.decode("utf-8").split(";"):
        if "=" in item:
            k, v = item.split("=", 1)
            ret[k] = float(v)
    return ret


def device_count():
    """Number of HIP devices visible to the native library (0 without a GPU)."""
    n = ctypes.c_int(0)
    _safe_call(_load_lib().LGBM_AMD_DeviceCount(ctypes.byref(n)))
    return n.value


def device_synchronize():
    """Wait for all work queued on the current HIP device (no-op without a GPU)."""
    _safe_call(_load_lib().LGBM_AMD_DeviceSynchronize())
