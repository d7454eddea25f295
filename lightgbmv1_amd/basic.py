"""Dataset, Booster and the prediction front end (the LightGBM v3 Python API; reference
python-package/lightgbm/basic.py defines the public contract -- lazy Dataset construction,
reference datasets for validation binning, pandas categorical handling, Booster training /
evaluation / prediction / model IO -- implemented here over the C API of
``lib_lightgbmv1_amd.so``).  With ``device_type='gpu'`` training runs on the MI355X learner.

Layout: `_native` (ctypes calls, enum codes, buffers), `_inputs` (torch / pandas / vector
normalisation), and here the three objects built on them:
  * `Dataset`: a recipe (raw data + fields + params) that `construct()` turns into a native
    handle through one of the builders in `_BUILDERS` (file, dense, list of dense, CSR,
    CSC) or as a row subset of a constructed reference;
  * `_InnerPredictor`: prediction over a native booster handle, dispatched on the input
    kind (`_PREDICT_KINDS`), with the SHAP sparse output re-assembled per class;
  * `Booster`: a native booster plus the Python-side caches of evaluation metadata and of
    per-dataset scores used by custom objectives / metrics.
"""
import copy
import ctypes
import json
import os
import tempfile
import warnings
from collections import OrderedDict

import numpy as np
import scipy.sparse

from . import _inputs as inp
from . import _native as nat
from ._native import LightGBMError
from .compat import PANDAS_INSTALLED, dt_DataTable, integer_types, string_type
from .utils.param_table import PARAMETERS as _PARAMETERS

__all__ = ["Dataset", "Booster", "LightGBMError", "get_timers", "device_count", "device_synchronize"]


def _load_lib():
    """The native library (kept for callers that use the C API directly)."""
    return nat.lib()


def _safe_call(ret):
    nat.check(ret)


class _ConfigAliases:
    """Parameter alias table, generated from the single parameter spec (tools/param_spec.py)."""

    aliases = {name: {name} | set(spec["aliases"]) for name, spec in _PARAMETERS.items()}
    aliases.setdefault("group_column", {"group_column", "group", "group_id", "query_column", "query", "query_id"})

    @classmethod
    def get(cls, *names):
        out = set()
        for n in names:
            out |= cls.aliases.get(n, {n})
        return out


def _any_alias(params, name):
    return any(params.get(a) for a in _ConfigAliases.get(name))


def _quiet(params, silent):
    """`silent` means verbose=-1 unless the params set a verbosity themselves."""
    if silent and not any(a in params for a in _ConfigAliases.get("verbosity")):
        params["verbose"] = -1
    return params


# ---------------------------------------------------------------------------------- data
_DATASET_PARAMS = ("bin_construct_sample_cnt", "categorical_feature", "data_random_seed", "enable_bundle",
                   "feature_pre_filter", "forcedbins_filename", "group_column", "header", "ignore_column",
                   "is_enable_sparse", "label_column", "max_bin", "max_bin_by_feature", "min_data_in_bin",
                   "pre_partition", "two_round", "use_missing", "weight_column", "zero_as_missing")

# field name -> numpy dtype on the Python side and the C API dtype code the library stores
_FIELDS = {"label": (np.float32, nat.DTYPE_FLOAT32), "weight": (np.float32, nat.DTYPE_FLOAT32),
           "init_score": (np.float64, nat.DTYPE_FLOAT64), "group": (np.int32, nat.DTYPE_INT32)}


def _dense_block(mat):
    """2-D array -> (contiguous row-major float32/64 buffer, rows, cols)."""
    mat = np.asarray(mat)
    if mat.ndim != 2:
        raise ValueError("Input numpy.ndarray must be 2 dimensional")
    if mat.dtype not in (np.float32, np.float64):
        mat = mat.astype(np.float32)
    if isinstance(mat.base, np.ndarray) and not mat.flags.c_contiguous:
        warnings.warn("Usage of np.ndarray subset (sliced data) is not recommended "
                      "due to it will double the peak memory cost in LightGBM.")
    return np.ascontiguousarray(mat).reshape(-1), mat.shape[0], mat.shape[1]


def _sparse_parts(m):
    """(indptr, int32 indices, data) buffers of a CSR / CSC matrix, kept alive by the caller."""
    if len(m.indices) != len(m.data):
        raise ValueError("Length mismatch: {} vs {}".format(len(m.indices), len(m.data)))
    return (nat.as_index_vector(m.indptr), np.ascontiguousarray(m.indices, dtype=np.int32),
            nat.as_float_vector(m.data))


def _build_from_file(data, params_str, ref):
    out = ctypes.c_void_p()
    nat.call("LGBM_DatasetCreateFromFile", nat.cstr(data), nat.cstr(params_str), ref, ctypes.byref(out))
    return out


def _build_from_dense(data, params_str, ref):
    buf, nrow, ncol = _dense_block(data)
    ptr, code = nat.pointer(buf)
    out = ctypes.c_void_p()
    nat.call("LGBM_DatasetCreateFromMat", ptr, nat.c_int(code), ctypes.c_int32(nrow), ctypes.c_int32(ncol),
             nat.c_int(1), nat.cstr(params_str), ref, ctypes.byref(out))
    return out


def _build_from_blocks(blocks, params_str, ref):
    flat = [_dense_block(b) for b in blocks]
    ncol = flat[0][2]
    if any(f[2] != ncol for f in flat):
        raise ValueError("Input arrays must have same number of columns")
    dtype = flat[0][0].dtype
    if any(f[0].dtype != dtype for f in flat):
        raise ValueError("Input chunks must have same type")
    code = nat.pointer(flat[0][0])[1]
    elem = ctypes.c_double if dtype == np.float64 else ctypes.c_float
    ptrs = (ctypes.POINTER(elem) * len(flat))(*[f[0].ctypes.data_as(ctypes.POINTER(elem)) for f in flat])
    rows = np.array([f[1] for f in flat], dtype=np.int32)
    out = ctypes.c_void_p()
    nat.call("LGBM_DatasetCreateFromMats", ctypes.c_int32(len(flat)),
             ctypes.cast(ptrs, ctypes.POINTER(ctypes.POINTER(ctypes.c_double))), nat.c_int(code),
             rows.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.c_int32(ncol), nat.c_int(1),
             nat.cstr(params_str), ref, ctypes.byref(out))
    return out


def _build_from_sparse(m, params_str, ref):
    indptr, indices, values = _sparse_parts(m)
    p_ptr, p_code = nat.pointer(indptr)
    v_ptr, v_code = nat.pointer(values)
    csr = scipy.sparse.isspmatrix_csr(m)
    out = ctypes.c_void_p()
    nat.call("LGBM_DatasetCreateFromCSR" if csr else "LGBM_DatasetCreateFromCSC", p_ptr, nat.c_int(p_code),
             indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), v_ptr, nat.c_int(v_code),
             ctypes.c_int64(len(indptr)), ctypes.c_int64(len(values)), ctypes.c_int64(m.shape[1] if csr else m.shape[0]),
             nat.cstr(params_str), ref, ctypes.byref(out))
    return out


def _input_kind(data):
    """Which builder / predictor handles `data` (None: try converting to CSR)."""
    if isinstance(data, string_type):
        return "file"
    if scipy.sparse.isspmatrix_csr(data):
        return "csr"
    if scipy.sparse.isspmatrix_csc(data):
        return "csc"
    if isinstance(data, np.ndarray):
        return "dense"
    if dt_DataTable is not None and isinstance(data, dt_DataTable):
        return "datatable"
    if isinstance(data, list):
        if data and all(isinstance(x, np.ndarray) for x in data):
            return "blocks"
        return "list"
    return None


_BUILDERS = {
    "file": _build_from_file,
    "dense": _build_from_dense,
    "blocks": _build_from_blocks,
    "csr": _build_from_sparse,
    "csc": _build_from_sparse,
    "datatable": lambda d, p, r: _build_from_dense(d.to_numpy(), p, r),
}


class Dataset:
    """Training / validation data, constructed lazily on the native side."""

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
        self.used_indices = None   # row subset of `reference` (Dataset.subset)
        self.need_slice = True     # self.data not yet sliced from the reference's raw data
        self._predictor = None     # init_model predictor: its raw scores become init_score
        self.pandas_categorical = None
        self.params_back_up = None
        self.version = 0           # bumped by field updates (Booster.update re-syncs)

    def __del__(self):
        try:
            self._free_handle()
        except Exception:  # noqa: BLE001 -- interpreter shutdown
            pass

    # ------------------------------------------------------------------ construction
    def get_params(self):
        """The parameters that shape the binned data (those a validation set must share)."""
        if not self.params:
            return {}
        keys = _ConfigAliases.get(*_DATASET_PARAMS)
        return {k: v for k, v in self.params.items() if k in keys}

    def _free_handle(self):
        if self.handle is not None:
            nat.call("LGBM_DatasetFree", self.handle)
            self.handle = None
        self.need_slice = True
        if self.used_indices is not None:
            self.data = None
        return self

    def construct(self):
        """Build the native dataset if not built yet; returns self."""
        if self.handle is not None:
            return self
        if self.reference is None:
            self._build(self.data, self.label, None, self.weight, self.group, self.init_score, self._predictor,
                        self.feature_name, self.categorical_feature, self.params)
        else:
            ref_params = self.reference.get_params()
            if self.get_params() != ref_params:
                warnings.warn("Overriding the parameters from Reference Dataset.")
                self._update_params(ref_params)
            if self.used_indices is None:
                self._build(self.data, self.label, self.reference, self.weight, self.group, self.init_score,
                            self._predictor, self.feature_name, "auto", self.params)
            else:
                self._build_subset()
        if self.free_raw_data:
            self.data = None
        return self

    def _build(self, data, label, reference, weight, group, init_score, predictor, feature_name,
               categorical_feature, params):
        if data is None:
            self.handle = None
            return self
        data, label, weight, init_score = (inp.to_host(x) for x in (data, label, weight, init_score))
        if reference is not None:
            self.pandas_categorical = reference.pandas_categorical
            categorical_feature = reference.categorical_feature
        data, feature_name, categorical_feature, self.pandas_categorical = inp.frame_to_array(
            data, feature_name, categorical_feature, self.pandas_categorical)
        label = inp.label_vector(label)
        params = {} if params is None else params
        for key in params:
            if key in ("data", "label", "reference", "weight", "group", "init_score", "predictor",
                       "feature_name", "categorical_feature", "silent"):
                warnings.warn("{0} keyword has been found in `params` and will be ignored.\n"
                              "Please use {0} argument of the Dataset constructor to pass this parameter."
                              .format(key))
        _quiet(params, self.silent)
        cat_idx = self._categorical_indices(categorical_feature, feature_name)
        if cat_idx:
            for alias in _ConfigAliases.get("categorical_feature"):
                if alias in params:
                    warnings.warn("{} in param dict is overridden.".format(alias))
                    params.pop(alias)
            params["categorical_column"] = sorted(cat_idx)
        self.params = params
        if reference is not None and not isinstance(reference, Dataset):
            raise TypeError("Reference dataset should be None or dataset instance")
        ref_handle = reference.construct().handle if reference is not None else None
        kind = _input_kind(data)
        if kind == "list":
            kind = None
        if kind is None:
            try:
                data = scipy.sparse.csr_matrix(data)
            except Exception:  # noqa: BLE001
                raise TypeError("Cannot initialize Dataset from {}".format(type(data).__name__))
            kind = "csr"
        self.handle = _BUILDERS[kind](data, nat.params_str(params), ref_handle)
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
            self._init_score_from(predictor, data)
        elif init_score is not None:
            self.set_init_score(init_score)
        elif predictor is not None:
            raise TypeError("Wrong predictor type {}".format(type(predictor).__name__))
        return self.set_feature_name(feature_name)

    @staticmethod
    def _categorical_indices(categorical_feature, feature_name):
        if categorical_feature is None:
            return set()
        index_of = {name: i for i, name in enumerate(feature_name or [])}
        out = set()
        for c in categorical_feature:
            if isinstance(c, string_type) and c in index_of:
                out.add(index_of[c])
            elif isinstance(c, integer_types):
                out.add(int(c))
            else:
                raise TypeError("Wrong type({}) or unknown name({}) in categorical_feature".format(
                    type(c).__name__, c))
        return out

    def _build_subset(self):
        idx = np.ascontiguousarray(inp.vector(self.used_indices, np.int32, "used_indices"))
        if self.reference.group is not None:
            # group sizes of the subset: the reference's query of every kept row
            query_of_row = np.repeat(np.arange(len(self.reference.group)), np.asarray(self.reference.group))
            _, self.group = np.unique(query_of_row[idx], return_counts=True)
        self.handle = ctypes.c_void_p()
        nat.call("LGBM_DatasetGetSubset", self.reference.construct().handle,
                 idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ctypes.c_int32(len(idx)),
                 nat.cstr(nat.params_str(self.params)), ctypes.byref(self.handle))
        if not self.free_raw_data:
            self.get_data()
        if self.group is not None:
            self.set_group(self.group)
        if self.get_label() is None:
            raise ValueError("Label should not be None.")
        if isinstance(self._predictor, _InnerPredictor) and self._predictor is not self.reference._predictor:
            self.get_data()
            self._init_score_from(self._predictor, self.data, idx)

    def _init_score_from(self, predictor, data, used_indices=None):
        """Raw scores of the init_model on this dataset's rows (class-major for the library)."""
        header = isinstance(data, string_type) and _any_alias(self.params or {}, "header")
        n = self.num_data()
        if predictor is None:
            if self.init_score is not None:
                self.set_init_score(np.zeros(np.shape(self.init_score), dtype=np.float32))
            return self
        k = predictor.num_class
        score = predictor.predict(data, raw_score=True, data_has_header=header, is_reshape=False)
        if used_indices is not None and isinstance(data, string_type):
            score = score.reshape(-1, k)[used_indices].reshape(-1)
        if k > 1:
            score = score.reshape(n, k).T.reshape(-1)  # row-major (row, class) -> class-major
        return self.set_init_score(score.astype(np.float32))

    def create_valid(self, data, label=None, weight=None, group=None, init_score=None, silent=False, params=None):
        """A validation Dataset binned like this one."""
        ret = Dataset(data, label=label, reference=self, weight=weight, group=group, init_score=init_score,
                      silent=silent, params=params, free_raw_data=self.free_raw_data)
        ret._predictor = self._predictor
        ret.pandas_categorical = self.pandas_categorical
        return ret

    def subset(self, used_indices, params=None):
        """A Dataset of some rows of this one (shares its bin mappers)."""
        ret = Dataset(None, reference=self, feature_name=self.feature_name,
                      categorical_feature=self.categorical_feature,
                      params=self.params if params is None else params, free_raw_data=self.free_raw_data)
        ret._predictor = self._predictor
        ret.pandas_categorical = self.pandas_categorical
        ret.used_indices = sorted(used_indices)
        return ret

    def save_binary(self, filename):
        """Write the binned dataset (reloadable as a data file)."""
        nat.call("LGBM_DatasetSaveBinary", self.construct().handle, nat.cstr(filename))
        return self

    def _update_params(self, params):
        if not params:
            return self
        params = copy.deepcopy(params)
        if self.handle is None:
            if self.params:
                self.params_back_up = copy.deepcopy(self.params)
                self.params.update(params)
            else:
                self.params = params
            return self
        ok = nat.lib().LGBM_DatasetUpdateParamChecking(nat.cstr(nat.params_str(self.params)),
                                                       nat.cstr(nat.params_str(params)))
        if ok != 0:
            if self.data is None:  # the binned data cannot be rebuilt
                nat.check(ok)
            self.params_back_up = copy.deepcopy(self.params)
            self.params.update(params)
            self._free_handle()
        return self

    def _reverse_update_params(self):
        if self.handle is None:
            self.params = copy.deepcopy(self.params_back_up)
            self.params_back_up = None
        return self

    # ------------------------------------------------------------------ fields
    def set_field(self, field_name, data):
        """Store a field (label, weight, init_score, group) on the native dataset."""
        if self.handle is None:
            raise Exception("Cannot set %s before construct dataset" % field_name)
        np_dtype, code = _FIELDS[field_name]
        if data is None:
            nat.call("LGBM_DatasetSetField", self.handle, nat.cstr(field_name), None, nat.c_int(0), nat.c_int(code))
            return self
        arr = np.ascontiguousarray(inp.vector(data, np_dtype, field_name))
        ptr, got = nat.pointer(arr)
        if got != code:
            raise TypeError("Input type error for set_field")
        nat.call("LGBM_DatasetSetField", self.handle, nat.cstr(field_name), ptr, nat.c_int(len(arr)), nat.c_int(code))
        self.version += 1
        return self

    def get_field(self, field_name):
        """A field of the native dataset as a numpy array (None if unset)."""
        if self.handle is None:
            raise Exception("Cannot get %s before construct Dataset" % field_name)
        n = ctypes.c_int(0)
        code = ctypes.c_int(0)
        ptr = ctypes.c_void_p()
        nat.call("LGBM_DatasetGetField", self.handle, nat.cstr(field_name), ctypes.byref(n), ctypes.byref(ptr),
                 ctypes.byref(code))
        if code.value != _FIELDS[field_name][1]:
            raise TypeError("Return type error for get_field")
        return nat.copy_out(ptr, n.value, code.value) if n.value else None

    def set_label(self, label):
        self.label = label
        if self.handle is not None:
            self.set_field("label", inp.vector(inp.label_vector(label), np.float32, "label"))
            self.label = self.get_field("label")  # as the library stored it
        return self

    def set_weight(self, weight):
        if weight is not None and np.all(np.asarray(inp.to_host(weight)) == 1):
            weight = None  # unit weights: none
        self.weight = weight
        if self.handle is not None:
            self.set_field("weight", None if weight is None else inp.vector(weight, np.float32, "weight"))
            if weight is not None:
                self.weight = self.get_field("weight")
        return self

    def set_init_score(self, init_score):
        self.init_score = init_score
        if self.handle is not None:
            self.set_field("init_score", None if init_score is None else
                           inp.vector(init_score, np.float64, "init_score"))
            if init_score is not None:
                self.init_score = self.get_field("init_score")
        return self

    def set_group(self, group):
        self.group = group
        if self.handle is not None and group is not None:
            self.set_field("group", inp.vector(group, np.int32, "group"))
        return self

    def get_label(self):
        if self.label is None:
            self.label = self.get_field("label")
        return self.label

    def get_weight(self):
        if self.weight is None:
            self.weight = self.get_field("weight")
        return self.weight

    def get_init_score(self):
        if self.init_score is None:
            self.init_score = self.get_field("init_score")
        return self.init_score

    def get_group(self):
        """Group sizes (the library keeps query boundaries)."""
        if self.group is None:
            bounds = self.get_field("group")
            self.group = np.diff(bounds) if bounds is not None else None
        return self.group

    def get_data(self):
        """The raw data (sliced from the reference's for a subset)."""
        if self.handle is None:
            raise Exception("Cannot get data before construct Dataset")
        if self.need_slice and self.used_indices is not None and self.reference is not None:
            src = self.reference.data
            if src is not None:
                if isinstance(src, np.ndarray) or scipy.sparse.issparse(src):
                    src = src[self.used_indices, :]
                elif inp.is_frame(src):
                    src = src.iloc[self.used_indices].copy()
                elif dt_DataTable is not None and isinstance(src, dt_DataTable):
                    src = src[self.used_indices, :]
                else:
                    warnings.warn("Cannot subset {} type of raw data.\nReturning original raw data".format(
                        type(src).__name__))
            self.data = src
            self.need_slice = False
        if self.data is None:
            raise LightGBMError("Cannot call `get_data` after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        return self.data

    # ------------------------------------------------------------------ features / links
    def set_categorical_feature(self, categorical_feature):
        if self.categorical_feature == categorical_feature:
            return self
        if self.data is None:
            raise LightGBMError("Cannot set categorical feature after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        if self.categorical_feature is None:
            self.categorical_feature = categorical_feature
            return self._free_handle()
        if categorical_feature == "auto":
            warnings.warn("Using categorical_feature in Dataset.")
            return self
        warnings.warn("categorical_feature in Dataset is overridden.\nNew categorical_feature is {}".format(
            sorted(categorical_feature)))
        self.categorical_feature = categorical_feature
        return self._free_handle()

    def _set_predictor(self, predictor):
        same = predictor is self._predictor and (
            predictor is None or predictor.current_iteration() == self._predictor.current_iteration())
        if same:
            return self
        if self.handle is None:
            self._predictor = predictor
        elif self.data is not None:
            self._predictor = predictor
            self._init_score_from(predictor, self.data)
        elif self.used_indices is not None and self.reference is not None and self.reference.data is not None:
            self._predictor = predictor
            self._init_score_from(predictor, self.reference.data, self.used_indices)
        else:
            raise LightGBMError("Cannot set predictor after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        return self

    def set_reference(self, reference):
        self.set_categorical_feature(reference.categorical_feature).set_feature_name(reference.feature_name)
        self._set_predictor(reference._predictor)
        if self.get_ref_chain() & reference.get_ref_chain():
            return self  # already binned with the same upstream reference
        if self.data is None:
            raise LightGBMError("Cannot set reference after freed raw data, "
                                "set free_raw_data=False when construct Dataset to avoid this.")
        self.reference = reference
        return self._free_handle()

    def set_feature_name(self, feature_name):
        if feature_name != "auto":
            self.feature_name = feature_name
        if self.handle is not None and feature_name not in (None, "auto"):
            if len(feature_name) != self.num_feature():
                raise ValueError("Length of feature_name({}) and num_feature({}) don't match".format(
                    len(feature_name), self.num_feature()))
            nat.call("LGBM_DatasetSetFeatureNames", self.handle, nat.string_array(list(feature_name)),
                     nat.c_int(len(feature_name)))
        return self

    def get_feature_name(self):
        if self.handle is None:
            raise LightGBMError("Cannot get feature_name before construct dataset")
        return nat.read_names(lambda n, got, size, need, bufs: nat.call(
            "LGBM_DatasetGetFeatureNames", self.handle, n, got, size, need, bufs), self.num_feature())

    def num_data(self):
        if self.handle is None:
            raise LightGBMError("Cannot get num_data before construct dataset")
        out = ctypes.c_int(0)
        nat.call("LGBM_DatasetGetNumData", self.handle, ctypes.byref(out))
        return out.value

    def num_feature(self):
        if self.handle is None:
            raise LightGBMError("Cannot get num_feature before construct dataset")
        out = ctypes.c_int(0)
        nat.call("LGBM_DatasetGetNumFeature", self.handle, ctypes.byref(out))
        return out.value

    def get_ref_chain(self, ref_limit=100):
        """This dataset and its chain of references."""
        chain, node = set(), self
        while isinstance(node, Dataset) and node not in chain and len(chain) < ref_limit:
            chain.add(node)
            node = node.reference
        return chain

    def add_features_from(self, other):
        if self.handle is None or other.handle is None:
            raise ValueError("Both source and target Datasets must be constructed before adding features")
        nat.call("LGBM_DatasetAddFeaturesFrom", self.handle, other.handle)
        return self

    def _dump_text(self, filename):
        nat.call("LGBM_DatasetDumpText", self.construct().handle, nat.cstr(filename))
        return self


# ---------------------------------------------------------------------------- predict
def _num_preds(handle, nrow, ptype, start, num):
    if nrow > nat.MAX_INT32:
        raise LightGBMError("LightGBM cannot perform prediction for data with number of rows greater than "
                            "MAX_INT32 (%d).\nYou can split your data into chunks and then concatenate "
                            "predictions for them" % nat.MAX_INT32)
    out = ctypes.c_int64(0)
    nat.call("LGBM_BoosterCalcNumPredict", handle, nat.c_int(nrow), nat.c_int(ptype), nat.c_int(start),
             nat.c_int(num), ctypes.byref(out))
    return out.value


class _InnerPredictor:
    """Prediction over a native booster: from a model file (owned handle) or a Booster's
    handle (borrowed)."""

    def __init__(self, model_file=None, booster_handle=None, pred_parameter=None):
        self.handle = ctypes.c_void_p()
        self._owns = model_file is not None
        if model_file is not None:
            iters = ctypes.c_int(0)
            nat.call("LGBM_BoosterCreateFromModelfile", nat.cstr(model_file), ctypes.byref(iters),
                     ctypes.byref(self.handle))
            self.num_total_iteration = iters.value
            self.pandas_categorical = inp.categories_from_file(model_file)
        elif booster_handle is not None:
            self.handle = booster_handle
            self.num_total_iteration = self.current_iteration()
            self.pandas_categorical = None
        else:
            raise TypeError("Need model_file or booster_handle to create a predictor")
        k = ctypes.c_int(0)
        nat.call("LGBM_BoosterGetNumClasses", self.handle, ctypes.byref(k))
        self.num_class = k.value
        self.pred_parameter = nat.params_str(pred_parameter or {})

    def __del__(self):
        try:
            if self._owns:
                nat.call("LGBM_BoosterFree", self.handle)
        except Exception:  # noqa: BLE001
            pass

    def __getstate__(self):
        state = self.__dict__.copy()
        state.pop("handle", None)
        return state

    def current_iteration(self):
        out = ctypes.c_int(0)
        nat.call("LGBM_BoosterGetCurrentIteration", self.handle, ctypes.byref(out))
        return out.value

    def predict(self, data, start_iteration=0, num_iteration=-1, raw_score=False, pred_leaf=False,
                pred_contrib=False, data_has_header=False, is_reshape=True):
        if isinstance(data, Dataset):
            raise TypeError("Cannot use Dataset instance for prediction, please use raw data instead")
        data = inp.frame_to_array(inp.to_host(data), None, None, self.pandas_categorical)[0]
        ptype = (nat.PREDICT_CONTRIB if pred_contrib else nat.PREDICT_LEAF_INDEX if pred_leaf
                 else nat.PREDICT_RAW_SCORE if raw_score else nat.PREDICT_NORMAL)
        kind = _input_kind(data)
        if kind == "list":
            try:
                data = np.array(data)
            except Exception:  # noqa: BLE001
                raise ValueError("Cannot convert data list to numpy array.")
            kind = "dense"
        elif kind == "datatable":
            data, kind = data.to_numpy(), "dense"
        elif kind is None:
            try:
                warnings.warn("Converting data to scipy sparse matrix.")
                data, kind = scipy.sparse.csr_matrix(data), "csr"
            except Exception:  # noqa: BLE001
                raise TypeError("Cannot predict data for type {}".format(type(data).__name__))
        if kind == "file":
            preds, nrow = self._predict_file(data, data_has_header, ptype, start_iteration, num_iteration)
        elif kind in ("csr", "csc"):
            preds, nrow = self._predict_sparse(data, ptype, start_iteration, num_iteration)
        else:
            preds, nrow = self._predict_dense(data, ptype, start_iteration, num_iteration)
        if pred_leaf:
            preds = preds.astype(np.int32)
        if is_reshape and isinstance(preds, np.ndarray) and preds.size != nrow:
            if preds.size % nrow:
                raise ValueError("Length of predict result (%d) cannot be divide nrow (%d)" % (preds.size, nrow))
            preds = preds.reshape(nrow, -1)
        return preds

    def _predict_file(self, path, header, ptype, start, num):
        fd, out_path = tempfile.mkstemp(prefix="lgbm_amd_pred_")
        os.close(fd)
        try:
            nat.call("LGBM_BoosterPredictForFile", self.handle, nat.cstr(path), nat.c_int(1 if header else 0),
                     nat.c_int(ptype), nat.c_int(start), nat.c_int(num), nat.cstr(self.pred_parameter),
                     nat.cstr(out_path))
            with open(out_path) as f:
                rows = [line.split("\t") for line in f.read().splitlines() if line]
        finally:
            os.remove(out_path)
        return np.asarray([float(v) for r in rows for v in r], dtype=np.float64), len(rows)

    def _predict_dense(self, mat, ptype, start, num):
        mat = np.asarray(mat)
        if mat.ndim != 2:
            raise ValueError("Input numpy.ndarray or list must be 2 dimensional")
        nrow = mat.shape[0]
        # the C API takes int32 row counts: cut very tall inputs into chunks
        bounds = list(range(0, nrow, nat.MAX_INT32)) + [nrow]
        counts = [_num_preds(self.handle, b - a, ptype, start, num) for a, b in zip(bounds[:-1], bounds[1:])]
        out = np.zeros(sum(counts), dtype=np.float64)
        at = 0
        for (a, b), cnt in zip(zip(bounds[:-1], bounds[1:]), counts):
            buf, rows, cols = _dense_block(mat[a:b])
            ptr, code = nat.pointer(buf)
            got = ctypes.c_int64(0)
            view = out[at:at + cnt]
            nat.call("LGBM_BoosterPredictForMat", self.handle, ptr, nat.c_int(code), ctypes.c_int32(rows),
                     ctypes.c_int32(cols), nat.c_int(1), nat.c_int(ptype), nat.c_int(start), nat.c_int(num),
                     nat.cstr(self.pred_parameter), ctypes.byref(got), view.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
            if got.value != cnt:
                raise ValueError("Wrong length for predict results")
            at += cnt
        return out, nrow

    def _predict_sparse(self, m, ptype, start, num):
        csr = scipy.sparse.isspmatrix_csr(m)
        nrow = m.shape[0]
        if not csr and nrow > nat.MAX_INT32:
            return self._predict_sparse(m.tocsr(), ptype, start, num)
        indptr, indices, values = _sparse_parts(m)
        p_ptr, p_code = nat.pointer(indptr)
        v_ptr, v_code = nat.pointer(values)
        i_ptr = indices.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        ncross = m.shape[1] if csr else m.shape[0]  # columns (CSR) or rows (CSC)
        common = (p_ptr, ctypes.c_int32(p_code), i_ptr, v_ptr, nat.c_int(v_code), ctypes.c_int64(len(indptr)),
                  ctypes.c_int64(len(values)), ctypes.c_int64(ncross), nat.c_int(ptype), nat.c_int(start),
                  nat.c_int(num), nat.cstr(self.pred_parameter))
        if ptype == nat.PREDICT_CONTRIB:
            return self._contrib_sparse(m, csr, common, p_code, v_code), nrow
        cnt = _num_preds(self.handle, nrow, ptype, start, num)
        out = np.zeros(cnt, dtype=np.float64)
        got = ctypes.c_int64(0)
        nat.call("LGBM_BoosterPredictForCSR" if csr else "LGBM_BoosterPredictForCSC", self.handle, *common,
                 ctypes.byref(got), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        if got.value != cnt:
            raise ValueError("Wrong length for predict results")
        return out, nrow

    def _contrib_sparse(self, m, csr, common, p_code, v_code):
        """SHAP values of sparse input as sparse matrices (one per class if multiclass)."""
        out_indptr = ctypes.c_void_p()
        out_indices = ctypes.c_void_p()
        out_data = ctypes.c_void_p()
        shape = np.zeros(2, dtype=np.int64)
        nat.call("LGBM_BoosterPredictSparseOutput", self.handle, *common,
                 nat.c_int(nat.MATRIX_CSR if csr else nat.MATRIX_CSC),
                 shape.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), ctypes.byref(out_indptr),
                 ctypes.byref(out_indices), ctypes.byref(out_data))
        nnz, nptr = int(shape[0]), int(shape[1])
        try:
            indptr = nat.copy_out(out_indptr, nptr, p_code)
            indices = nat.copy_out(out_indices, nnz, nat.DTYPE_INT32)
            values = nat.copy_out(out_data, nnz, v_code)
        finally:
            nat.call("LGBM_BoosterFreePredictSparse", out_indptr, out_indices, out_data, nat.c_int(p_code),
                     nat.c_int(v_code))
        shape_k = (m.shape[0], m.shape[1] + 1)
        make = scipy.sparse.csr_matrix if csr else scipy.sparse.csc_matrix
        if self.num_class <= 1:
            return make((values, indices, indptr), shape_k)
        # the classes' compressed arrays are concatenated, each indptr with its own offsets
        per = (shape_k[0] if csr else shape_k[1]) + 1
        mats = []
        for c in range(self.num_class):
            p = indptr[c * per:(c + 1) * per]
            lo, hi = p[0], p[-1]
            mats.append(make((values[lo:hi], indices[lo:hi], p - lo), shape_k))
        return mats


# ----------------------------------------------------------------------------- booster
class _EvalInfo:
    """Names / directions of the booster's built-in metrics (loaded once)."""

    def __init__(self):
        self.names = None
        self.higher_better = None

    def load(self, handle):
        if self.names is not None:
            return self
        n = ctypes.c_int(0)
        nat.call("LGBM_BoosterGetEvalCounts", handle, ctypes.byref(n))
        self.names = [] if n.value == 0 else nat.read_names(
            lambda c, got, size, need, bufs: nat.call("LGBM_BoosterGetEvalNames", handle, c, got, size, need, bufs),
            n.value)
        self.higher_better = [nm.startswith(("auc", "ndcg@", "map@", "average_precision")) for nm in self.names]
        return self


class _ScoreCache:
    """Raw scores of the training / validation datasets, fetched once per iteration (for
    custom objectives and metrics)."""

    def __init__(self):
        self.buffers = []
        self.fresh = []

    def add(self):
        self.buffers.append(None)
        self.fresh.append(False)

    def invalidate(self):
        self.fresh = [False] * len(self.buffers)

    def get(self, handle, idx, n):
        if self.buffers[idx] is None:
            self.buffers[idx] = np.zeros(n, dtype=np.float64)
        if not self.fresh[idx]:
            got = ctypes.c_int64(0)
            nat.call("LGBM_BoosterGetPredict", handle, nat.c_int(idx), ctypes.byref(got),
                     self.buffers[idx].ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
            if got.value != n:
                raise ValueError("Wrong length of predict results for data %d" % idx)
            self.fresh[idx] = True
        return self.buffers[idx]


def _network_params(params):
    """machines=... in params: (machine list string, count) or None."""
    for alias in _ConfigAliases.get("machines"):
        if alias in params:
            m = params[alias]
            if isinstance(m, string_type):
                return m, len(m.split(","))
            if isinstance(m, (list, set, tuple)):
                return ",".join(m), len(m)
            raise ValueError("Invalid machines in params.")
    return None


class Booster:
    """A gradient boosting model: trained from a Dataset, or loaded from a file / string."""

    def __init__(self, params=None, train_set=None, model_file=None, model_str=None, silent=False):
        self.handle = None
        self.network = False
        self._train_data_name = "training"
        self._attrs = {}
        self._objective_none = False  # a custom objective replaced the built-in one
        self.best_iteration = -1
        self.best_score = {}
        self._evals = _EvalInfo()
        self._scores = _ScoreCache()
        self._num_class = 1
        self._init_predictor = None
        params = _quiet({} if params is None else copy.deepcopy(params), silent)
        if train_set is not None:
            if not isinstance(train_set, Dataset):
                raise TypeError("Training data should be Dataset instance, met {}".format(type(train_set).__name__))
            net = _network_params(params)
            if net is not None:
                self.set_network(net[0], local_listen_port=params.get("local_listen_port", 12400),
                                 listen_time_out=params.get("listen_time_out", 120),
                                 num_machines=params.setdefault("num_machines", net[1]))
            train_set.construct()
            params.update(train_set.get_params())
            self.handle = ctypes.c_void_p()
            nat.call("LGBM_BoosterCreate", train_set.handle, nat.cstr(nat.params_str(params)),
                     ctypes.byref(self.handle))
            self.train_set = train_set
            self.valid_sets = []
            self.name_valid_sets = []
            self._scores.add()
            self._init_predictor = train_set._predictor
            if self._init_predictor is not None:
                nat.call("LGBM_BoosterMerge", self.handle, self._init_predictor.handle)
            self._num_class = self._query_int("LGBM_BoosterGetNumClasses")
            self._evals.load(self.handle)
            self.pandas_categorical = train_set.pandas_categorical
            self.train_set_version = train_set.version
        elif model_file is not None:
            iters = ctypes.c_int(0)
            self.handle = ctypes.c_void_p()
            nat.call("LGBM_BoosterCreateFromModelfile", nat.cstr(model_file), ctypes.byref(iters),
                     ctypes.byref(self.handle))
            self._num_class = self._query_int("LGBM_BoosterGetNumClasses")
            self.pandas_categorical = inp.categories_from_file(model_file)
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
        except Exception:  # noqa: BLE001
            pass
        try:
            if self.handle is not None:
                nat.call("LGBM_BoosterFree", self.handle)
        except Exception:  # noqa: BLE001
            pass

    def __copy__(self):
        return self.__deepcopy__(None)

    def __deepcopy__(self, _):
        return Booster(model_str=self.model_to_string(num_iteration=-1))

    def __getstate__(self):
        state = self.__dict__.copy()
        state.pop("train_set", None)
        state.pop("valid_sets", None)
        if state.get("handle") is not None:
            state["handle"] = self.model_to_string(num_iteration=-1)
        return state

    def __setstate__(self, state):
        text = state.get("handle")
        if text is not None:
            handle = ctypes.c_void_p()
            nat.call("LGBM_BoosterLoadModelFromString", nat.cstr(text), ctypes.byref(ctypes.c_int(0)),
                     ctypes.byref(handle))
            state["handle"] = handle
        self.__dict__.update(state)

    def _query_int(self, fn):
        out = ctypes.c_int(0)
        nat.call(fn, self.handle, ctypes.byref(out))
        return out.value

    def _query_double(self, fn):
        out = ctypes.c_double(0)
        nat.call(fn, self.handle, ctypes.byref(out))
        return out.value

    def _num_datasets(self):
        return len(self._scores.buffers)

    # ------------------------------------------------------------------ data / network
    def free_dataset(self):
        self.__dict__.pop("train_set", None)
        self.__dict__.pop("valid_sets", None)
        self._scores = _ScoreCache()
        return self

    def _free_buffer(self):
        self._scores = _ScoreCache()
        return self

    def set_network(self, machines, local_listen_port=12400, listen_time_out=120, num_machines=1):
        """Join a TCP mesh of training machines."""
        nat.call("LGBM_NetworkInit", nat.cstr(machines), nat.c_int(local_listen_port), nat.c_int(listen_time_out),
                 nat.c_int(num_machines))
        self.network = True
        return self

    def free_network(self):
        nat.call("LGBM_NetworkFree")
        self.network = False
        return self

    def set_train_data_name(self, name):
        self._train_data_name = name
        return self

    def add_valid(self, data, name):
        if not isinstance(data, Dataset):
            raise TypeError("Validation data should be Dataset instance, met {}".format(type(data).__name__))
        if data._predictor is not self._init_predictor:
            raise LightGBMError("Add validation data failed, you should use same predictor for these data")
        nat.call("LGBM_BoosterAddValidData", self.handle, data.construct().handle)
        self.valid_sets.append(data)
        self.name_valid_sets.append(name)
        self._scores.add()
        return self

    def reset_parameter(self, params):
        text = nat.params_str(params)
        if text:
            nat.call("LGBM_BoosterResetParameter", self.handle, nat.cstr(text))
        self.params.update(params)
        return self

    # ------------------------------------------------------------------ training
    def update(self, train_set=None, fobj=None):
        """One boosting iteration; True when training cannot continue."""
        stale = self.train_set_version != self.train_set.version
        if train_set is None and stale:
            train_set = self.train_set
        if train_set is not None and (train_set is not self.train_set or stale):
            if not isinstance(train_set, Dataset):
                raise TypeError("Training data should be Dataset instance, met {}".format(type(train_set).__name__))
            if train_set._predictor is not self._init_predictor:
                raise LightGBMError("Replace training data failed, you should use same predictor for these data")
            self.train_set = train_set
            nat.call("LGBM_BoosterResetTrainingData", self.handle, train_set.construct().handle)
            self._scores.buffers[0] = None
            self.train_set_version = train_set.version
        if fobj is None:
            if self._objective_none:
                raise LightGBMError("Cannot update due to null objective function.")
            finished = ctypes.c_int(0)
            nat.call("LGBM_BoosterUpdateOneIter", self.handle, ctypes.byref(finished))
            self._scores.invalidate()
            return finished.value == 1
        if not self._objective_none:
            self.reset_parameter({"objective": "none"})
            self._objective_none = True
        grad, hess = fobj(self._dataset_scores(0), self.train_set)
        return self._boost_custom(grad, hess)

    def _boost_custom(self, grad, hess):
        grad = np.ascontiguousarray(inp.vector(grad, np.float32, "gradient"))
        hess = np.ascontiguousarray(inp.vector(hess, np.float32, "hessian"))
        if len(grad) != len(hess):
            raise ValueError("Lengths of gradient({}) and hessian({}) don't match".format(len(grad), len(hess)))
        finished = ctypes.c_int(0)
        nat.call("LGBM_BoosterUpdateOneIterCustom", self.handle, grad.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                 hess.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), ctypes.byref(finished))
        self._scores.invalidate()
        return finished.value == 1

    def rollback_one_iter(self):
        nat.call("LGBM_BoosterRollbackOneIter", self.handle)
        self._scores.invalidate()
        return self

    def current_iteration(self):
        return self._query_int("LGBM_BoosterGetCurrentIteration")

    def num_model_per_iteration(self):
        return self._query_int("LGBM_BoosterNumModelPerIteration")

    def num_trees(self):
        return self._query_int("LGBM_BoosterNumberOfTotalModel")

    def upper_bound(self):
        return self._query_double("LGBM_BoosterGetUpperBoundValue")

    def lower_bound(self):
        return self._query_double("LGBM_BoosterGetLowerBoundValue")

    # ------------------------------------------------------------------ evaluation
    def _dataset_scores(self, idx):
        ds = self.train_set if idx == 0 else self.valid_sets[idx - 1]
        return self._scores.get(self.handle, idx, ds.num_data() * self._num_class)

    def _evaluate(self, name, idx, feval):
        if idx >= self._num_datasets():
            raise ValueError("Data_idx should be smaller than number of dataset")
        info = self._evals.load(self.handle)
        out = []
        if info.names:
            vals = np.zeros(len(info.names), dtype=np.float64)
            got = ctypes.c_int(0)
            nat.call("LGBM_BoosterGetEval", self.handle, nat.c_int(idx), ctypes.byref(got),
                     vals.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
            if got.value != len(info.names):
                raise ValueError("Wrong length of eval results")
            out += [(name, m, v, hb) for m, v, hb in zip(info.names, vals, info.higher_better)]
        fns = [feval] if callable(feval) else (feval or [])
        if fns:
            data = self.train_set if idx == 0 else self.valid_sets[idx - 1]
            for fn in fns:
                if fn is None:
                    continue
                res = fn(self._dataset_scores(idx), data)
                for metric, val, hb in (res if isinstance(res, list) else [res]):
                    out.append((name, metric, val, hb))
        return out

    def eval(self, data, name, feval=None):
        if not isinstance(data, Dataset):
            raise TypeError("Can only eval for Dataset instance")
        if data is self.train_set:
            idx = 0
        else:
            idx = next((i + 1 for i, v in enumerate(self.valid_sets) if v is data), -1)
            if idx < 0:
                self.add_valid(data, name)
                idx = self._num_datasets() - 1
        return self._evaluate(name, idx, feval)

    def eval_train(self, feval=None):
        return self._evaluate(self._train_data_name, 0, feval)

    def eval_valid(self, feval=None):
        return [r for i, nm in enumerate(self.name_valid_sets) for r in self._evaluate(nm, i + 1, feval)]

    # ------------------------------------------------------------------ model IO
    def _iterations(self, num_iteration):
        return self.best_iteration if num_iteration is None else num_iteration

    def save_model(self, filename, num_iteration=None, start_iteration=0, importance_type="split"):
        nat.call("LGBM_BoosterSaveModel", self.handle, nat.c_int(start_iteration),
                 nat.c_int(self._iterations(num_iteration)), nat.c_int(nat.IMPORTANCE_TYPES[importance_type]),
                 nat.cstr(filename))
        with open(filename, "a") as f:
            f.write(inp.categories_line(self.pandas_categorical))
        return self

    def model_to_string(self, num_iteration=None, start_iteration=0, importance_type="split"):
        args = (self.handle, nat.c_int(start_iteration), nat.c_int(self._iterations(num_iteration)),
                nat.c_int(nat.IMPORTANCE_TYPES[importance_type]))
        text = nat.read_string(lambda size, need, buf: nat.call("LGBM_BoosterSaveModelToString", *args, size, need, buf))
        return text + inp.categories_line(self.pandas_categorical)

    def dump_model(self, num_iteration=None, start_iteration=0, importance_type="split"):
        args = (self.handle, nat.c_int(start_iteration), nat.c_int(self._iterations(num_iteration)),
                nat.c_int(nat.IMPORTANCE_TYPES[importance_type]))
        out = json.loads(nat.read_string(lambda size, need, buf: nat.call("LGBM_BoosterDumpModel", *args, size, need,
                                                                          buf)))
        out["pandas_categorical"] = inp.categories_json(self.pandas_categorical)
        return out

    def model_from_string(self, model_str, verbose=True):
        if self.handle is not None:
            nat.call("LGBM_BoosterFree", self.handle)
        self._free_buffer()
        self.handle = ctypes.c_void_p()
        iters = ctypes.c_int(0)
        nat.call("LGBM_BoosterLoadModelFromString", nat.cstr(model_str), ctypes.byref(iters), ctypes.byref(self.handle))
        self._num_class = self._query_int("LGBM_BoosterGetNumClasses")
        if verbose:
            print("Finished loading model, total used %d iterations" % iters.value)
        self.pandas_categorical = inp.categories_from_text(model_str)
        return self

    def model_to_if_else(self, num_iteration=None):
        """Standalone C++ source of the model (the CLI's convert_model task): it defines
        ``extern "C"`` ``lgbm_predict_raw(const double* row, double* out)`` and
        ``lgbm_predict_leaf``, so rows can be scored without this library."""
        fd, path = tempfile.mkstemp(prefix="lgbm_amd_ifelse_", suffix=".cpp")
        os.close(fd)
        try:
            nat.call("LGBM_AMD_BoosterSaveModelToIfElse", self.handle, nat.c_int(self._iterations(num_iteration)),
                     nat.cstr(path))
            with open(path) as f:
                return f.read()
        finally:
            os.remove(path)

    def shuffle_models(self, start_iteration=0, end_iteration=-1):
        nat.call("LGBM_BoosterShuffleModels", self.handle, nat.c_int(start_iteration), nat.c_int(end_iteration))
        return self

    # ------------------------------------------------------------------ prediction
    def _to_predictor(self, pred_parameter=None):
        pred = _InnerPredictor(booster_handle=self.handle, pred_parameter=pred_parameter)
        pred.pandas_categorical = self.pandas_categorical
        return pred

    def predict(self, data, start_iteration=0, num_iteration=None, raw_score=False, pred_leaf=False,
                pred_contrib=False, data_has_header=False, is_reshape=True, **kwargs):
        """Predictions for raw data (numpy, pandas, scipy sparse, lists, torch tensors or a file)."""
        if num_iteration is None:
            num_iteration = self.best_iteration if start_iteration <= 0 else -1
        return self._to_predictor(copy.deepcopy(kwargs)).predict(
            data, start_iteration, num_iteration, raw_score, pred_leaf, pred_contrib, data_has_header, is_reshape)

    def refit(self, data, label, decay_rate=0.9, **kwargs):
        """A copy of the model with leaf values refitted on new data."""
        if self._objective_none:
            raise LightGBMError("Cannot refit due to null objective function.")
        pred = self._to_predictor(copy.deepcopy(kwargs))
        leaves = pred.predict(data, -1, pred_leaf=True)
        nrow, ncol = leaves.shape
        params = copy.deepcopy(self.params)
        params["refit_decay_rate"] = decay_rate
        refitted = Booster(params, Dataset(data, label, silent=True))
        nat.call("LGBM_BoosterMerge", refitted.handle, pred.handle)
        flat = np.ascontiguousarray(leaves.reshape(-1), dtype=np.int32)
        nat.call("LGBM_BoosterRefit", refitted.handle, flat.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                 ctypes.c_int32(nrow), ctypes.c_int32(ncol))
        refitted.network = self.network
        refitted._attrs = dict(self._attrs)
        return refitted

    def get_leaf_output(self, tree_id, leaf_id):
        out = ctypes.c_double(0)
        nat.call("LGBM_BoosterGetLeafValue", self.handle, nat.c_int(tree_id), nat.c_int(leaf_id), ctypes.byref(out))
        return out.value

    # ------------------------------------------------------------------ introspection
    def num_feature(self):
        return self._query_int("LGBM_BoosterGetNumFeature")

    def feature_name(self):
        return nat.read_names(lambda n, got, size, need, bufs: nat.call(
            "LGBM_BoosterGetFeatureNames", self.handle, n, got, size, need, bufs), self.num_feature())

    def feature_importance(self, importance_type="split", iteration=None):
        kind = nat.IMPORTANCE_TYPES[importance_type]
        out = np.zeros(self.num_feature(), dtype=np.float64)
        nat.call("LGBM_BoosterFeatureImportance", self.handle, nat.c_int(self._iterations(iteration)),
                 nat.c_int(kind), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        return out.astype(np.int32) if kind == 0 else out

    def _walk_trees(self):
        """(tree index, node dict, depth, parent node id) over every node of the JSON dump."""
        model = self.dump_model()
        for info in model["tree_info"]:
            stack = [(info["tree_structure"], 1, None)]
            while stack:
                node, depth, parent = stack.pop()
                yield info["tree_index"], node, depth, parent, model.get("feature_names")
                if "split_index" in node:
                    me = "{}-S{}".format(info["tree_index"], node["split_index"])
                    stack.append((node["right_child"], depth + 1, me))
                    stack.append((node["left_child"], depth + 1, me))

    def get_split_value_histogram(self, feature, bins=None, xgboost_style=False):
        """Histogram of the thresholds the model uses for one numerical feature."""
        values = []
        for _, node, _, _, names in self._walk_trees():
            if "split_index" not in node:
                continue
            f = node["split_feature"]
            if names is not None and isinstance(feature, string_type):
                f = names[f]
            if f == feature:
                if isinstance(node["threshold"], string_type):
                    raise LightGBMError("Cannot compute split value histogram for the categorical feature")
                values.append(node["threshold"])
        if bins is None or (isinstance(bins, integer_types) and xgboost_style):
            n_unique = len(np.unique(values))
            bins = max(min(n_unique, bins) if bins is not None else n_unique, 1)
        hist, edges = np.histogram(values, bins=bins)
        if not xgboost_style:
            return hist, edges
        table = np.column_stack((edges[1:], hist))
        table = table[table[:, 1] > 0]
        if PANDAS_INSTALLED:
            from pandas import DataFrame
            return DataFrame(table, columns=["SplitValue", "Count"])
        return table

    def trees_to_dataframe(self):
        """One row per node of every tree (pandas DataFrame)."""
        if not PANDAS_INSTALLED:
            raise LightGBMError("This method cannot be run without pandas installed")
        if self.num_trees() == 0:
            raise LightGBMError("There are no trees in this Booster and thus nothing to parse")
        from pandas import DataFrame

        def node_id(tree, node):
            split = "split_index" in node
            return "{}-{}{}".format(tree, "S" if split else "L", node.get("split_index" if split else "leaf_index", 0))

        rows = []
        for tree, node, depth, parent, names in self._walk_trees():
            split = "split_index" in node
            row = OrderedDict([
                ("tree_index", tree), ("node_depth", depth), ("node_index", node_id(tree, node)),
                ("left_child", node_id(tree, node["left_child"]) if split else None),
                ("right_child", node_id(tree, node["right_child"]) if split else None),
                ("parent_index", parent),
                ("split_feature", (names[node["split_feature"]] if names is not None else node["split_feature"])
                 if split else None),
                ("split_gain", node.get("split_gain") if split else None),
                ("threshold", node.get("threshold") if split else None),
                ("decision_type", node.get("decision_type") if split else None),
                ("missing_direction", ("left" if node["default_left"] else "right") if split else None),
                ("missing_type", node.get("missing_type") if split else None),
                ("value", node["internal_value"] if split else node["leaf_value"]),
                ("weight", node["internal_weight"] if split else node.get("leaf_weight")),
                ("count", node["internal_count"] if split else node.get("leaf_count")),
            ])
            rows.append(row)
        return DataFrame(rows, columns=list(rows[0].keys()))

    def attr(self, key):
        return self._attrs.get(key)

    def set_attr(self, **kwargs):
        for key, value in kwargs.items():
            if value is None:
                self._attrs.pop(key, None)
            elif not isinstance(value, string_type):
                raise ValueError("Only string values are accepted")
            else:
                self._attrs[key] = value
        return self


# ------------------------------------------------------------------------ device helpers
def get_timers():
    """Phase timers of the native library (enabled with LGBM_AMD_TIMETAG=1) as {name: seconds}."""
    text = nat.read_string(lambda size, need, buf: nat.call("LGBM_AMD_GetTimers", size, need, buf), 1 << 16)
    return {k: float(v) for k, v in (item.split("=", 1) for item in text.split(";") if "=" in item)}


def device_count():
    """Number of HIP devices visible to the native library (0 without a GPU)."""
    n = ctypes.c_int(0)
    nat.call("LGBM_AMD_DeviceCount", ctypes.byref(n))
    return n.value


def device_synchronize():
    """Wait for all work queued on the current HIP device (no-op without a GPU)."""
    nat.call("LGBM_AMD_DeviceSynchronize")
