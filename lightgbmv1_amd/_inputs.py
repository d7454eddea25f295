"""Input normalisation for Dataset / prediction: torch tensors, pandas frames (with
categorical columns), label / weight / group vectors, and the ``pandas_categorical`` line
that models carry so prediction re-encodes categories exactly as training did (the
reference Python package's model-file convention)."""
import json
import os

import numpy as np

from .compat import pd_DataFrame, pd_Series

_OK_KINDS = ("b", "i", "u", "f")  # numpy dtype kinds a frame column may have
CATEGORICAL_KEY = "pandas_categorical:"


def to_host(x):
    """torch.Tensor (CPU or a HIP device) -> numpy; anything else unchanged.  The library
    bins the values and keeps its own device copy of the binned matrix."""
    if type(x).__module__.startswith("torch") and hasattr(x, "detach"):
        return x.detach().cpu().numpy()
    return x


def is_frame(x):
    return pd_DataFrame is not None and isinstance(x, pd_DataFrame)


def is_series(x):
    return pd_Series is not None and isinstance(x, pd_Series)


def _column_ok(dtype):
    s = str(dtype)
    if s.startswith("Sparse"):
        return True
    try:
        return np.dtype(dtype).kind in _OK_KINDS
    except TypeError:
        return False


def frame_to_array(data, feature_name, categorical_feature, categories):
    """pandas -> (float array, feature names, categorical features, category lists).

    Category columns become their codes (unknown -> NaN).  `categories` is None for a
    training frame (its categories are recorded) and the training lists otherwise (the
    frame's categories are aligned to them).  Non-frames pass through, with "auto"
    resolved to None."""
    if not is_frame(data):
        return (data, None if feature_name == "auto" else feature_name,
                None if categorical_feature == "auto" else categorical_feature, categories)
    if data.ndim != 2 or data.shape[0] < 1:
        raise ValueError("Input data must be 2 dimensional and non empty.")
    if feature_name in ("auto", None):
        data = data.rename(columns=str)
    cat_cols = [c for c, t in zip(data.columns, data.dtypes) if str(t) == "category"]
    unordered = [c for c in cat_cols if not data[c].cat.ordered]
    if categories is None:
        categories = [list(data[c].cat.categories) for c in cat_cols]
    elif len(categories) != len(cat_cols):
        raise ValueError("train and valid dataset categorical_feature do not match.")
    if cat_cols:
        data = data.copy()  # the caller's frame stays as it is
        for col, cats in zip(cat_cols, categories):
            if list(data[col].cat.categories) != list(cats):
                data[col] = data[col].cat.set_categories(cats)
            codes = data[col].cat.codes.astype(np.float64)
            data[col] = codes.where(codes >= 0, np.nan)
    if categorical_feature is not None:
        if feature_name is None:
            feature_name = list(data.columns)
        categorical_feature = unordered if categorical_feature == "auto" else list(categorical_feature)
    if feature_name == "auto":
        feature_name = list(data.columns)
    bad = [str(c) for c, t in zip(data.columns, data.dtypes) if not _column_ok(t)]
    if bad:
        raise ValueError("DataFrame.dtypes for data must be int, float or bool.\n"
                         "Did not expect the data types in the following fields: " + ", ".join(bad))
    arr = data.values
    if arr.dtype not in (np.float32, np.float64):
        arr = arr.astype(np.float32)
    return arr, feature_name, categorical_feature, categories


def label_vector(label):
    """A one-column label frame -> 1-D float32 array; anything else unchanged."""
    if is_frame(label):
        if label.shape[1] > 1:
            raise ValueError("DataFrame for label cannot have multiple columns")
        if not all(_column_ok(t) for t in label.dtypes):
            raise ValueError("DataFrame.dtypes for label must be int, float or bool")
        return np.ravel(label.values.astype(np.float32, copy=False))
    return label


def vector(data, dtype, name):
    """list / 1-D array / Series -> 1-D numpy array of `dtype`."""
    data = to_host(data)
    if is_series(data):
        if not _column_ok(data.dtype):
            raise ValueError("Series.dtypes must be int, float or bool")
        return np.asarray(data, dtype=dtype)
    if isinstance(data, np.ndarray) and data.ndim == 1:
        return data if data.dtype == dtype else data.astype(dtype)
    if isinstance(data, (list, tuple)):
        return np.asarray(data, dtype=dtype)
    raise TypeError("Wrong type({}) for {}.\nIt should be list, numpy 1-D array or pandas Series".format(
        type(data).__name__, name))


def _json_safe(obj):
    if isinstance(obj, (np.integer, np.floating, np.bool_)):
        return obj.item()
    if isinstance(obj, np.ndarray):
        return obj.tolist()
    return obj


def categories_line(categories):
    """The trailing model line recording the training frame's category lists."""
    return "\n" + CATEGORICAL_KEY + json.dumps(categories, default=_json_safe) + "\n"


def categories_json(categories):
    return json.loads(json.dumps(categories, default=_json_safe))


def categories_from_text(text):
    """Category lists from the last non-empty line(s) of a model text, or None."""
    for line in reversed(text.rstrip().splitlines()[-2:]):
        line = line.strip()
        if line.startswith(CATEGORICAL_KEY):
            return json.loads(line[len(CATEGORICAL_KEY):])
    return None


def categories_from_file(path):
    """Same, reading only the end of a (possibly large) model file."""
    size = os.path.getsize(path)
    chunk = 4096
    with open(path, "rb") as f:
        while True:
            f.seek(max(0, size - chunk))
            tail = f.read().decode("utf-8", errors="replace")
            if chunk >= size or tail.count("\n") >= 3:
                return categories_from_text(tail)
            chunk *= 4
