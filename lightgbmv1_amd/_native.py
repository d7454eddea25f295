"""ctypes layer over ``lib_lightgbmv1_amd.so`` (C API: include/lgbm_amd/c_api.h).

Everything the Python classes need from the native side goes through here: loading the
library (and routing its log output to Python), error checking, the C API's enum codes,
numpy <-> pointer conversion, parameter serialisation and the two-pass string-buffer
protocol of the ``Get...Names`` / ``SaveModelToString`` calls.
"""
import ctypes

import numpy as np

from .libpath import find_lib_path


class LightGBMError(Exception):
    """Error raised by the native library."""


# C API enum values (c_api.h)
DTYPE_FLOAT32, DTYPE_FLOAT64, DTYPE_INT32, DTYPE_INT64 = 0, 1, 2, 3
PREDICT_NORMAL, PREDICT_RAW_SCORE, PREDICT_LEAF_INDEX, PREDICT_CONTRIB = 0, 1, 2, 3
MATRIX_CSR, MATRIX_CSC = 0, 1
IMPORTANCE_TYPES = {"split": 0, "gain": 1}
MAX_INT32 = (1 << 31) - 1

# numpy dtype -> (ctypes element type, C API dtype code)
_NP_TO_C = {
    np.dtype(np.float32): (ctypes.c_float, DTYPE_FLOAT32),
    np.dtype(np.float64): (ctypes.c_double, DTYPE_FLOAT64),
    np.dtype(np.int32): (ctypes.c_int32, DTYPE_INT32),
    np.dtype(np.int64): (ctypes.c_int64, DTYPE_INT64),
}
_C_TO_NP = {code: dt for dt, (_, code) in _NP_TO_C.items()}
_C_ELEM = {code: ct for (ct, code) in _NP_TO_C.values()}


class _Library:
    """The loaded native library; attribute access returns its functions."""

    def __init__(self):
        self._dll = None
        self._log_cb = None

    def dll(self):
        if self._dll is None:
            dll = ctypes.cdll.LoadLibrary(find_lib_path()[0])
            dll.LGBM_GetLastError.restype = ctypes.c_char_p

            def _forward(msg):
                print(msg.decode("utf-8"), end="")

            self._log_cb = ctypes.CFUNCTYPE(None, ctypes.c_char_p)(_forward)
            if dll.LGBM_RegisterLogCallback(self._log_cb) != 0:
                raise LightGBMError(dll.LGBM_GetLastError().decode("utf-8"))
            self._dll = dll
        return self._dll


_LIBRARY = _Library()


def lib():
    """The native library (loaded on first use)."""
    return _LIBRARY.dll()


def check(ret):
    """Raise the library's last error if a C API call failed."""
    if ret != 0:
        raise LightGBMError(lib().LGBM_GetLastError().decode("utf-8"))


def call(name, *args):
    """Call C API function `name` and check its status."""
    check(getattr(lib(), name)(*args))


def cstr(s):
    return ctypes.c_char_p(s.encode("utf-8"))


def c_int(v):
    return ctypes.c_int(int(v))


def pointer(arr, allowed=None):
    """(typed pointer, dtype code) of a C-contiguous 1-D numpy array of a C API dtype."""
    if arr.dtype not in _NP_TO_C or (allowed is not None and arr.dtype not in allowed):
        raise TypeError("unsupported array dtype {}".format(arr.dtype))
    if not arr.flags.c_contiguous:
        raise ValueError("array must be C-contiguous")
    ctype, code = _NP_TO_C[arr.dtype]
    return arr.ctypes.data_as(ctypes.POINTER(ctype)), code


def as_float_vector(arr):
    """float32 / float64 stay, anything else becomes float32; contiguous 1-D."""
    arr = np.asarray(arr)
    if arr.dtype not in (np.float32, np.float64):
        arr = arr.astype(np.float32)
    return np.ascontiguousarray(arr.reshape(-1))


def as_index_vector(arr):
    """int32 / int64 stay, anything else becomes int32; contiguous 1-D."""
    arr = np.asarray(arr)
    if arr.dtype not in (np.int32, np.int64):
        arr = arr.astype(np.int32)
    return np.ascontiguousarray(arr.reshape(-1))


def copy_out(ptr, length, code):
    """numpy copy of `length` elements behind a native pointer of dtype `code`."""
    typed = ctypes.cast(ptr, ctypes.POINTER(_C_ELEM[code]))
    return np.ctypeslib.as_array(typed, shape=(length,)).copy() if length else np.zeros(0, _C_TO_NP[code])


def params_str(params):
    """``key=value`` pairs separated by spaces (lists comma-joined, nested lists bracketed)."""
    if not params:
        return ""

    def one(v):
        if isinstance(v, (list, tuple)):
            return "[" + ",".join(str(x) for x in v) + "]"
        return str(v)

    out = []
    for key, val in params.items():
        if val is None:
            continue
        if isinstance(val, (list, tuple, set, np.ndarray)):
            out.append("{}={}".format(key, ",".join(one(v) for v in val)))
        elif isinstance(val, (str, bool, int, float, np.integer, np.floating)):
            out.append("{}={}".format(key, val))
        else:
            try:
                float(val)
            except (TypeError, ValueError):
                raise TypeError("Unknown type of parameter:{}, got:{}".format(key, type(val).__name__))
            out.append("{}={}".format(key, val))
    return " ".join(out)


def read_string(fn, initial=1 << 20):
    """Two-pass string protocol: fn(buffer_len, out_len_ptr, buffer) fills `buffer` and
    reports the needed length; retried once with a large-enough buffer."""
    size = initial
    for _ in range(2):
        needed = ctypes.c_int64(0)
        buf = ctypes.create_string_buffer(size)
        fn(ctypes.c_int64(size), ctypes.byref(needed), ctypes.c_char_p(ctypes.addressof(buf)))
        if needed.value <= size:
            return buf.value.decode("utf-8")
        size = needed.value
    raise LightGBMError("native string output kept growing")


def read_names(fn, count):
    """Name-list protocol: fn(count, out_count_ptr, buffer_size, needed_size_ptr, buffers)."""
    size = 256
    for _ in range(2):
        got = ctypes.c_int(0)
        needed = ctypes.c_size_t(0)
        bufs = [ctypes.create_string_buffer(size) for _ in range(count)]
        ptrs = (ctypes.c_char_p * count)(*[ctypes.addressof(b) for b in bufs])
        fn(ctypes.c_int(count), ctypes.byref(got), ctypes.c_size_t(size), ctypes.byref(needed), ptrs)
        if got.value != count:
            raise ValueError("expected {} names, the library returned {}".format(count, got.value))
        if needed.value <= size:
            return [b.value.decode("utf-8") for b in bufs]
        size = needed.value
    raise LightGBMError("native name output kept growing")


def string_array(strings):
    return (ctypes.c_char_p * len(strings))(*[s.encode("utf-8") for s in strings])
