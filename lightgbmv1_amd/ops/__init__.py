"""Device ops: the HIP kernels of one boosting iteration, callable on torch tensors.

Each op runs the same kernel the device learner launches inside training (see
src/capi/ops_api.cpp) on caller-owned ``torch.Tensor`` buffers that live on the GPU, so
the kernels can be checked one by one against plain PyTorch references
(tests/test_ops.py) and reused outside a Booster:

* :func:`gradients` -- point-wise objective gradients / hessians
  (src/device/objective_kernels.hip; reference src/objective/*.hpp GetGradients)
* :func:`metric` -- validation metrics incl. AUC (src/device/metric_kernels.hip;
  reference src/metric/*.hpp Eval)
* :func:`sample_rows` -- bagging / GOSS row sampling with the reference's per-1024-row
  generators (src/device/sample_kernels.hip; reference gbdt.cpp:162-243, goss.hpp:103-179)

There is no host fallback: the ops need a GPU and the in-tree library.
"""
import ctypes

import numpy as np

from .._native import LightGBMError, params_str as param_dict_to_str
from ..basic import _load_lib

__all__ = ["gradients", "metric", "sample_rows"]


def _torch():
    import torch
    return torch


def _lib():
    lib = _load_lib()
    lib.LGBMAMD_OpLastError.restype = ctypes.c_char_p
    return lib


def _check(ret):
    if ret != 0:
        raise LightGBMError(_lib().LGBMAMD_OpLastError().decode("utf-8"))


def _dev_ptr(t, dtype, name):
    torch = _torch()
    if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
        raise LightGBMError("%s must be a torch tensor on the GPU" % name)
    if t.dtype != dtype or not t.is_contiguous():
        raise LightGBMError("%s must be a contiguous %s tensor" % (name, dtype))
    return ctypes.c_void_p(t.data_ptr())


def _host_f32(a, n, name):
    if a is None:
        return None, None
    if type(a).__module__.startswith("torch"):
        a = a.detach().cpu().numpy()
    a = np.ascontiguousarray(np.asarray(a, dtype=np.float32).reshape(-1))
    if a.shape[0] != n:
        raise LightGBMError("%s has %d entries, expected %d" % (name, a.shape[0], n))
    return a, a.ctypes.data_as(ctypes.POINTER(ctypes.c_float))


def _params(params):
    return param_dict_to_str(params).encode("utf-8") if isinstance(params, dict) else str(params).encode("utf-8")


def gradients(params, score, label, weight=None):
    """Gradients and hessians of objective ``params`` (e.g. ``{"objective": "binary"}``).

    ``score``: float64 GPU tensor ``[n]`` (multiclass: ``[num_class, n]``).  Returns
    float32 GPU tensors ``(grad, hess)`` of the same shape."""
    torch = _torch()
    n = score.shape[-1]
    _dev_ptr(score, torch.float64, "score")
    lab, lab_p = _host_f32(label, n, "label")
    w, w_p = _host_f32(weight, n, "weight")
    grad = torch.empty(score.shape, dtype=torch.float32, device=score.device)
    hess = torch.empty_like(grad)
    torch.cuda.synchronize(score.device)
    _check(_lib().LGBMAMD_OpGradients(ctypes.c_char_p(_params(params)), lab_p, w_p, ctypes.c_int32(n),
                                      _dev_ptr(score, torch.float64, "score"), _dev_ptr(grad, torch.float32, "grad"),
                                      _dev_ptr(hess, torch.float32, "hess")))
    del lab, w
    return grad, hess


def metric(params, score, label, weight=None):
    """Value of ``params["metric"]`` on raw GPU scores (float64 ``[n]``, or class-major
    ``[num_class, n]`` for multiclass metrics), with the output transform of
    ``params["objective"]`` (e.g. sigmoid for binary, softmax for multiclass)."""
    torch = _torch()
    n = score.shape[-1]
    lab, lab_p = _host_f32(label, n, "label")
    w, w_p = _host_f32(weight, n, "weight")
    out = ctypes.c_double(0.0)
    torch.cuda.synchronize(score.device)
    _check(_lib().LGBMAMD_OpMetric(ctypes.c_char_p(_params(params)), lab_p, w_p, ctypes.c_int32(n),
                                   _dev_ptr(score, torch.float64, "score"), ctypes.byref(out)))
    del lab, w
    return out.value


def sample_rows(n, fraction=1.0, seed=3, goss=False, top_rate=0.2, other_rate=0.1, grad=None, hess=None,
                device="cuda"):
    """One bagging (``goss=False``: keep ``fraction`` of every 1024-row block) or GOSS draw
    with fresh generators ``Random(seed + block)``.  Returns ``(bag, oob)`` int32 GPU
    tensors: in-bag rows ascending and the out-of-bag rows.  GOSS needs float32 GPU
    ``grad`` / ``hess`` (``[n]`` or ``[num_class, n]``) and rescales the sampled rows in place."""
    torch = _torch()
    bag = torch.empty(n, dtype=torch.int32, device=device)
    oob = torch.empty(n, dtype=torch.int32, device=device)
    num_class = 1
    gp = hp = ctypes.c_void_p(0)
    if goss:
        if grad is None or hess is None:
            raise LightGBMError("GOSS sampling needs grad and hess")
        num_class = 1 if grad.dim() == 1 else grad.shape[0]
        gp = _dev_ptr(grad, torch.float32, "grad")
        hp = _dev_ptr(hess, torch.float32, "hess")
    cnt = ctypes.c_int32(0)
    torch.cuda.synchronize(bag.device)
    _check(_lib().LGBMAMD_OpSampleRows(ctypes.c_int64(n), ctypes.c_int32(seed), ctypes.c_int32(1 if goss else 0),
                                       ctypes.c_int32(num_class), ctypes.c_double(fraction),
                                       ctypes.c_double(top_rate), ctypes.c_double(other_rate), gp, hp,
                                       _dev_ptr(bag, torch.int32, "bag"), _dev_ptr(oob, torch.int32, "oob"),
                                       ctypes.byref(cnt)))
    k = cnt.value
    return bag[:k], oob[:n - k]
