"""Host collectives of the calling thread's training network (the TCP mesh of
``machines=``, in-process thread ranks, or the torch.distributed callbacks), for user code
that exchanges its own data over the same mesh and for testing the collective algorithms
(src/network/collectives.cpp: Bruck / ring allgather, recursive-halving / ring
reduce-scatter).  Without a network (one machine) every call is the identity."""
import ctypes

import numpy as np

from .. import _native as nat


def world():
    """(rank, num_machines) of the calling thread's network."""
    return _rank(), _num_machines()


def allgather(arr):
    """Every rank's 1-D array (any length, same dtype on every rank), as a list by rank."""
    arr = np.ascontiguousarray(arr)
    lens = np.zeros(_num_machines(), dtype=np.int64)
    mine = np.array([arr.nbytes], dtype=np.int64)
    lens8 = np.full(len(lens), 8, dtype=np.int64)
    nat.call("LGBM_AMD_NetworkAllgather", mine.ctypes.data_as(ctypes.c_void_p),
             lens8.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), lens.ctypes.data_as(ctypes.c_void_p))
    out = np.zeros(int(lens.sum()), dtype=np.uint8)
    nat.call("LGBM_AMD_NetworkAllgather", arr.ctypes.data_as(ctypes.c_void_p),
             lens.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), out.ctypes.data_as(ctypes.c_void_p))
    bounds = np.concatenate([[0], np.cumsum(lens)])
    return [out[bounds[i]:bounds[i + 1]].view(arr.dtype) for i in range(len(lens))]


def reduce_scatter_sum(arr, counts):
    """Sum over ranks of a float64 vector; rank r receives items
    [sum(counts[:r]), sum(counts[:r+1])) of the sum."""
    arr = np.ascontiguousarray(arr, dtype=np.float64)
    counts = np.ascontiguousarray(counts, dtype=np.int64)
    if counts.sum() != arr.size:
        raise ValueError("counts must add up to the vector length")
    out = np.zeros(int(counts[_rank()]), dtype=np.float64)
    nat.call("LGBM_AMD_NetworkReduceScatterSumF64", arr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
             counts.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return out


def allreduce_sum(arr):
    """Sum over ranks of a float64 vector (bitwise identical on every rank)."""
    arr = np.ascontiguousarray(arr, dtype=np.float64)
    out = np.zeros_like(arr)
    nat.call("LGBM_AMD_NetworkAllreduceSumF64", arr.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
             ctypes.c_int64(arr.size), out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
    return out


def _num_machines():
    n = ctypes.c_int(0)
    nat.call("LGBM_AMD_NetworkNumMachines", ctypes.byref(n))
    return n.value


def _rank():
    r = ctypes.c_int(0)
    nat.call("LGBM_AMD_NetworkRank", ctypes.byref(r))
    return r.value
