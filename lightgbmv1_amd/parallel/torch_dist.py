"""Distributed bootstrap over torch.distributed (one process per GPU).

The native library needs two kinds of collectives:
  * host collectives (bin-mapper exchange, split-info sync, metric sums): provided to
    ``LGBM_NetworkInitWithFunctions`` as an allgather callback backed by a CPU (gloo)
    process group -- the analogue of the reference's socket/MPI linkers
    (reference src/network/linkers_socket.cpp, c_api.h LGBM_NetworkInitWithFunctions);
  * device collectives (per-round histogram reduce-scatter, split-record allgather, root
    statistics), one of:
      - "peer" (default): one-shot collectives that read the peers' HBM over xGMI, one kernel
        each, captured in the learner's graphs; windows exported with hipIpc handles
        exchanged through the process group (src/network/peer_comm.cpp).  A self test of every
        collective (eager and graph-replayed) runs first; if it fails on any rank, every rank
        falls back to RCCL;
      - "rccl": an RCCL communicator created natively from an ncclUniqueId that rank 0 draws
        and broadcasts through the same process group (src/network/rccl_comm.cpp).
    Chosen by `device_comm` or LGBM_AMD_DEVICE_COMM.

torch itself never touches the GPU here, so the HIP runtime is owned by the library.
Rendezvous uses MASTER_ADDR / MASTER_PORT / RANK / WORLD_SIZE (torchrun); always use
127.0.0.1 on a single node.
"""
import ctypes
import os

import numpy as np

from ..basic import _load_lib, _safe_call

_ALLGATHER_T = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_int),
                                ctypes.POINTER(ctypes.c_int), ctypes.c_int, ctypes.c_void_p, ctypes.c_int)

_STATE = {"callbacks": None, "group": None, "rccl": False, "device_comm": None, "self_test": None}


def _make_allgather(dist, group):
    import torch

    def allgather(input_ptr, input_size, block_start, block_len, num_block, output_ptr, output_size):
        # an exception must not escape a ctypes callback (ctypes would print it and return,
        # leaving the native caller with an unfilled buffer): report it, the caller raises
        try:
            _allgather(input_ptr, input_size, block_start, block_len, num_block, output_ptr)
        except BaseException as e:  # noqa: BLE001
            _load_lib().LGBM_AMD_NetworkReportExternalError(
                ("%s: %s" % (type(e).__name__, e)).encode("utf-8", "replace"))

    def _allgather(input_ptr, input_size, block_start, block_len, num_block, output_ptr):
        lens = [block_len[i] for i in range(num_block)]
        starts = [block_start[i] for i in range(num_block)]
        max_len = max(lens) if lens else 0
        mine = np.zeros(max(1, max_len), dtype=np.uint8)
        if input_size > 0:
            ctypes.memmove(mine.ctypes.data, input_ptr, input_size)
        send = torch.from_numpy(mine)
        recv = [torch.empty_like(send) for _ in range(num_block)]
        dist.all_gather(recv, send, group=group)
        for r in range(num_block):
            if lens[r] > 0:
                ctypes.memmove(output_ptr + starts[r], recv[r].numpy().ctypes.data, lens[r])
    return _ALLGATHER_T(allgather)


def _all_ok(dist, group, ok):
    """True when `ok` holds on every rank (a host all-reduce)."""
    import torch
    t = torch.tensor([1 if ok else 0], dtype=torch.int64)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(t.item())


def _init_peer(lib, dist, group, device, timeout_s):
    """The peer comm on every rank, self-tested; False (and nothing left behind) otherwise."""
    ok = lib.LGBM_AMD_PeerCommInit(ctypes.c_int(device), ctypes.c_double(timeout_s)) == 0
    if not _all_ok(dist, group, ok):
        if ok:
            lib.LGBM_AMD_DeviceCommFree()
        return False
    a, b = ctypes.c_int(0), ctypes.c_int(0)
    ok = (lib.LGBM_AMD_RcclSelfTest(ctypes.byref(a)) == 0 and a.value == 1 and
          lib.LGBM_AMD_RcclGraphSelfTest(ctypes.byref(b)) == 0 and b.value == 1)
    _STATE["self_test"] = {"eager": a.value == 1, "graph": b.value == 1}
    if not _all_ok(dist, group, ok):
        lib.LGBM_AMD_DeviceCommFree()
        return False
    return True


def init_network(use_rccl=True, backend="gloo", timeout_s=600, device_comm=None):
    """Initialise host (and, with use_rccl, device) collectives for the current process group.

    device_comm: "peer" or "rccl" (default: LGBM_AMD_DEVICE_COMM, else "peer" with RCCL as
    the fallback).  Returns (rank, world_size, local_rank).
    """
    import datetime

    import torch.distributed as dist
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", str(rank)))
    if world <= 1:
        return rank, world, local_rank
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if not dist.is_initialized():
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=datetime.timedelta(seconds=timeout_s))
    group = dist.group.WORLD
    lib = _load_lib()
    cb = _make_allgather(dist, group)
    _STATE["callbacks"] = cb
    _STATE["group"] = group
    _safe_call(lib.LGBM_NetworkInitWithFunctions(ctypes.c_int(world), ctypes.c_int(rank), None, cb))
    if use_rccl:
        ndev = ctypes.c_int(0)
        _safe_call(lib.LGBM_AMD_DeviceCount(ctypes.byref(ndev)))
        kind = device_comm or os.environ.get("LGBM_AMD_DEVICE_COMM", "peer")
        if ndev.value > 0 and kind == "peer":
            # (the learner raises the device-side wait bound to its time_out minutes)
            if _init_peer(lib, dist, group, local_rank % ndev.value, float(timeout_s)):
                _STATE["device_comm"] = "peer"
            else:
                kind = "rccl"
                if rank == 0:
                    print("[lightgbmv1_amd] peer device comm unavailable; using RCCL", flush=True)
        if ndev.value > 0 and kind == "rccl":
            import torch
            size = ctypes.c_int(0)
            _safe_call(lib.LGBM_AMD_RcclUniqueIdSize(ctypes.byref(size)))
            uid = np.zeros(size.value, dtype=np.uint8)
            ok = True
            if rank == 0:
                ok = lib.LGBM_AMD_RcclGetUniqueId(uid.ctypes.data_as(ctypes.c_char_p)) == 0
            t = torch.from_numpy(uid)
            dist.broadcast(t, src=0, group=group)
            uid = t.numpy()
            ok = _all_ok(dist, group, ok)
            if ok:
                ok = lib.LGBM_AMD_RcclInit(ctypes.c_int(world), ctypes.c_int(rank),
                                           ctypes.c_int(local_rank % ndev.value),
                                           uid.ctypes.data_as(ctypes.c_char_p)) == 0
            if _all_ok(dist, group, ok):
                _STATE["rccl"] = True
                _STATE["device_comm"] = "rccl"
            else:
                # neither device communicator: the learners' collectives go through the host
                # process group (slower, same trees)
                if ok:
                    lib.LGBM_AMD_DeviceCommFree()
                if rank == 0:
                    print("[lightgbmv1_amd] RCCL unavailable; device collectives over the host process group",
                          flush=True)
    return rank, world, local_rank


def device_comm_kind():
    """"peer", "rccl" or None: the device communicator init_network set up."""
    return _STATE["device_comm"]


def device_topology():
    """This rank's view of the device topology (dict), for run records: the device comm kind,
    the peer comm's self-test outcome and, per peer rank, its PCI bus id and either
    ``same_device`` or the link type (``xgmi`` / ``pcie``) and hop count
    (hipExtGetLinkTypeAndHopCount), or ``visible: false`` under per-process device isolation."""
    import json
    out = {"device_comm": _STATE["device_comm"], "self_test": _STATE["self_test"]}
    if _STATE["device_comm"] == "peer" or _STATE["self_test"] is not None:
        lib = _load_lib()
        n = ctypes.c_int(0)
        lib.LGBM_AMD_DeviceCommTopology(None, ctypes.c_int(0), ctypes.byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        lib.LGBM_AMD_DeviceCommTopology(buf, ctypes.c_int(n.value + 1), ctypes.byref(n))
        try:
            out.update(json.loads(buf.value.decode() or "{}"))
        except ValueError:
            out["raw"] = buf.value.decode(errors="replace")
    return out


def barrier():
    import torch.distributed as dist
    if dist.is_initialized():
        dist.barrier()


def allreduce_max(value):
    """Max of a float over ranks (host)."""
    import torch
    import torch.distributed as dist
    if not dist.is_initialized():
        return value
    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shutdown():
    lib = _load_lib()
    if _STATE["device_comm"] is not None:
        lib.LGBM_AMD_DeviceCommFree()  # (after every rank's kernels are done with the windows)
        _STATE["rccl"] = False
        _STATE["device_comm"] = None
    lib.LGBM_NetworkFree()
    try:
        import torch.distributed as dist
        if dist.is_initialized():
            # every rank is done with the group before any destroys it: rank 0 hosts the
            # rendezvous store, and a peer still using the group when the store goes away
            # fails inside c10d's own threads (a process abort, not a Python error)
            dist.barrier()
            dist.destroy_process_group()
    except Exception:  # pragma: no cover
        pass
