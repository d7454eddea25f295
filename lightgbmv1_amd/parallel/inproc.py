"""In-process ranks: several training ranks as threads of one process.

The native Network state is thread-local (as the reference's THREAD_LOCAL network,
src/network/network.cpp:17-27), so each thread can join a shared hub of thread transports
and train as one rank of a data- / feature- / voting-parallel job -- no sockets, no extra
processes.  The hub bounds every collective with a timeout and can inject a fault into
one rank: the failing rank raises, its peers raise "peer rank failed" instead of hanging
(the fault-injecting fake backend of SURVEY.md §5.3).

    ranks = ThreadRanks(world=2, timeout_s=30)
    results = ranks.run(lambda rank: train_my_shard(rank))

With device_comm every rank thread also joins an in-process device communicator (the
threads share one GPU), so the data- / feature-parallel device learners run their device
collective path without RCCL:
  * device_comm=True / "peer": the capture-safe peer comm (src/network/peer_comm.cpp) --
    one kernel per collective reading the peers' windows, captured in the round graphs like
    the multi-process path; device_fail_at_call stops rank fail_rank at that collective
    (counted on the device), its peers time out after timeout_s;
  * device_comm="host": collectives rendezvous on the host (eager launches, no graphs);
    device_fail_at_call makes rank fail_rank raise at that call.
"""
import ctypes
import threading

from ..basic import _load_lib, _safe_call


class RankResult:
    """Outcome of one rank: `value` if it returned, `error` (the exception) if it raised."""

    def __init__(self, rank, value=None, error=None):
        self.rank = rank
        self.value = value
        self.error = error

    @property
    def ok(self):
        return self.error is None


class ThreadRanks:
    def __init__(self, world, timeout_s=0.0, fail_rank=-1, fail_at_call=0, device_comm=False, device_fail_at_call=0):
        self.world = int(world)
        self._hub = ctypes.c_void_p()
        self._dev_hub = ctypes.c_void_p()
        lib = _load_lib()
        _safe_call(lib.LGBM_AMD_NetworkCreateThreadHub(
            ctypes.c_int(self.world), ctypes.c_double(timeout_s), ctypes.c_int(fail_rank),
            ctypes.c_int(fail_at_call), ctypes.byref(self._hub)))
        if device_comm:
            kind = 0 if device_comm == "host" else 1
            _safe_call(lib.LGBM_AMD_DeviceCommCreateThreadHubEx(
                ctypes.c_int(self.world), ctypes.c_double(timeout_s), ctypes.c_int(fail_rank),
                ctypes.c_int(device_fail_at_call), ctypes.c_int(kind), ctypes.byref(self._dev_hub)))

    def run(self, fn):
        """Call fn(rank) in one thread per rank (joined to the hub); returns [RankResult]."""
        results = [None] * self.world
        lib = _load_lib()

        def body(rank):
            try:
                _safe_call(lib.LGBM_AMD_NetworkJoinThreadHub(self._hub, ctypes.c_int(rank)))
                if self._dev_hub:
                    _safe_call(lib.LGBM_AMD_DeviceCommJoinThreadHub(self._dev_hub, ctypes.c_int(rank)))
                results[rank] = RankResult(rank, value=fn(rank))
            except Exception as e:  # noqa: BLE001 -- reported per rank
                results[rank] = RankResult(rank, error=e)
            finally:
                lib.LGBM_NetworkFree()

        threads = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.world)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        return results

    def close(self):
        if self._hub:
            _load_lib().LGBM_AMD_NetworkFreeThreadHub(self._hub)
            self._hub = ctypes.c_void_p()
        if self._dev_hub:
            _load_lib().LGBM_AMD_DeviceCommFreeThreadHub(self._dev_hub)
            self._dev_hub = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
