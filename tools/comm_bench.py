"""Per-collective latency of the device communicators on thread ranks sharing one MI355X.

    python tools/comm_bench.py [--worlds 2,4,8] [--comms peer,host]

For each world size and communicator, every rank thread runs the learner's round collectives
back to back: the int64 reduce-scatter of one Higgs-sized round (6 expansions x 28 features x
256 bins x (g, h) x 8 bytes = 688 KB), the per-round split-record allgather (2 x 6 x 4
records x 64 bytes per rank) and a small all-reduce (3 values).  The peer comm is timed from
a captured graph (as the learner launches it) and eagerly; the host-rendezvous comm only
eagerly (it cannot be captured).  Ranks on one GPU signal each other through the same HBM,
so these numbers are the comm's own overhead without the xGMI hop (~1-2 us per flag exchange
across GPUs).  Prints one JSON line per case.
"""
import argparse
import ctypes
import json
import os
import sys

if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 16:
    os.environ["GPU_MAX_HW_QUEUES"] = "16"  # one hardware queue per rank's stream
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from lightgbmv1_amd.basic import _load_lib  # noqa: E402
from lightgbmv1_amd.parallel.inproc import ThreadRanks  # noqa: E402

CASES = [("reduce_scatter_round", 0, 6 * 28 * 256 * 2 * 8), ("allgather_records", 1, 2 * 6 * 4 * 64),
         ("allreduce_root", 2, 24), ("reduce_scatter_8MB", 0, 8 << 20)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--comms", default="peer,host")
    ap.add_argument("--iters", type=int, default=200)
    args = ap.parse_args()
    lib = _load_lib()
    for comm in args.comms.split(","):
        for world in [int(w) for w in args.worlds.split(",")]:
            for name, kind, nbytes in CASES:
                for graph in ([1, 0] if comm == "peer" else [0]):
                    iters = args.iters if comm == "peer" else max(10, args.iters // 10)

                    def fn(r, kind=kind, nbytes=nbytes, graph=graph, iters=iters):
                        us = ctypes.c_double(0)
                        rc = lib.LGBM_AMD_DeviceCommBench(ctypes.c_int(kind), ctypes.c_int64(nbytes),
                                                          ctypes.c_int(iters), ctypes.c_int(graph), ctypes.byref(us))
                        if rc != 0:
                            raise RuntimeError("bench failed on rank %d" % r)
                        return us.value

                    with ThreadRanks(world, timeout_s=60, device_comm=comm) as tr:
                        res = tr.run(fn)
                    errs = [str(r.error) for r in res if not r.ok]
                    out = {"comm": comm, "world": world, "case": name, "bytes": nbytes, "graph": bool(graph),
                           "iters": iters}
                    if errs:
                        out["error"] = errs[0]
                    else:
                        out["us_per_collective_max_rank"] = round(max(r.value for r in res), 2)
                    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
