#!/usr/bin/env python3
"""Per-iteration budget of device-resident round growth from a rocprofv3 kernel trace: for the
iterations between consecutive k_tree_begin launches, the summed duration of each kernel, its
launches per iteration, and the idle gaps between kernels (launch latency, graph boundaries,
host round trips).

  rocprofv3 --kernel-trace -d gpurun_out/rt -o run -- python3 bench.py --rows 1250000 --steps 20
  python tools/round_trace.py gpurun_out/rt/run_results.db [--skip 5]

The trace is rocprofv3's SQLite output (its `kernels` view) or a `*_kernel_trace.csv`.

Prints a markdown table (mean us per iteration) and, with --last, the kernel sequence of the
last iteration (gap-before / duration per launch).
"""
import argparse
import collections
import csv
import sqlite3


def short(name):
    """the kernel's name with its template arguments, without namespaces and parameters"""
    for ns in ("void ", "(anonymous namespace)::", "lgbm_amd::dev::", "lgbm_amd::"):
        name = name.replace(ns, "")
    depth, out = 0, []
    for ch in name:  # cut at the parameter list (the first '(' outside template brackets)
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out)[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=3, help="iterations skipped at the start (warm-up)")
    ap.add_argument("--last", action="store_true", help="print the last iteration's launches")
    args = ap.parse_args()
    if args.trace.endswith(".db"):
        con = sqlite3.connect(args.trace)
        ev = sorted((int(s), int(e), short(n)) for s, e, n in con.execute("select start, end, name from kernels"))
    else:
        rows = list(csv.DictReader(open(args.trace)))
        ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in rows)
    starts = [i for i, e in enumerate(ev) if "k_tree_begin" in e[2]]
    if len(starts) < args.skip + 2:
        print("too few iterations: %d tree starts" % len(starts))
        return
    iters = [(starts[k], starts[k + 1]) for k in range(args.skip, len(starts) - 1)]
    dur = collections.defaultdict(float)
    cnt = collections.defaultdict(int)
    gaps = 0.0
    wall = 0.0
    for a, b in iters:
        wall += (ev[b][0] - ev[a][0]) / 1e3
        prev_end = ev[a][0]
        for s, e, n in ev[a:b]:
            dur[n] += (e - s) / 1e3
            cnt[n] += 1
            gaps += max(0, s - prev_end) / 1e3
            prev_end = max(prev_end, e)
    n = len(iters)
    print("iterations %d: %.1f us each (kernels %.1f, idle gaps %.1f)" % (n, wall / n, sum(dur.values()) / n, gaps / n))
    print()
    print("| kernel | launches / iter | us / iter | us / launch |")
    print("|---|---|---|---|")
    for k in sorted(dur, key=lambda k: -dur[k]):
        print("| `%s` | %.1f | %.1f | %.2f |" % (k, cnt[k] / n, dur[k] / n, dur[k] / cnt[k]))
    if args.last:
        a, b = iters[-1]
        prev_end = ev[a][0]
        print()
        for s, e, nm in ev[a:b]:
            print("%7.1f %7.1f  %s" % ((s - prev_end) / 1e3, (e - s) / 1e3, nm))
            prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
