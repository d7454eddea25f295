#!/usr/bin/env python3
"""Per-step kernel durations and the gaps between them, for the last profiled tree, from a
rocprofv3 kernel trace (device-resident growth: k_split [k_hist_reduce<1>] k_find<false>
[k_pick] per split).

  python tools/step_trace.py gpurun_out/prof/run_kernel_trace.csv

Prints one line per split (kernel: gap-before/duration in us) and the totals.
"""
import csv
import sys


def short(name):
    for k in ("k_split", "k_hist_reduce<1", "k_find<false", "k_pick", "k_find<true", "k_hist<0", "k_hist_reduce<0"):
        if k in name:
            return k
    return None


def main():
    tr = list(csv.DictReader(open(sys.argv[1])))
    tr.sort(key=lambda r: int(r["Start_Timestamp"]))
    ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in tr]
    ev = [e for e in ev if e[0] is not None]
    roots = [i for i, e in enumerate(ev) if e[0] == "k_find<true"]
    if not roots:
        print("no tree found")
        return
    start = roots[-2] if len(roots) > 1 else roots[-1]  # the last complete tree
    end = roots[-1] if len(roots) > 1 else len(ev)
    tree = ev[start:end]
    steps = []
    cur = []
    for e in tree[1:]:
        if e[0] == "k_split" and cur:
            steps.append(cur)
            cur = []
        cur.append(e)
    if cur:
        steps.append(cur)
    tot_k = tot_g = 0.0
    prev_end = tree[0][2]
    for i, st in enumerate(steps):
        parts = []
        for name, b, en in st:
            gap = (b - prev_end) / 1e3
            dur = (en - b) / 1e3
            tot_g += gap
            tot_k += dur
            parts.append(f"{name}: {gap:5.1f}/{dur:6.1f}")
            prev_end = en
        print(f"{i:3d}  " + "   ".join(parts))
    n = max(1, len(steps))
    print(f"splits {len(steps)}: kernels {tot_k:.1f} us, gaps {tot_g:.1f} us; per split {tot_k / n:.2f} + {tot_g / n:.2f} us")


if __name__ == "__main__":
    main()
