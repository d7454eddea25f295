#!/usr/bin/env python3
"""Per-step kernel durations of the last profiled tree from a rocprofv3 kernel trace.

  python tools/step_trace.py gpurun_out/prof/run_kernel_trace.csv [num_steps]
"""
import csv
import sys

tr = list(csv.DictReader(open(sys.argv[1])))
tr.sort(key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 62
names = ["k_partition", "k_hist<1", "k_hist_reduce<1", "k_find<false", "k_pick<false"]
cols = {k: [] for k in names}
gaps = []
for r in tr:
    for k in names:
        if k in r["Kernel_Name"]:
            cols[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
# wall time of the last tree's steps: first partition start -> last pick end
parts = [r for r in tr if "k_partition" in r["Kernel_Name"]][-n:]
picks = [r for r in tr if "k_pick<false" in r["Kernel_Name"]][-n:]
print("step " + " ".join(f"{k[:14]:>14}" for k in names))
for i in range(n):
    print(f"{i:4d} " + " ".join(f"{cols[k][-n + i]:14.1f}" for k in names))
w = (int(picks[-1]["End_Timestamp"]) - int(parts[0]["Start_Timestamp"])) / 1e3
busy = sum(sum(cols[k][-n:]) for k in names)
print(f"steps wall {w:.1f} us, kernels {busy:.1f} us, gaps {w - busy:.1f} us ({(w - busy) / (5 * n):.2f} us per boundary)")
