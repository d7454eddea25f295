#!/usr/bin/env python3
"""Per-kernel time of the last TREES trees of a rocprofv3 kernel trace (round growth), split
at each tree's root plan kernel.  usage: late_tree_trace.py run_kernel_trace.csv [TREES]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
trees = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_tree_begin" in r["Kernel_Name"]]
sel = rows[starts[-trees - 1]:starts[-1]] if len(starts) > trees else rows
tot = collections.defaultdict(float)
cnt = collections.Counter()
for r in sel:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lgbm_amd::dev::", "")
    tot[name] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    cnt[name] += 1
span = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3
busy = sum(tot.values())
print("last %d trees: span %.1f us per tree, kernel-busy %.1f us per tree" % (trees, span / trees, busy / trees))
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print("  %-60s calls/tree %6.1f  us/tree %8.1f  avg %6.2f" % (k[:60], cnt[k] / trees, v / trees, v / cnt[k]))
