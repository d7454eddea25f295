#!/usr/bin/env python3
"""Per-kernel time of the last TREES whole trees of a rocprofv3 kernel trace (round growth),
split at each tree's k_tree_begin, and the timeline of the last of them (start offset, duration,
gap to the previous kernel).  usage: late_tree_trace.py run_kernel_trace.csv [TREES]"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
trees = int(sys.argv[2]) if len(sys.argv) > 2 else 3
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "k_tree_begin" in r["Kernel_Name"]]
if len(starts) <= trees:
    sys.exit("need %d tree starts, trace has %d" % (trees + 1, len(starts)))
sel = rows[starts[-trees - 1]:starts[-1]]
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

last = rows[starts[-2]:starts[-1]]
t0 = int(last[0]["Start_Timestamp"])
prev_end = t0
print("timeline of the last tree (us: start, duration, gap)")
for r in last:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("lgbm_amd::dev::", "")
    print("  %8.1f %7.1f %6.1f  %s" % ((st - t0) / 1e3, (en - st) / 1e3, (st - prev_end) / 1e3, name[:50]))
    prev_end = max(prev_end, en)
