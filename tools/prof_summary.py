#!/usr/bin/env python3
"""Turn rocprofv3 `--kernel-trace --stats -f csv` output into a markdown summary.

  python tools/prof_summary.py gpurun_out/prof/run_kernel_stats.csv "title" [notes] > profiles/x.md

With a `run_kernel_trace.csv` next to the stats file, a per-tree breakdown of the first
histogram-step kernel durations is appended (useful to see the small-leaf floor).
"""
import csv
import os
import sys


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else "kernel stats"
    notes = sys.argv[3] if len(sys.argv) > 3 else ""
    rows = list(csv.DictReader(open(path)))
    print(f"# {title}\n")
    if notes:
        print(notes + "\n")
    print("| kernel | calls | total us | avg us | min us | max us | % |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        name = r["Name"].replace("|", "\\|")
        print(f"| {name} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e3:.1f} | "
              f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | "
              f"{float(r['MaxNs']) / 1e3:.2f} | {float(r['Percentage']):.2f} |")
    trace = os.path.join(os.path.dirname(path), os.path.basename(path).replace("kernel_stats", "kernel_trace"))
    if os.path.exists(trace):
        tr = list(csv.DictReader(open(trace)))
        tr.sort(key=lambda r: int(r["Start_Timestamp"]))
        steps = [r for r in tr if "k_hist<1" in r["Kernel_Name"]]
        if steps:
            d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in steps]
            print("\nPer-step histogram kernel durations (us), last profiled tree:\n")
            n = 62 if len(d) >= 62 else len(d)
            print(", ".join(f"{x:.1f}" for x in d[-n:]))
        t0 = int(tr[0]["Start_Timestamp"])
        t1 = int(tr[-1]["End_Timestamp"])
        busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in tr)
        print(f"\nGPU busy {busy / 1e6:.2f} ms of {(t1 - t0) / 1e6:.2f} ms traced "
              f"({100.0 * busy / max(1, t1 - t0):.1f}%)")


if __name__ == "__main__":
    main()
