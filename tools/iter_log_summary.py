#!/usr/bin/env python3
"""Per-tree time, rounds and expansions of an LGBM_AMD_ITER_LOG file, averaged over iteration
buckets.  usage: iter_log_summary.py iters.jsonl [BUCKET]"""
import json
import sys

rows = [json.loads(line) for line in open(sys.argv[1])]
bucket = int(sys.argv[2]) if len(sys.argv) > 2 else 50
for b0 in range(0, len(rows), bucket):
    sel = rows[b0:b0 + bucket]
    n = sum(len(r["tree_ms"]) for r in sel)
    ms = sum(sum(r["tree_ms"]) for r in sel) / n
    it = sum(r["ms"] for r in sel) / len(sel)
    rd = sum(sum(r["rounds"]) for r in sel) / n
    ex = sum(sum(r.get("expansions", [0])) for r in sel) / n
    lv = sum(sum(r["leaves"]) for r in sel) / n
    print("iters %4d-%4d  iter_ms %.3f  tree_ms %.3f  rounds %.1f  expansions %.1f  leaves %.1f"
          % (b0, b0 + len(sel) - 1, it, ms, rd, ex, lv))
