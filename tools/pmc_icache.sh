#!/bin/bash
# Instruction-fetch counters over a short headline-bench run (two passes, each within the
# SQ / SQC slot limits): wave cycles waiting on instruction issue and I-cache misses per kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
tag=${1:-ic}
mkdir -p "$ROOT/gpurun_out/$tag"
cd /tmp && export TMPDIR=/tmp
run_pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/gpurun_out/$tag/$name" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --test-rows 0 > "$ROOT/gpurun_out/$tag/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"
  return $rc
}
run_pass sq SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_BUSY_CYCLES SQ_WAIT_ANY &&
run_pass sqc SQC_ICACHE_MISSES SQC_ICACHE_HITS
cd "$ROOT" && python3 - "$tag" <<'PY'
import csv, glob, os, sys
from collections import defaultdict
tag = sys.argv[1]
s = defaultdict(lambda: defaultdict(float)); d = defaultdict(set)
for p in glob.glob(f"gpurun_out/{tag}/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"].replace("lgbm_amd::dev::", "")[:50]
        s[k][r["Counter_Name"]] += float(r["Counter_Value"]); d[k].add((p, r["Dispatch_Id"]))
for k in sorted(s, key=lambda k: -s[k].get("SQ_WAVE_CYCLES", 0)):
    c = s[k]; n = max(1, len(d[k]) // 2)
    print("%-50s disp %4d waitinst/wavecyc %.2f wait_any/wavecyc %.2f ic_miss/disp %8.0f ic_hit/disp %9.0f ifetch/wave %.0f" % (
        k, n, c["SQ_WAIT_INST_ANY"] / max(1, c["SQ_WAVE_CYCLES"]), c["SQ_WAIT_ANY"] / max(1, c["SQ_WAVE_CYCLES"]),
        c["SQC_ICACHE_MISSES"] / n, c["SQC_ICACHE_HITS"] / n, c["SQ_IFETCH"] / max(1, c["SQ_WAVES"])))
PY
