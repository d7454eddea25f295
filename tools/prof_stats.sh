#!/bin/bash
# rocprofv3 kernel stats of a short headline run under extra env settings.
# usage: tools/prof_stats.sh TAG STEPS [VAR=VALUE ...]
tag=$1; steps=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for kv in "$@"; do export "$kv"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${tag} -o run -- python3 $R/bench.py --steps $steps --warmup 2 --test-rows 0 > $R/gpurun_out/${tag}.log 2>&1 || { echo "rocprof failed"; tail -5 $R/gpurun_out/${tag}.log; exit 3; }
f=$(find $R/gpurun_out/${tag} -name 'run_kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print("%-60s calls %6s  total %9.1f us  avg %8.2f us" % (r["Name"][:60], r["Calls"], float(r["TotalDurationNs"]) / 1e3, float(r["AverageNs"]) / 1e3))
PY
