#!/bin/bash
# rocprofv3 kernel stats of the Criteo-shaped shard benchmark (tools/bench_criteo.py)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/criteo_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_criteo.py --steps 3 --warmup 1 "$@" > $GRAFT_REPO_ROOT/gpurun_out/criteo_prof.log 2>&1 || { echo "rocprof failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/criteo_prof.log; exit 3; }
cd $GRAFT_REPO_ROOT
s=$(find gpurun_out/criteo_prof -name 'run_kernel_stats.csv' | head -1)
python3 tools/prof_summary.py "$s" criteo > gpurun_out/criteo_stats.md
head -16 gpurun_out/criteo_stats.md
rm -rf gpurun_out/criteo_prof
