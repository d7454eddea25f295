#!/bin/bash
# rocprofv3 kernel trace of a short headline-bench run + the per-step breakdown of the last tree.
# usage: tools/gpu_prof.sh TAG [env assignments...]
tag=${1:-prof}; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --test-rows 0 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/${tag}_prof -name 'run_kernel_trace.csv' | head -1)
s=$(find gpurun_out/${tag}_prof -name 'run_kernel_stats.csv' | head -1)
python3 tools/step_trace.py "$f" > gpurun_out/${tag}_steps.txt
tail -3 gpurun_out/${tag}_steps.txt
python3 tools/prof_summary.py "$s" "$tag" > gpurun_out/${tag}_stats.md
head -14 gpurun_out/${tag}_stats.md
