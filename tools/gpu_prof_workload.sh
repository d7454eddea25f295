#!/bin/bash
# rocprofv3 kernel trace of a short tools/bench_workload.py run + the per-step breakdown of the last tree.
# usage: tools/gpu_prof_workload.sh TAG WORKLOAD [extra bench_workload args...]
tag=${1:-wl}; shift
name=${1:-expo}; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -f csv -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_workload.py --name $name --steps 4 --warmup 1 --test-rows 1000 "$@" > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.log; exit 3; }
cd $GRAFT_REPO_ROOT
f=$(find gpurun_out/${tag}_prof -name 'run_kernel_trace.csv' | head -1)
s=$(find gpurun_out/${tag}_prof -name 'run_kernel_stats.csv' | head -1)
python3 tools/step_trace.py "$f" > gpurun_out/${tag}_steps.txt
tail -3 gpurun_out/${tag}_steps.txt
python3 tools/prof_summary.py "$s" "$tag" > gpurun_out/${tag}_stats.md
head -24 gpurun_out/${tag}_stats.md
rm -rf gpurun_out/${tag}_prof
