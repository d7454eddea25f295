#!/bin/bash
# per-kernel summary of late trees: ITERS untraced headline iterations, then 4 traced ones (3 whole trees between them)
# continued from that model (tools/prof_late.py).  usage: tools/gpu_prof_late.sh TAG ITERS [env...]
tag=${1:-late}; iters=${2:-150}; shift 2
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
for kv in "$@"; do export "$kv"; done
timeout -k 10 300 python3 $R/tools/prof_late.py train $iters /tmp/late_model.txt > $R/gpurun_out/${tag}_train.log 2>&1 || { echo "train failed"; tail -3 $R/gpurun_out/${tag}_train.log; exit 3; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $R/gpurun_out/${tag}_prof -o run -- python3 $R/tools/prof_late.py cont 4 /tmp/late_model.txt > $R/gpurun_out/${tag}_prof.log 2>&1 || { echo "rocprof failed"; tail -5 $R/gpurun_out/${tag}_prof.log; exit 3; }
cd $R
f=$(find gpurun_out/${tag}_prof -name 'run_kernel_trace.csv' | head -1)
python3 tools/late_tree_trace.py "$f" 3 > gpurun_out/${tag}_late.txt
cat gpurun_out/${tag}_late.txt
