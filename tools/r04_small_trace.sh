# per-round latency at a small shard: kernel timeline of the last trees + in-kernel phase times
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04s
mkdir -p $O
ROWS=${ROWS:-1250000}
LGBM_AMD_KTRACE=1 timeout -k 10 120 python3 $R/bench.py --steps 12 --warmup 3 --rows $ROWS --test-rows 0 > $O/ktrace_$ROWS.log 2>&1 || { tail -5 $O/ktrace_$ROWS.log; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/prof_$ROWS -o run -- python3 $R/bench.py --steps 12 --warmup 3 --rows $ROWS --test-rows 0 > $O/prof_$ROWS.log 2>&1 || { tail -5 $O/prof_$ROWS.log; exit 1; }
cd $R
f=$(find $O/prof_$ROWS -name 'run_kernel_trace.csv' | head -1)
python3 tools/late_tree_trace.py "$f" 3 > $O/late_$ROWS.txt
head -20 $O/late_$ROWS.txt
