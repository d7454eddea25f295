# kernel stats of training-set AUC evaluation every iteration (bench.py --eval-train)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04auc
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 3 --test-rows 0 > $O/base.log 2>&1 || { tail -5 $O/base.log; exit 1; }
timeout -k 10 200 python3 $R/bench.py --steps 20 --warmup 3 --test-rows 0 --eval-train > $O/eval.log 2>&1 || { tail -5 $O/eval.log; exit 1; }
echo "no eval $(grep -o '"ms_per_step": [0-9.]*' $O/base.log)  eval $(grep -o '"ms_per_step": [0-9.]*' $O/eval.log)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/p -o run -- python3 $R/bench.py --steps 20 --warmup 3 --test-rows 0 --eval-train > $O/p.log 2>&1 || { tail -5 $O/p.log; exit 1; }
f=$(find $O/p -name 'run_kernel_stats.csv' | head -1)
python3 $R/tools/prof_summary.py $f "eval-train kernel stats" > $O/p.md
head -30 $O/p.md | cut -c1-250
