# kernel stats at HEAD: headline (10M) and the 8-way shard (1.25M), 60 timed iterations each
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r04hp
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rows in 10000000 1250000; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/p$rows -o run -- python3 $R/bench.py --rows $rows --steps 60 --warmup 3 --test-rows 0 > $O/p$rows.log 2>&1 || { tail -5 $O/p$rows.log; exit 1; }
  grep -o '"ms_per_step": [0-9.]*' $O/p$rows.log
  f=$(find $O/p$rows -name 'run_kernel_stats.csv' | head -1)
  python3 $R/tools/prof_summary.py $f "kernel stats rows=$rows" > $O/p$rows.md
  head -16 $O/p$rows.md
done
