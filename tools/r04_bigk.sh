# round-growth K on a throughput-bound shard (Criteo-shaped 125M rows, serial) + the training-AUC
# evaluation's kernels (rocprofv3 kernel stats of bench.py --eval-train)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04bk
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/evalprof -o run -- python3 bench.py --steps 10 --warmup 3 --eval-train > $O/evalprof.log 2>&1 || { tail -5 $O/evalprof.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/evalprof.log
for k in 1 2 3 6; do
  LGBM_AMD_ROUND_K=$k timeout -k 10 600 python -u tools/bench_criteo.py --rows 125000000 --steps 6 --warmup 2 > $O/criteo_k$k.json 2> $O/criteo_k$k.err || { tail -5 $O/criteo_k$k.err; exit 1; }
  echo "K=$k $(tail -1 $O/criteo_k$k.json | cut -c1-200)"
done
