# per-tree times and rounds along 300 iterations, K=6 and K=8 (ITER_LOG)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04kl
mkdir -p $O
for k in 6 8 10; do
  LGBM_AMD_ROUND_K=$k LGBM_AMD_ITER_LOG=$GRAFT_REPO_ROOT/$O/iters_$k.jsonl timeout -k 10 200 python bench.py --steps 300 --warmup 5 --test-rows 0 > $O/l_$k.log 2>&1 || { tail -5 $O/l_$k.log; exit 1; }
  echo "300 K=$k $(grep -o '"ms_per_step": [0-9.]*' $O/l_$k.log)"
done
