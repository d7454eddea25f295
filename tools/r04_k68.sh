# K=6 vs K=8 on the headline: driver window (20 after 5) x3 interleaved, and 300 iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k
mkdir -p $O
for rep in 1 2 3; do
  for k in 6 8; do
    LGBM_AMD_ROUND_K=$k timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/w_${k}_$rep.log 2>&1 || { tail -5 $O/w_${k}_$rep.log; exit 1; }
    echo "window K=$k rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/w_${k}_$rep.log)"
  done
done
for k in 6 8; do
  LGBM_AMD_ROUND_K=$k timeout -k 10 200 python bench.py --steps 300 --warmup 5 --test-rows 0 > $O/l_$k.log 2>&1 || { tail -5 $O/l_$k.log; exit 1; }
  echo "300 K=$k $(grep -o '"ms_per_step": [0-9.]*' $O/l_$k.log)"
done
