# adaptive round width vs fixed K=6: driver window x3 interleaved, 300 iterations, round tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ka
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_rounds.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/w_a_$rep.log 2>&1 || { tail -5 $O/w_a_$rep.log; exit 1; }
  echo "window adaptive rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/w_a_$rep.log) $(grep -o '"auc_heldout": [0-9.]*' $O/w_a_$rep.log)"
  LGBM_AMD_ROUND_K=6 timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/w_6_$rep.log 2>&1 || { tail -5 $O/w_6_$rep.log; exit 1; }
  echo "window K=6 rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/w_6_$rep.log) $(grep -o '"auc_heldout": [0-9.]*' $O/w_6_$rep.log)"
done
timeout -k 10 200 python bench.py --steps 300 --warmup 5 --test-rows 0 > $O/l_a.log 2>&1 || { tail -5 $O/l_a.log; exit 1; }
echo "300 adaptive $(grep -o '"ms_per_step": [0-9.]*' $O/l_a.log)"
timeout -k 10 150 python bench.py --rows 1250000 --steps 100 --warmup 5 --test-rows 0 > $O/s_a.log 2>&1 || { tail -5 $O/s_a.log; exit 1; }
echo "1.25M adaptive $(grep -o '"ms_per_step": [0-9.]*' $O/s_a.log)"
