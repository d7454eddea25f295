set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04sh
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_rounds.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
LGBM_AMD_ROUND_K=1 LGBM_AMD_KTRACE=1 timeout -k 10 200 python3 bench.py --steps 6 --warmup 3 --test-rows 0 > $O/k1_ktrace.log 2>&1 || { tail -5 $O/k1_ktrace.log; exit 1; }
head -1 $O/k1_ktrace.log | cut -c1-500
for rep in 1 2; do
LGBM_AMD_ROUND_K=1 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --test-rows 0 > $O/k1_$rep.log 2>&1 || { tail -5 $O/k1_$rep.log; exit 1; }
echo "k1 $(grep -o '"ms_per_step": [0-9.]*' $O/k1_$rep.log)"
done
