# step-path pick with DPP argmaxes: rounds-vs-steps tests, the learner tests, K=1 / bynode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04pk
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_rounds.py tests/test_gpu_learner.py tests/test_cegb.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
LGBM_AMD_ROUND_K=1 timeout -k 10 200 python bench.py --steps 50 --warmup 5 --test-rows 0 > $O/k1_$rep.log 2>&1 || { tail -5 $O/k1_$rep.log; exit 1; }
echo "k1 $(grep -o '"ms_per_step": [0-9.]*' $O/k1_$rep.log)"
timeout -k 10 200 python bench.py --steps 50 --warmup 5 --test-rows 0 --params '{"feature_fraction_bynode": 0.8}' > $O/bynode_$rep.log 2>&1 || { tail -5 $O/bynode_$rep.log; exit 1; }
echo "bynode $(grep -o '"ms_per_step": [0-9.]*' $O/bynode_$rep.log)"
done
