# round tests + headline + 1.25M shard + scan-phase trace of the phases variant
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O gpurun_out/r04p
timeout -k 10 600 python -u -m pytest tests/test_gpu_rounds.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rows in 10000000 1250000; do
  timeout -k 10 300 python -u bench.py --steps 60 --warmup 5 --rows $rows --test-rows 0 > $O/b_$rows.log 2>&1 || { tail -5 $O/b_$rows.log; exit 1; }
  echo "rows=$rows $(tail -1 $O/b_$rows.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("rounds_per_tree"))')"
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
echo "driver window: $(tail -1 $O/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["auc_heldout"])')"
LIGHTGBM_AMD_LIB=$GRAFT_REPO_ROOT/variants/phases/lib_lightgbmv1_amd.so LGBM_AMD_KTRACE=1 timeout -k 10 120 python3 bench.py --steps 12 --warmup 3 --rows 1250000 --test-rows 0 > gpurun_out/r04p/k.log 2>&1
grep -A2 "^plan" gpurun_out/r04p/k.log | tail -9
