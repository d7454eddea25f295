set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r04_base_bench.log 2>&1 && tail -1 gpurun_out/r04_base_bench.log &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -k "training_metrics_on_device" -x -v --timeout 120 --timeout-method thread > gpurun_out/r04_trainmetric.log 2>&1 && tail -3 gpurun_out/r04_trainmetric.log &&
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --eval-train > gpurun_out/r04_evaltrain_bench.log 2>&1 && tail -1 gpurun_out/r04_evaltrain_bench.log &&
LGBM_AMD_KTRACE=1 timeout -k 10 300 python -u bench.py --steps 40 --warmup 5 --test-rows 0 > gpurun_out/r04_base_ktrace.log 2>&1 &&
bash tools/gpu_prof_late.sh r04late 150
