# training AUC: tests, then eval latency of the float-key path vs the 64-bit sort
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04auc
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_learner.py -k "metrics or auc" > gpurun_out/r04auc/tests.txt 2>&1 || { tail -30 gpurun_out/r04auc/tests.txt; exit 1; }
tail -1 gpurun_out/r04auc/tests.txt
timeout -k 10 200 python3 tools/r04_auc_eval_time.py
LGBM_AMD_AUC_SORT64=1 timeout -k 10 200 python3 tools/r04_auc_eval_time.py
