set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_learner.py -k "sparse or layouts" -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_sparse.log 2>&1 || { tail -40 gpurun_out/gpu_sparse.log; exit 1; }
tail -1 gpurun_out/gpu_sparse.log
for n in bosch expo yahoo_ltr; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --steps 20 --max-bin 63 2> /dev/null | tail -1 | cut -c1-220 || exit 1
  LGBM_AMD_SPARSE_ROWS=0 timeout -k 10 600 python -u tools/bench_workload.py --name $n --steps 20 --max-bin 63 2> /dev/null | tail -1 | cut -c1-220 || exit 1
done
