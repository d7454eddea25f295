set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_learner.py -k "sparse or mixed or uniform or layouts or numeric" -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_sparse.log 2>&1 || { tail -40 gpurun_out/gpu_sparse.log; exit 1; }
tail -3 gpurun_out/gpu_sparse.log
timeout -k 10 600 python -u tools/bench_workload.py --name expo --steps 20 --max-bin 63 > gpurun_out/expo_sparse.log 2>&1 || { tail -20 gpurun_out/expo_sparse.log; exit 1; }
tail -1 gpurun_out/expo_sparse.log
