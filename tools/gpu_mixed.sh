set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread > gpurun_out/gpu_kernels.log 2>&1 || { tail -40 gpurun_out/gpu_kernels.log; exit 1; }
tail -3 gpurun_out/gpu_kernels.log
timeout -k 10 600 python -u tools/bench_workload.py --name expo --steps 20 --max-bin 63 > gpurun_out/expo_mixed.log 2>&1 || { tail -20 gpurun_out/expo_mixed.log; exit 1; }
tail -1 gpurun_out/expo_mixed.log
LGBM_AMD_UNIFORM_BINS=1 timeout -k 10 600 python -u tools/bench_workload.py --name expo --steps 20 --max-bin 63 > gpurun_out/expo_uniform.log 2>&1 || { tail -20 gpurun_out/expo_uniform.log; exit 1; }
tail -1 gpurun_out/expo_uniform.log
