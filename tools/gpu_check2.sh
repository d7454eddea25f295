set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 python -u bench.py --steps 500 --warmup 20 > gpurun_out/bench500.log 2>&1 || { tail -20 gpurun_out/bench500.log; exit 1; }
tail -1 gpurun_out/bench500.log
bash tools/gpu_prof_workload.sh eps epsilon --max-bin 63 | grep -E "k_find|k_split|splits"
