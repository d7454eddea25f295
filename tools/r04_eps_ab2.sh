set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_distributed.py tests/test_gpu_rounds.py > gpurun_out/r04_ab2_tests.log 2>&1 || { tail -30 gpurun_out/r04_ab2_tests.log; exit 1; }
tail -1 gpurun_out/r04_ab2_tests.log
bash tools/r04_eps_ab.sh
