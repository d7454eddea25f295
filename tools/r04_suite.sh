# full GPU suite + smoke
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_suite_r04.log 2>&1
e=$?
tail -5 gpurun_out/gpu_suite_r04.log
[ $e -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_suite_r04.log | head -10; exit $e; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04.log 2>&1 || { tail -10 gpurun_out/smoke_r04.log; exit 1; }
tail -3 gpurun_out/smoke_r04.log
