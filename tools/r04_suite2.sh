# full GPU suite + smoke + headline window x3 + shard floor
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/gpu_suite_r04b.log 2>&1
e=$?
tail -3 gpurun_out/gpu_suite_r04b.log
[ $e -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gpu_suite_r04b.log | head -10; exit $e; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r04b.log 2>&1 || { tail -10 gpurun_out/smoke_r04b.log; exit 1; }
tail -1 gpurun_out/smoke_r04b.log
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 > gpurun_out/win_$rep.log 2>&1 || { tail -5 gpurun_out/win_$rep.log; exit 1; }
  echo "window $rep $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/win_$rep.log)"
done
timeout -k 10 150 python bench.py --rows 1250000 --steps 100 --warmup 5 --test-rows 0 > gpurun_out/s125.log 2>&1 || { tail -5 gpurun_out/s125.log; exit 1; }
echo "1.25M $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/s125.log)"
