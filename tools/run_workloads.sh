# every published workload shape at its full row count, 1x MI355X (tools/bench_workload.py)
set -o pipefail
mkdir -p gpurun_out/wl
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread > gpurun_out/wl/kernels.log 2>&1 || { tail -30 gpurun_out/wl/kernels.log; exit 1; }
tail -1 gpurun_out/wl/kernels.log
for n in epsilon bosch yahoo_ltr ms_ltr expo; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > gpurun_out/wl/$n.json 2> gpurun_out/wl/$n.err || { tail -5 gpurun_out/wl/$n.err; exit 1; }
  cat gpurun_out/wl/$n.json
done
