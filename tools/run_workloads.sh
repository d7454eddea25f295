mkdir -p gpurun_out/wl
for n in epsilon bosch yahoo_ltr ms_ltr; do
  timeout -k 10 300 python tools/bench_workload.py --name $n --max-bin 63 --steps 50 --warmup 3 > gpurun_out/wl/$n.json 2> gpurun_out/wl/$n.err || exit 1
  cat gpurun_out/wl/$n.json
done
timeout -k 10 300 python tools/bench_workload.py --name expo --rows 2000000 --max-bin 63 --steps 50 --warmup 3 > gpurun_out/wl/expo.json 2> gpurun_out/wl/expo.err && cat gpurun_out/wl/expo.json
