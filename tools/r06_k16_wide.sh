#!/bin/bash
# Round width 16 against the default width on the 255-leaf shapes: config #2 at 63 / 15 bins
# and the config #3 workloads (interleaved; one step per bench set, each under its own limit)
mkdir -p gpurun_out
timeout -k 10 500 python tools/ab.py --out gpurun_out/k16a --reps 2 \
  --bench "bench.py --leaves 255 --max-bin 63 --steps 150 --warmup 5 --test-rows 0 --params '{\"min_sum_hessian_in_leaf\": 100}'" \
  --bench "bench.py --leaves 255 --max-bin 15 --steps 150 --warmup 5 --test-rows 0 --params '{\"min_sum_hessian_in_leaf\": 100}'" \
  --variant default --variant k16:LGBM_AMD_ROUND_K=16 || exit 1
timeout -k 10 600 python tools/ab.py --out gpurun_out/k16b --reps 1 --timeout 200 \
  --bench "tools/bench_workload.py --name epsilon --steps 30 --warmup 3" \
  --bench "tools/bench_workload.py --name bosch --steps 30 --warmup 3" \
  --bench "tools/bench_workload.py --name yahoo_ltr --steps 30 --warmup 3" \
  --bench "tools/bench_workload.py --name ms_ltr --steps 30 --warmup 3" \
  --bench "tools/bench_workload.py --name expo --steps 30 --warmup 3" \
  --variant default --variant k16:LGBM_AMD_ROUND_K=16 || exit 1
