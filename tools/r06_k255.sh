#!/bin/bash
# Round width at 255 leaves (BASELINE config #2, the reference's published configuration):
# adaptive (8 / 6) against fixed widths, interleaved
mkdir -p gpurun_out
timeout -k 10 900 python tools/ab.py --out gpurun_out/k255 --reps 2 \
  --bench "bench.py --leaves 255 --max-bin 255 --steps 150 --warmup 5 --test-rows 0 --params '{\"min_sum_hessian_in_leaf\": 100}'" \
  --variant adaptive --variant k8:LGBM_AMD_ROUND_K=8 --variant k12:LGBM_AMD_ROUND_K=12 --variant k16:LGBM_AMD_ROUND_K=16 \
  --variant vmax8:LGBM_AMD_ROUND_VMAX=8 || exit 1
