#!/bin/bash
# the leaf-scaled round width at HEAD: GPU suite, config #2 over 500 trees, and 127 leaves at
# widths 8 / 12 / 16 (each step under its own limit; stops at the first failure)
mkdir -p gpurun_out/wv
O=gpurun_out/wv
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/suite.log 2>&1 || { echo "suite failed"; tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for b in 255 63 15; do
  timeout -k 10 200 python bench.py --leaves 255 --max-bin $b --steps 500 --params '{"min_sum_hessian_in_leaf": 100}' > $O/published_$b.log 2>&1 || exit 1
  tail -1 $O/published_$b.log
done
timeout -k 10 400 python tools/ab.py --out $O/l127 --reps 2 \
  --bench "bench.py --leaves 127 --steps 150 --warmup 5 --test-rows 0" \
  --variant default --variant k12:LGBM_AMD_ROUND_K=12 --variant k16:LGBM_AMD_ROUND_K=16 || exit 1
