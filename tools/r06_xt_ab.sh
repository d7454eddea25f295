#!/bin/bash
# extra_trees deferred-fold A/B: the round-growth xt tests on the current library, then the
# headline shape with extra_trees under the previous library (variants/xt_old) and this one
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_learner.py \
  -k "extra_trees or split_rules or deterministic or round" > gpurun_out/xt_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/xt_tests.log; exit 1; }
tail -2 gpurun_out/xt_tests.log
timeout -k 10 600 python tools/ab.py --out gpurun_out/xt_ab --reps 3 \
  --bench "bench.py --steps 100 --warmup 5 --test-rows 0 --params '{\"extra_trees\":true}'" \
  --variant old:LIGHTGBM_AMD_LIB=variants/xt_old/lib_lightgbmv1_amd.so --variant new || exit 1
