#!/bin/bash
# A/B of round-growth knobs on the headline bench: each argument is a space-free list of
# env assignments joined by ',' (e.g. LGBM_AMD_ROUND_GR=8,LGBM_AMD_ROUND_GRID=512); prints
# ms/iter per configuration.  usage: tools/round_sweep.sh TAG STEPS CFG...
tag=$1; steps=$2; shift 2
mkdir -p gpurun_out
for cfg in "$@"; do
  env_args=$(echo "$cfg" | tr ',' ' ')
  out=gpurun_out/${tag}_$(echo "$cfg" | tr ',=' '__').log
  env $env_args timeout -k 10 240 python3 bench.py --steps $steps --warmup 5 --test-rows 0 > $out 2>&1 || { echo "FAILED $cfg"; tail -3 $out; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' $out)"
done
