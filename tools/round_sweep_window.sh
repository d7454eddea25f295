#!/bin/bash
# round_sweep.sh at the driver's short window (STEPS after 5 warm-up, default 20) with the
# held-out rows: usage tools/round_sweep_window.sh TAG STEPS CFG...
tag=$1; steps=$2; shift 2
mkdir -p gpurun_out
for cfg in "$@"; do
  env_args=$(echo "$cfg" | tr ',' ' ')
  out=gpurun_out/${tag}_$(echo "$cfg" | tr ',=' '__').log
  env $env_args timeout -k 10 240 python3 bench.py --steps $steps --warmup 5 > $out 2>&1 || { echo "FAILED $cfg"; tail -3 $out; exit 1; }
  echo "$cfg $(grep -o '"ms_per_step": [0-9.]*' $out)"
done
