#!/bin/bash
# Headline bench under several environment settings (one bench process each, 100 timed
# iterations): each argument is a space-separated list of VAR=VALUE assignments ("" = none).
# usage: tools/sweep_env.sh TAG "" "LGBM_AMD_BLK_MIN_ROWS=4096" ...
tag=$1; shift
mkdir -p gpurun_out
out=gpurun_out/${tag}_sweep.txt
: > $out
for cfg in "$@"; do
  line=$(env $cfg timeout -k 10 120 python bench.py --steps 100 --warmup 3 --test-rows 0 2>/dev/null | tail -1) || { echo "[$cfg] failed" | tee -a $out; exit 3; }
  ms=$(echo "$line" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
  echo "[$cfg] ms/iter $ms" | tee -a $out
done
