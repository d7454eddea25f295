#!/bin/bash
# ITER_LOG summaries of the headline bench per speculation depth.  usage: tools/vmax_logs.sh STEPS VMAX...
steps=$1; shift
mkdir -p gpurun_out
for v in "$@"; do
  rm -f gpurun_out/it_v$v.jsonl
  LGBM_AMD_ROUND_VMAX=$v LGBM_AMD_ITER_LOG=gpurun_out/it_v$v.jsonl timeout -k 10 240 python3 bench.py --steps $steps --warmup 5 --test-rows 0 > gpurun_out/it_v$v.log 2>&1 || { echo "FAILED $v"; tail -3 gpurun_out/it_v$v.log; exit 1; }
  echo "vmax $v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/it_v$v.log)"
  python3 tools/iter_log_summary.py gpurun_out/it_v$v.jsonl 60
done
