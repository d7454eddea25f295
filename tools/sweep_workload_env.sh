#!/bin/bash
# tools/bench_workload.py under several environment settings:
#   tools/sweep_workload_env.sh TAG WORKLOAD "" "LGBM_AMD_SPLIT_GRID=64" ...
tag=$1; wl=$2; shift 2
mkdir -p gpurun_out
out=gpurun_out/${tag}_${wl}_sweep.txt
: > $out
for cfg in "$@"; do
  line=$(env $cfg timeout -k 10 300 python tools/bench_workload.py --name $wl --max-bin 63 --steps 20 --warmup 3 2>/dev/null | tail -1) || { echo "[$cfg] failed" | tee -a $out; exit 3; }
  ms=$(echo "$line" | python3 -c 'import json,sys; print(1000*json.loads(sys.stdin.read())["sec_per_iter"])')
  echo "[$wl $cfg] ms/iter $ms" | tee -a $out
done
