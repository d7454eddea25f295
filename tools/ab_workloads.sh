#!/bin/bash
# tools/bench_workload.py per library variant: tools/ab_workloads.sh TAG "wl1 wl2" base g8 ...
tag=$1; wls=$2; shift 2
mkdir -p gpurun_out
out=gpurun_out/${tag}_wl_ab.txt
: > $out
for wl in $wls; do
  for v in "$@"; do
    lib=""
    [ "$v" != "base" ] && lib=$GRAFT_REPO_ROOT/variants/$v/lib_lightgbmv1_amd.so
    line=$(LIGHTGBM_AMD_LIB=$lib timeout -k 10 300 python tools/bench_workload.py --name $wl --max-bin 63 --steps 20 --warmup 3 2>/dev/null | tail -1) || { echo "[$wl $v] failed" | tee -a $out; exit 3; }
    ms=$(echo "$line" | python3 -c 'import json,sys; print(1000*json.loads(sys.stdin.read())["sec_per_iter"])')
    echo "[$wl $v] ms/iter $ms" | tee -a $out
  done
done
