#!/bin/bash
# Headline bench per library variant, interleaved twice (A B C A B C): each argument is a
# variant name under variants/ ("base" = the in-tree library).
# usage: tools/ab_libs.sh TAG base g16 ...
tag=$1; shift
mkdir -p gpurun_out
out=gpurun_out/${tag}_ab.txt
: > $out
for rep in 1 2; do
  for v in "$@"; do
    lib=""
    [ "$v" != "base" ] && lib=$GRAFT_REPO_ROOT/variants/$v/lib_lightgbmv1_amd.so
    line=$(LIGHTGBM_AMD_LIB=$lib timeout -k 10 150 python bench.py --steps 150 --warmup 3 --test-rows 0 2>/dev/null | tail -1) || { echo "[$v] failed" | tee -a $out; exit 3; }
    ms=$(echo "$line" | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')
    echo "[$v] rep $rep ms/iter $ms" | tee -a $out
  done
done
