set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w8
mkdir -p $O
for rep in 1 2; do
  for v in base w8; do
    lib=""; [ "$v" = "w8" ] && lib=$GRAFT_REPO_ROOT/variants/w8/lib_lightgbmv1_amd.so
    LIGHTGBM_AMD_LIB=$lib timeout -k 10 150 python bench.py --steps 60 --warmup 5 --test-rows 0 > $O/${v}_$rep.log 2>&1 || { tail -5 $O/${v}_$rep.log; exit 1; }
    LIGHTGBM_AMD_LIB=$lib timeout -k 10 150 python bench.py --rows 1250000 --steps 60 --warmup 5 --test-rows 0 > $O/s_${v}_$rep.log 2>&1 || { tail -5 $O/s_${v}_$rep.log; exit 1; }
    echo "$v rep $rep 10M $(grep -o '"ms_per_step": [0-9.]*' $O/${v}_$rep.log) 1.25M $(grep -o '"ms_per_step": [0-9.]*' $O/s_${v}_$rep.log)"
  done
done
