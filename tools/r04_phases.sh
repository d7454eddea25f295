cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04p
LIGHTGBM_AMD_LIB=$GRAFT_REPO_ROOT/variants/phases/lib_lightgbmv1_amd.so LGBM_AMD_KTRACE=1 timeout -k 10 120 python3 bench.py --steps 12 --warmup 3 --rows 1250000 --test-rows 0 > gpurun_out/r04p/k.log 2>&1
grep -A2 "^plan" gpurun_out/r04p/k.log | tail -24
