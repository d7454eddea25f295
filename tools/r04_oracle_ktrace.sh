# k_round_split phase times (LGBM_AMD_KTRACE, workgroup 0 of every round) for the in-tree library
# and the sequential-gather timing oracles (variants/oseq1, oseq2): gather us per row
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04o
mkdir -p $O
for v in base oseq1 oseq2; do
  lib=""; [ "$v" != "base" ] && lib=$GRAFT_REPO_ROOT/variants/$v/lib_lightgbmv1_amd.so
  LIGHTGBM_AMD_LIB=$lib LGBM_AMD_KTRACE=1 timeout -k 10 200 python -u bench.py --steps 12 --warmup 3 --test-rows 0 > $O/$v.log 2>&1 || { echo "$v failed"; tail -3 $O/$v.log; exit 1; }
  echo "$v $(grep -c '^round' $O/$v.log) round lines"
done
