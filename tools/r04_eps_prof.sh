# per-kernel stats of the Epsilon-shaped workload: library at a9dbf59 vs HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ep
mkdir -p $O
export TMPDIR=/tmp
for v in a9 head; do
  lib=""; [ "$v" = "a9" ] && lib=$GRAFT_REPO_ROOT/variants/a9/lib_lightgbmv1_amd.so
  LIGHTGBM_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/$v -o run -- python3 tools/bench_workload.py --name epsilon --max-bin 63 --steps 10 --warmup 3 > $O/$v.log 2>&1 || { tail -5 $O/$v.log; exit 1; }
  echo "$v done"
done
