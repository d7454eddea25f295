# Epsilon-shaped workload: the library at a9dbf59 (variants/a9) vs HEAD, interleaved
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ea
mkdir -p $O
for rep in 1 2; do
  for v in a9 head; do
    lib=""; [ "$v" = "a9" ] && lib=$GRAFT_REPO_ROOT/variants/a9/lib_lightgbmv1_amd.so
    LIGHTGBM_AMD_LIB=$lib timeout -k 10 600 python -u tools/bench_workload.py --name epsilon --max-bin 63 --steps 30 --warmup 3 > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { tail -5 $O/${v}_$rep.err; exit 1; }
    echo "$v rep $rep $(tail -1 $O/${v}_$rep.json | grep -o '"sec_per_iter": [0-9.]*')"
  done
done
