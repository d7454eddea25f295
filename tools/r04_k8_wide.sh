# fixed K=8 vs the adaptive width on the small-row workload shapes (and MS-LTR)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k8w
mkdir -p $O
for n in epsilon bosch yahoo_ltr ms_ltr; do
  for k in adapt 8; do
    if [ $k = adapt ]; then unset LGBM_AMD_ROUND_K; else export LGBM_AMD_ROUND_K=$k; fi
    timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/${n}_$k.json 2> $O/${n}_$k.err || { tail -5 $O/${n}_$k.err; exit 1; }
    echo "$n K=$k $(tail -1 $O/${n}_$k.json | grep -o '"value": [0-9.e-]*')"
  done
done
