# adaptive round width on the wide workload shapes (after the split-scan fixes)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w3
mkdir -p $O
for n in epsilon bosch yahoo_ltr expo; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n adaptive $(tail -1 $O/$n.json | grep -o '"sec_per_iter": [0-9.]*')"
  LGBM_AMD_ROUND_K=6 timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/${n}_6.json 2> $O/${n}_6.err || { tail -5 $O/${n}_6.err; exit 1; }
  echo "$n K=6 $(tail -1 $O/${n}_6.json | grep -o '"sec_per_iter": [0-9.]*')"
done
