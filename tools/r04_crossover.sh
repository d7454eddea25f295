# where one split per step overtakes round growth: Criteo-shaped (255 leaves) and Higgs-shaped
# (63 leaves) at growing row counts, K=1 vs K=6
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04x
mkdir -p $O
for r in 15000000 30000000 60000000; do
  for k in 1 6; do
    LGBM_AMD_ROUND_K=$k timeout -k 10 500 python -u tools/bench_criteo.py --rows $r --steps 6 --warmup 2 > $O/c_${r}_k$k.json 2> $O/c_${r}_k$k.err || { tail -5 $O/c_${r}_k$k.err; exit 1; }
    echo "criteo rows $r K $k $(tail -1 $O/c_${r}_k$k.json | grep -o '"value": [0-9.]*')"
  done
done
for r in 40000000; do
  for k in 1 6; do
    LGBM_AMD_ROUND_K=$k timeout -k 10 500 python bench.py --rows $r --steps 30 --warmup 3 --test-rows 0 > $O/h_${r}_k$k.log 2>&1 || { tail -5 $O/h_${r}_k$k.log; exit 1; }
    echo "higgs rows $r K $k $(grep -o '"ms_per_step": [0-9.]*' $O/h_${r}_k$k.log)"
  done
done
