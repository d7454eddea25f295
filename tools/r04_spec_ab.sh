# speculation budget (LGBM_AMD_SPEC_ROWS) A/B: headline 10M, the 1.25M shard, Criteo 125M shard
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04spec
mkdir -p $O
for b in 0 2000000 4000000 8000000; do
  for r in 10000000 1250000; do
    LGBM_AMD_SPEC_ROWS=$b timeout -k 10 150 python bench.py --rows $r --steps 100 --warmup 5 --test-rows 0 > $O/b_${r}_$b.log 2>&1 || { tail -5 $O/b_${r}_$b.log; exit 1; }
    echo "rows $r spec $b $(grep -o '"ms_per_step": [0-9.]*' $O/b_${r}_$b.log | cut -d' ' -f2) rounds $(grep -o '"rounds_per_tree": [0-9.]*' $O/b_${r}_$b.log | cut -d' ' -f2)"
  done
done
for b in 0 2000000 8000000; do
  LGBM_AMD_SPEC_ROWS=$b timeout -k 10 600 python -u tools/bench_criteo.py --rows 125000000 --steps 6 --warmup 2 > $O/criteo_$b.json 2> $O/criteo_$b.err || { tail -5 $O/criteo_$b.err; exit 1; }
  echo "criteo spec $b $(tail -1 $O/criteo_$b.json | grep -o '"value": [0-9.]*')"
done
