set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ab
mkdir -p $O
timeout -k 10 120 python -u tools/debug/round_diff.py min_data > $O/diff.txt 2>&1; head -70 $O/diff.txt
timeout -k 10 120 python -u tools/debug/self_check.py > $O/self_check.txt 2>&1; cat $O/self_check.txt | cut -c1-1500
for pif in 1 0; do
  for rows in 10000000 1250000; do
    LGBM_AMD_PLAN_IN_FIND=$pif timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --rows $rows --test-rows 0 > $O/b_${pif}_${rows}.log 2>&1 || exit 1
    echo "plan_in_find=$pif rows=$rows $(tail -1 $O/b_${pif}_${rows}.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("rounds_per_tree"))')"
  done
done
for tw in 4 2; do
  LGBM_AMD_HIST_TILE_WORDS=$tw timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --test-rows 0 > $O/tw_$tw.log 2>&1 || exit 1
  echo "tile_words=$tw $(tail -1 $O/tw_$tw.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
