# round width on latency-bound shards: fixed K vs the adaptive default, 100 iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04ks
mkdir -p $O
for rows in 1250000 2500000; do
  for k in adapt 6 8 10 12 16; do
    if [ $k = adapt ]; then unset LGBM_AMD_ROUND_K; else export LGBM_AMD_ROUND_K=$k; fi
    LGBM_AMD_ITER_LOG=$O/it_${rows}_$k.jsonl timeout -k 10 120 python3 bench.py --rows $rows --steps 100 --warmup 5 --test-rows 0 > $O/b_${rows}_$k.log 2>&1 || { tail -5 $O/b_${rows}_$k.log; exit 1; }
    python3 - $O/it_${rows}_$k.jsonl $rows $k $O/b_${rows}_$k.log <<'PY'
import json, sys
rows = [json.loads(l) for l in open(sys.argv[1])][-100:]
r = [x for row in rows for x in row["rounds"]]
e = [x for row in rows for x in row["expansions"]]
b = [json.loads(l) for l in open(sys.argv[4]) if l.startswith("{")][-1]
print("rows %s K=%s ms/iter %.4f rounds/tree %.2f exp/tree %.1f" % (sys.argv[2], sys.argv[3], b["ms_per_step"], sum(r)/len(r), sum(e)/len(e)))
PY
  done
done
