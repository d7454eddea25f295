# inputs of the strong-scaling projection: per-shard compute at HEAD and the peer comm's
# per-collective latency (thread ranks on one GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04proj
mkdir -p $O
for r in 10000000 5000000 2500000 1250000; do
  for k in 6 8; do
    LGBM_AMD_ROUND_K=$k timeout -k 10 150 python bench.py --rows $r --steps 100 --warmup 5 --test-rows 0 > $O/b_${r}_k$k.log 2>&1 || { tail -5 $O/b_${r}_k$k.log; exit 1; }
    echo "rows $r K $k $(grep -o '"ms_per_step": [0-9.]*' $O/b_${r}_k$k.log | cut -d' ' -f2) rounds $(grep -o '"rounds_per_tree": [0-9.]*' $O/b_${r}_k$k.log | cut -d' ' -f2)"
  done
done
timeout -k 10 300 python tools/comm_bench.py --worlds 2,4 --comms peer > $O/comm.jsonl 2> $O/comm.err || { tail -5 $O/comm.err; exit 1; }
cat $O/comm.jsonl | cut -c1-200
