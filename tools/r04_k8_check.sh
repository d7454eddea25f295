# after the width rule (fixed 8 below 4M rows per rank): headline window, 1.25M shard, torchrun 4 / 2
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04k8c
mkdir -p $O
for i in 1 2; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 5 > $O/w$i.log 2>&1 || { tail -5 $O/w$i.log; exit 1; }
  echo "window $(grep -o '"ms_per_step": [0-9.]*\|"auc_heldout": [0-9.]*' $O/w$i.log | tr '\n' ' ')"
done
timeout -k 10 200 python3 bench.py --rows 1250000 --steps 100 --warmup 5 --test-rows 0 > $O/s.log 2>&1 || { tail -5 $O/s.log; exit 1; }
echo "1.25M $(grep -o '"ms_per_step": [0-9.]*\|"rounds_per_tree": [0-9.]*' $O/s.log | tr '\n' ' ')"
bash tools/r04_torchrun4.sh
