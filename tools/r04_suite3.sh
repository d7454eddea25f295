# end-of-round: full GPU suite + smoke + headline window x3 + 500 trees + shard floor + torchrun 2/4
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04end
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $O/gpu_suite.log 2>&1
e=$?
tail -3 $O/gpu_suite.log
[ $e -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_suite.log | head -10; exit $e; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -10 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/win_$rep.log 2>&1 || { tail -5 $O/win_$rep.log; exit 1; }
  echo "window $rep $(grep -o '"ms_per_step": [0-9.]*\|"auc_heldout": [0-9.]*' $O/win_$rep.log | tr '\n' ' ')"
done
timeout -k 10 300 python bench.py > $O/def.log 2>&1 || { tail -5 $O/def.log; exit 1; }
echo "500 trees $(grep -o '"ms_per_step": [0-9.]*\|"auc_heldout": [0-9.]*' $O/def.log | tr '\n' ' ')"
for rows in 5000000 2500000 1250000; do
  timeout -k 10 150 python bench.py --rows $rows --steps 100 --warmup 5 --test-rows 0 > $O/s$rows.log 2>&1 || { tail -5 $O/s$rows.log; exit 1; }
  echo "$rows $(grep -o '"ms_per_step": [0-9.]*\|"rounds_per_tree": [0-9.]*' $O/s$rows.log | tr '\n' ' ')"
done
bash tools/r04_torchrun4.sh
