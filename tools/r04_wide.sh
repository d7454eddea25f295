# round width on wide data (Epsilon-shaped 2000 features) and the headline window
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04wd
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 600 python -u tools/bench_workload.py --name epsilon --max-bin 63 --steps 30 --warmup 3 > $O/eps_$rep.json 2> $O/eps_$rep.err || { tail -5 $O/eps_$rep.err; exit 1; }
  echo "epsilon $(tail -1 $O/eps_$rep.json | grep -o '"sec_per_iter": [0-9.]*')"
done
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/window.log 2>&1 || { tail -5 $O/window.log; exit 1; }
echo "window $(grep -o '"ms_per_step": [0-9.]*' $O/window.log)"
