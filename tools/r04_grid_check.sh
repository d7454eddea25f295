set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04gc
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_rounds.py tests/test_gpu_kernels.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/win_$rep.log 2>&1 || { tail -5 $O/win_$rep.log; exit 1; }
  echo "window $rep $(grep -o '"ms_per_step": [0-9.]*' $O/win_$rep.log)"
done
for n in epsilon bosch yahoo_ltr ms_ltr expo; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "$n $(tail -1 $O/$n.json | grep -o '"sec_per_iter": [0-9.]*')"
done
timeout -k 10 600 python -u tools/bench_criteo.py --rows 20000000 --steps 6 --warmup 3 > $O/criteo20.json 2> $O/criteo20.err || { tail -5 $O/criteo20.err; exit 1; }
echo "criteo 20M $(tail -1 $O/criteo20.json | grep -o '"value": [0-9.]*')"
