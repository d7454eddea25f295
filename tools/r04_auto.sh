# timed growth-mode choice: GPU round tests, the headline (below the size threshold: rounds),
# the 125M Criteo shard (probes and picks)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04auto
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_rounds.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/bench.log
timeout -k 10 700 python -u tools/bench_criteo.py --rows 125000000 --steps 8 --warmup 6 > $O/criteo.json 2> $O/criteo.err || { tail -5 $O/criteo.err; exit 1; }
grep -h "growth timed" $O/criteo.err $O/criteo.json || echo "(no growth log: verbose off)"
tail -1 $O/criteo.json | grep -o '"value": [0-9.]*'
