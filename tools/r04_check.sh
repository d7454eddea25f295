# correctness + speed check of a round-kernel change: round / kernel GPU tests, the driver-window
# headline, and the 1.25M-row shard with its kernel timeline
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rounds.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-260
timeout -k 10 300 python -u bench.py --steps 100 --warmup 5 --rows 1250000 --test-rows 0 > $O/bench_1p25.log 2>&1 || { tail -5 $O/bench_1p25.log; exit 1; }
tail -1 $O/bench_1p25.log | cut -c1-200
if [ -n "$TRACE" ]; then ROWS=1250000 bash tools/r04_small_trace.sh; fi
