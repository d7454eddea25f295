#!/bin/bash
# GPU check used with gpurun: device tests, then (unless a test run crashed or hung) the
# headline bench and an in-kernel trace run.  Output under gpurun_out/<tag>_*.
# usage: tools/gpu_check.sh TAG [pytest-args...]
tag=${1:-chk}; shift
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${tag}_pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 180 python bench.py --steps 200 --warmup 5 > gpurun_out/${tag}_bench.log 2>&1 || { echo "bench failed"; tail -5 gpurun_out/${tag}_bench.log; exit 3; }
tail -1 gpurun_out/${tag}_bench.log
LGBM_AMD_KTRACE=1 timeout -k 10 120 python bench.py --steps 3 --warmup 1 --test-rows 0 > gpurun_out/${tag}_ktrace.log 2>&1 || exit 4
grep ktrace gpurun_out/${tag}_ktrace.log | tail -2
exit $rc
