#!/bin/bash
# One GPU-box session: GPU tests, 1-GPU bench, optional rocprofv3 kernel stats.
# Stops at the first step that times out, aborts or segfaults (exit 124/134/137/139).
#   tools/gpu_check.sh [tests] [bench] [prof] [env VAR=VAL ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
fatal() { case "$1" in 124|134|137|139) return 0;; *) return 1;; esac; }
want() { [[ " $STEPS " == *" $1 "* ]]; }
STEPS="$*"
[ -z "$STEPS" ] && STEPS="tests bench prof"
if want tests; then
  timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest_exit=$rc" >> gpurun_out/pytest_gpu.log
  fatal $rc && exit $rc
fi
if want bench; then
  timeout -k 10 420 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1
  rc=$?; echo "bench_exit=$rc" >> gpurun_out/bench.log
  fatal $rc && exit $rc
fi
if want prof; then
  ROOT=$(pwd)
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 420 rocprofv3 --kernel-trace --stats -f csv -d "$ROOT/gpurun_out/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 2 --test-rows 0 > "$ROOT/gpurun_out/prof.log" 2>&1
  rc=$?; echo "prof_exit=$rc" >> "$ROOT/gpurun_out/prof.log"
  fatal $rc && exit $rc
fi
exit 0
