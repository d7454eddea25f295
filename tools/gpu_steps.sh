#!/bin/bash
# Run GPU steps in order on the GPU box, each under its own time limit, and stop at the first
# step that crashed, faulted or timed out (exit status > 1; status 1 -- e.g. failing tests --
# goes on).  Each step's output goes to gpurun_out/<name>.log.
#   tools/gpu_steps.sh NAME SECONDS "command" [NAME SECONDS "command" ...]
mkdir -p gpurun_out
while [ $# -ge 3 ]; do
  name=$1; secs=$2; cmd=$3; shift 3
  echo "[gpu_steps] $name (limit ${secs}s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[gpu_steps] $name rc=$rc"
  tail -3 "gpurun_out/$name.log"
  if [ $rc -gt 1 ]; then
    echo "[gpu_steps] stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit 0
