#!/bin/bash
# Hardware-counter passes (as tools/pmc_profile.sh) over a short tools/bench_workload.py run.
# usage: tools/pmc_workload.sh WORKLOAD [extra bench_workload args...]; writes gpurun_out/pmc_<workload>/
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
name=${1:-epsilon}; shift
out="$ROOT/gpurun_out/pmc_$name"
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
run_pass() {
  local pass=$1; shift
  timeout -s KILL 180 rocprofv3 --pmc "$@" --output-format csv -d "$out/$pass" -o run -- \
    python3 "$ROOT/tools/bench_workload.py" --name $name --steps 2 --warmup 1 --test-rows 1000 $EXTRA > "$out/$pass.log" 2>&1
  local rc=$?
  echo "$pass exit=$rc"
  return $rc
}
EXTRA="$*"
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU &&
run_pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_ACCUM_PREV_HIRES SQ_LEVEL_WAVES SQ_INSTS_BRANCH &&
cd "$ROOT" && python3 tools/pmc_summary.py "$out" > gpurun_out/pmc_$name.md && head -30 gpurun_out/pmc_$name.md
