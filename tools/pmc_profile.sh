#!/bin/bash
# Hardware-counter passes (rocprofv3 --pmc, one pass per counter set, each within the
# per-block slot limits) over a short headline-bench run; writes gpurun_out/pmc/<pass>/.
# Summarise with: python tools/pmc_summary.py gpurun_out/pmc
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
ROOT=$(pwd)
mkdir -p "$ROOT/gpurun_out/pmc"
cd /tmp && export TMPDIR=/tmp
run_pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$ROOT/gpurun_out/pmc/$name" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --test-rows 0 > "$ROOT/gpurun_out/pmc/$name.log" 2>&1
  local rc=$?
  echo "$name exit=$rc"
  return $rc
}
run_pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_ANY &&
run_pass sq2 SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAIT_INST_ANY SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES &&
run_pass fetch FETCH_SIZE GRBM_GUI_ACTIVE &&
run_pass write WRITE_SIZE TCC_HIT_sum TCC_MISS_sum
