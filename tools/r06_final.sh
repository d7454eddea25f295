#!/bin/bash
# Round-6 end-of-round re-measurement of every BASELINE configuration at HEAD (1x MI355X).
# Each step has its own time limit; the script stops at the first crash or timeout.
set -o pipefail
mkdir -p gpurun_out/r06_final
O=gpurun_out/r06_final
run() {  # name seconds command...
  local name=$1 secs=$2; shift 2
  echo "[r06_final] $name"
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  tail -1 "$O/$name.log"
  if [ $rc -ne 0 ]; then echo "[r06_final] $name rc=$rc: stopping"; exit $rc; fi
}
run headline_window 200 python bench.py --steps 20 --warmup 5
run headline_500 300 python bench.py
for b in 255 63 15; do
  run published_${b} 300 python bench.py --leaves 255 --max-bin $b --steps 500 --params '{"min_sum_hessian_in_leaf": 100}'
done
for s in 5000000 2500000 1250000; do
  run shard_$s 200 python bench.py --rows $s --steps 100 --warmup 5 --test-rows 0
done
for w in epsilon bosch yahoo_ltr ms_ltr expo; do
  run workload_$w 400 python tools/bench_workload.py --name $w --steps 30 --warmup 3
done
run ltr_config4 400 python tools/bench_ltr.py
echo "[r06_final] done"
