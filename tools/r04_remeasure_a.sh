# HEAD re-measurement, part A (1x MI355X): headline at 500 trees (fx32 / fx64 AUC parity),
# the reference's exact published Higgs configuration (255 leaves, 255/63/15 bins, 500 iterations),
# and the strong-scaling floor (per-GPU compute of a 1/2/4/8-way row shard) with ITER_LOG.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04a
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; tail -1 $O/$tag.log; }
run h63_fx32_500 --steps 495 --warmup 5 &&
run h63_fx64_500 --steps 495 --warmup 5 --hist-precision fx64 &&
run h255_b255 --steps 495 --warmup 5 --leaves 255 --max-bin 255 --params '{"min_data_in_leaf": 1}' &&
run h255_b63 --steps 495 --warmup 5 --leaves 255 --max-bin 63 &&
run h255_b15 --steps 495 --warmup 5 --leaves 255 --max-bin 15 &&
for r in 10000000 5000000 2500000 1250000; do
  LGBM_AMD_ITER_LOG=$O/iters_$r.jsonl run rows_$r --steps 100 --warmup 5 --rows $r --test-rows 0 || exit 1
done
