# end-of-round re-measure, part A: driver window x3, 500-tree fx32 / fx64 AUC parity, the
# published 255-leaf configurations, the shard floor
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04fa
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; echo "$tag $(tail -1 $O/$tag.log | cut -c1-150) $(grep -o '"ms_per_step": [0-9.]*\|"auc_heldout": [0-9.]*\|"rounds_per_tree": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; }
run window1 && run window2 && run window3 &&
run h63_fx32_500 --steps 495 --warmup 5 &&
run h63_fx64_500 --steps 495 --warmup 5 --hist-precision fx64 &&
run h255_b255 --steps 495 --warmup 5 --leaves 255 --max-bin 255 &&
run h255_b63 --steps 495 --warmup 5 --leaves 255 --max-bin 63 &&
run h255_b15 --steps 495 --warmup 5 --leaves 255 --max-bin 15 &&
for r in 5000000 2500000 1250000; do
  run rows_$r --steps 100 --warmup 5 --rows $r --test-rows 0 || exit 1
done
