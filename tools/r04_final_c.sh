# end-of-round numbers after the grid change: 500 trees fx32/fx64, 255-leaf configs, shards
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04fc
mkdir -p $O
run() { local tag=$1; shift; timeout -k 10 300 python -u bench.py "$@" > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }; echo "$tag $(grep -o '"ms_per_step": [0-9.]*\|"auc_heldout": [0-9.]*\|"rounds_per_tree": [0-9.]*' $O/$tag.log | tr '\n' ' ')"; }
run default500 &&
run h63_fx64_500 --steps 495 --warmup 5 --hist-precision fx64 &&
run h255_b255 --steps 495 --warmup 5 --leaves 255 --max-bin 255 &&
run h255_b63 --steps 495 --warmup 5 --leaves 255 --max-bin 63 &&
run h255_b15 --steps 495 --warmup 5 --leaves 255 --max-bin 15 &&
for r in 5000000 2500000 1250000; do run rows_$r --steps 100 --warmup 5 --rows $r --test-rows 0 || exit 1; done
timeout -k 10 600 python -u tools/bench_ltr.py > $O/ltr.json 2> $O/ltr.err || { tail -5 $O/ltr.err; exit 1; }
echo "ltr $(tail -1 $O/ltr.json | grep -o '"ms_per_step": [0-9.]*')"
