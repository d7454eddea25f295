set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w2
mkdir -p $O
for n in epsilon bosch yahoo_ltr ms_ltr expo; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | cut -c1-200
done
timeout -k 10 600 python -u tools/bench_ltr.py > $O/ltr.json 2> $O/ltr.err || { tail -5 $O/ltr.err; exit 1; }
tail -1 $O/ltr.json | cut -c1-200
for b in 255 63 15; do
  timeout -k 10 300 python bench.py --steps 495 --warmup 5 --leaves 255 --max-bin $b > $O/h255_$b.log 2>&1 || { tail -5 $O/h255_$b.log; exit 1; }
  echo "255 leaves $b bins $(grep -o '"ms_per_step": [0-9.]*\|"auc_heldout": [0-9.]*' $O/h255_$b.log | tr '\n' ' ')"
done
