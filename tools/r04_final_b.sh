# end-of-round re-measure, part B: the five workload shapes, MS-LTR lambdarank + GOSS, the
# Criteo-shaped 125M-row shard (serial) and 4 voting processes x 31.25M rows
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04fb
mkdir -p $O
for rep in 1 2 3; do timeout -k 10 150 python bench.py --steps 20 --warmup 5 > $O/window$rep.log 2>&1 || { tail -5 $O/window$rep.log; exit 1; }; echo "window $rep $(grep -o "\"ms_per_step\": [0-9.]*" $O/window$rep.log)"; done
for n in epsilon bosch yahoo_ltr ms_ltr expo; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | cut -c1-260
done
timeout -k 10 600 python -u tools/bench_ltr.py > $O/ltr.json 2> $O/ltr.err || { tail -5 $O/ltr.err; exit 1; }
tail -1 $O/ltr.json | cut -c1-300
timeout -k 10 900 python -u tools/bench_criteo.py --rows 125000000 --steps 8 --warmup 6 > $O/criteo.json 2> $O/criteo.err || { tail -5 $O/criteo.err; exit 1; }
tail -1 $O/criteo.json | cut -c1-300
timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29561 \
  tools/bench_criteo.py --rows 31250000 --learner voting --steps 6 --warmup 6 > $O/criteo_vote4.json 2> $O/criteo_vote4.err || { tail -20 $O/criteo_vote4.err; exit 1; }
tail -1 $O/criteo_vote4.json | cut -c1-300
