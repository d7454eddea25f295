# HEAD workload shapes at 255 leaves / 63 bins (bench_workload.py) + the Criteo-shaped 125M-row shard
# (1/8 of config #5's 1B rows), serial learner
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04w
mkdir -p $O
for n in epsilon bosch yahoo_ltr ms_ltr expo; do
  timeout -k 10 600 python -u tools/bench_workload.py --name $n --max-bin 63 --steps 30 --warmup 3 > $O/$n.json 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  tail -1 $O/$n.json | cut -c1-400
done
timeout -k 10 900 python -u tools/bench_criteo.py --rows 125000000 --steps 8 --warmup 2 > $O/criteo_125M.json 2> $O/criteo_125M.err || { tail -5 $O/criteo_125M.err; exit 1; }
tail -1 $O/criteo_125M.json | cut -c1-500
