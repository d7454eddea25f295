# config #5 shape at 125M rows: 4 processes (voting, 31.25M rows each) sharing the box's one GPU,
# round growth (default) vs one split per step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04cv
mkdir -p $O
run() {  # name env port
  env $2 timeout -k 10 1000 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $3 tools/bench_criteo.py --rows 31250000 --learner voting --steps 5 --warmup 2 > $O/$1.json 2> $O/$1.err \
    || { tail -20 $O/$1.err; exit 1; }
  tail -1 $O/$1.json | cut -c1-460
}
run k6 LGBM_AMD_ROUND_K=6 29541 && run k1 LGBM_AMD_ROUND_K=1 29542
