# config #5 voting rehearsal: 4 processes sharing the box's one MI355X (peer comm over hipIpc),
# 5M Criteo-shaped rows per rank; one split per step (ROUND_K=1) vs round growth (default K=6)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04vote
mkdir -p $O
run() {  # name, extra env
  env $2 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port $3 tools/bench_criteo.py --rows 5000000 --learner voting --steps 6 --warmup 2 > $O/$1.json 2> $O/$1.err \
    || { tail -20 $O/$1.err; exit 1; }
  tail -1 $O/$1.json | cut -c1-420
}
run k1 LGBM_AMD_ROUND_K=1 29531 && run k6 LGBM_AMD_ROUND_K=6 29532
