# the driver's multi-GPU bench shape on the box's one GPU: 4 processes (ranks share the GPU)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04tr
mkdir -p $O
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29571 \
  bench.py --gpus 4 --steps 20 --warmup 5 > $O/tr4.json 2> $O/tr4.err || { tail -20 $O/tr4.err; exit 1; }
grep '^{' $O/tr4.json | tail -1 | cut -c1-700
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29572 \
  bench.py --gpus 2 --steps 20 --warmup 5 > $O/tr2.json 2> $O/tr2.err || { tail -20 $O/tr2.err; exit 1; }
grep '^{' $O/tr2.json | tail -1 | cut -c1-700
