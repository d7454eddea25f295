# kernel time per tree of the Criteo-shaped 125M-row shard: round growth (K=6) vs one split per step
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04cp
mkdir -p $O
export TMPDIR=/tmp
for k in 6 1; do
  LGBM_AMD_ROUND_K=$k timeout -k 10 700 rocprofv3 --kernel-trace --stats -f csv -d $O/k$k -o run -- python3 tools/bench_criteo.py --rows 125000000 --steps 4 --warmup 1 > $O/k$k.log 2>&1 || { tail -5 $O/k$k.log; exit 1; }
  grep -o '"value": [0-9.]*' $O/k$k.log
done
