# kernel stats of one split per step on the headline (K=1) and with per-node sampling
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04sp
mkdir -p $O
export TMPDIR=/tmp
LGBM_AMD_ROUND_K=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv -d $O/k1 -o run -- python3 bench.py --steps 20 --warmup 3 --test-rows 0 > $O/k1.log 2>&1 || { tail -5 $O/k1.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' $O/k1.log
LGBM_AMD_ROUND_K=1 LGBM_AMD_KTRACE=1 timeout -k 10 200 python3 bench.py --steps 6 --warmup 3 --test-rows 0 > $O/k1_ktrace.log 2>&1 || { tail -5 $O/k1_ktrace.log; exit 1; }
grep -c "" $O/k1_ktrace.log
