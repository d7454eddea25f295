# round grid and minimum block rows at HEAD (10M window-length runs and the 1.25M shard)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04gs
mkdir -p $O
run() {  # name rows env
  local n=$1 r=$2; shift 2
  env "$@" timeout -k 10 150 python bench.py --rows $r --steps 60 --warmup 5 --test-rows 0 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log | cut -d' ' -f2)"
}
for rep in 1 2; do
for g in 256 384 512 768; do run g${g}_10M_$rep 10000000 LGBM_AMD_ROUND_GRID=$g; run g${g}_1p25_$rep 1250000 LGBM_AMD_ROUND_GRID=$g; done
done
for b in 2048 8192; do run b${b}_10M 10000000 LGBM_AMD_BLK_MIN_ROWS=$b; done
