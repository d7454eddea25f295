# knob sweep of the strong-scaling floor: 1.25M-row shard (and 10M for the K choices)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04sw
mkdir -p $O
run() {  # name rows env...
  local n=$1 r=$2; shift 2
  env "$@" timeout -k 10 120 python bench.py --rows $r --steps 60 --warmup 5 --test-rows 0 > $O/$n.log 2>&1 || { tail -5 $O/$n.log; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/$n.log | cut -d' ' -f2) rounds $(grep -o '"rounds_per_tree": [0-9.]*' $O/$n.log | cut -d' ' -f2)"
}
for k in 6 8 10 12 16; do run k${k}_1p25 1250000 LGBM_AMD_ROUND_K=$k; done
for b in 2048 8192 16384; do run blk${b}_1p25 1250000 LGBM_AMD_BLK_MIN_ROWS=$b; done
for v in 4 8; do run vmax${v}_1p25 1250000 LGBM_AMD_ROUND_VMAX=$v; done
for g in 256 1024; do run grid${g}_1p25 1250000 LGBM_AMD_ROUND_GRID=$g; done
for k in 6 8 10; do run k${k}_10M 10000000 LGBM_AMD_ROUND_K=$k; done
