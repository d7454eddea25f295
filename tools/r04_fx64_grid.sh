set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04fg
mkdir -p $O
for rep in 1 2; do
  for g in 256 512; do
    LGBM_AMD_ROUND_GRID=$g timeout -k 10 150 python bench.py --steps 100 --warmup 5 --test-rows 0 --hist-precision fx64 > $O/g${g}_$rep.log 2>&1 || { tail -5 $O/g${g}_$rep.log; exit 1; }
    echo "fx64 grid $g rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/g${g}_$rep.log)"
  done
done
