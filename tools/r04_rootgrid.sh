# root histogram workgroups per CU: headline window and 100 iterations
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04rg
mkdir -p $O
for rep in 1 2; do
  for w in 2 1 3 4; do
    LGBM_AMD_ROOT_WG_PER_CU=$w timeout -k 10 150 python3 bench.py --steps 100 --warmup 5 --test-rows 0 > $O/h_${w}_$rep.log 2>&1 || { tail -5 $O/h_${w}_$rep.log; exit 1; }
    echo "per_cu $w rep $rep $(grep -o '"ms_per_step": [0-9.]*' $O/h_${w}_$rep.log)"
  done
done
