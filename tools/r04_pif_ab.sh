# split scan without the plan body when the plan has its own kernel (PIF=false): previous
# library (variants/prev) vs HEAD on wide data and the 255-leaf configuration, + round tests
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04pif
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_gpu_rounds.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in prev head; do
    lib=""; [ "$v" = "prev" ] && lib=$GRAFT_REPO_ROOT/variants/prev/lib_lightgbmv1_amd.so
    LIGHTGBM_AMD_LIB=$lib timeout -k 10 600 python -u tools/bench_workload.py --name epsilon --max-bin 63 --steps 30 --warmup 3 > $O/eps_${v}_$rep.json 2> $O/eps_${v}_$rep.err || { tail -5 $O/eps_${v}_$rep.err; exit 1; }
    LIGHTGBM_AMD_LIB=$lib timeout -k 10 300 python bench.py --steps 100 --warmup 5 --leaves 255 --test-rows 0 > $O/l255_${v}_$rep.log 2>&1 || { tail -5 $O/l255_${v}_$rep.log; exit 1; }
    echo "$v rep $rep epsilon $(tail -1 $O/eps_${v}_$rep.json | grep -o '"sec_per_iter": [0-9.]*') 255-leaf $(grep -o '"ms_per_step": [0-9.]*' $O/l255_${v}_$rep.log)"
  done
done
