# direct_from_split sweep on 255-leaf workloads (see profiles/r01_v8_direct_sweep_255leaves.txt)
mkdir -p gpurun_out/sweep
for w in expo ms_ltr epsilon; do
  for d in 16 64 128 255; do
    rows=0; [ $w = expo ] && rows=2000000
    LGBM_AMD_DIRECT_FROM_SPLIT=$d timeout -k 10 200 python tools/bench_workload.py --name $w --rows $rows --steps 20 --warmup 2 --test-rows 1000 > gpurun_out/sweep/${w}_$d.json 2>&1 || exit 1
    echo "$w $d $(grep -o '"sec_per_iter": [0-9.]*' gpurun_out/sweep/${w}_$d.json)"
  done
done
