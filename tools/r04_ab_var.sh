# A/B of library variants (base = in-tree) at two shard sizes, interleaved: tools/r04_ab_var.sh v1 v2 ...
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04v
for rep in 1 2; do
  for v in "$@"; do
    lib=""; [ "$v" != "base" ] && lib=$GRAFT_REPO_ROOT/variants/$v/lib_lightgbmv1_amd.so
    for rows in 10000000 1250000; do
      LIGHTGBM_AMD_LIB=$lib timeout -k 10 200 python -u bench.py --steps 60 --warmup 5 --rows $rows --test-rows 0 > gpurun_out/r04v/${v}_$rows.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/r04v/${v}_$rows.log; exit 1; }
      echo "[$v] rep $rep rows $rows $(tail -1 gpurun_out/r04v/${v}_$rows.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("rounds_per_tree"))')"
    done
  done
done
