# round provisioning A/B: history / margin / segment size / root graph rounds
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04prov
mkdir -p $O
run() {  # tag env... -- bench args
  tag=$1; shift
  envs=(); while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 150 python3 bench.py "$@" --test-rows 0 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; exit 1; }
  echo "$tag $(grep -o '"ms_per_step": [0-9.]*' $O/$tag.log)"
}
for rep in 1 2; do
  for cfg in "A" "B LGBM_AMD_ROUND_HIST=5 LGBM_AMD_ROUND_MARGIN=0 LGBM_AMD_ROUND_SEG=2 LGBM_AMD_ROUND_ROOT=8" \
             "C LGBM_AMD_ROUND_HIST=5 LGBM_AMD_ROUND_MARGIN=0 LGBM_AMD_ROUND_SEG=1 LGBM_AMD_ROUND_ROOT=8" \
             "D LGBM_AMD_ROUND_HIST=3 LGBM_AMD_ROUND_MARGIN=0" \
             "E LGBM_AMD_ROUND_HIST=5 LGBM_AMD_ROUND_MARGIN=0 LGBM_AMD_ROUND_SEG=2"; do
    set -- $cfg; t=$1; shift
    run ${t}_s_$rep "X=1" "$@" -- --rows 1250000 --steps 100 --warmup 5 || exit 1
    run ${t}_w_$rep "X=1" "$@" -- --steps 20 --warmup 5 || exit 1
    run ${t}_h_$rep "X=1" "$@" -- --steps 100 --warmup 5 || exit 1
  done
done
