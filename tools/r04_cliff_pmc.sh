# order-dependent modes on the headline (one split per step) vs plain round growth, then the
# hardware-counter passes of the headline at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r04cl
mkdir -p $O
run() {  # name params
  timeout -k 10 200 python bench.py --steps 50 --warmup 5 --test-rows 0 --params "$2" > $O/$1.log 2>&1 || { tail -5 $O/$1.log; exit 1; }
  echo "$1 $(grep -o '"ms_per_step": [0-9.]*' $O/$1.log) rounds $(grep -o '"rounds_per_tree": [0-9.]*' $O/$1.log | cut -d' ' -f2)"
}
run plain '{}' && run bynode '{"feature_fraction_bynode": 0.8}' && run extra_trees '{"extra_trees": true}' && \
run cegb '{"cegb_penalty_split": 0.0001}' && run mono_inter '{"monotone_constraints": [1,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,0,-1], "monotone_constraints_method": "intermediate"}' && \
LGBM_AMD_ROUND_K=1 run plain_k1 "{}" || exit 1
bash tools/pmc_profile.sh && python3 tools/pmc_summary.py gpurun_out/pmc > $O/pmc_summary.md && head -12 $O/pmc_summary.md
