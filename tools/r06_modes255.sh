#!/bin/bash
# order-dependent modes at 255 leaves: the leaf-scaled width (16) against width 8 -- the same
# trees (held-out AUC) and the time per iteration
mkdir -p gpurun_out/m255
for m in xt bynode cegb; do
  case $m in
    xt) P='{"extra_trees": true, "min_sum_hessian_in_leaf": 100}' ;;
    bynode) P='{"feature_fraction_bynode": 0.8, "min_sum_hessian_in_leaf": 100}' ;;
    cegb) P='{"cegb_penalty_feature_coupled": [1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1], "cegb_tradeoff": 0.5, "min_sum_hessian_in_leaf": 100}' ;;
  esac
  for k in 16 8; do
    LGBM_AMD_ROUND_K=$k timeout -k 10 200 python bench.py --leaves 255 --steps 60 --warmup 3 --params "$P" > gpurun_out/m255/${m}_k$k.log 2>&1 || { echo "$m k$k failed"; exit 1; }
    tail -1 gpurun_out/m255/${m}_k$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$m', 'k$k', d['ms_per_step'], d['auc_heldout'], d['rounds_per_tree'])"
  done
done
