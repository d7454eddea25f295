#!/bin/bash
# smoke() plus the order-dependent modes' cost against plain growth on the headline shape
# (each step under its own limit; stops at the first failure)
mkdir -p gpurun_out
step() { local n=$1 s=$2; shift 2; timeout -k 10 $s "$@" > gpurun_out/$n.log 2>&1 || { echo "$n failed"; exit 1; }; tail -1 gpurun_out/$n.log; }
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step plain 200 python bench.py --steps 100 --warmup 5 --test-rows 0
step xt 200 python bench.py --steps 100 --warmup 5 --test-rows 0 --params '{"extra_trees": true}'
step bynode 200 python bench.py --steps 100 --warmup 5 --test-rows 0 --params '{"feature_fraction_bynode": 0.8}'
step cegb 200 python bench.py --steps 100 --warmup 5 --test-rows 0 --params '{"cegb_penalty_feature_coupled": [1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1,1], "cegb_tradeoff": 0.5}'
