#!/bin/bash
mkdir -p gpurun_out
LGBM_AMD_KTRACE=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 --test-rows 0 --params '{"extra_trees": true}' > gpurun_out/xt_kt.log 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace -f csv -d $GRAFT_REPO_ROOT/gpurun_out/xt_rt -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 30 --warmup 5 --test-rows 0 --params '{"extra_trees": true}' > $GRAFT_REPO_ROOT/gpurun_out/xt_rt.log 2>&1 || exit 1
