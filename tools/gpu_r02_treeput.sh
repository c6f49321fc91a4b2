#!/bin/bash
# Round 2: reduce_tree_put (LFA_ALGO_P2P kernel) on local HBM: A/B of scope
# bits and tiling, kernel trace, and FETCH/WRITE PMC passes of the product.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh tune_treeput 300 python3 bench.py --tune-treeput --tune-rounds 10 && \
tools/gpu_step.sh prof_treeput 200 $P -d gpurun_out/prof_treeput -o run -- python3 bench.py --only-extra tree_put && \
tools/gpu_step.sh pmc_fetch_tp 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_tp -o run -- python3 bench.py --only-extra tree_put && \
tools/gpu_step.sh pmc_write_tp 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_tp -o run -- python3 bench.py --only-extra tree_put
