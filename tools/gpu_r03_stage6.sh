#!/bin/bash
# Round 3: u-major tree_put stores and the nt-drained readwrite body —
# their GPU tests, the tree_put A/B against the output-major form, and the
# combine-vs-size evidence for VERDICT r2 #5 (kernel trace + PMC passes over
# bench.py --only-extra sizes).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh gpu_subset 400 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "tree_put or treeput or fetch or readwrite or swap or oneshot or p2p" && \
tools/gpu_step.sh tune_treeput 300 python3 -u bench.py --tune-treeput --variants 0,18,22 --tune-rounds 10 && \
tools/gpu_step.sh prof_sizes 300 $P -d gpurun_out/prof_sizes -o run -- python3 bench.py --only-extra sizes --sizes-reps 100 && \
tools/gpu_step.sh pmc_sizes_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_sizes_fetch -o run -- python3 bench.py --only-extra sizes --sizes-reps 10 --prewarm-s 0 && \
tools/gpu_step.sh pmc_sizes_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_sizes_write -o run -- python3 bench.py --only-extra sizes --sizes-reps 10 --prewarm-s 0
