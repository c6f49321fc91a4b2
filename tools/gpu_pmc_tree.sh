#!/bin/bash
# HBM traffic of the fused tree kernel (8 -> 1 among others): FETCH_SIZE and
# WRITE_SIZE in separate rocprofv3 --pmc passes (no tracing domains).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
CMD="python3 bench.py --tune-tree --variants -1 --tune-rounds 1"
tools/gpu_step.sh pmc_tree_fetch 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_tree_fetch -o run -- $CMD && \
tools/gpu_step.sh pmc_tree_write 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_tree_write -o run -- $CMD
