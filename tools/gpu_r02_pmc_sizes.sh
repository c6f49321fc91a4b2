#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE, separate runs) of the headline kernel at
# 8..256 MiB per operand: roofline.traffic at the strong-scaling shard sizes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh pmc_fetch_sizes 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_sizes -o run -- python3 bench.py --only-extra sizes --sizes-reps 10 --prewarm-s 0 && \
tools/gpu_step.sh pmc_write_sizes 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_sizes -o run -- python3 bench.py --only-extra sizes --sizes-reps 10 --prewarm-s 0
