#!/bin/bash
# Remaining cache-policy bits on the headline body (variants 56-59) against
# the product (30), 256 MiB, under rocprofv3 kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh tune_cpol256 240 $P -d gpurun_out/prof_cpol256 -o run -- python3 bench.py --tune --variants 30,56,57,58,59,50 --tune-rounds 12
