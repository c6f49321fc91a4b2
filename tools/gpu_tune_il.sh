#!/bin/bash
# Workgroup-interleaved LDS-DMA tiles (variants 60-63) against the product
# (30), 256 MiB and 64 MiB, under rocprofv3 kernel trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh tune_il256 240 $P -d gpurun_out/prof_il256 -o run -- python3 bench.py --tune --variants 30,60,61,62,63 --tune-rounds 12 && \
tools/gpu_step.sh tune_il64 240 $P -d gpurun_out/prof_il64 -o run -- python3 bench.py --tune --variants 30,60,61,62,63 --tune-rounds 12 --tune-bytes 67108864
