#!/bin/bash
# rocprofv3 kernel durations: product (buffer-store nt at 256 MiB) vs the
# global-store nt form (variant 20) in one process.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh prof_tune256 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tune256 -o run -- python3 bench.py --tune --variants 30,20,51 --tune-rounds 15
