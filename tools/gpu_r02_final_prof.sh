#!/bin/bash
# End-of-session evidence: smoke(), then the driver-shaped N=1 bench (extras
# included) under rocprofv3 kernel-trace stats, so the profile and the bench
# line come from the same command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
tools/gpu_step.sh smoke 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" && \
tools/gpu_step.sh prof_bench 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
