#!/bin/bash
# Round 2: the bench as the driver runs it (N=1, 20/5), the default bench,
# and a rocprofv3 kernel-trace summary of the driver-shaped command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh bench_driver 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 && \
tools/gpu_step.sh prof_driver 240 $P -d gpurun_out/prof_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-extras
