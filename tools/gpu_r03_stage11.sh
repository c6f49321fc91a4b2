#!/bin/bash
# Round 3, after the container re-creation: validate HEAD on one GPU —
# smoke(), the whole GPU suite, and the driver-shaped bench under rocprofv3.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" && \
tools/gpu_step.sh gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread && \
tools/gpu_step.sh prof_bench 500 $P -d gpurun_out/prof_bench -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5
