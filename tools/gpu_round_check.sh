#!/bin/bash
# Round check: smoke, GPU parity suite, rocprofv3 of the headline kernel, then
# the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh pytest_gpu 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh prof_headline 240 $P -d gpurun_out/prof_headline -o run -- python3 bench.py --steps 60 --warmup 40 --no-cpu --no-extras && \
tools/gpu_step.sh bench 300 python3 bench.py
