#!/bin/bash
# Round check: GPU parity suite, then the loopback allreduce profile (tree
# kernel) and the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh pytest_gpu 500 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh prof_loopback 240 $P -d gpurun_out/prof_loopback -o run -- python3 tools/prof_loopback.py && \
tools/gpu_step.sh bench 300 python3 bench.py
