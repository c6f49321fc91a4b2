#!/bin/bash
# Round 3: random programs of collectives over three groups on GPU peer
# domains (2-5 processes sharing the GPU; every algorithm, IPC workspaces,
# one-shot kernels), then the whole GPU suite.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out/stress_logs
STRESS_LOG_DIR=gpurun_out/stress_logs STRESS_STALL_S=40 tools/gpu_step.sh gpu_stress 600 python3 -u -m pytest tests/test_coll_stress.py -m gpu -x -v --timeout 200 --timeout-method thread && \
tools/gpu_step.sh gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
