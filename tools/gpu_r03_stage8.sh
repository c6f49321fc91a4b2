#!/bin/bash
# Round 3: group chunk with a host member across processes (peer suite's
# c_executor test at 2..8), and the 2-process host-buffer 256 MiB allreduce
# with and without a group chunk.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh peer_cexec 600 python3 -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 200 --timeout-method thread -k "c_executor" && \
tools/gpu_step.sh host_group_chunk 300 python3 -u tools/probe_host_group_chunk.py --reps 5
