#!/bin/bash
# Round 3: peer domains honour the group chunk under P2P (async staged
# H2D / D2H, issued-hop ordering): the whole peer suite, the off_lfa device
# tests, then the 2-process host-buffer 256 MiB allreduce probe.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh peer_suite 700 python3 -u -m pytest tests/test_coll_peer_gpu.py tests/test_off_lfa.py -m gpu -x -v --timeout 200 --timeout-method thread && \
tools/gpu_step.sh host_group_chunk 300 python3 -u tools/probe_host_group_chunk.py --reps 5
