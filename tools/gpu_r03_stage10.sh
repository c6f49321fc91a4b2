#!/bin/bash
# Round 3: the mixed one-shot test with more seeds / longer sequences, then
# the 2-process host-buffer 256 MiB allreduce with and without a group chunk.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh mixed 500 python3 -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 200 --timeout-method thread -k "mixed" && \
tools/gpu_step.sh host_group_chunk 400 python3 -u tools/probe_host_group_chunk.py --reps 5
