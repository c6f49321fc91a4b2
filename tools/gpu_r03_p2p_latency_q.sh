#!/bin/bash
# 8 processes sharing the GPU: small-bucket latency with fewer hardware queues
# per process (GPU_MAX_HW_QUEUES; the box default is 4).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for q in 2 1; do
  GPU_MAX_HW_QUEUES=$q tools/gpu_step.sh p2p_lat_8_q$q 200 python3 -u tools/probe_p2p_latency.py --world 8 --reps 300 || exit 1
done
