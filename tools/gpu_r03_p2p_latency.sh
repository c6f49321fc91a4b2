#!/bin/bash
# Round 3: provider-path small-bucket latency of LFA_ALGO_P2P (one-shot and
# flag-barrier paths) with 2, 4 and 8 processes sharing the GPU.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for w in 2 4 8; do
  tools/gpu_step.sh p2p_lat_$w 200 python3 -u tools/probe_p2p_latency.py --world $w --reps 300 || exit 1
done
