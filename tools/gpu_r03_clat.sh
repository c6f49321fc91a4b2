#!/bin/bash
# Round 3: provider latency with the C-timed loop beside the Python-timed one:
# P2P peer domains at 2 and 4 processes, and the N = 1 bench's collectives
# extras (RCCL device domain at world size 1).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for w in 2 4; do
  tools/gpu_step.sh clat_$w 200 python3 -u tools/probe_p2p_latency.py --world $w --reps 300 || exit 1
done
tools/gpu_step.sh bench_n1 400 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
