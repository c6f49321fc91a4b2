#!/bin/bash
# Round 3: soak of the random programs on GPU peer domains, many seeds
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh soak_dev 420 python3 -u tools/stress_soak.py --dev --worlds 2,3,4,5 --seeds 100-107 --nops 160 && \
tools/gpu_step.sh soak_mixed 240 python3 -u tools/stress_soak.py --dev --worlds 3,4 --seeds 200-205 --nops 160 --host-rank 0 --refuse-every 6
