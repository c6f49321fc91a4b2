#!/bin/bash
# Round 3: a longer soak of the random programs on GPU peer domains
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh soak2_dev 900 python3 -u tools/stress_soak.py --dev --worlds 2,3,4,5 --seeds 300-339 --nops 200
