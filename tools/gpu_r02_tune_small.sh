#!/bin/bash
# Register-staged and block-shape variants against the product at the
# strong-scaling shard sizes (16 / 32 / 64 MiB per operand).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for b in 16777216 33554432 67108864; do
  tools/gpu_step.sh tune_small_$b 300 python3 bench.py --tune --tune-bytes $b --tune-rounds 12 --variants 30,0,1,2,3,12,13,14,15,18,19,23,33 || exit 1
done
