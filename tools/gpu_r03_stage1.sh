#!/bin/bash
# Round 3, first GPU call: the tree_put narrow-lane probe and
# the drained-in-steps combine forms at the N = 8 shard, config-3 and headline
# sizes.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_step.sh treeput_narrow 400 python3 -u tools/probe_treeput_narrow.py --out gpurun_out/treeput_narrow.json && \
tools/gpu_step.sh tune_drain_32 300 python3 bench.py --tune --tune-rounds 12 --tune-bytes 33554432 --variants 30,70,71,72,73,74,75,76 && \
tools/gpu_step.sh tune_drain_64 300 python3 bench.py --tune --tune-rounds 12 --tune-bytes 67108864 --variants 30,70,71,72,73,74,75,76 && \
tools/gpu_step.sh tune_drain_256 300 python3 bench.py --tune --tune-rounds 10 --variants 30,70,71,72,75,76
