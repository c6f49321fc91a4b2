#!/bin/bash
# Round 3: the fixed part of one combine launch from below (4 KiB .. 4 MiB
# kernel-trace durations), and the tree_put tests after the store-order revert.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh floor 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/floor -o run -- python3 tools/probe_launch_floor.py && \
tools/gpu_step.sh treeput_tests 300 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "tree_put or treeput"
