#!/bin/bash
# Round 3: the N -> 1 fused tree against what HBM gives its access mix (read
# side alone in the tree's load shape, write side alone, the tree), in
# separate allocations and in the collective's slot layout; 8 and 2 inputs.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh probe_tree_mix 240 python3 -u tools/probe_hbm.py --tree
