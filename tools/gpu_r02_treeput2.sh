#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh tune_treeput2 300 python3 bench.py --tune-treeput --tune-rounds 10 --variants 0,2,10,12,13,14,15,16,17
