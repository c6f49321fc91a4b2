#!/bin/bash
# Round 3: tree_put store pacing A/B (8 -> 1 / 8 -> 8), the readwrite drained
# body confirmed against the round-2 form, then the full GPU suite.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh tune_treeput 300 python3 -u bench.py --tune-treeput --variants 0,14,18,19,20,21,22 --tune-rounds 10 && \
FETCH_VARIANTS=4,6,7 tools/gpu_step.sh tune_fetch 240 python3 -u tools/probe_fetch.py --tune && \
tools/gpu_step.sh gpu_suite 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
