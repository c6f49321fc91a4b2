#!/bin/bash
# Round 3: the hypothesis property tests through the gfx950 kernels (random
# table entries, lengths, byte offsets, fan-ins and edge lanes vs the oracle),
# then the whole GPU suite (the one-shot and tree launchers changed).
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh gpu_props 700 python3 -u -m pytest tests/test_properties.py -m gpu -x -v --timeout 400 --timeout-method thread --hypothesis-show-statistics && \
tools/gpu_step.sh gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread
