#!/bin/bash
# Round 3, second GPU call: the tree_put register-regime probe, the
# back-to-back combine A/B (scalar wave index vs round 2, drained steps), and
# the GPU suite with 4 / 5 / 8 members on the one-shot and flag-barrier paths.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_step.sh treeput_probe 400 python3 -u tools/probe_treeput_narrow.py --probe --out gpurun_out/treeput_probe.json && \
tools/gpu_step.sh tune_combine 300 python3 -u tools/tune_combine.py --sizes 32,64,128,256 --variants 30,77,70,76 --rounds 15 && \
tools/gpu_step.sh gpu_tests 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
