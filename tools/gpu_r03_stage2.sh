#!/bin/bash
# Round 3, second GPU call: liblfa.so load cost (this build vs round 2's), the
# tree_put register-regime probe, the back-to-back combine A/B (scalar wave
# index vs round 2, drained steps), and the GPU suite with 4 / 5 / 8 members
# on the one-shot and flag-barrier paths.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_step.sh probe_load 200 python3 -u tools/probe_load.py --reps 3 && \
tools/gpu_step.sh probe_load_r2 200 python3 -u tools/probe_load.py --reps 3 --lib tools/_r2/liblfa.so && \
tools/gpu_step.sh treeput_probe 300 python3 -u tools/probe_treeput_narrow.py --probe --out gpurun_out/treeput_probe.json && \
tools/gpu_step.sh tune_combine 200 python3 -u tools/tune_combine.py --sizes 32,64,128,256 --variants 30,77,70,76 --rounds 15 && \
tools/gpu_step.sh gpu_tests 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
