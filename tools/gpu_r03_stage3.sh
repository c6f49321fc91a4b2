#!/bin/bash
# Round 3, third GPU call: the drained nt-path product kernel (every op
# family at 200 MiB, the headline sizes), the narrow-lane tree_put tests, the
# multi-member one-shot tests with every rank's outcome reported, the
# back-to-back A/B at 192-256 MiB, then the driver-shaped bench.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_step.sh combine_tests 400 python3 -u -m pytest tests/test_combine_gpu.py -x -v --timeout 200 --timeout-method thread && \
tools/gpu_step.sh peer_tests 700 python3 -u -m pytest tests/test_coll_peer_gpu.py -v --timeout 200 --timeout-method thread -k "mixed or every_reducing or c_executor" && \
tools/gpu_step.sh tune_combine 200 python3 -u tools/tune_combine.py --sizes 192,256 --variants 30,77,75 --rounds 15 && \
tools/gpu_step.sh bench 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5
