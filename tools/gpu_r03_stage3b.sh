#!/bin/bash
# Round 3: the combine tests again (fixed nt-path test) and the diagnosis of
# the mixed one-shot test at 3 / 4 members: the default mix (one-shots with
# two-barrier allreduces between them) and one-shots alone.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_step.sh combine_tests 400 python3 -u -m pytest tests/test_combine_gpu.py -x -v --timeout 200 --timeout-method thread && \
tools/gpu_step.sh mixed_all 300 python3 -u -m pytest tests/test_coll_peer_gpu.py -v --timeout 200 --timeout-method thread -k "mixed and (3 or 4)" && \
ONESHOT_MIX=small tools/gpu_step.sh mixed_small 300 python3 -u -m pytest tests/test_coll_peer_gpu.py -v --timeout 200 --timeout-method thread -k "mixed and (3 or 4)"
