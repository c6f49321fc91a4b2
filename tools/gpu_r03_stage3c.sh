#!/bin/bash
# Round 3: the mixed one-shot test at 3..8 members with the P2P staging copy
# now through write-through stores (twice), then the rest of the peer suite.
set -o pipefail
cd "$(dirname "$0")/.."
tools/gpu_step.sh mixed_a 400 python3 -u -m pytest tests/test_coll_peer_gpu.py -v --timeout 200 --timeout-method thread -k "mixed" && \
tools/gpu_step.sh mixed_b 400 python3 -u -m pytest tests/test_coll_peer_gpu.py -v --timeout 200 --timeout-method thread -k "mixed" && \
tools/gpu_step.sh peer_rest 500 python3 -u -m pytest tests/test_coll_peer_gpu.py -v --timeout 200 --timeout-method thread -k "not mixed"
