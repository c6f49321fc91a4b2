# One-shot kernel after the fence change: GPU time (probe), the peer-domain
# tests (flag barrier, one-shot every entry, mixed in flight), whole suite.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_step.sh probe_oneshot 150 python -u tools/probe_oneshot.py && \
bash tools/gpu_step.sh peer_tests 300 python -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 200 --timeout-method thread && \
bash tools/gpu_step.sh gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
