# The mixed in-flight one-shot test, then the whole -m gpu suite.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_step.sh peer_tests 300 python -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 150 --timeout-method thread && \
bash tools/gpu_step.sh gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread
