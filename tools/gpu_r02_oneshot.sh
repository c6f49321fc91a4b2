# Flag barrier + one-shot allreduce (LFA_ALGO_P2P) on the GPU: the peer-domain
# cross-process tests first, then the whole -m gpu suite, then the latency probe.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_step.sh peer_tests 300 python -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 150 --timeout-method thread && \
bash tools/gpu_step.sh gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread && \
bash tools/gpu_step.sh p2p_latency 240 python -u tools/probe_p2p_latency.py --world 2 --reps 300 && \
bash tools/gpu_step.sh p2p_latency3 240 python -u tools/probe_p2p_latency.py --world 3 --reps 300
