# One-shot reduce_scatter / reduce (LFA_ALGO_P2P): peer-domain tests, the
# whole -m gpu suite, the latency probe, and its rocprofv3 kernel trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/gpu_step.sh peer_tests 300 python -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 150 --timeout-method thread && \
bash tools/gpu_step.sh gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread && \
bash tools/gpu_step.sh p2p_latency 240 python -u tools/probe_p2p_latency.py --world 2 --reps 300 && \
bash tools/gpu_step.sh p2p_latency_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p2p -o p2p -- python3 -u tools/probe_p2p_latency.py --world 2 --reps 100
