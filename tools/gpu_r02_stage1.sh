# P2P staging as one copy: the whole -m gpu suite, then the 2-process latency probe.
set -o pipefail
mkdir -p gpurun_out
bash tools/gpu_step.sh gpu_tests 600 python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread && \
bash tools/gpu_step.sh p2p_latency 240 python -u tools/probe_p2p_latency.py --world 2 --reps 300
