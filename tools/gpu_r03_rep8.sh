#!/bin/bash
cd "$(dirname "$0")" 2>/dev/null; cd $GRAFT_REPO_ROOT || exit 1
export TMPDIR=/tmp
for i in 1 2 3 4; do
  mkdir -p gpurun_out/peer_logs/run$i
  PEER_LOG_DIR=gpurun_out/peer_logs/run$i LFA_TRACE=1 LFA_SIG_TIMEOUT_MS=30000 tools/gpu_step.sh gpu_exec8_$i 300 python3 -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 250 --timeout-method thread -k "test_c_executor_gpu_kernels_across_processes and 8" || exit 1
  grep -q "1 passed" gpurun_out/gpu_exec8_$i.log || exit 0
done
