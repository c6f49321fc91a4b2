#!/bin/bash
# test_oneshot_every_reducing_entry[8] with 2 and with 4 hardware queues per process
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
for q in 2 4; do
  LFA_TEST_HW_QUEUES=$q tools/gpu_step.sh every8_q$q 250 python3 -u -m pytest tests/test_coll_peer_gpu.py -x -v --timeout 240 --timeout-method thread --durations=3 -k "test_oneshot_every_reducing_entry and 8" || exit 1
done
