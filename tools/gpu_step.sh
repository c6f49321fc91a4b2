#!/bin/bash
# Run one GPU step under its own time limit; stop the whole call on a fault.
#   tools/gpu_step.sh <name> <seconds> <cmd...>
# rc 0/1 (pass / ordinary test failure) → continue; anything else (abort 134,
# segfault 139, timeout 124/137, …) → exit 99 so the caller's && chain stops.
name=$1; secs=$2; shift 2
mkdir -p gpurun_out
echo "== $name: $*" >> gpurun_out/steps.log
timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
rc=$?
echo "== $name rc=$rc" >> gpurun_out/steps.log
tail -5 "gpurun_out/$name.log"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
  echo "STOP: $name exited $rc"; exit 99
fi
exit 0
