#!/bin/bash
# rocprofv3 kernel durations of the store-policy variants (nt product vs sc1
# write-through) at several buffer sizes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
for mib in 16 32 64 128 256; do
  tools/gpu_step.sh prof_tune$mib 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_tune$mib -o run -- python3 bench.py --tune --variants 30,51 --tune-rounds 10 --tune-bytes $((mib * 1048576)) || exit 1
done
