#!/bin/bash
# Round 2: product combine vs size, config-3 kernels traced + PMC, and tuning
# variants at the strong-scaling shard sizes (32 / 64 MiB per operand).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh sizes 200 python3 bench.py --only-extra sizes && \
tools/gpu_step.sh prof_config3 200 $P -d gpurun_out/prof_config3 -o run -- python3 bench.py --only-extra config3 && \
tools/gpu_step.sh pmc_fetch_config3 120 timeout -s KILL 100 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch_c3 -o run -- python3 bench.py --only-extra config3 && \
tools/gpu_step.sh pmc_write_config3 120 timeout -s KILL 100 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write_c3 -o run -- python3 bench.py --only-extra config3 && \
tools/gpu_step.sh tune32 300 python3 bench.py --tune --tune-bytes 33554432 --tune-rounds 12 --variants 30,20,24,25,31,32,33,34,51,22,40,47 && \
tools/gpu_step.sh tune64 300 python3 bench.py --tune --tune-bytes 67108864 --tune-rounds 12 --variants 30,20,24,25,31,32,33,34,51,22,40,47
