#!/bin/bash
# Round 3 final: smoke(), the driver-shaped N = 1 bench under rocprofv3
# kernel-trace stats, and the headline kernel's PMC traffic in separate
# FETCH_SIZE / WRITE_SIZE passes.
cd "$(dirname "$0")/.." || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" && \
tools/gpu_step.sh prof_bench 500 $P -d gpurun_out/prof_bench -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 && \
tools/gpu_step.sh pmc_fetch 150 timeout -s KILL 140 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extras && \
tools/gpu_step.sh pmc_write 150 timeout -s KILL 140 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu --no-extras
