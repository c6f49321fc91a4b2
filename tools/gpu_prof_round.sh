#!/bin/bash
# Round profiling: rocprofv3 kernel-trace summaries (CSV) of the headline
# kernel, the P2P tree-put kernel and the 8-rank loopback allreduce.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
P="rocprofv3 --kernel-trace --stats --output-format csv"
tools/gpu_step.sh prof_headline 240 $P -d gpurun_out/prof_headline -o run -- python3 bench.py --steps 60 --warmup 40 --no-cpu --no-extras && \
tools/gpu_step.sh prof_treeput 240 $P -d gpurun_out/prof_treeput -o run -- python3 bench.py --only-extra tree_put && \
tools/gpu_step.sh prof_loopback 240 $P -d gpurun_out/prof_loopback -o run -- python3 tools/prof_loopback.py
