#!/bin/bash
# GPU parity suite + the P2P kernel extra.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
tools/gpu_step.sh smoke 200 python3 -c "import __graft_entry__ as g; g.smoke()" && \
tools/gpu_step.sh pytest_gpu 700 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread && \
tools/gpu_step.sh treeput 200 python3 bench.py --only-extra tree_put
