#!/usr/bin/env python3
"""Exercise the collective schedules' GPU work on one MI355X for profiling:
8 ranks' allreduce of 256 MiB float SUM each (configs[3] shape) through
lfa_coll_loopback, TREE, RD and P2P algorithms, then print per-op wall times.
Run under rocprofv3 --kernel-trace --stats to see the kernel mix."""
import sys
import time

import torch

sys.path.insert(0, ".")
from libfabric_amd import coll  # noqa: E402

N, COUNT = 8, 64 * 1024 * 1024
sends = [torch.rand(COUNT, device="cuda") for _ in range(N)]
results = [torch.empty_like(s) for s in sends]
for name, algo in (("tree", coll.ALGO_TREE), ("rd", coll.ALGO_RD), ("p2p", coll.ALGO_P2P)):
    coll.loopback(3, algo, N, -1, 8, 2, COUNT, sends, results)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        coll.loopback(3, algo, N, -1, 8, 2, COUNT, sends, results)
    torch.cuda.synchronize()
    print(name, "ms per 8-rank allreduce on one GPU:",
          round((time.perf_counter() - t0) / 3 * 1e3, 2))
# exactness across algorithms: both equal the reference order
a = [torch.empty_like(s) for s in sends]
coll.loopback(3, coll.ALGO_TREE, N, -1, 8, 2, COUNT, sends, a)
b = [torch.empty_like(s) for s in sends]
coll.loopback(3, coll.ALGO_RD, N, -1, 8, 2, COUNT, sends, b)
c = [torch.empty_like(s) for s in sends]
coll.loopback(3, coll.ALGO_P2P, N, -1, 8, 2, COUNT, sends, c)
torch.cuda.synchronize()
print("tree == rd bitwise:", all(torch.equal(x, y) for x, y in zip(a, b)))
print("tree == p2p bitwise:", all(torch.equal(x, y) for x, y in zip(a, c)))
