#!/usr/bin/env python3
"""The fixed part of one combine_lds launch, measured from
below: float SUM combines of 4 KiB … 4 MiB per operand, 200 launches each,
back to back on one stream.  Run it under

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/floor \
        -o run -- python3 tools/probe_launch_floor.py

and read the per-grid kernel durations from the trace (tools/kernel_sizes.py).
At 4 KiB one wave loads its two 4 KiB tiles and stores one, so the kernel's
duration is one dispatch + one HBM load round trip + one write-through store:
the floor under which no launch of this kernel, at any size, can finish.
Every result is checked against dst + src.
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from libfabric_amd import atomic  # noqa: E402

FI_SUM, FI_FLOAT = 2, 8


def main():
    torch.cuda.set_device(0)
    s = torch.cuda.current_stream()
    for kib in (4, 16, 64, 256, 1024, 4096):
        n = kib * 256
        d = torch.rand(n, device="cuda")
        x = torch.rand(n, device="cuda")
        want = d + x
        atomic.write(FI_SUM, FI_FLOAT, d, x, n, s)
        torch.cuda.synchronize()
        assert torch.equal(d, want), kib
        for _ in range(200):
            atomic.write(FI_SUM, FI_FLOAT, d, x, n, s)
        torch.cuda.synchronize()
        print(f"{kib} KiB: 201 launches", flush=True)


if __name__ == "__main__":
    main()
