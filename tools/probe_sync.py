#!/usr/bin/env python3
"""Fixed wall-clock cost of bench.py's timed region (dev probe, GPU box).

The timed region is: barrier, synchronize, t0, K launches, synchronize, t1.
Its wall time minus the K kernels' GPU time is a fixed cost (first-launch
latency + the wake-up of the final synchronize) that a short strong-scaled
region (K = 20 launches of a 32 MiB shard) pays in full.  This probe
measures it per host wait mode, each mode in its own child process because
the HIP device flags must be set before the runtime creates the context:

  auto   HIP default (hipDeviceScheduleAuto)
  spin   hipSetDeviceFlags(hipDeviceScheduleSpin) before the first GPU call
  yield  hipSetDeviceFlags(hipDeviceScheduleYield)

Prints one JSON line per (mode, operand size, K).
"""
from __future__ import annotations

import json
import os
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FLAGS = {"auto": None, "spin": 1, "yield": 2}


def child(mode: str) -> None:
    import ctypes
    import torch
    if FLAGS[mode] is not None:
        # the HIP runtime torch already loaded (same instance liblfa.so binds)
        path = next(ln.split()[-1] for ln in open("/proc/self/maps")
                    if "libamdhip64.so" in ln)
        rc = ctypes.CDLL(path).hipSetDeviceFlags(ctypes.c_uint(FLAGS[mode]))
        assert rc == 0, rc
    from libfabric_amd import atomic
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    for mib in (256, 32):
        count = mib * (1 << 20) // 4
        nsets = max(4, (1 << 30) // (8 * count))
        sets = [(torch.rand(count, device="cuda"), torch.rand(count, device="cuda"))
                for _ in range(nsets)]

        def step(i):
            d, s = sets[i % nsets]
            atomic.write(2, 8, d, s, count, stream)
        t = time.perf_counter()
        n = 0
        while time.perf_counter() - t < 0.3:
            step(n)
            n += 1
        torch.cuda.synchronize()
        for k in (0, 1, 20):
            walls, gpus = [], []
            for rep in range(40):
                e0 = torch.cuda.Event(enable_timing=True)
                e1 = torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                e0.record(stream)
                for i in range(k):
                    step(i + rep)
                e1.record(stream)
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                walls.append((t1 - t0) * 1e6)
                gpus.append(e0.elapsed_time(e1) * 1e3)
            w, g = statistics.median(walls), statistics.median(gpus)
            print(json.dumps({"mode": mode, "mib": mib, "k": k, "wall_us": round(w, 1),
                              "gpu_us": round(g, 1), "fixed_us": round(w - g, 1),
                              "wall_p90_us": round(statistics.quantiles(walls, n=10)[-1], 1)}),
                  flush=True)
        del sets
        torch.cuda.empty_cache()


def main() -> int:
    if len(sys.argv) > 2 and sys.argv[1] == "--child":
        child(sys.argv[2])
        return 0
    rc = 0
    for mode in FLAGS:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), "--child", mode],
                           timeout=120)
        rc = rc or r.returncode
        if r.returncode != 0:
            break
    return rc


if __name__ == "__main__":
    sys.exit(main())
