#!/usr/bin/env python3
"""Soak run of tests/test_coll_stress.py's random programs over many seeds
(dev tool; GPU box for --dev).  Prints one line per program and stops at the
first failure.

  python tools/stress_soak.py [--dev] [--worlds 2,3,4,5] [--seeds 100-119] [--nops 160]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dev", action="store_true")
    ap.add_argument("--worlds", default="2,3,4,5")
    ap.add_argument("--seeds", default="100-109")
    ap.add_argument("--nops", type=int, default=160)
    ap.add_argument("--host-rank", type=int, default=-1)
    ap.add_argument("--refuse-every", type=int, default=0)
    a = ap.parse_args()
    import test_coll_stress as T
    lo, hi = (int(x) for x in a.seeds.split("-"))
    n = 0
    for seed in range(lo, hi + 1):
        for w in (int(x) for x in a.worlds.split(",")):
            t0 = time.time()
            T._run(w, seed, a.nops, dev=a.dev, timeout=100,
                   host_rank=a.host_rank if w > 1 else -1, refuse_every=a.refuse_every)
            n += 1
            print(f"ok world={w} seed={seed} ({time.time() - t0:.1f} s)", flush=True)
    print(f"SOAK OK: {n} programs", flush=True)


if __name__ == "__main__":
    main()
