"""Cost of loading liblfa.so and of its first kernel launch, per process
(VERDICT r2 #7).  Each measurement runs in a FRESH child process (the code
objects are registered at dlopen and loaded on first use), timed from
inside: torch + HIP init, ctypes load of liblfa.so, the first combine launch
+ synchronize (code-object load), a second launch + synchronize.

    python tools/probe_load.py [--reps 3]
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, time, sys
sys.path.insert(0, %r)
t0 = time.perf_counter()
import torch
torch.cuda.init(); torch.zeros(1, device="cuda"); torch.cuda.synchronize()
t1 = time.perf_counter()
import ctypes, os
path = os.environ.get("PROBE_LIB") or os.path.join(%r, "libfabric_amd", "liblfa.so")
L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
L.lfa_atomic_write_async.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                                     ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
t2 = time.perf_counter()
a = torch.ones(1 << 20, device="cuda"); b = torch.ones(1 << 20, device="cuda")
torch.cuda.synchronize()
t3 = time.perf_counter()
assert L.lfa_atomic_write_async(2, 8, a.data_ptr(), b.data_ptr(), 1 << 20, None) == 0
torch.cuda.synchronize()
t4 = time.perf_counter()
assert L.lfa_atomic_write_async(6, 6, a.data_ptr(), b.data_ptr(), 1 << 19, None) == 0
torch.cuda.synchronize()
t5 = time.perf_counter()
assert L.lfa_atomic_write_async(2, 8, a.data_ptr(), b.data_ptr(), 1 << 20, None) == 0
torch.cuda.synchronize()
t6 = time.perf_counter()
print(json.dumps({"torch_hip_init_s": round(t1 - t0, 3), "dlopen_liblfa_ms": round((t2 - t1) * 1e3, 2),
                  "first_launch_ms": round((t4 - t3) * 1e3, 2),
                  "first_launch_other_op_ms": round((t5 - t4) * 1e3, 2),
                  "warm_launch_ms": round((t6 - t5) * 1e3, 3)}))
""" % (ROOT, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--lib", default="", help="another liblfa.so to time (A/B)")
    args = ap.parse_args()
    env = dict(os.environ, PROBE_LIB=os.path.abspath(args.lib) if args.lib else "")
    rows = []
    for _ in range(args.reps):
        r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True,
                           timeout=300, env=env)
        line = [x for x in r.stdout.splitlines() if x.startswith("{")]
        if r.returncode or not line:
            raise SystemExit(r.stdout + r.stderr)
        rows.append(json.loads(line[-1]))
        print(line[-1], flush=True)
    keys = rows[0].keys()
    med = {k: statistics.median(r[k] for r in rows) for k in keys}
    size = os.path.getsize(os.path.abspath(args.lib) if args.lib else
                           os.path.join(ROOT, "libfabric_amd", "liblfa.so"))
    print(json.dumps({"probe_load": med, "lib": args.lib or "libfabric_amd/liblfa.so",
                      "liblfa_so_bytes": size, "reps": args.reps}))


if __name__ == "__main__":
    main()
