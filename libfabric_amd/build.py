"""Build the in-tree native libraries for gfx950.

  libfabric_amd/liblfa.so       combine kernels + C ABI (include/lfa_atomic.h)
  libfabric_amd/liblfa_coll.so  C host provider (include/lfa_coll.h), links
                                liblfa.so + RCCL

hipcc cross-compiles gfx950 without a GPU.  Objects are cached under
build/ by source mtime; the kernel file is compiled once per write op in
parallel (-DLFA_OP=<op>).  Run:  python -m libfabric_amd.build
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
INC = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build", "lfa")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"
# every enum fi_op row of the three tables: write+fetch 0..11, compare 12..18
WRITE_OPS = list(range(19))

HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-ffp-contract=off", "-fPIC",
             "-std=c++17", "-Wall", "-Wno-unused-function", "-I" + INC]

LIB_LFA = os.path.join(PKG, "liblfa.so")
LIB_TUNE = os.path.join(PKG, "liblfa_tune.so")
LIB_COLL = os.path.join(PKG, "liblfa_coll.so")


def _newer(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _run(cmd: list[str]) -> None:
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        sys.stderr.write(" ".join(cmd) + "\n" + r.stdout + r.stderr)
        raise RuntimeError(f"build step failed: {cmd[0]} … {cmd[-1]}")


def build_lfa(jobs: int = 8, verbose: bool = False) -> str:
    os.makedirs(BUILD, exist_ok=True)
    kern = os.path.join(CSRC, "lfa_combine.hip")
    hdrs = [os.path.join(CSRC, "lfa_ops.hpp"), os.path.join(CSRC, "lfa_kernels.hpp"),
            *(os.path.join(CSRC, f"lfa_k_{p}.hpp") for p in ("tree", "oneshot", "fetch", "launch")),
            os.path.join(INC, "lfa_atomic.h"), os.path.join(INC, "lfa_fabric.h")]
    steps = []
    objs = []
    for op in WRITE_OPS:
        o = os.path.join(BUILD, f"combine_op{op}.o")
        objs.append(o)
        if _newer(o, [kern] + hdrs):
            steps.append([HIPCC, *HIP_FLAGS, f"-DLFA_OP={op}", "-c", kern, "-o", o])
    # tuning-only kernel forms (bench.py --tune*): their own library
    tune_objs = []
    for name in ("lfa_tune", "lfa_tune_b"):
        tune = os.path.join(CSRC, name + ".hip")
        tune_o = os.path.join(BUILD, name + ".o")
        tune_objs.append(tune_o)
        if _newer(tune_o, [tune] + hdrs):
            steps.append([HIPCC, *HIP_FLAGS, "-c", tune, "-o", tune_o])
    # the tree_put register-pressure probe (tools/probe_treeput_narrow.py)
    probe = os.path.join(CSRC, "lfa_probe.hip")
    probe_o = os.path.join(BUILD, "lfa_probe.o")
    tune_objs.append(probe_o)
    if _newer(probe_o, [probe] + hdrs):
        steps.append([HIPCC, *HIP_FLAGS, "-c", probe, "-o", probe_o])
    # op-independent device code: the P2P flag barrier
    sig = os.path.join(CSRC, "lfa_signal.hip")
    o = os.path.join(BUILD, "lfa_signal.o")
    objs.append(o)
    if _newer(o, [sig, os.path.join(CSRC, "lfa_signal.h"), os.path.join(CSRC, "lfa_solo_body.hpp"),
                  os.path.join(INC, "lfa_fabric.h")]):
        steps.append([HIPCC, *HIP_FLAGS, "-c", sig, "-o", o])
    # the direct-dispatch code object: a plain gfx950 ELF of lfa_direct_k.hip,
    # embedded as bytes (lfa_direct.cpp loads it into its own HSA executable)
    dk = os.path.join(CSRC, "lfa_direct_k.hip")
    co_c = os.path.join(BUILD, "lfa_direct_co.c")
    co_o = os.path.join(BUILD, "lfa_direct_co.o")
    objs.append(co_o)
    if _newer(co_o, [dk, os.path.join(CSRC, "lfa_solo_body.hpp")]):
        # two code objects: the kernel as is, and with its arguments preloaded
        # into SGPRs by the packet processor (lfa_direct_k.hip)
        with open(co_c, "w") as f:
            f.write("#include <stddef.h>\n")
            for sym, extra in (("lfa_direct_co", []),
                               ("lfa_direct_co_pl",
                                ["-DLFA_DIRECT_NAME=lfa_direct_solo_copy_pl", "-mllvm",
                                 "-amdgpu-kernarg-preload-count=14"])):
                co = os.path.join(BUILD, sym + ".hsaco")
                _run([os.path.join(ROCM, "lib", "llvm", "bin", "clang++"), "-x", "hip",
                      "--offload-device-only", "--offload-arch=" + ARCH,
                      "--no-gpu-bundle-output", "-O3", "-std=c++17", *extra, "-o", co, dk])
                data = open(co, "rb").read()
                f.write(f"const unsigned char {sym}[] __attribute__((aligned(4096))) = {{\n")
                for i in range(0, len(data), 16):
                    f.write(",".join(str(b) for b in data[i:i + 16]) + ",\n")
                f.write(f"}};\nconst size_t {sym}_size = sizeof({sym});\n")
        _run(["gcc", "-O2", "-fPIC", "-c", co_c, "-o", co_o])
    direct = os.path.join(CSRC, "lfa_direct.cpp")
    o = os.path.join(BUILD, "lfa_direct.o")
    objs.append(o)
    if _newer(o, [direct, os.path.join(CSRC, "lfa_signal.h")]):
        steps.append(["g++", "-O2", "-fPIC", "-std=c++17", "-Wall",
                      "-D__HIP_PLATFORM_AMD__", "-I" + INC,
                      "-I" + os.path.join(ROCM, "include"), "-c", direct, "-o", o])
    capi = os.path.join(CSRC, "lfa_capi.cpp")
    o = os.path.join(BUILD, "lfa_capi.o")
    objs.append(o)
    if _newer(o, [capi] + hdrs):
        # host-only C++ (hipcc would compile .cpp as HIP): g++ + HIP C API
        steps.append(["g++", "-O2", "-fPIC", "-std=c++17", "-Wall",
                      "-D__HIP_PLATFORM_AMD__", "-I" + INC,
                      "-I" + os.path.join(ROCM, "include"), "-c", capi, "-o", o])
    host = os.path.join(CSRC, "lfa_host.cpp")
    o = os.path.join(BUILD, "lfa_host.o")
    objs.append(o)
    if _newer(o, [host] + hdrs):
        # the host-memory combine: the kernels' functors compiled by g++,
        # no FMA contraction (as the reference's x86-64 build)
        steps.append(["g++", "-O3", "-fPIC", "-std=c++17", "-Wall", "-ffp-contract=off",
                      "-I" + INC, "-c", host, "-o", o])
    if steps:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for f in [ex.submit(_run, s) for s in steps]:
                f.result()
    if steps or _newer(LIB_LFA, objs):
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB_LFA,
              *objs, "-L" + os.path.join(ROCM, "lib"), "-lhsa-runtime64",
              "-Wl,-soname,liblfa.so"])
    if _newer(LIB_TUNE, tune_objs + [LIB_LFA]):
        # the tuning forms share the product's launchers, which call into
        # liblfa.so (lfa__wallclock_ticks_per_us)
        _run([HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", LIB_TUNE,
              *tune_objs, "-L" + PKG, "-llfa", "-Wl,-rpath,$ORIGIN",
              "-Wl,-soname,liblfa_tune.so"])
    if verbose:
        print(f"built {LIB_LFA} ({len(steps)} objects recompiled)")
    return LIB_LFA


def build_coll(verbose: bool = False) -> str | None:
    src = os.path.join(CSRC, "lfa_coll.c")
    if not os.path.exists(src):
        return None
    # API + endpoints, completion words, P2P workspaces, host buffers, group
    # join, executor + transports, planner, single-GPU loopback
    srcs = [src] + [os.path.join(CSRC, f) for f in
                    ("lfa_coll_word.c", "lfa_coll_ws.c", "lfa_coll_host.c",
                     "lfa_coll_group.c", "lfa_coll_exec.c", "lfa_coll_plan.c",
                     "lfa_coll_loopback.c")]
    hdrs = [os.path.join(INC, "lfa_coll.h"), os.path.join(INC, "lfa_atomic.h"),
            os.path.join(INC, "lfa_fabric.h"), os.path.join(CSRC, "lfa_coll_plan.h"),
            os.path.join(CSRC, "lfa_coll_int.h"), os.path.join(CSRC, "lfa_signal.h"), LIB_LFA]
    if _newer(LIB_COLL, srcs + hdrs):
        # Plain C (the reference's host language), calling HIP's and RCCL's
        # C APIs; no HIP device code in this library.
        _run(["gcc", "-O2", "-fPIC", "-std=gnu11", "-Wall", "-Wextra",
              "-Wno-unused-parameter", "-D__HIP_PLATFORM_AMD__", "-I" + INC,
              "-I" + os.path.join(ROCM, "include"), "-shared", "-o", LIB_COLL, *srcs,
              "-L" + PKG, "-llfa", "-L" + os.path.join(ROCM, "lib"), "-lamdhip64",
              "-lrccl", "-lpthread", "-Wl,-rpath,$ORIGIN",
              "-Wl,-soname,liblfa_coll.so"])
        if verbose:
            print(f"built {LIB_COLL}")
    return LIB_COLL


LIB_BENCH = os.path.join(PKG, "liblfa_bench.so")


def build_bench(verbose: bool = False) -> str | None:
    """liblfa_bench.so: bench-only C helpers (lfa_bench_loop), linked to the
    provider; never loaded by the product path."""
    src = os.path.join(CSRC, "lfa_bench.c")
    if not os.path.exists(src):
        return None
    if _newer(LIB_BENCH, [src, os.path.join(INC, "lfa_coll.h"), LIB_COLL, LIB_LFA]):
        _run(["gcc", "-O2", "-fPIC", "-std=gnu11", "-Wall", "-Wextra",
              "-Wno-unused-parameter", "-D__HIP_PLATFORM_AMD__", "-I" + INC,
              "-I" + os.path.join(ROCM, "include"), "-shared", "-o", LIB_BENCH, src,
              "-L" + PKG, "-llfa_coll", "-llfa", "-L" + os.path.join(ROCM, "lib"),
              "-lamdhip64", "-Wl,-rpath,$ORIGIN", "-Wl,-soname,liblfa_bench.so"])
        if verbose:
            print(f"built {LIB_BENCH}")
    return LIB_BENCH


EXAMPLE = os.path.join(ROOT, "examples", "c_drop_in")


def build_example(verbose: bool = False) -> str | None:
    """Plain-C caller of both libraries (no torch): examples/c_drop_in."""
    src = EXAMPLE + ".c"
    if not os.path.exists(src):
        return None
    if _newer(EXAMPLE, [src, LIB_LFA, LIB_COLL]):
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-D__HIP_PLATFORM_AMD__",
              "-I" + INC, "-I" + os.path.join(ROCM, "include"), "-o", EXAMPLE, src,
              "-L" + PKG, "-llfa", "-llfa_coll", "-L" + os.path.join(ROCM, "lib"),
              "-lamdhip64", "-Wl,-rpath," + PKG, "-Wl,-rpath,$ORIGIN/../libfabric_amd"])
        if verbose:
            print(f"built {EXAMPLE}")
    return EXAMPLE


# libfabric's public headers: only this container has them.  The provider
# shell and its host driver compile against them here; the built files travel
# to the GPU box with the snapshot (as oracle/_ref does).
FABRIC_INC = os.environ.get("LFA_FABRIC_INCLUDE", "/root/reference/include")
LIB_OFF = os.path.join(PKG, "liboff_lfa-fi.so")
OFF_HOST = os.path.join(ROOT, "examples", "off_lfa_host")
OFF_PEER = os.path.join(ROOT, "examples", "off_lfa_peer")


def have_fabric_headers() -> bool:
    return os.path.exists(os.path.join(FABRIC_INC, "rdma", "providers", "fi_peer.h"))


def build_off_lfa(verbose: bool = False) -> str | None:
    """libfabric offload-collective provider (liboff_lfa-fi.so) over
    liblfa_coll.so, plus the rxm-shaped host driver examples/off_lfa_host."""
    src = os.path.join(CSRC, "off_lfa.c")
    srcs = [src, os.path.join(CSRC, "off_lfa_ep.c")]
    host = OFF_HOST + ".c"
    if not have_fabric_headers():
        if verbose:
            print("libfabric headers absent: off_lfa not rebuilt "
                  f"({'prebuilt present' if os.path.exists(LIB_OFF) else 'missing'})")
        return LIB_OFF if os.path.exists(LIB_OFF) else None
    hdrs = [os.path.join(INC, "lfa_coll.h"), os.path.join(INC, "off_lfa.h"),
            os.path.join(CSRC, "off_lfa_int.h"), LIB_COLL]
    if _newer(LIB_OFF, srcs + hdrs):
        _run(["gcc", "-O2", "-fPIC", "-std=gnu11", "-Wall", "-Wextra",
              "-Wno-unused-parameter", "-I" + INC, "-I" + FABRIC_INC, "-shared",
              "-o", LIB_OFF, *srcs, "-L" + PKG, "-llfa_coll", "-llfa", "-lpthread",
              "-Wl,-rpath,$ORIGIN", "-Wl,-soname,liboff_lfa-fi.so"])
        if verbose:
            print(f"built {LIB_OFF}")
    stub = os.path.join(ROOT, "examples", "fi_param_stub.h")
    if _newer(OFF_HOST, [host, os.path.join(INC, "off_lfa.h"), stub]):
        # -rdynamic: the provider's fi_param_* references resolve to the
        # owner's stubs (examples/fi_param_stub.h), as to libfabric's core
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Wno-unused-parameter",
              "-rdynamic", "-D__HIP_PLATFORM_AMD__", "-I" + INC, "-I" + FABRIC_INC,
              "-I" + os.path.join(ROCM, "include"), "-o", OFF_HOST, host,
              "-L" + os.path.join(ROCM, "lib"), "-lamdhip64", "-ldl"])
        if verbose:
            print(f"built {OFF_HOST}")
    if _newer(OFF_PEER, [OFF_PEER + ".c", os.path.join(INC, "off_lfa.h"), stub]):
        # the multi-process owner with its own tagged transport: no HIP
        _run(["gcc", "-O2", "-std=gnu11", "-Wall", "-Wextra", "-Wno-unused-parameter",
              "-rdynamic", "-I" + INC, "-I" + FABRIC_INC, "-o", OFF_PEER, OFF_PEER + ".c", "-ldl",
              "-lpthread"])
        if verbose:
            print(f"built {OFF_PEER}")
    return LIB_OFF


def build_all(verbose: bool = False) -> None:
    build_lfa(verbose=verbose)
    build_coll(verbose=verbose)
    build_bench(verbose=verbose)
    build_example(verbose=verbose)
    build_off_lfa(verbose=verbose)


if __name__ == "__main__":
    build_all(verbose=True)
