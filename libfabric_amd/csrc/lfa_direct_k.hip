// The direct-dispatch code object (lfa_direct.cpp): kernels that liblfa
// launches with its own AQL packets on its own HSA queue, not through HIP.
// Built device-only into a plain gfx950 ELF (build.py) and embedded in
// liblfa.so.  They read no hidden kernel arguments — the workgroup count
// comes as an explicit argument and the group size is fixed at 256 — so the
// packet's kernarg block is exactly the arguments below.
#include <hip/hip_runtime.h>
#include <stdint.h>

// lfa_solo_copy_async's kernel (lfa_solo_body.hpp: 16 KiB per workgroup
// when both pointers are 16-B aligned, 4 KiB byte-wise otherwise; the last
// workgroup to finish publishes `val`, a single one without the counter).
// Built twice: as lfa_direct_solo_copy, and as lfa_direct_solo_copy_pl with
// -mllvm -amdgpu-kernarg-preload-count=14, where the packet processor loads
// the 56-byte argument block into SGPRs before the wave starts instead of the
// wave's first scalar loads fetching it from host memory (build.py).
#include "lfa_solo_body.hpp"

#ifndef LFA_DIRECT_NAME
#define LFA_DIRECT_NAME lfa_direct_solo_copy
#endif
extern "C" __global__ __launch_bounds__(256) void LFA_DIRECT_NAME(
    char *dst, const char *src, uint64_t bytes, uint32_t nblocks, uint32_t *ctr,
    uint64_t *word, uint64_t val) {
  lfa_solo_body(dst, src, bytes, nblocks, ctr, word, val);
}
