// The direct-dispatch code object (lfa_direct.cpp): kernels that liblfa
// launches with its own AQL packets on its own HSA queue, not through HIP.
// Built device-only into a plain gfx950 ELF (build.py) and embedded in
// liblfa.so.  They read no hidden kernel arguments — the workgroup count
// comes as an explicit argument and the group size is fixed at 256 — so the
// packet's kernarg block is exactly the arguments below.
#include <hip/hip_runtime.h>
#include <stdint.h>

// lfa_solo_copy_async's kernel (lfa_signal.hip solo_copy), same body and
// completion word: workgroup b copies bytes [b·4 KiB, (b+1)·4 KiB), 16 B per
// lane when both pointers are 16-B aligned, byte-wise otherwise and for the
// tail; the last workgroup to finish publishes `val` (a single workgroup
// publishes it without the counter).
// Built twice: as lfa_direct_solo_copy, and as lfa_direct_solo_copy_pl with
// -mllvm -amdgpu-kernarg-preload-count=14, where the packet processor loads
// the 56-byte argument block into SGPRs before the wave starts instead of the
// wave's first scalar loads fetching it from host memory (build.py).
#ifndef LFA_DIRECT_NAME
#define LFA_DIRECT_NAME lfa_direct_solo_copy
#endif
extern "C" __global__ __launch_bounds__(256) void LFA_DIRECT_NAME(
    char *dst, const char *src, uint64_t bytes, uint32_t nblocks, uint32_t *ctr,
    uint64_t *word, uint64_t val) {
  const unsigned t = __builtin_amdgcn_workitem_id_x();
  const uint64_t lo = (uint64_t)__builtin_amdgcn_workgroup_id_x() * 4096;
  const uint64_t hi = lo + 4096 < bytes ? lo + 4096 : bytes;
  const bool vec = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const uint64_t vhi = vec ? lo + ((hi - lo) & ~(uint64_t)15) : lo;
  if (lo + (uint64_t)t * 16 < vhi) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // write-through (sc0 sc1): nothing of the result stays dirty in this
    // XCD's L2, so the release before the word has no lines to write back
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + lo, 0, 4096, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)(src + lo + (uint64_t)t * 16), r,
                                           t * 16, 0, 17);
  }
  for (uint64_t o = vhi + t; o < hi; o += 256) dst[o] = src[o];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (nblocks == 1) {
    // one workgroup (up to 4 KiB): no counter to count in
    if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  if (t == 0) {
    // lfa_signal.hip solo_copy's ordering: a workgroup whose stores were all
    // write-through adds with no fence; byte-wise stores are released first
    if (vhi != hi) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const uint32_t seen =
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen + 1 == nblocks) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}
