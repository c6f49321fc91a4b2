// lfa_solo_body.hpp — the world-1 copy that ends in the completion word
// (lfa_signal.h), shared by lfa_solo_copy_async's HIP kernel (lfa_signal.hip)
// and the direct-dispatch kernel (lfa_direct_k.hip, built on its own into
// the code object liblfa's HSA queue runs).  Device code only.
//
// Workgroup b copies bytes [b·tile, (b+1)·tile) of `bytes`: tile = 16 KiB
// when both pointers are 16-B aligned — four 16-B loads in flight per lane,
// all issued before the write-through stores, then the tail byte-wise —
// and 4 KiB byte-wise otherwise (lfa_solo_blocks gives the host the same
// grid).  16 KiB tiles took 0.8-1.4 us less from launch to word than 4 KiB
// ones between 16 KiB and 1 MiB (round 5, tools/probe_solo_multi.py).
//
// The word: write-through stores are in memory once acknowledged (the
// s_waitcnt), so a workgroup that made only those adds to the counter
// relaxed, with no release of its own; one with byte-wise (plain) stores
// releases them at system scope first.  The last workgroup acquires the
// others' adds, resets the counter for the next launch and releases before
// it publishes `val`; a single workgroup publishes with no counter.  A
// release per workgroup (an L2 write-back, and one more inside an acq_rel
// add) cost 3.3 us at 1 MiB.
#pragma once
#include <stdint.h>

__device__ __forceinline__ void lfa_solo_body(char *dst, const char *src, uint64_t bytes,
                                              uint32_t nblocks, uint32_t *ctr, uint64_t *word,
                                              uint64_t val) {
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const unsigned t = __builtin_amdgcn_workitem_id_x();
  const bool vec = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const uint64_t tile = vec ? 16384 : 4096;
  const uint64_t lo = (uint64_t)__builtin_amdgcn_workgroup_id_x() * tile;
  const uint64_t hi = lo + tile < bytes ? lo + tile : bytes;
  const uint64_t vhi = vec ? lo + ((hi - lo) & ~(uint64_t)15) : lo;
  if (vec && vhi > lo) {
    // buffer descriptors sized to the tile's whole vectors: lanes past it
    // load 0 and their stores are dropped
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char *>(src) + lo, 0, (int)(vhi - lo), 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(dst + lo, 0, (int)(vhi - lo), 0x00020000);
    u32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; k++)
      v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                           rs, (unsigned)(k * 4096 + t * 16), 0, 0));
#pragma unroll
    for (int k = 0; k < 4; k++)
      // write-through (sc0 sc1): nothing of the result stays dirty in L2
      __builtin_amdgcn_raw_buffer_store_b128(v[k], rd, (unsigned)(k * 4096 + t * 16), 0, 17);
  }
  for (uint64_t o = vhi + t; o < hi; o += 256) dst[o] = src[o];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t != 0) return;
  if (nblocks == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (vhi != hi) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // plain stores
  const uint32_t seen = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (seen + 1 == nblocks) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
