// lfa_kernels.hpp — the gfx950 combine kernels and their host launchers.
//
// Included by lfa_combine.hip (the product entry points of liblfa.so, one
// object per write op) and by lfa_tune.hip (the on-GPU A/B sweep of
// bench.py --tune*, built into the separate liblfa_tune.so).  Templates only:
// a kernel form is compiled into a library only where a launcher
// instantiates it, so the tuning forms never reach liblfa.so.
#pragma once

#include <hip/hip_runtime.h>
#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <type_traits>

#include "lfa_ops.hpp"
#include "lfa_signal.h"
#include "../../include/lfa_atomic.h"

namespace lfa {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------
// memory access helpers
// ---------------------------------------------------------------------------
template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4 *p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4 *p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// The wave's index in its workgroup, as a SCALAR.  threadIdx.x / 64 is the
// same on every lane of a wave, but the compiler cannot prove it: a buffer
// descriptor built from it counts as divergent, so every buffer load / store
// through it was wrapped in a readfirstlane loop (4 v_readfirstlane, a
// compare, an exec save and a branch per access) and the 64-bit tile base was
// kept per lane in VGPRs.  readfirstlane makes it uniform: the descriptors
// live in SGPRs and each access is one instruction.  UW = false keeps the
// round-2 (divergent) form for the A/B in liblfa_tune.so.
template <bool UW = true>
__device__ __forceinline__ unsigned wave_id() {
  if constexpr (UW) return __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
  else return threadIdx.x / 64;
}

// OP applied lane-wise to the 16/sizeof(T) elements packed in a 16-B vector.
template <int OP, typename T>
__device__ __forceinline__ u32x4 apply_vec(u32x4 d, u32x4 s) {
  constexpr int N = 16 / sizeof(T);
  T a[N], b[N];
  __builtin_memcpy(a, &d, 16);
  __builtin_memcpy(b, &s, 16);
#pragma unroll
  for (int i = 0; i < N; i++) a[i] = apply<OP, T>(a[i], b[i]);
  u32x4 r;
  __builtin_memcpy(&r, a, 16);
  return r;
}

// ---------------------------------------------------------------------------
// binary combine, vector body
// ---------------------------------------------------------------------------
constexpr int kBlock = 256;  // 4 waves of 64

// Chunked: workgroup b owns vectors [b·kBlock·U, (b+1)·kBlock·U); step u of
// thread t touches base + u·kBlock + t, i.e. each wave-instruction reads 1 KiB
// of consecutive bytes.  All 2·U loads issue before the first op.
template <int OP, typename T, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlock) void combine_vec(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * (kBlock * U) + threadIdx.x;
  if (base + (size_t)(U - 1) * kBlock < nvec) {  // full chunk: no guards
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<NTL>(dst + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; u++) b[u] = ld<NTL>(src + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; u++)
      st<NTS>(dst + base + u * kBlock, apply_vec<OP, T>(a[u], b[u]));
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * kBlock;
      if (i < nvec)
        st<NTS>(dst + i, apply_vec<OP, T>(ld<NTL>(dst + i), ld<NTL>(src + i)));
    }
  }
}

// LDS-DMA staged form — the PRODUCT body (bench.py --tune, DESIGN.md
// "Kernel tuning": 1-2 % faster than register staging at 256 MiB).  Each wave
// owns U consecutive KiB of both operands and moves them HBM -> LDS with
// global_load_lds_dwordx4 (aux = nt, no VGPR round trip; 2·U KiB in flight per
// wave), waits on its own vmcnt, reads its lane's 16 B back with
// ds_read_b128, applies OP and streams the result out with nt stores.  Waves
// never share LDS, so there is no barrier; a wave whose chunk runs past nvec
// takes the guarded register path.
typedef __attribute__((address_space(3))) void lds_void;
constexpr int kLdsWaves = 4;

// Store cache policy of the body (gfx950 cpol bits): nt keeps the line in
// the XCD's L2 for the end-of-kernel writeback; sc1 writes through.  sc1 is
// 1.6-6.7 % faster per launch from 16 to 128 MiB per operand and level at
// 256 MiB (rocprofv3 kernel durations, profiles/r01_rocprof_store_policy.csv),
// so launches below kSc1Bytes write through.
constexpr int kStoreNt = 2, kStoreSc1 = 16;
constexpr size_t kSc1Bytes = (size_t)192 << 20;

// s_waitcnt vmcnt(N) alone (expcnt / lgkmcnt fields at their no-wait
// maximum): every vector-memory operation of this wave but the N youngest
// has completed — loads, LDS-DMA and stores count together, in issue order.
template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt is 6 bits");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// Step u of a drained tile: wait until the pair of 1-KiB loads of vector u
// has landed — in issue order the loads of u+1..U-1 (2 each, or 1 each for
// ATOMIC_WRITE, which reads no dst) and the u stores already issued may stay
// in flight — then combine and store vector u while the later loads arrive.
template <int OP, typename T, int U, int SAUX, int u>
__device__ __forceinline__ void combine_drain(u32x4 (*lds)[kLdsWaves][U][64], unsigned w,
                                              unsigned l, u32x4 *dst,
                                              __amdgpu_buffer_rsrc_t r) {
  if constexpr (u < U) {
    constexpr int per = OP == OP_WRITE ? 1 : 2;
    wait_vmcnt<per * (U - 1 - u) + u>();
    u32x4 v;
    if constexpr (OP == OP_WRITE) v = lds[1][w][u][l];
    else v = apply_vec<OP, T>(lds[0][w][u][l], lds[1][w][u][l]);
    if constexpr (SAUX == kStoreNt)
      st<true>(dst + u * 64 + l, v);
    else
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
    combine_drain<OP, T, U, SAUX, u + 1>(lds, w, l, dst, r);
  }
}

// DRAIN: the wave's loads issue pairwise (dst u, src u, dst u+1, ...) and
// step u stores vector u as soon as its pair has landed (combine_drain),
// instead of waiting vmcnt(0) for the whole 2·U KiB before the first store.
// Back-to-back launches at 256 MiB per operand (tools/tune_combine.py,
// profiles/r03_tune_combine_backtoback.log): 119.4 us against 120.7 us; no
// change within noise at 32-128 MiB (write-through stores there), so the
// product drains on the nt-store path only.
template <int OP, typename T, int U, int SAUX, bool UW = true,
          bool DRAIN = SAUX == kStoreNt>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_lds(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned w = wave_id<UW>(), l = threadIdx.x % 64;
  const size_t base =
      (size_t)blockIdx.x * (kLdsWaves * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U <= nvec) {
    if constexpr (DRAIN) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        if constexpr (OP != OP_WRITE)  // ATOMIC_WRITE never reads dst
          __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                           (lds_void *)&lds[0][w][u][0], 16, 0,
                                           /*aux: nt*/ 2);
        __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                         (lds_void *)&lds[1][w][u][0], 16, 0, 2);
      }
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
      combine_drain<OP, T, U, SAUX, 0>(lds, w, l, dst + base, r);
      return;
    }
    if constexpr (OP != OP_WRITE) {  // ATOMIC_WRITE never reads dst
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0,
                                         /*aux: nt*/ 2);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // sc1: the wave's tile through one buffer descriptor whose stores carry
    // the bits; nt: plain global stores (0.5 % faster than the buffer form
    // at 256 MiB in rocprofv3)
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      u32x4 v;
      if constexpr (OP == OP_WRITE) v = lds[1][w][u][l];
      else v = apply_vec<OP, T>(lds[0][w][u][l], lds[1][w][u][l]);
      if constexpr (SAUX == kStoreNt)
        st<true>(dst + base + u * 64 + l, v);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
    }
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * 64 + l;
      if (i < nvec)
        st<true>(dst + i, apply_vec<OP, T>(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

// Tapered tail.  Per-wave timestamps (tools/probe_ramp.py)
// put a launch's fixed cost in its drain: the waves still running at the end
// each live ~4.6 us, and at 32 MiB per operand the last ones finish over
// ~2.4 us.  Here workgroups [0, head) take U-KiB tiles (the body above) up to
// vector `split`, and the rest — dispatched last, the highest block ids —
// take 1-KiB tiles, so the waves that end the launch are short ones.  Worth
// it where the launch runs at least two rounds of waves; below that the extra
// waves cost more than the drain saves (tools/tune_combine.py variants 85-88,
// profiles/r04_tune_combine_taper*.json: 32 MiB -1.9 %, 48 and 64 MiB -1.3 %,
// 16 MiB +2.1 %, 256 MiB on the nt path +1 %).
template <int OP, typename T, int U, int UA, int SAUX>
__device__ __forceinline__ void lds_tile(u32x4 *__restrict__ dst, const u32x4 *__restrict__ src,
                                         size_t nvec, size_t base,
                                         u32x4 (*lds)[kLdsWaves][UA][64], unsigned w,
                                         unsigned l) {
  if (base + 64 * U <= nvec) {
    if constexpr (OP != OP_WRITE) {  // ATOMIC_WRITE never reads dst
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0, /*aux: nt*/ 2);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      u32x4 v;
      if constexpr (OP == OP_WRITE) v = lds[1][w][u][l];
      else v = apply_vec<OP, T>(lds[0][w][u][l], lds[1][w][u][l]);
      if constexpr (SAUX == kStoreNt)
        st<true>(dst + base + u * 64 + l, v);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
    }
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * 64 + l;
      if (i < nvec)
        st<true>(dst + i, apply_vec<OP, T>(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

template <int OP, typename T, int U, int SAUX>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_lds_taper(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec, size_t split,
    unsigned head) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const unsigned b = blockIdx.x;
  if (b < head)
    lds_tile<OP, T, U, U, SAUX>(dst, src, split,
                                (size_t)b * (kLdsWaves * 64 * U) + (size_t)w * 64 * U, lds, w, l);
  else
    lds_tile<OP, T, 1, U, SAUX>(dst, src, nvec,
                                split + (size_t)(b - head) * (kLdsWaves * 64) + (size_t)w * 64,
                                lds, w, l);
}

// Grid-stride variant (for the tuning sweep): a fixed grid of G workgroups
// walks the buffer; each thread holds U vectors spaced kBlock apart.
template <int OP, typename T, int U, bool NTL, bool NTS>
__global__ __launch_bounds__(kBlock) void combine_vec_gs(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec) {
  const size_t step = (size_t)gridDim.x * kBlock * U;
  size_t base = (size_t)blockIdx.x * (kBlock * U) + threadIdx.x;
  for (; base + (size_t)(U - 1) * kBlock < nvec; base += step) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) a[u] = ld<NTL>(dst + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; u++) b[u] = ld<NTL>(src + base + u * kBlock);
#pragma unroll
    for (int u = 0; u < U; u++)
      st<NTS>(dst + base + u * kBlock, apply_vec<OP, T>(a[u], b[u]));
  }
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + (size_t)u * kBlock;
    if (i < nvec)
      st<NTS>(dst + i, apply_vec<OP, T>(ld<NTL>(dst + i), ld<NTL>(src + i)));
  }
}

// ---------------------------------------------------------------------------
// binary combine, element-wise (heads, tails, non-co-aligned buffers)
// ---------------------------------------------------------------------------
// Up to two index ranges [0, n0) and [off1, off1 + n1) in one launch, so a
// misaligned head and tail cost a single extra dispatch.
template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void combine_elem(
    T *__restrict__ dst, const T *__restrict__ src, size_t n0, size_t off1,
    size_t n1) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n0 + n1; i += stride) {
    size_t k = i < n0 ? i : off1 + (i - n0);
    dst[k] = apply<OP, T>(dst[k], src[k]);
  }
}

// Element pointers not even aligned to sizeof(T): byte-wise access.
template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void combine_unaligned(
    unsigned char *dst, const unsigned char *src, size_t n) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n; i += stride) {
    T a, b;
    __builtin_memcpy(&a, dst + i * sizeof(T), sizeof(T));
    __builtin_memcpy(&b, src + i * sizeof(T), sizeof(T));
    a = apply<OP, T>(a, b);
    __builtin_memcpy(dst + i * sizeof(T), &a, sizeof(T));
  }
}

}  // namespace lfa

// The rest of the kernels and the launchers, split by concern in round 6:
#include "lfa_k_tree.hpp"
#include "lfa_k_oneshot.hpp"
#include "lfa_k_fetch.hpp"
#include "lfa_k_launch.hpp"
