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

// ---------------------------------------------------------------------------
// N-input tree reduction in recursive-doubling order
// ---------------------------------------------------------------------------
// Leaf k (k < nleaf, nleaf = largest power of two <= nsrc) is either a pair
// (in[hi] OP in[lo]) — the non-power-of-two pre-step, coll_coll.c:366-389 —
// or a single input.  Leaves are then combined pairwise, higher-index
// partial OP lower-index partial, level by level (coll_coll.c:392-433).
// The kernel evaluates that tree with a stack: push leaves left to right and
// merge the two top entries while they cover equal-size groups, so only
// log2(nleaf)+1 partials are live per element.
constexpr int kMaxLeaf = 32;

struct TreeArgs {
  const void *in[kMaxLeaf];  // nsrc <= 32 inputs (LFA_TREE_MAX)
  signed char hi[kMaxLeaf];  // input index of the leaf's (higher-rank) value
  signed char lo[kMaxLeaf];  // paired lower-rank input, or -1
};

template <int OP, typename T, typename V>
__device__ __forceinline__ V apply_any(V d, V s) {
  if constexpr (sizeof(V) == 16 && sizeof(T) <= 16 && !__is_same(V, T))
    return apply_vec<OP, T>(d, s);
  else
    return apply<OP, T>(d, s);
}

// Evaluate the tree for one element (or one 16-B vector); load(k) fetches
// input k.  Leaf order, pairing and merge order are compile-time except the
// kernel-argument (wave-uniform) pair test.
template <int OP, typename T, typename V, int NLEAF, typename L, typename A = TreeArgs>
__device__ __forceinline__ V tree_eval_with(const A &a, L &&load) {
  V stack[6];
  int depth = 0;
#pragma unroll
  for (int k = 0; k < NLEAF; k++) {
    V v = load(a.hi[k]);
    if (a.lo[k] >= 0)  // wave-uniform: kernel-argument branch
      v = apply_any<OP, T, V>(v, load(a.lo[k]));
    stack[depth++] = v;
    // after leaf k, merge the two top partials once per trailing zero bit
    // of (k + 1): that is when they cover equal-size rank groups
#pragma unroll
    for (int m = 1; m < NLEAF; m <<= 1) {
      if (((k + 1) & (2 * m - 1)) == 0) {
        V hi = stack[--depth];
        V lo = stack[--depth];
        stack[depth++] = apply_any<OP, T, V>(hi, lo);
      }
    }
  }
  return stack[0];
}

template <int OP, typename T, typename V, int NLEAF>
__device__ __forceinline__ V tree_eval(const TreeArgs &a, size_t i) {
  return tree_eval_with<OP, T, V, NLEAF>(
      a, [&](int k) { return ((const V *)a.in[k])[i]; });
}

// Grid-stride form (tuning reference): plain loads, one vector per lane.
template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void reduce_tree_vec(TreeArgs a,
                                                          u32x4 *dst,
                                                          size_t nvec) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < nvec; i += stride)
    st<true>(dst + i, tree_eval<OP, T, u32x4, NLEAF>(a, i));
}

// Chunked register form: workgroup b owns [b·kBlock·U, (b+1)·kBlock·U),
// every input read with nt loads (U·nsrc 16-B loads in flight per lane).
// SAUX = kStoreSc1: the result is written through (buffer stores, sc1).
template <int OP, typename T, int NLEAF, int U, int SAUX = kStoreNt>
__global__ __launch_bounds__(kBlock) void reduce_tree_chunk(TreeArgs a,
                                                            u32x4 *dst,
                                                            size_t nvec) {
  const size_t base = (size_t)blockIdx.x * (kBlock * U) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + (size_t)u * kBlock;
    if (i < nvec) {
      u32x4 v = tree_eval_with<OP, T, u32x4, NLEAF>(
          a, [&](int k) { return ld<true>((const u32x4 *)a.in[k] + i); });
      if constexpr (SAUX == kStoreNt) {
        st<true>(dst + i, v);
      } else {
        // the wave's first vector, as a scalar (wave_id)
        const size_t wb = (size_t)blockIdx.x * (kBlock * U) + (size_t)u * kBlock +
                          (size_t)wave_id() * 64;
        __builtin_amdgcn_raw_buffer_store_b128(
            v, __builtin_amdgcn_make_buffer_rsrc(dst + wb, 0, 64 * 16, 0x00020000),
            (threadIdx.x % 64) * 16, 0, SAUX);
      }
    }
  }
}

// Tapered chunk form (variant 12, the combine's tapered tail applied to the
// tree): workgroups [0, head) take U = 2 vectors per lane up to vector
// `split`, the rest — dispatched last — one vector per lane, so the waves that
// end the launch are shorter.  Write-through stores (the chunk form's sc1).
template <int OP, typename T, int NLEAF, int U>
__device__ __forceinline__ void tree_chunk_at(const TreeArgs &a, u32x4 *dst, size_t nvec,
                                              size_t wg0) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    const size_t i = wg0 + (size_t)u * kBlock + threadIdx.x;
    if (i < nvec) {
      u32x4 v = tree_eval_with<OP, T, u32x4, NLEAF>(
          a, [&](int k) { return ld<true>((const u32x4 *)a.in[k] + i); });
      const size_t wb = wg0 + (size_t)u * kBlock + (size_t)wave_id() * 64;
      __builtin_amdgcn_raw_buffer_store_b128(
          v, __builtin_amdgcn_make_buffer_rsrc(dst + wb, 0, 64 * 16, 0x00020000),
          (threadIdx.x % 64) * 16, 0, kStoreSc1);
    }
  }
}

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void reduce_tree_taper(TreeArgs a, u32x4 *dst, size_t nvec,
                                                            size_t split, unsigned head) {
  const unsigned b = blockIdx.x;
  if (b < head)
    tree_chunk_at<OP, T, NLEAF, 2>(a, dst, split, (size_t)b * (kBlock * 2));
  else
    tree_chunk_at<OP, T, NLEAF, 1>(a, dst, nvec, split + (size_t)(b - head) * kBlock);
}

// LDS-DMA form: each wave DMAs U KiB of every input into its own LDS slots
// (global_load_lds_dwordx4, nt), waits on its vmcnt, then evaluates U trees
// per lane from LDS and stores nt.  Dynamic LDS: nin · W · U KiB per
// workgroup.  Waves never share LDS, so no barrier.
template <int OP, typename T, int NLEAF, int W, int U>
__global__ __launch_bounds__(W * 64) void reduce_tree_lds(TreeArgs a, int nin,
                                                          u32x4 *dst,
                                                          size_t nvec) {
  extern __shared__ u32x4 tlds[];  // [nin][W][U][64]
  const unsigned w = wave_id(), l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (W * 64 * U) + (size_t)w * 64 * U;
  auto slot = [&](int k, int u) { return ((k * W + w) * U + u) * 64; };
  if (base + 64 * U <= nvec) {
    for (int k = 0; k < nin; k++)  // uniform loop over the inputs
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds(
            (const void *)((const u32x4 *)a.in[k] + base + u * 64 + l),
            (lds_void *)&tlds[slot(k, u)], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++)
      st<true>(dst + base + u * 64 + l,
               tree_eval_with<OP, T, u32x4, NLEAF>(
                   a, [&](int k) { return tlds[slot(k, u) + l]; }));
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * 64 + l;
      if (i < nvec)
        st<true>(dst + i, tree_eval_with<OP, T, u32x4, NLEAF>(a, [&](int k) {
                   return ld<true>((const u32x4 *)a.in[k] + i);
                 }));
    }
  }
}

// Wave-contiguous register form: wave w of workgroup b owns U consecutive KiB
// of every input (longer DRAM bursts per input stream than the chunked form).
template <int OP, typename T, int NLEAF, int U>
__global__ __launch_bounds__(kBlock) void reduce_tree_wave(TreeArgs a,
                                                           u32x4 *dst,
                                                           size_t nvec) {
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U + l;
#pragma unroll
  for (int u = 0; u < U; u++) {
    size_t i = base + (size_t)u * 64;
    if (i < nvec)
      st<true>(dst + i, tree_eval_with<OP, T, u32x4, NLEAF>(a, [&](int k) {
                 return ld<true>((const u32x4 *)a.in[k] + i);
               }));
  }
}

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void reduce_tree_elem(TreeArgs a, T *dst,
                                                           size_t n0,
                                                           size_t off1,
                                                           size_t n1) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n0 + n1; i += stride) {
    size_t k = i < n0 ? i : off1 + (i - n0);
    dst[k] = tree_eval<OP, T, T, NLEAF>(a, k);
  }
}

// Operands not aligned to sizeof(T) — a caller's byte offset into a buffer,
// which the reference's host loops take as they come (coll_coll.c:763 hands
// the table whatever the caller passed).  Element i of such an operand is
// moved byte-wise, and the tree is walked with a runtime leaf count: one
// kernel per (OP, T) for a path only odd caller buffers take.
template <typename T>
__device__ __forceinline__ T ld_bytes(const void *p, size_t i) {
  T v;
  __builtin_memcpy(&v, (const char *)p + i * sizeof(T), sizeof(T));
  return v;
}

template <typename T>
__device__ __forceinline__ void st_bytes(void *p, size_t i, T v) {
  __builtin_memcpy((char *)p + i * sizeof(T), &v, sizeof(T));
}

// tree_eval_with's order (same leaves, same merges) for a runtime nleaf.
template <int OP, typename T, typename L>
__device__ __forceinline__ T tree_eval_rt(const TreeArgs &a, int nleaf, L &&load) {
  T stack[6];
  int depth = 0;
  for (int k = 0; k < nleaf; k++) {
    T v = load(a.hi[k]);
    if (a.lo[k] >= 0) v = apply<OP, T>(v, load(a.lo[k]));
    stack[depth++] = v;
    for (int m = 1; m < nleaf; m <<= 1) {
      if (((k + 1) & (2 * m - 1)) == 0) {
        T hi = stack[--depth];
        T lo = stack[--depth];
        stack[depth++] = apply<OP, T>(hi, lo);
      }
    }
  }
  return stack[0];
}

template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void reduce_tree_unaligned(TreeArgs a, int nleaf,
                                                                void *dst, size_t n) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n; i += stride)
    st_bytes<T>(dst, i, tree_eval_rt<OP, T>(a, nleaf, [&](int k) {
                  return ld_bytes<T>(a.in[k], i);
                }));
}

// ---------------------------------------------------------------------------
// N-input tree with fan-out, across GPUs (LFA_ALGO_P2P)
// ---------------------------------------------------------------------------
// Inputs and outputs may be other GPUs' HBM mapped into this process over
// IPC (xGMI).  Every access is system scope (sc0 sc1): such loads miss in any
// cache that is not coherent with the owning GPU's memory, and such stores
// write through instead of leaving dirty lines in this XCD's L2, so a peer
// that orders itself after this kernel (a stream-ordered barrier) reads the
// bytes, and the next operation here reads the peer's fresh input.
constexpr int kSysAux = 17;      // cpol sc0 | sc1: system scope (stores)
constexpr int kSysLoadAux = 19;  // sc0 | sc1 | nt: system scope + streaming
// The nt hint on the loads is worth 63 % -> 73 % of HBM peak on local memory
// (8 -> 1, 8 x 32 MiB), U = 4 a further 2 points; the scope bits themselves
// cost nothing (default-policy loads: 62.6 %).  bench.py --tune-treeput,
// profiles/r02_tune_treeput*.log.
constexpr int kMaxPut = 32;

struct PutArgs {
  TreeArgs t;
  void *out[kMaxPut];
  int nout;
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t tile_rsrc(const void *base,
                                                            unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(base), 0, (int)bytes,
                                           0x00020000);
}

// Vector body: wave w of workgroup b owns U KiB (64·U vectors) of every
// input; its loads and stores go through buffer descriptors sized to the
// wave's tile, so the last, partial tile needs no guards (out-of-range lanes
// load 0 and their stores are dropped by the hardware).
template <int OP, typename T, int NLEAF, int U, bool UW>
__device__ __forceinline__ void tree_put_body(const PutArgs &a, size_t nvec) {
  const unsigned w = wave_id<UW>(), l = threadIdx.x % 64;
  const size_t wbase = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP, T, u32x4, NLEAF>(a.t, [&](int k) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0,
                     kSysLoadAux));
    });
  }
  // Output-major issue.  Pacing the outputs (a vmcnt wait or s_sleep between
  // them) or u-major order (every output's u-th vector, then u + 1) gained
  // 4.5 us at 8 -> 8 on one box and lost 2.5 us on the next (8 x 32 MiB,
  // local HBM, bench.py --tune-treeput variants 18-22,
  // profiles/r03_tune_treeput*.log): not a reproducible difference.
  for (int j = 0; j < a.nout; j++) {  // wave-uniform
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0,
                                             kSysAux);
  }
}

template <int OP, typename T, int NLEAF, int U, bool UW = true>
__global__ __launch_bounds__(kBlock) void reduce_tree_put(PutArgs a, size_t nvec) {
  tree_put_body<OP, T, NLEAF, U, UW>(a, nvec);
}

// One element at system scope (relaxed atomics of the element's width; a
// 16-byte element as two 8-byte halves — the halves of one element are
// written by one lane, so no reader sees a torn value after the barrier).
template <typename T>
__device__ __forceinline__ T sys_load(const T *p) {
  T v;
  if constexpr (sizeof(T) == 16) {
    uint64_t h[2];
    h[0] = __hip_atomic_load((const uint64_t *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    h[1] = __hip_atomic_load((const uint64_t *)p + 1, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_memcpy(&v, h, 16);
  } else {
    typedef typename std::conditional<
        sizeof(T) == 1, uint8_t,
        typename std::conditional<
            sizeof(T) == 2, uint16_t,
            typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type>::type U;
    U x = __hip_atomic_load((const U *)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __builtin_memcpy(&v, &x, sizeof(T));
  }
  return v;
}

template <typename T>
__device__ __forceinline__ void sys_store(T *p, T v) {
  if constexpr (sizeof(T) == 16) {
    uint64_t h[2];
    __builtin_memcpy(h, &v, 16);
    __hip_atomic_store((uint64_t *)p, h[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store((uint64_t *)p + 1, h[1], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    typedef typename std::conditional<
        sizeof(T) == 1, uint8_t,
        typename std::conditional<
            sizeof(T) == 2, uint16_t,
            typename std::conditional<sizeof(T) == 4, uint32_t, uint64_t>::type>::type>::type U;
    U x;
    __builtin_memcpy(&x, &v, sizeof(T));
    __hip_atomic_store((U *)p, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void reduce_tree_put_elem(PutArgs a, size_t n0,
                                                               size_t off1, size_t n1) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n0 + n1; i += stride) {
    size_t k = i < n0 ? i : off1 + (i - n0);
    T v = tree_eval_with<OP, T, T, NLEAF>(
        a.t, [&](int s) { return sys_load<T>((const T *)a.t.in[s] + k); });
    for (int j = 0; j < a.nout; j++) sys_store<T>((T *)a.out[j] + k, v);
  }
}

// Some operand not aligned to sizeof(T).  In the P2P schedules that is only
// ever the caller's own buffer (its block read in place, its result written
// in place: local memory), never a peer's workspace slot (256-B aligned), so
// element-aligned operands keep their system-scope element accesses (bit k
// of `in_sys` / `out_sys`) and the others are moved byte-wise.
template <int OP, typename T>
__global__ __launch_bounds__(kBlock) void reduce_tree_put_unaligned(PutArgs a, int nleaf,
                                                                    uint32_t in_sys,
                                                                    uint32_t out_sys,
                                                                    size_t n) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n; i += stride) {
    T v = tree_eval_rt<OP, T>(a.t, nleaf, [&](int k) {
      return (in_sys >> k) & 1 ? sys_load<T>((const T *)a.t.in[k] + i)
                               : ld_bytes<T>(a.t.in[k], i);
    });
    for (int j = 0; j < a.nout; j++) {
      if ((out_sys >> j) & 1) sys_store<T>((T *)a.out[j] + i, v);
      else st_bytes<T>(a.out[j], i, v);
    }
  }
}

// ---------------------------------------------------------------------------
// one-shot reduction (LFA_STEP_ONESHOT, lfa_signal.h): push, post, wait,
// reduce — one launch for a small bucket instead of copy + barrier + tree +
// barrier.  Destination k receives bytes [soff[k], soff[k] + slen[k]) of this
// rank's input (the whole vector for allreduce, block k for reduce_scatter,
// the root alone for reduce).  Workgroup b owns bytes [b·chunk, (b+1)·chunk)
// of every such range and synchronises only with the peers' workgroup b.
// ---------------------------------------------------------------------------
constexpr int kOsMax = LFA_OS_MAX_RANKS;

// One system-scope release / acquire per workgroup (0, the product) or per
// wave (1, round 2's first form).  A workgroup's waves share a CU and so an
// L2, which makes the single pair sufficient on one GPU — every
// cross-process test runs on one MI355X — but its ordering across GPUs over
// xGMI has not run anywhere yet, so the per-wave form stays
// selectable: build with -DLFA_OS_WAVE_FENCES=1.
#ifndef LFA_OS_WAVE_FENCES
#define LFA_OS_WAVE_FENCES 0
#endif

// The one-shot's association tree over at most kOsMax leaves (TreeArgs has
// room for 32): the kernel's argument block is 376 bytes instead of ~670, one
// 64-byte line of it read per 64 bytes on every launch — the n = 1 kernel
// with the larger block took ~1 us longer from launch to completion word
// than a 48-byte one (profiles/r04_solo_2.json).
struct OsTree {
  const void *in[kOsMax];      // own input range (k == rank) or own slot k
  signed char hi[kOsMax];
  signed char lo[kOsMax];
};

struct OsArgs {
  OsTree t;
  char *push[kOsMax];          // peer k's slot of this rank (k != rank)
  uint32_t *post[kOsMax];      // peer k's one-shot rows, column `rank`
  uint32_t soff[kOsMax];       // input range pushed to k (k == rank: reduced)
  uint32_t slen[kOsMax];
  const uint32_t *wait;        // own one-shot rows
  const char *send;
  char *result;
  uint64_t *status;
  uint64_t timeout;            // wall-clock ticks
  size_t chunk;                // a multiple of 16
  uint64_t ticket;
  uint32_t epoch;
  int n, rank;
  int vec;                     // every range start and result 16-B aligned
  int unal;                    // send or result not aligned to the element
  uint32_t *done_ctr;          // completion word (lfa_signal.h), optional
  uint64_t *done_word;
  uint64_t done_val;
};
static_assert(sizeof(OsArgs) == 376, "the one-shot's argument block (see OsTree)");

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void oneshot_reduce(OsArgs a) {
  constexpr size_t E = sizeof(T);
  const unsigned t = threadIdx.x;
  const size_t b = blockIdx.x;
  const size_t lo = b * a.chunk;
  // 1. push this rank's chunk of each destination's range into its slot on
  //    that peer (system-scope write-through stores over xGMI)
  for (int k = 0; k < a.n; k++) {  // wave-uniform
    if (k == a.rank || lo >= a.slen[k]) continue;
    const size_t hi = lo + a.chunk < a.slen[k] ? lo + a.chunk : a.slen[k];
    const size_t vhi = a.vec ? hi & ~(size_t)15 : lo;
    const char *src = a.send + a.soff[k];
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(a.push[k], (unsigned)a.slen[k]);
    for (size_t o = lo + (size_t)t * 16; o < vhi; o += (size_t)kBlock * 16)
      __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)(src + o), r, (unsigned)o, 0,
                                             kSysAux);
    for (size_t o = vhi + t; o < hi; o += kBlock)
      sys_store<uint8_t>((uint8_t *)a.push[k] + o, (uint8_t)src[o]);
  }
  // 2. every wave's pushes acknowledged (write-through, so in the peer's
  //    memory), then ONE system-scope release for the workgroup — its waves
  //    share a CU and so an L2 — and one post per peer
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (a.n > 1 && (LFA_OS_WAVE_FENCES || t < 64))  // wave 0: the posting lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if ((int)t < a.n && (int)t != a.rank) {
    __hip_atomic_store(a.post[t] + b * LFA_SIG_MAX, a.epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    // 3. wait for peer t's workgroup b (bounded: *status on timeout)
    const uint32_t *w = a.wait + b * LFA_SIG_MAX + t;
    const uint64_t t0 = wall_clock64();
    while ((int32_t)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                     a.epoch) < 0) {
      if (wall_clock64() - t0 > a.timeout) {
        lfa_sig_note_timeout(a.status, a.ticket);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  // the waiting wave acquires for the workgroup (same CU, same L2), then
  // every wave may read what the peers pushed
  if (a.n > 1 && (LFA_OS_WAVE_FENCES || t < 64)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  // 4. reduce chunk b of this rank's own range over every rank's input, rank
  //    order (system-scope loads: the slots were written by peers over xGMI)
  const size_t own = a.slen[a.rank];
  bool plain = false;  // this workgroup wrote result bytes with plain stores
  if (lo < own) {
    const size_t hi = lo + a.chunk < own ? lo + a.chunk : own;
    const size_t vhi = a.vec ? hi & ~(size_t)15 : lo;
    plain = a.unal || vhi < hi;
    for (size_t o = lo + (size_t)t * 16; o < vhi; o += (size_t)kBlock * 16) {
      u32x4 v = tree_eval_with<OP, T, u32x4, NLEAF>(a.t, [&](int k) {
        return __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.t.in[k], (unsigned)own),
                                                         (unsigned)o, 0, kSysLoadAux));
      });
      // write-through: the release before the completion word then has no
      // dirty result lines to write back
      __builtin_amdgcn_raw_buffer_store_b128(v, tile_rsrc(a.result, (unsigned)own), (unsigned)o,
                                             0, kSysAux);
    }
    if (a.unal) {
      // the caller's own input and result, byte-wise (local memory); the
      // peers' slots (256-B aligned) keep their system-scope loads
      for (size_t e = lo / E + t; e < hi / E; e += kBlock)
        st_bytes<T>(a.result, e, tree_eval_with<OP, T, T, NLEAF>(a.t, [&](int k) {
                      return k == a.rank ? ld_bytes<T>(a.t.in[k], e)
                                         : sys_load<T>((const T *)a.t.in[k] + e);
                    }));
    } else {
      for (size_t e = vhi / E + t; e < hi / E; e += kBlock) {
        T v = tree_eval_with<OP, T, T, NLEAF>(
            a.t, [&](int k) { return sys_load<T>((const T *)a.t.in[k] + e); });
        ((T *)a.result)[e] = v;
      }
    }
  }
  // 5. completion word: this workgroup's result stores acknowledged, then it
  //    counts itself; the last workgroup resets the counter for the next
  //    launch on the stream and publishes done_val to the host.  Write-
  //    through stores are in memory once acknowledged, so a workgroup that
  //    made only those adds relaxed with no release of its own (an L2
  //    write-back saved per workgroup, as in lfa_signal.hip solo_copy); one
  //    with plain (byte-wise or tail) stores releases them first at system
  //    scope (its waves share a CU and an L2).  The last one acquires the
  //    others' adds, then releases before the word.
  if (a.done_word) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0 && gridDim.x == 1) {
      // one workgroup: no counter to count in (one device atomic less)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (t == 0) {
      if (plain) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      const uint32_t seen = __hip_atomic_fetch_add(a.done_ctr, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      if (seen + 1 == gridDim.x) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(a.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LL one-shot (lfa_signal.h): parts of at most LFA_OS_LL_BYTES.  Lane c owns
// bytes [16c, 16c + 16) of every part: it pushes its 16 bytes of each peer's
// part as two 16-byte stores of {data, flag, data, flag} into that peer's LL
// slot for this rank, then polls its own slots' words until every peer's four
// flags read 2·epoch + 1 — the 8-byte {data, flag} pairs are written and read
// whole, so a matching flag carries its data — and reduces the values in
// prov/coll's association order.  No acknowledgement wait, fence or flag post
// between push and wait, and the poll is the read.  Same completion word and
// timeout as oneshot_reduce.
// ---------------------------------------------------------------------------
struct LlArgs {
  const char *send;
  char *result;
  char *push[kOsMax];          // peer k's LL slot of this rank, this parity
  const char *own;             // this rank's LL slots, this parity
  uint64_t *status;
  uint64_t ticket, timeout;    // timeout: wall-clock ticks
  uint32_t *done_ctr;
  uint64_t *done_word;
  uint64_t done_val;
  uint32_t soff[kOsMax], slen[kOsMax];
  uint32_t flag;
  int n, rank, vec;            // vec: every part start and result 16-B aligned
  signed char hi[kOsMax], lo[kOsMax];  // the association tree's leaves
};

// 16 bytes at base + off, bytes at or past len read as zero (registers only)
__device__ __forceinline__ u32x4 ll_in(const char *base, uint32_t off, uint32_t len, int vec) {
  if (vec && off + 16 <= len) return *(const u32x4 *)(base + off);
  u32x4 v = {0, 0, 0, 0};
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t x = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t i = off + 4 * w + b;
      if (i < len) x |= (uint32_t)(unsigned char)base[i] << (8 * b);
    }
    v[w] = x;
  }
  return v;
}

__device__ __forceinline__ void ll_out(char *base, uint32_t off, uint32_t len, int vec, u32x4 v) {
  if (vec && off + 16 <= len) {
    *(u32x4 *)(base + off) = v;
    return;
  }
#pragma unroll
  for (int w = 0; w < 4; w++)
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t i = off + 4 * w + b;
      if (i < len) base[i] = (char)(v[w] >> (8 * b));
    }
}

// vals[k] for a wave-uniform k without indexing registers dynamically
__device__ __forceinline__ u32x4 ll_pick(const u32x4 (&v)[kOsMax], int k) {
  u32x4 r = v[0];
#pragma unroll
  for (int i = 1; i < kOsMax; i++)
    if (k == i) r = v[i];
  return r;
}

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void oneshot_ll(LlArgs a) {
  const unsigned t = threadIdx.x;
  const uint32_t off = ((uint32_t)blockIdx.x * kBlock + t) * 16u;
  // 1. push this lane's 16 bytes of every peer's part
#pragma unroll
  for (int k = 0; k < kOsMax; k++) {
    if (k >= a.n || k == a.rank || off >= a.slen[k]) continue;
    const u32x4 v = ll_in(a.send + a.soff[k], off, a.slen[k], a.vec);
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(a.push[k], LFA_SIG_LL_SLOT);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[0], a.flag, v[1], a.flag}, r, 2 * off, 0,
                                           kSysAux);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[2], a.flag, v[3], a.flag}, r, 2 * off + 16,
                                           0, kSysAux);
  }
  // 2. this rank's part.  First one lane per wave polls, per peer, the words
  //    of the wave's last chunk (one 16-B load per peer per round instead of
  //    the wave's 128), then every lane reads its own words and polls them
  //    until their flags match — most do on the first read
  const uint32_t own = a.slen[a.rank];
  const uint32_t lane = t & 63u, wave0 = off - lane * 16u;
  if (wave0 < own && lane == 0) {
    const uint32_t last_chunk = (own - 1u) / 16u * 16u;
    const uint32_t last = wave0 + 63u * 16u < last_chunk ? wave0 + 63u * 16u : last_chunk;
    uint32_t pending = 0;
#pragma unroll
    for (int k = 0; k < kOsMax; k++)
      if (k < a.n && k != a.rank) pending |= 1u << k;
    const uint64_t t0 = wall_clock64();
    while (pending) {
#pragma unroll
      for (int k = 0; k < kOsMax; k++) {
        if (!(pending >> k & 1u)) continue;
        const u32x4 w1 = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       tile_rsrc(a.own + (size_t)k * LFA_SIG_LL_SLOT, LFA_SIG_LL_SLOT),
                       2 * last + 16, 0, kSysLoadAux));
        if (w1[1] == a.flag && w1[3] == a.flag) pending &= ~(1u << k);
      }
      if (pending) {
        if (wall_clock64() - t0 > a.timeout) break;   // the lanes below note it
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  if (off < own) {
    u32x4 vals[kOsMax];
    uint32_t pending = 0;
    const u32x4 mine = ll_in(a.send + a.soff[a.rank], off, own, a.vec);
#pragma unroll
    for (int k = 0; k < kOsMax; k++) {
      vals[k] = k == a.rank ? mine : u32x4{0, 0, 0, 0};
      if (k < a.n && k != a.rank) pending |= 1u << k;
    }
    const uint64_t t0 = wall_clock64();
    while (pending) {
#pragma unroll
      for (int k = 0; k < kOsMax; k++) {
        if (!(pending >> k & 1u)) continue;
        const __amdgpu_buffer_rsrc_t r =
            tile_rsrc(a.own + (size_t)k * LFA_SIG_LL_SLOT, LFA_SIG_LL_SLOT);
        const u32x4 w0 = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, 2 * off, 0, kSysLoadAux));
        const u32x4 w1 = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, 2 * off + 16, 0, kSysLoadAux));
        if (w0[1] == a.flag && w0[3] == a.flag && w1[1] == a.flag && w1[3] == a.flag) {
          vals[k] = u32x4{w0[0], w0[2], w1[0], w1[2]};
          pending &= ~(1u << k);
        }
      }
      if (pending) {
        if (wall_clock64() - t0 > a.timeout) {
          lfa_sig_note_timeout(a.status, a.ticket);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    ll_out(a.result, off, own, a.vec,
           tree_eval_with<OP, T, u32x4, NLEAF>(a, [&](int k) { return ll_pick(vals, k); }));
  }
  // 3. completion word, as oneshot_reduce's step 5
  if (a.done_word) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0 && gridDim.x == 1) {
      // one workgroup: no counter to count in (one device atomic less)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      const uint32_t seen = __hip_atomic_fetch_add(a.done_ctr, 1u, __ATOMIC_ACQ_REL,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      if (seen + 1 == gridDim.x) {
        __hip_atomic_store(a.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// fetch (readwrite) and compare-swap tables
// ---------------------------------------------------------------------------
// One launch shape for both: a functor F carries the operand pointers and
// knows how to process one 16-B vector (vec) or one element (elem); the
// kernels only map indices.  res[] receives the old destination, as every
// shipping readwrite / swap handler returns it (util_atomic.c:345-760).
template <int OP, typename T, bool ALIGNED>
struct RwF {
  char *d;
  const char *s;
  char *r;
  u32x4 *dv;
  const u32x4 *sv;
  u32x4 *rv;
  // fetch_lds interface: inputs dst, src; outputs res (old dst), dst
  static constexpr int kIn = OP == OP_READ ? 1 : 2;
  static constexpr bool kWriteDst = OP != OP_READ;
  __device__ __forceinline__ const u32x4 *in(int k) const { return k ? sv : dv; }
  __device__ __forceinline__ u32x4 op(u32x4 a, u32x4 b, u32x4) const {
    return apply_vec<OP, T>(a, b);
  }
  __device__ __forceinline__ void vec(size_t i) const {
    u32x4 a = ld<true>(dv + i);
    st<true>(rv + i, a);
    if constexpr (OP != OP_READ)
      st<true>(dv + i, apply_vec<OP, T>(a, ld<true>(sv + i)));
  }
  __device__ __forceinline__ void elem(size_t k) const {
    T a;
    if constexpr (ALIGNED) a = ((T *)d)[k];
    else __builtin_memcpy(&a, d + k * sizeof(T), sizeof(T));
    if constexpr (ALIGNED) ((T *)r)[k] = a;
    else __builtin_memcpy(r + k * sizeof(T), &a, sizeof(T));
    if constexpr (OP != OP_READ) {
      T b;
      if constexpr (ALIGNED) b = ((const T *)s)[k];
      else __builtin_memcpy(&b, s + k * sizeof(T), sizeof(T));
      a = apply<OP, T>(a, b);
      if constexpr (ALIGNED) ((T *)d)[k] = a;
      else __builtin_memcpy(d + k * sizeof(T), &a, sizeof(T));
    }
  }
};

template <int OP, typename T>
__device__ __forceinline__ u32x4 swap_vec(u32x4 a, u32x4 b, u32x4 c) {
  constexpr int N = 16 / sizeof(T);
  T x[N], y[N], z[N];
  __builtin_memcpy(x, &a, 16);
  __builtin_memcpy(y, &b, 16);
  __builtin_memcpy(z, &c, 16);
#pragma unroll
  for (int i = 0; i < N; i++) x[i] = swap_apply<OP, T>(x[i], y[i], z[i]);
  u32x4 out;
  __builtin_memcpy(&out, x, 16);
  return out;
}

template <int OP, typename T, bool ALIGNED>
struct SwapF {
  char *d;
  const char *s;
  const char *c;
  char *r;
  u32x4 *dv;
  const u32x4 *sv;
  const u32x4 *cv;
  u32x4 *rv;
  // fetch_lds interface: inputs dst, src, cmp; outputs res, dst
  static constexpr int kIn = 3;
  static constexpr bool kWriteDst = true;
  __device__ __forceinline__ const u32x4 *in(int k) const {
    return k == 0 ? dv : k == 1 ? sv : cv;
  }
  __device__ __forceinline__ u32x4 op(u32x4 a, u32x4 b, u32x4 m) const {
    return swap_vec<OP, T>(a, b, m);
  }
  __device__ __forceinline__ void vec(size_t i) const {
    u32x4 a = ld<true>(dv + i);
    u32x4 b = ld<true>(sv + i);
    u32x4 m = ld<true>(cv + i);
    st<true>(rv + i, a);
    st<true>(dv + i, swap_vec<OP, T>(a, b, m));
  }
  __device__ __forceinline__ void elem(size_t k) const {
    T a, b, m;
    if constexpr (ALIGNED) {
      a = ((T *)d)[k];
      b = ((const T *)s)[k];
      m = ((const T *)c)[k];
      ((T *)r)[k] = a;
      ((T *)d)[k] = swap_apply<OP, T>(a, b, m);
    } else {
      __builtin_memcpy(&a, d + k * sizeof(T), sizeof(T));
      __builtin_memcpy(&b, s + k * sizeof(T), sizeof(T));
      __builtin_memcpy(&m, c + k * sizeof(T), sizeof(T));
      __builtin_memcpy(r + k * sizeof(T), &a, sizeof(T));
      a = swap_apply<OP, T>(a, b, m);
      __builtin_memcpy(d + k * sizeof(T), &a, sizeof(T));
    }
  }
};

constexpr int kFetchUnroll = 2;

template <typename F>
__global__ __launch_bounds__(kBlock) void fetch_vec(F f, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * (kBlock * kFetchUnroll) + threadIdx.x;
#pragma unroll
  for (int u = 0; u < kFetchUnroll; u++) {
    size_t i = base + (size_t)u * kBlock;
    if (i < nvec) f.vec(i);
  }
}

template <typename F>
__global__ __launch_bounds__(kBlock) void fetch_elem(F f, size_t n0, size_t off1,
                                                     size_t n1) {
  size_t i = (size_t)blockIdx.x * kBlock + threadIdx.x;
  size_t stride = (size_t)gridDim.x * kBlock;
  for (; i < n0 + n1; i += stride) f.elem(i < n0 ? i : off1 + (i - n0));
}

// LDS-DMA staged fetch / compare body, combine_lds's shape: each wave moves
// U KiB of each of its F::kIn inputs (dst, src[, cmp]) HBM -> LDS with nt
// global_load_lds (all in flight together), then writes res = the old dst
// and, unless ATOMIC_READ, the new dst, with SAUX stores.  The register form
// above interleaves its loads with stores that may alias them, so each lane
// had only one or two loads in flight (75.7 % of HBM peak for a 256 MiB float
// SUM readwrite, tools/probe_fetch.py).
// Step u of a drained fetch tile (combine_drain's scheme): the kIn loads of
// vector u have landed once every op but the kIn·(U-1-u) younger loads and
// the stores of steps 0..u-1 (res, and dst unless ATOMIC_READ) is done.
template <int U, int SAUX, typename F, int u>
__device__ __forceinline__ void fetch_drain(const F &f, u32x4 (*lds)[kLdsWaves][U][64],
                                            unsigned w, unsigned l, size_t base,
                                            __amdgpu_buffer_rsrc_t rr,
                                            __amdgpu_buffer_rsrc_t rd) {
  if constexpr (u < U) {
    constexpr int nst = F::kWriteDst ? 2 : 1;
    wait_vmcnt<F::kIn * (U - 1 - u) + nst * u>();
    const u32x4 a = lds[0][w][u][l];
    const u32x4 b = F::kIn > 1 ? lds[F::kIn > 1 ? 1 : 0][w][u][l] : a;
    const u32x4 c = F::kIn > 2 ? lds[F::kIn > 2 ? 2 : 0][w][u][l] : a;
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    if constexpr (SAUX == kStoreNt) {
      st<true>(f.rv + base + u * 64 + l, a);
      if constexpr (F::kWriteDst) st<true>(f.dv + base + u * 64 + l, f.op(a, b, c));
    } else {
      __builtin_amdgcn_raw_buffer_store_b128(a, rr, off, 0, SAUX);
      if constexpr (F::kWriteDst)
        __builtin_amdgcn_raw_buffer_store_b128(f.op(a, b, c), rd, off, 0, SAUX);
    }
    fetch_drain<U, SAUX, F, u + 1>(f, lds, w, l, base, rr, rd);
  }
}

template <int U, int SAUX, typename F, bool DRAIN = false>
__global__ __launch_bounds__(kLdsWaves * 64) void fetch_lds(F f, size_t nvec) {
  __shared__ u32x4 lds[F::kIn][kLdsWaves][U][64];
  const unsigned w = wave_id(), l = threadIdx.x % 64;
  const size_t base =
      (size_t)blockIdx.x * (kLdsWaves * 64 * U) + (size_t)w * 64 * U;
  if (DRAIN && base + 64 * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int k = 0; k < F::kIn; k++)
        __builtin_amdgcn_global_load_lds((const void *)(f.in(k) + base + u * 64 + l),
                                         (lds_void *)&lds[k][w][u][0], 16, 0,
                                         /*aux: nt*/ 2);
    fetch_drain<U, SAUX, F, 0>(
        f, lds, w, l, base,
        __builtin_amdgcn_make_buffer_rsrc(f.rv + base, 0, 64 * U * 16, 0x00020000),
        __builtin_amdgcn_make_buffer_rsrc(f.dv + base, 0, 64 * U * 16, 0x00020000));
    return;
  }
  if (base + 64 * U <= nvec) {
#pragma unroll
    for (int k = 0; k < F::kIn; k++)
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(f.in(k) + base + u * 64 + l),
                                         (lds_void *)&lds[k][w][u][0], 16, 0,
                                         /*aux: nt*/ 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc(f.rv + base, 0, 64 * U * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(f.dv + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u32x4 a = lds[0][w][u][l];
      const u32x4 b = F::kIn > 1 ? lds[F::kIn > 1 ? 1 : 0][w][u][l] : a;
      const u32x4 c = F::kIn > 2 ? lds[F::kIn > 2 ? 2 : 0][w][u][l] : a;
      const unsigned off = (unsigned)(u * 64 + l) * 16;
      if constexpr (SAUX == kStoreNt) {
        st<true>(f.rv + base + u * 64 + l, a);
        if constexpr (F::kWriteDst) st<true>(f.dv + base + u * 64 + l, f.op(a, b, c));
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(a, rr, off, 0, SAUX);
        if constexpr (F::kWriteDst)
          __builtin_amdgcn_raw_buffer_store_b128(f.op(a, b, c), rd, off, 0, SAUX);
      }
    }
  } else {
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * 64 + l;
      if (i < nvec) f.vec(i);
    }
  }
}

// ---------------------------------------------------------------------------
// host-side launchers
// ---------------------------------------------------------------------------
// Product configuration of the vector body (chosen by the on-GPU sweep in
// bench.py --tune; see DESIGN.md "Kernel tuning"): LDS-DMA staging, 4 KiB of
// each operand per wave, nt loads and stores.
constexpr int kUnroll = 4;
// combine_lds_taper from this many bytes per operand (up to kSc1Bytes; the
// nt-store path above keeps the uniform grid), the last 1/kTaperDiv tapered
constexpr size_t kTaperBytes = (size_t)32 << 20;
constexpr size_t kTaperDiv = 8;

static inline unsigned grid_for(size_t work, size_t per_block, unsigned cap) {
  size_t g = (work + per_block - 1) / per_block;
  if (g == 0) g = 1;
  return (unsigned)(g < cap ? g : cap);
}
constexpr unsigned kElemGridCap = 256 * 8;  // 8 workgroups per CU, grid-stride

template <int OP, typename T>
static int launch_write(void *dst, const void *src, size_t cnt,
                        hipStream_t s, bool mapped = false) {
  if constexpr (!supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    constexpr size_t E = sizeof(T);
    uintptr_t pd = (uintptr_t)dst, ps = (uintptr_t)src;
    if (cnt == 0) return 0;
    if (pd % E || ps % E) {
      hipLaunchKernelGGL((combine_unaligned<OP, T>),
                         dim3(grid_for(cnt, kBlock, kElemGridCap)), dim3(kBlock),
                         0, s, (unsigned char *)dst, (const unsigned char *)src,
                         cnt);
    } else if ((pd ^ ps) % 16 == 0 && E <= 16) {
      size_t head = ((16 - pd % 16) % 16) / E;
      if (head > cnt) head = cnt;
      size_t nvec = (cnt - head) * E / 16;
      size_t body = nvec * 16 / E;
      size_t tail = cnt - head - body;
      if (nvec) {
        u32x4 *d = (u32x4 *)((char *)dst + head * E);
        const u32x4 *v = (const u32x4 *)((const char *)src + head * E);
        const dim3 grid(grid_for(nvec, (size_t)kLdsWaves * 64 * kUnroll, 0x7fffffffu));
        if (mapped) {
          // host-mapped operands (lfa_atomic_write_staged's zero-copy form):
          // PCIe-bound, so the tiling does not matter; the plain write-through
          // body at every size keeps these ~10 ms launches out of the device
          // kernels' instantiations in traces (rocprofv3 stats per kernel)
          hipLaunchKernelGGL((combine_lds<OP, T, kUnroll, kStoreSc1>), grid,
                             dim3(kLdsWaves * 64), 0, s, d, v, nvec);
        } else if (nvec * 16 >= kTaperBytes && nvec * 16 < kSc1Bytes) {
          // the last 1/kTaperDiv of the vectors in 1-KiB tiles
          const size_t hv = (size_t)kLdsWaves * 64 * kUnroll;
          size_t split = nvec - nvec / kTaperDiv;
          split -= split % hv;
          const unsigned head = (unsigned)(split / hv);
          const unsigned tail = (unsigned)((nvec - split + kLdsWaves * 64 - 1) / (kLdsWaves * 64));
          hipLaunchKernelGGL((combine_lds_taper<OP, T, kUnroll, kStoreSc1>), dim3(head + tail),
                             dim3(kLdsWaves * 64), 0, s, d, v, nvec, split, head);
        } else if (nvec * 16 < kSc1Bytes)
          hipLaunchKernelGGL((combine_lds<OP, T, kUnroll, kStoreSc1>), grid,
                             dim3(kLdsWaves * 64), 0, s, d, v, nvec);
        else
          hipLaunchKernelGGL((combine_lds<OP, T, kUnroll, kStoreNt>), grid,
                             dim3(kLdsWaves * 64), 0, s, d, v, nvec);
      }
      if (head + tail)
        hipLaunchKernelGGL((combine_elem<OP, T>),
                           dim3(grid_for(head + tail, kBlock, kElemGridCap)),
                           dim3(kBlock), 0, s, (T *)dst, (const T *)src, head,
                           head + body, tail);
    } else {
      hipLaunchKernelGGL((combine_elem<OP, T>),
                         dim3(grid_for(cnt, kBlock, kElemGridCap)), dim3(kBlock),
                         0, s, (T *)dst, (const T *)src, cnt, (size_t)0,
                         (size_t)0);
    }
    return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
  }
}

// Vector body of the tree (bench.py --tune-tree): LDS-DMA for
// 2 inputs, chunked nt register loads for more (U=2 above 8 inputs).
template <int OP, typename T, int NLEAF, int W, int U>
static void launch_tree_lds(const TreeArgs &b, int nsrc, u32x4 *dst,
                            size_t nvec, hipStream_t s) {
  hipLaunchKernelGGL((reduce_tree_lds<OP, T, NLEAF, W, U>),
                     dim3(grid_for(nvec, (size_t)W * 64 * U, 0x7fffffffu)),
                     dim3(W * 64), (size_t)nsrc * W * U * 64 * sizeof(u32x4), s,
                     b, nsrc, dst, nvec);
}

constexpr unsigned kTreeCapLds = 41u << 10;

template <int OP, typename T, int NLEAF, bool ALL = false>
static void launch_tree_body(const TreeArgs &b, int nsrc, u32x4 *dst,
                             size_t nvec, hipStream_t s, int variant = -1) {
  // Product choice (bench.py --tune-tree, profiles/r01_tune_tree_sc1.log):
  // below kSc1Bytes of output the U=2 chunk form with write-through stores
  // wins at every fan-in (2..16 inputs: 58.9/53.4/52.1/51.7 us against
  // 63.2/58.2/53.9/51.7 for the nt-store forms, 256 MiB of inputs).
  //
  // Round 5: at 3..8 inputs that form runs with 41 KiB of dynamic LDS the body
  // never touches, so at most 3 workgroups (12 waves) share a CU: fewer input
  // streams in flight per CU.  Interleaved A/B on two boxes, 256 MiB of inputs
  // (bench.py --tune-tree variants -1 / 20, profiles/r05_tune_tree_occupancy_*.json):
  // 4 inputs 55.44 -> 53.10 and 55.00 -> 53.52 us, 8 inputs 53.98 -> 52.84 and
  // 53.84 -> 52.92 us; 2 inputs lose (58.8 -> 61.8) and 16 tie, so they keep
  // the full occupancy.
  const unsigned cap_lds =
      (variant < 0 && nvec * 16 < kSc1Bytes && nsrc >= 3 && nsrc <= 8) ? kTreeCapLds : 0u;
  // Round 5: at 8-15 inputs of >= 4-byte lanes the P2P push kernel's body
  // with one output (4 KiB per wave per input through tile-sized buffer
  // descriptors, nt loads, write-through stores) beat that form: 8 inputs
  // 52.28 -> 50.56 us, 16 (as U = 4 float) 52.26 -> 50.68 us; at 4 inputs it
  // lost (52.74 -> 53.22), at 2 tied (bench.py --tune-tree variants -1 / 25,
  // profiles/r05_tune_tree_putbody.json)
  constexpr bool kPutBody = NLEAF == 8 && sizeof(T) >= 4;
  if (variant < 0 && nvec * 16 < kSc1Bytes && kPutBody) variant = 25;
  if (variant < 0 && nvec * 16 < kSc1Bytes) variant = 11;
  if (variant < 0) variant = nsrc <= 2 ? 3 : nsrc > 8 ? 2 : 1;
  // nsrc lies in [NLEAF, 2·NLEAF): only these forms are reachable from the
  // product choice, so only they are instantiated into liblfa.so (ALL: the
  // tuning library, which times every form at every fan-in)
  constexpr bool has3 = ALL || NLEAF == 2;   // nsrc <= 2
  constexpr bool has2 = ALL || NLEAF >= 8;   // nsrc > 8
  constexpr bool has1 = ALL || NLEAF <= 8;   // 3 <= nsrc <= 8
  if (variant == 2) {
    if constexpr (has2) {
      hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 2>),
                         dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)),
                         dim3(kBlock), 0, s, b, dst, nvec);
      return;
    }
  } else if (variant == 3) {
    if constexpr (has3) {
      launch_tree_lds<OP, T, NLEAF, kLdsWaves, 1>(b, nsrc, dst, nvec, s);
      return;
    }
  } else if (variant == 1) {
    if constexpr (has1) {
      hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 1>),
                         dim3(grid_for(nvec, (size_t)kBlock, 0x7fffffffu)),
                         dim3(kBlock), 0, s, b, dst, nvec);
      return;
    }
  } else if (variant >= 20 && variant <= 24) {
    if constexpr (ALL) {
      // round 5: the write-through chunk form at capped occupancy (dynamic
      // LDS the body never touches) and at 4 vectors per lane
      constexpr unsigned kCap[5] = {41u << 10, 54u << 10, 81u << 10, 0u, 54u << 10};
      const unsigned lds = kCap[variant - 20];
      if (variant < 23)
        hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 2, kStoreSc1>),
                           dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)),
                           dim3(kBlock), lds, s, b, dst, nvec);
      else
        hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 4, kStoreSc1>),
                           dim3(grid_for(nvec, (size_t)kBlock * 4, 0x7fffffffu)),
                           dim3(kBlock), lds, s, b, dst, nvec);
      return;
    }
  } else if (variant == 27 || variant == 28) {
    if constexpr (ALL) {
      // round 5: the push kernel's body with one output at 2 KiB per wave per
      // input; 28 at <= 3 workgroups per CU
      PutArgs pa;
      pa.t = b;
      memset(pa.out, 0, sizeof(pa.out));
      pa.out[0] = dst;
      pa.nout = 1;
      hipLaunchKernelGGL((reduce_tree_put<OP, T, NLEAF, 2>),
                         dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)), dim3(kBlock),
                         variant == 28 ? (41u << 10) : 0u, s, pa, nvec);
      return;
    }
  } else if (variant == 25 || variant == 26) {
    if constexpr (ALL || kPutBody) {
      // round 5: the P2P push kernel's body with one output (4 KiB per wave
      // per input through tile-sized buffer descriptors, system-scope nt
      // loads, write-through stores); 26 at <= 3 workgroups per CU
      PutArgs pa;
      pa.t = b;
      memset(pa.out, 0, sizeof(pa.out));
      pa.out[0] = dst;
      pa.nout = 1;
      hipLaunchKernelGGL((reduce_tree_put<OP, T, NLEAF, 4>),
                         dim3(grid_for(nvec, (size_t)kBlock * 4, 0x7fffffffu)), dim3(kBlock),
                         variant == 26 ? (41u << 10) : 0u, s, pa, nvec);
      return;
    }
  } else if (variant == 12) {
    if constexpr (ALL) {
      // the last 1/8 of the vectors one per lane (reduce_tree_taper)
      size_t split = nvec - nvec / 8;
      split -= split % ((size_t)kBlock * 2);
      const unsigned head = (unsigned)(split / ((size_t)kBlock * 2));
      const unsigned tail = (unsigned)((nvec - split + kBlock - 1) / kBlock);
      hipLaunchKernelGGL((reduce_tree_taper<OP, T, NLEAF>), dim3(head + tail), dim3(kBlock), 0,
                         s, b, dst, nvec, split, head);
      return;
    }
  }
  // variant 11, or a form this fan-in never selects: the write-through
  // chunk form, correct at every size
  hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 2, kStoreSc1>),
                     dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)),
                     dim3(kBlock), cap_lds, s, b, dst, nvec);
}

// Leaf pairing of prov/coll's tree for nsrc ranks (see TreeArgs); returns
// the number of leaves (largest power of two <= nsrc).
static int tree_leaves(TreeArgs &a, const void *const *srcs, int nsrc) {
  int pof2 = 1;
  while (pof2 * 2 <= nsrc) pof2 *= 2;
  const int rem = nsrc - pof2;
  memset(&a, 0, sizeof(a));
  for (int k = 0; k < nsrc; k++) a.in[k] = srcs[k];
  for (int k = 0; k < pof2; k++) {
    if (k < rem) {
      a.hi[k] = (signed char)(2 * k + 1);
      a.lo[k] = (signed char)(2 * k);
    } else {
      a.hi[k] = (signed char)(k + rem);
      a.lo[k] = -1;
    }
  }
  return pof2;
}

// The vector body's launcher as a policy, so the tuning library
// (lfa_tune.hip, liblfa_tune.so) can time other forms through the same
// pairing / head / tail logic without linking them into liblfa.so.
struct ProductTreeBody {
  template <int OP, typename T, int NLEAF>
  static void launch(const TreeArgs &b, int nsrc, u32x4 *dst, size_t nvec,
                     hipStream_t s, int variant) {
    launch_tree_body<OP, T, NLEAF>(b, nsrc, dst, nvec, s, variant);
  }
};

template <int OP, typename T, int NLEAF, typename Body = ProductTreeBody>
static int launch_tree_n(const TreeArgs &a, int nsrc, void *dst, size_t cnt,
                         bool vec, size_t head, size_t nvec, hipStream_t s,
                         int variant) {
  constexpr size_t E = sizeof(T);
  if (vec && nvec) {
    TreeArgs b = a;
    for (int k = 0; k < kMaxLeaf; k++)
      if (b.in[k]) b.in[k] = (const char *)b.in[k] + head * E;
    Body::template launch<OP, T, NLEAF>(b, nsrc, (u32x4 *)((char *)dst + head * E),
                                        nvec, s, variant);
  }
  size_t body = vec ? nvec * 16 / E : 0;
  size_t n0 = vec ? head : cnt;
  size_t tail = vec ? cnt - head - body : 0;
  if (n0 + tail)
    hipLaunchKernelGGL((reduce_tree_elem<OP, T, NLEAF>),
                       dim3(grid_for(n0 + tail, kBlock, kElemGridCap)),
                       dim3(kBlock), 0, s, a, (T *)dst, n0, head + body, tail);
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

template <int OP, typename T, typename Body = ProductTreeBody>
static int launch_tree(void *dst, const void *const *srcs, int nsrc,
                       size_t cnt, hipStream_t s, int variant = -1) {
  if constexpr (!supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    constexpr size_t E = sizeof(T);
    if (nsrc < 1 || nsrc > kMaxLeaf) return -LFA_EINVAL;
    if (cnt == 0) return 0;
    if (nsrc == 1) {
      if (dst == srcs[0]) return 0;
      return hipMemcpyAsync(dst, srcs[0], cnt * E, hipMemcpyDeviceToDevice,
                            s) == hipSuccess ? 0 : -LFA_EIO;
    }
    TreeArgs a;
    const int pof2 = tree_leaves(a, srcs, nsrc);
    uintptr_t mis = (uintptr_t)dst % 16, anyelem = (uintptr_t)dst % E;
    for (int k = 0; k < nsrc; k++) {
      mis |= ((uintptr_t)srcs[k] % 16) ^ ((uintptr_t)dst % 16);
      anyelem |= (uintptr_t)srcs[k] % E;
    }
    if (anyelem) {
      hipLaunchKernelGGL((reduce_tree_unaligned<OP, T>),
                         dim3(grid_for(cnt, kBlock, kElemGridCap)), dim3(kBlock), 0, s,
                         a, pof2, dst, cnt);
      return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
    }
    bool vec = (mis == 0) && E <= 16;
    size_t head = vec ? ((16 - (uintptr_t)dst % 16) % 16) / E : 0;
    if (head > cnt) head = cnt;
    size_t nvec = vec ? (cnt - head) * E / 16 : 0;
    switch (pof2) {
      case 2: return launch_tree_n<OP, T, 2, Body>(a, nsrc, dst, cnt, vec, head, nvec, s, variant);
      case 4: return launch_tree_n<OP, T, 4, Body>(a, nsrc, dst, cnt, vec, head, nvec, s, variant);
      case 8: return launch_tree_n<OP, T, 8, Body>(a, nsrc, dst, cnt, vec, head, nvec, s, variant);
      case 16: return launch_tree_n<OP, T, 16, Body>(a, nsrc, dst, cnt, vec, head, nvec, s, variant);
      case 32: return launch_tree_n<OP, T, 32, Body>(a, nsrc, dst, cnt, vec, head, nvec, s, variant);
      default: return -LFA_EINVAL;
    }
  }
}

// Wide fan-out (LFA_ALGO_P2P's allreduce push: every member's block to all
// N members) with the occupancy held at ONE workgroup per CU.  The body never
// touches LDS; the dynamic LDS a launch reserves (over half of the CU's
// 160 KiB) only keeps a second workgroup off the CU.  At 8 inputs -> 8
// outputs the 136-VGPR body otherwise runs 12 waves per CU with ~32 KiB of
// loads and 32 KiB of stores in flight per wave, which over-subscribes HBM
// with 16 concurrent streams: 4 waves per CU with 2 KiB tiles (64 KiB of
// loads in flight per CU) ran 8 x 32 MiB -> 8 in 90.0 us against 96.1-97.1
// (two boxes, 3 fresh buffer sets rotated, bench.py --tune-treeput variants
// 39 vs 0, profiles/r05_tune_treeput_occupancy_*.json).  At 4 outputs the
// forms tie (66-68 us), at 1-2 outputs the reads want the full occupancy
// (49.3 vs 52.7 us at 8 -> 1), so only wide fan-outs take this form.
constexpr int kPutNarrowOuts = 6;
constexpr unsigned kPutNarrowLds = 96u << 10;

template <int OP, typename T, int NLEAF, int UF = 0>
static int launch_tree_put_n(const PutArgs &a, size_t cnt, bool vec, size_t head,
                             hipStream_t s) {
  constexpr size_t E = sizeof(T);
  // 4 KiB of every input per wave (tune variant 14: +2 points over 2 KiB at
  // 8 inputs) where the registers allow it: up to 8 leaves of 4-16 B
  // elements.  Wider fan-in or byte/short lanes keep 2 KiB (U = 4 there
  // needs > 256 VGPRs and gave wrong uint8 results at 16 leaves).
  constexpr int U = UF ? UF : (NLEAF <= 8 && E >= 4) ? 4 : 2;
  constexpr bool kNarrowable = UF == 0 && NLEAF <= 8 && E >= 4;
  size_t nvec = vec ? (cnt - head) * E / 16 : 0;
  if (nvec) {
    PutArgs b = a;
    for (int k = 0; k < kMaxLeaf; k++)
      if (b.t.in[k]) b.t.in[k] = (const char *)b.t.in[k] + head * E;
    for (int j = 0; j < b.nout; j++) b.out[j] = (char *)b.out[j] + head * E;
    if (kNarrowable && b.nout >= kPutNarrowOuts)
      hipLaunchKernelGGL((reduce_tree_put<OP, T, NLEAF, 2>),
                         dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)),
                         dim3(kBlock), kPutNarrowLds, s, b, nvec);
    else
      hipLaunchKernelGGL((reduce_tree_put<OP, T, NLEAF, U>),
                         dim3(grid_for(nvec, (size_t)kBlock * U, 0x7fffffffu)),
                         dim3(kBlock), 0, s, b, nvec);
  }
  size_t body = nvec * 16 / E;
  size_t n0 = vec ? head : cnt;
  size_t tail = vec ? cnt - head - body : 0;
  if (n0 + tail)
    hipLaunchKernelGGL((reduce_tree_put_elem<OP, T, NLEAF>),
                       dim3(grid_for(n0 + tail, kBlock, kElemGridCap)), dim3(kBlock),
                       0, s, a, n0, head + body, tail);
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

// UF != 0 forces the vector body's tile (KiB per wave) — liblfa_tune.so only.
template <int OP, typename T, int UF = 0>
static int launch_tree_put(void *const *dsts, int ndst, const void *const *srcs,
                           int nsrc, size_t cnt, hipStream_t s) {
  if constexpr (!supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    constexpr size_t E = sizeof(T);
    if (nsrc < 1 || nsrc > kMaxLeaf || ndst < 1 || ndst > kMaxPut) return -LFA_EINVAL;
    if (cnt == 0) return 0;
    PutArgs a;
    const int pof2 = tree_leaves(a.t, srcs, nsrc);
    memset(a.out, 0, sizeof(a.out));
    a.nout = ndst;
    const uintptr_t p0 = (uintptr_t)dsts[0];
    uintptr_t mis = 0, anyelem = 0;
    for (int k = 0; k < nsrc; k++) {
      mis |= ((uintptr_t)srcs[k] ^ p0) % 16;
      anyelem |= (uintptr_t)srcs[k] % E;
    }
    for (int j = 0; j < ndst; j++) {
      a.out[j] = dsts[j];
      mis |= ((uintptr_t)dsts[j] ^ p0) % 16;
      anyelem |= (uintptr_t)dsts[j] % E;
    }
    if (anyelem) {
      uint32_t in_sys = 0, out_sys = 0;
      for (int k = 0; k < nsrc; k++)
        if ((uintptr_t)srcs[k] % E == 0) in_sys |= 1u << k;
      for (int j = 0; j < ndst; j++)
        if ((uintptr_t)dsts[j] % E == 0) out_sys |= 1u << j;
      hipLaunchKernelGGL((reduce_tree_put_unaligned<OP, T>),
                         dim3(grid_for(cnt, kBlock, kElemGridCap)), dim3(kBlock), 0, s,
                         a, pof2, in_sys, out_sys, cnt);
      return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
    }
    const bool vec = mis == 0 && E <= 16;
    size_t head = vec ? ((16 - p0 % 16) % 16) / E : 0;
    if (head > cnt) head = cnt;
    switch (pof2) {
      case 1: return launch_tree_put_n<OP, T, 1, UF>(a, cnt, vec, head, s);
      case 2: return launch_tree_put_n<OP, T, 2, UF>(a, cnt, vec, head, s);
      case 4: return launch_tree_put_n<OP, T, 4, UF>(a, cnt, vec, head, s);
      case 8: return launch_tree_put_n<OP, T, 8, UF>(a, cnt, vec, head, s);
      case 16: return launch_tree_put_n<OP, T, 16, UF>(a, cnt, vec, head, s);
      case 32: return launch_tree_put_n<OP, T, 32, UF>(a, cnt, vec, head, s);
      default: return -LFA_EINVAL;
    }
  }
}

// LFA_OS_LL=1: the LL one-shot for small allreduce / reduce_scatter parts
// (the same setting on every member of a group, as both sides of the
// exchange follow it).  Off by default: on one MI355X shared by two processes
// it measured 0.6-1.7 us SLOWER than the flagged kernel (256 lanes polling
// uncached words against the peer's incoming stores).
// Not for reduce: its non-root members wait for nothing, so one could run two
// operations ahead and overwrite the root's words of the same parity before
// the root read them (the flagged kernel posts and waits on every member).
static inline bool ll_enabled() {
  static int on = -1;
  if (on < 0) {
    const char *e = lfa_param("LFA_OS_LL");
    on = e && e[0] == '1';
  }
  return on;
}

// The one-shot's smallest per-workgroup chunk (bytes, a multiple of 16):
// LFA_OS_MIN_CHUNK, the same on every member of a group (the grid and the
// flag columns follow it); 4096 by default.  A tuning knob.
static inline size_t os_min_chunk() {
  static long c = -1;
  if (c < 0) {
    const char *e = lfa_param("LFA_OS_MIN_CHUNK");
    const long v = e ? atol(e) : 0;
    c = v >= 16 && v <= (1l << 20) ? (v + 15) & ~15l : 4096;
  }
  return (size_t)c;
}

template <int OP, typename T>
static int launch_oneshot(const lfa_oneshot &h, hipStream_t s) {
  if constexpr (!supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    constexpr size_t E = sizeof(T);
    const int n = h.n, r = h.rank;
    if (n < 1 || n > kOsMax || r < 0 || r >= n || (n > 1 && (!h.sym || !h.status)) ||
        h.mode < LFA_ONESHOT_SCATTER || h.mode >= n || (h.done_word && !h.done_ctr))
      return -LFA_EINVAL;
    if (h.count == 0) return 0;
    OsArgs a;
    memset(&a, 0, sizeof(a));
    size_t most = 0, slen[kOsMax] = {}, soff[kOsMax] = {};
    for (int k = 0; k < n; k++) {
      if (h.mode == LFA_ONESHOT_SCATTER) {  // lfa_coll_block's partition
        const size_t base = h.count / (size_t)n, extra = h.count % (size_t)n;
        const size_t kk = (size_t)k;
        slen[k] = (base + (kk < extra ? 1 : 0)) * E;
        soff[k] = (kk * base + (kk < extra ? kk : extra)) * E;
      } else {
        slen[k] = h.mode == LFA_ONESHOT_ALL || h.mode == k ? h.count * E : 0;
      }
      if (slen[k] > most) most = slen[k];
    }
    // 32-bit ranges in the argument block
    if (h.count > 0xffffffffu / E) return -LFA_EINVAL;
    for (int k = 0; k < n; k++) {
      a.slen[k] = (uint32_t)slen[k];
      a.soff[k] = (uint32_t)soff[k];
    }
    if (!h.send || (!h.result && a.slen[r]) || most > 0xffffffffu ||
        (n > 1 && (h.slot_bytes < most || h.slot_bytes % 256 || h.parity_off % 256 ||
                   (size_t)n * h.slot_bytes > h.parity_off)))
      return -LFA_EINVAL;
    for (int k = 0; k < n && n > 1; k++)
      if (!h.sym[k] || (uintptr_t)h.sym[k] % 256) return -LFA_EINVAL;
    const void *srcs[kOsMax];
    const size_t par = (size_t)(h.epoch & 1) * h.parity_off;
    uintptr_t mis = (uintptr_t)h.result % 16;
    for (int k = 0; k < n; k++) {
      mis |= ((uintptr_t)h.send + a.soff[k]) % 16;
      srcs[k] = k == r ? (const char *)h.send + a.soff[r]
                       : h.sym[r] + par + (size_t)k * h.slot_bytes;
      if (k != r) {
        a.push[k] = h.sym[k] + par + (size_t)r * h.slot_bytes;
        a.post[k] = (uint32_t *)(h.sym[k] + h.flag_off + LFA_SIG_OS_OFF) + r;
      }
    }
    TreeArgs tree;
    const int pof2 = tree_leaves(tree, srcs, n);
    for (int k = 0; k < kOsMax; k++) {
      a.t.in[k] = k < n ? tree.in[k] : nullptr;
      a.t.hi[k] = tree.hi[k];
      a.t.lo[k] = tree.lo[k];
    }
    if (n > 1 && most <= LFA_OS_LL_BYTES &&
        (h.mode == LFA_ONESHOT_ALL || h.mode == LFA_ONESHOT_SCATTER) && ll_enabled()) {
      // LL one-shot: the words live in the flag area (lfa_signal.h)
      LlArgs l;
      memset(&l, 0, sizeof(l));
      const size_t lpar = (size_t)(h.epoch & 1) * LFA_SIG_LL_PARITY;
      for (int k = 0; k < n; k++) {
        l.soff[k] = (uint32_t)a.soff[k];
        l.slen[k] = (uint32_t)a.slen[k];
        if (k != r)
          l.push[k] = h.sym[k] + h.flag_off + LFA_SIG_LL_OFF + lpar + (size_t)r * LFA_SIG_LL_SLOT;
        l.hi[k] = a.t.hi[k];
        l.lo[k] = a.t.lo[k];
      }
      l.own = h.sym[r] + h.flag_off + LFA_SIG_LL_OFF + lpar;
      l.send = (const char *)h.send;
      l.result = (char *)h.result;
      l.status = h.status;
      l.ticket = h.ticket;
      l.timeout = h.timeout_us * lfa__wallclock_ticks_per_us();
      l.done_ctr = h.done_ctr;
      l.done_word = h.done_word;
      l.done_val = h.done_val;
      l.flag = h.epoch * 2u + 1u;
      l.n = n;
      l.rank = r;
      l.vec = mis == 0;
      // the same grid on every member: `most` depends only on count and n
      const unsigned grid = (unsigned)(((most + 15) / 16 + kBlock - 1) / kBlock);
      switch (pof2) {
        case 2:
          hipLaunchKernelGGL((oneshot_ll<OP, T, 2>), dim3(grid), dim3(kBlock), 0, s, l);
          break;
        case 4:
          hipLaunchKernelGGL((oneshot_ll<OP, T, 4>), dim3(grid), dim3(kBlock), 0, s, l);
          break;
        case 8:
          hipLaunchKernelGGL((oneshot_ll<OP, T, 8>), dim3(grid), dim3(kBlock), 0, s, l);
          break;
        default:
          return -LFA_EINVAL;
      }
      return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
    }
    a.wait = n > 1 ? (const uint32_t *)(h.sym[r] + h.flag_off + LFA_SIG_OS_OFF) : nullptr;
    a.done_ctr = h.done_ctr;
    a.done_word = h.done_word;
    a.done_val = h.done_val;
    a.send = (const char *)h.send;
    a.result = (char *)h.result;
    a.status = h.status;
    a.timeout = h.timeout_us * lfa__wallclock_ticks_per_us();
    size_t chunk = (most + LFA_SIG_OS_CHUNKS - 1) / LFA_SIG_OS_CHUNKS;
    chunk = (chunk + 15) & ~(size_t)15;
    a.chunk = chunk < os_min_chunk() ? os_min_chunk() : chunk;
    a.epoch = h.epoch;
    a.ticket = h.ticket;
    a.n = n;
    a.rank = r;
    a.unal = (uintptr_t)h.send % E || (uintptr_t)h.result % E;
    a.vec = mis == 0 && E <= 16 && !a.unal;
    // the same grid on every member: `most` depends only on count and n
    const unsigned grid = (unsigned)((most + a.chunk - 1) / a.chunk);
    switch (pof2) {
      case 1:
        hipLaunchKernelGGL((oneshot_reduce<OP, T, 1>), dim3(grid), dim3(kBlock), 0, s, a);
        break;
      case 2:
        hipLaunchKernelGGL((oneshot_reduce<OP, T, 2>), dim3(grid), dim3(kBlock), 0, s, a);
        break;
      case 4:
        hipLaunchKernelGGL((oneshot_reduce<OP, T, 4>), dim3(grid), dim3(kBlock), 0, s, a);
        break;
      case 8:
        hipLaunchKernelGGL((oneshot_reduce<OP, T, 8>), dim3(grid), dim3(kBlock), 0, s, a);
        break;
      default:
        return -LFA_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
  }
}

// Shared launcher for the fetch / swap tables: vector body when every operand
// is co-aligned mod 16, element path for heads, tails and the rest.
template <typename T, typename MakeF>
static int launch_fetch(const void *const *ptrs, int nptr, size_t cnt,
                        hipStream_t s, MakeF &&make) {
  constexpr size_t E = sizeof(T);
  if (cnt == 0) return 0;
  uintptr_t p0 = (uintptr_t)ptrs[0], mis = 0, elem_mis = 0;
  for (int k = 0; k < nptr; k++) {
    mis |= ((uintptr_t)ptrs[k] ^ p0) % 16;
    elem_mis |= (uintptr_t)ptrs[k] % E;
  }
  if (elem_mis) {
    auto f = make(std::integral_constant<bool, false>(), (size_t)0);
    hipLaunchKernelGGL(fetch_elem<decltype(f)>, dim3(grid_for(cnt, kBlock, kElemGridCap)),
                       dim3(kBlock), 0, s, f, cnt, (size_t)0, (size_t)0);
  } else if (mis == 0 && E <= 16) {
    size_t head = ((16 - p0 % 16) % 16) / E;
    if (head > cnt) head = cnt;
    size_t nvec = (cnt - head) * E / 16, body = nvec * 16 / E;
    size_t tail = cnt - head - body;
    auto f = make(std::integral_constant<bool, true>(), head);
    using FF = decltype(f);
    // 4 KiB per input per wave and write-through (sc1) stores at every size:
    // at 256 MiB per operand 168.0 us (79.9 %) for a float SUM readwrite and
    // 199.9 us (83.9 %) for a float CSWAP, against 174.3 / 204.8 us for the
    // round-1 register form and 174.6 / 201.1 us with nt stores
    // (tools/probe_fetch.py --tune, profiles/r02_tune_fetch.log).  Two
    // output streams make write-through win even where combine_lds (one
    // output) keeps nt.  Round 3: two-input bodies (readwrite) store step by
    // step as their loads land (fetch_drain), and from kSc1Bytes per operand
    // with nt stores, as combine_lds does: 256 MiB float SUM 163.2 / 164.9 us
    // nt-drained vs 166.7 / 166.8 sc1-drained vs 172.2 sc1 (two boxes, back
    // to back, profiles/r03_tune_fetch*.log).  The three-input compare body
    // gains nothing measurable either way (212.5 - 217.6 us over every form)
    // and keeps round 2's.
    // Round 6: the three-input compare body takes the nt-drained form from
    // kSc1Bytes too — 256 MiB float CSWAP 212.5 us (79.0 %) against 215.2 us
    // for the sc1 body on one box, 167.0-167.9 / 173.8-175.8 us for the
    // readwrite pair (tools/probe_fetch.py --tune, profiles/r06_tune_fetch_*.jsonl);
    // cmp loaded into VGPRs instead of LDS (5 workgroups per CU instead of 3)
    // measured 213.7 us, no better.
    constexpr int U = 4;
    constexpr bool D = FF::kIn == 2;
    const dim3 grid(grid_for(nvec, (size_t)kLdsWaves * 64 * U, 0x7fffffffu));
    const bool nt = nvec * 16 >= kSc1Bytes;
    if (nt)
      hipLaunchKernelGGL((fetch_lds<U, kStoreNt, FF, true>), grid, dim3(kLdsWaves * 64), 0, s,
                         f, nvec);
    if (nvec && !nt)
      hipLaunchKernelGGL((fetch_lds<U, kStoreSc1, FF, D>), grid, dim3(kLdsWaves * 64), 0, s,
                         f, nvec);
    if (head + tail)
      hipLaunchKernelGGL(fetch_elem<decltype(f)>,
                         dim3(grid_for(head + tail, kBlock, kElemGridCap)),
                         dim3(kBlock), 0, s, f, head, head + body, tail);
  } else {
    auto f = make(std::integral_constant<bool, true>(), (size_t)0);
    hipLaunchKernelGGL(fetch_elem<decltype(f)>, dim3(grid_for(cnt, kBlock, kElemGridCap)),
                       dim3(kBlock), 0, s, f, cnt, (size_t)0, (size_t)0);
  }
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

template <int OP, typename T>
static int launch_readwrite(void *dst, const void *src, void *res, size_t cnt,
                            hipStream_t s) {
  if constexpr (!rw_supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    const void *ptrs[3] = {dst, res, OP == OP_READ ? dst : src};
    return launch_fetch<T>(ptrs, 3, cnt, s, [&](auto aligned, size_t head) {
      constexpr bool A = decltype(aligned)::value;
      const size_t hb = head * sizeof(T);
      return RwF<OP, T, A>{(char *)dst, (const char *)src, (char *)res,
                           (u32x4 *)((char *)dst + hb),
                           (const u32x4 *)((const char *)src + hb),
                           (u32x4 *)((char *)res + hb)};
    });
  }
}

template <int OP, typename T>
static int launch_swap(void *dst, const void *src, const void *cmp, void *res,
                       size_t cnt, hipStream_t s) {
  if constexpr (!swap_supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    const void *ptrs[4] = {dst, src, cmp, res};
    return launch_fetch<T>(ptrs, 4, cnt, s, [&](auto aligned, size_t head) {
      constexpr bool A = decltype(aligned)::value;
      const size_t hb = head * sizeof(T);
      return SwapF<OP, T, A>{(char *)dst, (const char *)src, (const char *)cmp,
                             (char *)res, (u32x4 *)((char *)dst + hb),
                             (const u32x4 *)((const char *)src + hb),
                             (const u32x4 *)((const char *)cmp + hb),
                             (u32x4 *)((char *)res + hb)};
    });
  }
}

}  // namespace lfa
