// lfa_k_tree.hpp — the N-input tree kernels: reduce_tree_* (the fused N -> 1 combine of LFA_ALGO_TREE) and reduce_tree_put (LFA_ALGO_P2P, system scope).
// Part of lfa_kernels.hpp (split in round 6); included by it, in order, after
// the shared helpers and the combine kernels.  Not included on its own.
#pragma once

namespace lfa {

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

}  // namespace lfa
