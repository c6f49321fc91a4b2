// lfa_k_fetch.hpp — the fetch (readwrite) and compare (swap) table kernels.
// Part of lfa_kernels.hpp (split in round 6); included by it, in order, after
// the shared helpers and the combine kernels.  Not included on its own.
#pragma once

namespace lfa {

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

// The drained fetch body with a tapered tail (round 6): the
// combine's taper (combine_lds_taper) applied to the fetch / compare kernel.
// Workgroups [0, head) run the drained U-KiB tiles up to vector `split`; the
// rest — dispatched last — take UT-KiB tiles, so the waves that end the
// launch are short ones.  The product runs it from kSc1Bytes (launch_fetch).
template <int U, int UT, int SAUX, typename F>
__global__ __launch_bounds__(kLdsWaves * 64) void fetch_lds_taper(F f, size_t nvec,
                                                                 size_t split, unsigned head) {
  __shared__ u32x4 lds[F::kIn][kLdsWaves][U][64];
  const unsigned w = wave_id(), l = threadIdx.x % 64, b = blockIdx.x;
  if (b < head) {
    // split is a multiple of a workgroup's tile: every head tile is whole
    const size_t base = (size_t)b * (kLdsWaves * 64 * U) + (size_t)w * 64 * U;
#pragma unroll
    for (int u = 0; u < U; u++)
#pragma unroll
      for (int k = 0; k < F::kIn; k++)
        __builtin_amdgcn_global_load_lds((const void *)(f.in(k) + base + u * 64 + l),
                                         (lds_void *)&lds[k][w][u][0], 16, 0, 2);
    fetch_drain<U, SAUX, F, 0>(
        f, lds, w, l, base,
        __builtin_amdgcn_make_buffer_rsrc(f.rv + base, 0, 64 * U * 16, 0x00020000),
        __builtin_amdgcn_make_buffer_rsrc(f.dv + base, 0, 64 * U * 16, 0x00020000));
    return;
  }
  const size_t base = split + (size_t)(b - head) * (kLdsWaves * 64 * UT) + (size_t)w * 64 * UT;
  if (base + 64 * UT <= nvec) {
#pragma unroll
    for (int u = 0; u < UT; u++)
#pragma unroll
      for (int k = 0; k < F::kIn; k++)
        __builtin_amdgcn_global_load_lds((const void *)(f.in(k) + base + u * 64 + l),
                                         (lds_void *)&lds[k][w][u][0], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc(f.rv + base, 0, 64 * UT * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(f.dv + base, 0, 64 * UT * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < UT; u++) {
      const u32x4 a = lds[0][w][u][l];
      const u32x4 bb = F::kIn > 1 ? lds[F::kIn > 1 ? 1 : 0][w][u][l] : a;
      const u32x4 c = F::kIn > 2 ? lds[F::kIn > 2 ? 2 : 0][w][u][l] : a;
      if constexpr (SAUX == kStoreNt) {
        st<true>(f.rv + base + u * 64 + l, a);
        if constexpr (F::kWriteDst) st<true>(f.dv + base + u * 64 + l, f.op(a, bb, c));
      } else {
        const unsigned off = (unsigned)(u * 64 + l) * 16;
        __builtin_amdgcn_raw_buffer_store_b128(a, rr, off, 0, SAUX);
        if constexpr (F::kWriteDst)
          __builtin_amdgcn_raw_buffer_store_b128(f.op(a, bb, c), rd, off, 0, SAUX);
      }
    }
  } else {
    for (int u = 0; u < UT; u++) {
      const size_t i = base + (size_t)u * 64 + l;
      if (i < nvec) f.vec(i);
    }
  }
}

}  // namespace lfa
