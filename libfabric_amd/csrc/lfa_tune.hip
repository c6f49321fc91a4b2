// lfa_tune.hip — alternative schedules of the headline kernel (float FI_SUM
// combine) for the on-GPU A/B sweep (bench.py --tune).  Not on the product
// path: the winner is folded back into combine_vec (lfa_combine.hip).
//
// Each variant is the same dst[i] += src[i] stream over 16-byte vectors; they
// differ only in how work maps to lanes, cache policy and staging:
//   layout 0  block-strided: step u of thread t -> base + u*B + t
//   layout 1  wave-contiguous: wave w owns U consecutive KiB
//   XCD       blockIdx remapped so XCD x sweeps one contiguous 1/8 of the buffer
//   LDSDMA    operands land in LDS through global_load_lds_dwordx4 (no VGPR
//             round trip), then ds_read_b128 -> add -> global store
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <errno.h>
#include <string.h>
#include <time.h>

#include "lfa_kernels.hpp"

namespace lfa_tune {

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

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
__device__ __forceinline__ u32x4 addf(u32x4 a, u32x4 b) {
  f32x4 x = __builtin_bit_cast(f32x4, a), y = __builtin_bit_cast(f32x4, b);
  return __builtin_bit_cast(u32x4, x + y);
}

__device__ __forceinline__ unsigned block_id(bool xcd) {
  unsigned b = blockIdx.x, nb = gridDim.x;
  if (xcd && nb % 8 == 0) b = (b % 8) * (nb / 8) + b / 8;
  return b;
}

template <int B, int U, bool NTL, bool NTS, int LAYOUT, bool XCD, bool INTERLEAVE>
__global__ __launch_bounds__(B) void sum_vec(u32x4 *__restrict__ dst,
                                             const u32x4 *__restrict__ src,
                                             size_t nvec) {
  const size_t blk = (size_t)block_id(XCD) * (B * U);
  const unsigned t = threadIdx.x;
  size_t idx[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    if constexpr (LAYOUT == 0) idx[u] = blk + (size_t)u * B + t;
    else idx[u] = blk + (size_t)(t / 64) * 64 * U + (size_t)u * 64 + (t % 64);
  }
  if (blk + (size_t)B * U <= nvec) {
    u32x4 a[U], b[U];
    if constexpr (INTERLEAVE) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        a[u] = ld<NTL>(dst + idx[u]);
        b[u] = ld<NTL>(src + idx[u]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++) a[u] = ld<NTL>(dst + idx[u]);
#pragma unroll
      for (int u = 0; u < U; u++) b[u] = ld<NTL>(src + idx[u]);
    }
#pragma unroll
    for (int u = 0; u < U; u++) st<NTS>(dst + idx[u], addf(a[u], b[u]));
  } else {
#pragma unroll
    for (int u = 0; u < U; u++)
      if (idx[u] < nvec)
        st<NTS>(dst + idx[u], addf(ld<NTL>(dst + idx[u]), ld<NTL>(src + idx[u])));
  }
}

// LDS-DMA staged: every wave pulls its U KiB of dst and src straight into
// LDS (global_load_lds_dwordx4, aux=nt), waits on its own vmcnt, reads back
// with ds_read_b128 and stores the sum.  No cross-wave sharing, no barrier.
// MODE 0: all dst then all src; 1: interleaved per step; 2: dst via LDS-DMA,
// src via register loads.
template <int W, int U, int AUX, int MODE>
__global__ __launch_bounds__(W * 64) void sum_ldsdma(u32x4 *__restrict__ dst,
                                                     const u32x4 *__restrict__ src,
                                                     size_t nvec) {
  __shared__ u32x4 lds[2][W][U][64];
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (W * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U <= nvec) {
    u32x4 b[U];
    if constexpr (MODE == 1) {
#pragma unroll
      for (int u = 0; u < U; u++) {
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0, AUX);
        __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                         (lds_void *)&lds[1][w][u][0], 16, 0, AUX);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0, AUX);
      if constexpr (MODE == 2) {
#pragma unroll
        for (int u = 0; u < U; u++) b[u] = ld<true>(src + base + u * 64 + l);
      } else {
#pragma unroll
        for (int u = 0; u < U; u++)
          __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                           (lds_void *)&lds[1][w][u][0], 16, 0, AUX);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) {
      u32x4 y = MODE == 2 ? b[u] : lds[1][w][u][l];
      st<true>(dst + base + u * 64 + l, addf(lds[0][w][u][l], y));
    }
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + u * 64 + l;
      if (i < nvec) st<true>(dst + i, addf(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

// Persistent LDS-DMA form: a grid sized to the resident capacity walks the
// chunks in a grid-stride loop (fewer workgroup launches, one tail).
// Workgroup-interleaved tiles: load u of wave w covers vectors
// wg_base + (u·W + w)·64 + l, so the W waves' u-th loads are one contiguous
// W KiB span (the product gives each wave U contiguous KiB instead).
template <int W, int U, int SAUX>
__global__ __launch_bounds__(W * 64) void sum_ldsdma_il(u32x4 *__restrict__ dst,
                                                        const u32x4 *__restrict__ src,
                                                        size_t nvec) {
  __shared__ u32x4 lds[2][W][U][64];
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t wg = (size_t)blockIdx.x * (W * 64 * U);
  if (wg + W * 64 * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(dst + wg + (u * W + w) * 64 + l),
                                       (lds_void *)&lds[0][w][u][0], 16, 0, 2);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(src + wg + (u * W + w) * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u32x4 v = addf(lds[0][w][u][l], lds[1][w][u][l]);
      if constexpr (SAUX == 2) {
        st<true>(dst + wg + (u * W + w) * 64 + l, v);
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(
            v, __builtin_amdgcn_make_buffer_rsrc(dst + wg + (u * W + w) * 64, 0, 64 * 16,
                                                 0x00020000),
            l * 16, 0, SAUX);
      }
    }
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = wg + (size_t)(u * W + w) * 64 + l;
      if (i < nvec) st<true>(dst + i, addf(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void sum_ldsdma_persist(u32x4 *__restrict__ dst,
                                                          const u32x4 *__restrict__ src,
                                                          size_t nvec) {
  __shared__ u32x4 lds[2][4][U][64];
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  for (size_t blk = blockIdx.x;; blk += gridDim.x) {
    const size_t base = blk * (256 * U) + (size_t)w * 64 * U;
    if (base >= nvec) break;
    if (base + 64 * U <= nvec) {
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0, 2);
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                         (lds_void *)&lds[1][w][u][0], 16, 0, 2);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
      for (int u = 0; u < U; u++)
        st<true>(dst + base + u * 64 + l, addf(lds[0][w][u][l], lds[1][w][u][l]));
      // the next iteration overwrites this wave's LDS slots: make sure the
      // ds_reads above have returned (their values feed the stores already)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    } else {
      for (int u = 0; u < U; u++) {
        size_t i = base + u * 64 + l;
        if (i < nvec) st<true>(dst + i, addf(ld<true>(dst + i), ld<true>(src + i)));
      }
    }
  }
}

// One wave's tile of U KiB per operand through LDS (the product body).
template <int U, int UMAX, int AUX>
__device__ __forceinline__ void ldsdma_tile(u32x4 *__restrict__ dst,
                                            const u32x4 *__restrict__ src, size_t nvec,
                                            size_t base, u32x4 (*lds)[UMAX][64],
                                            unsigned l) {
  if (base + 64 * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                       (lds_void *)&lds[0][u][0], 16, 0, AUX);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                       (lds_void *)&lds[1][u][0], 16, 0, AUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++)
      st<true>(dst + base + u * 64 + l, addf(lds[0][u][l], lds[1][u][l]));
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + u * 64 + l;
      if (i < nvec) st<true>(dst + i, addf(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

// Tapered grid: the first n4 workgroups take 4 KiB tiles per wave, the next
// n2 take 2 KiB, the rest 1 KiB.  Workgroups dispatch roughly in blockIdx
// order, so the last ones to start are the short ones and the drain at the
// end of the launch (CUs going idle one by one) is shorter.
template <int AUX>
__global__ __launch_bounds__(256) void sum_taper(u32x4 *__restrict__ dst,
                                                 const u32x4 *__restrict__ src,
                                                 size_t nvec, unsigned n4, unsigned n2) {
  __shared__ u32x4 lds[4][2][4][64];
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64, b = blockIdx.x;
  if (b < n4) {
    ldsdma_tile<4, 4, AUX>(dst, src, nvec, (size_t)b * 1024 + w * 256, lds[w], l);
  } else if (b < n4 + n2) {
    ldsdma_tile<2, 4, AUX>(dst, src, nvec,
                           (size_t)n4 * 1024 + (size_t)(b - n4) * 512 + w * 128, lds[w], l);
  } else {
    ldsdma_tile<1, 4, AUX>(dst, src, nvec,
                           (size_t)n4 * 1024 + (size_t)n2 * 512 +
                               (size_t)(b - n4 - n2) * 256 + w * 64,
                           lds[w], l);
  }
}

// LDS-DMA body with the stores issued as buffer stores carrying cache-policy
// bits SAUX (gfx950 cpol: sc0=1, nt=2, sc1=16).  sc1 stores write through
// the XCD L2 instead of leaving dirty lines for the end-of-kernel writeback.
template <int U, int SAUX>
__global__ __launch_bounds__(256) void sum_ldsdma_st(u32x4 *__restrict__ dst,
                                                     const u32x4 *__restrict__ src,
                                                     size_t nvec) {
  __shared__ u32x4 lds[2][4][U][64];
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (4 * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                       (lds_void *)&lds[0][w][u][0], 16, 0, 2);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(addf(lds[0][w][u][l], lds[1][w][u][l]), r,
                                             (u * 64 + l) * 16, 0, SAUX);
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + u * 64 + l;
      if (i < nvec) st<true>(dst + i, addf(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

static inline unsigned blocks(size_t nvec, size_t per) {
  return (unsigned)((nvec + per - 1) / per);
}

// Taper launch: the last s2 and s1 vectors (rounded) go to 2 KiB / 1 KiB tiles.
template <int AUX>
static void taper(u32x4 *d, const u32x4 *v, size_t nvec, size_t s2, size_t s1,
                  hipStream_t s) {
  size_t big = nvec > s2 + s1 ? nvec - s2 - s1 : 0;
  unsigned n4 = (unsigned)(big / 1024);
  size_t rest = nvec - (size_t)n4 * 1024;
  size_t r2 = rest > s1 ? rest - s1 : 0;
  unsigned n2 = (unsigned)(r2 / 512);
  size_t r1 = rest - (size_t)n2 * 512;
  unsigned n1 = blocks(r1, 256);
  hipLaunchKernelGGL((sum_taper<AUX>), dim3(n4 + n2 + n1), dim3(256), 0, s, d, v, nvec,
                     n4, n2);
}

}  // namespace lfa_tune

using namespace lfa_tune;

// Variants 12.. (0..11 live in lfa_combine.hip next to the product kernel).
extern "C" int lfa__tune2_sum_f32(int variant, void *dst, const void *src,
                                  size_t nvec, void *stream) {
  hipStream_t s = (hipStream_t)stream;
  u32x4 *d = (u32x4 *)dst;
  const u32x4 *v = (const u32x4 *)src;
#define RUN(B, U, NTL, NTS, L, X, I)                                             \
  hipLaunchKernelGGL((sum_vec<B, U, NTL, NTS, L, X, I>), dim3(blocks(nvec, B * U)), \
                     dim3(B), 0, s, d, v, nvec)
  switch (variant) {
    case 12: RUN(512, 4, true, true, 0, false, false); break;
    case 13: RUN(1024, 2, true, true, 0, false, false); break;
    case 14: RUN(256, 4, true, true, 1, false, false); break;
    case 15: RUN(256, 8, true, true, 1, false, false); break;
    case 16: RUN(256, 4, true, true, 0, true, false); break;
    case 17: RUN(256, 4, true, true, 0, false, true); break;
    case 18: RUN(64, 16, true, true, 1, false, false); break;
    case 19: RUN(256, 4, true, true, 0, false, false); break;  // = product, in this TU
#define LDSDMA(W, U, AUX, MODE)                                                  \
  hipLaunchKernelGGL((sum_ldsdma<W, U, AUX, MODE>), dim3(blocks(nvec, W * 64 * U)), \
                     dim3(W * 64), 0, s, d, v, nvec)
    case 20: LDSDMA(4, 4, 2, 0); break;
    case 21: LDSDMA(4, 4, 0, 0); break;
    case 22: LDSDMA(4, 8, 2, 0); break;
    case 24: LDSDMA(4, 2, 2, 0); break;
    case 25: LDSDMA(8, 4, 2, 0); break;
    case 26: LDSDMA(4, 4, 2, 2); break;
    case 27: LDSDMA(4, 4, 2, 1); break;
    case 28: LDSDMA(2, 4, 2, 0); break;
    case 29: LDSDMA(1, 4, 2, 0); break;
    case 31: LDSDMA(8, 2, 2, 0); break;
    case 32: LDSDMA(16, 1, 2, 0); break;
    case 33: LDSDMA(4, 3, 2, 0); break;
    case 34: LDSDMA(8, 1, 2, 0); break;
    case 35: LDSDMA(4, 4, 2, 2); break;
    case 36:
      hipLaunchKernelGGL((sum_ldsdma_persist<4>),
                         dim3(min(blocks(nvec, 256 * 4), 256u * 5)), dim3(256), 0, s,
                         d, v, nvec);
      break;
    case 37:
      hipLaunchKernelGGL((sum_ldsdma_persist<2>),
                         dim3(min(blocks(nvec, 256 * 2), 256u * 8)), dim3(256), 0, s,
                         d, v, nvec);
      break;
    case 38:
      hipLaunchKernelGGL((sum_ldsdma_persist<4>),
                         dim3(min(blocks(nvec, 256 * 4), 256u * 10)), dim3(256), 0, s,
                         d, v, nvec);
      break;
    case 23: RUN(256, 4, true, true, 1, true, true); break;
    // tapered tails (last workgroups take shorter tiles)
    case 40: taper<2>(d, v, nvec, 0, 1280 * 256, s); break;
    case 41: taper<2>(d, v, nvec, 0, 2560 * 256, s); break;
    case 42: taper<2>(d, v, nvec, 1280 * 512, 1280 * 256, s); break;
    case 43: taper<2>(d, v, nvec, 2560 * 512, 1280 * 256, s); break;
    case 47: taper<2>(d, v, nvec, 0, 640 * 256, s); break;
    // cache-policy bits on the LDS-DMA loads (gfx950 cpol: sc0=1, nt=2, sc1=16)
    case 44: LDSDMA(4, 4, 3, 0); break;
    case 45: LDSDMA(4, 4, 18, 0); break;
    case 46: LDSDMA(4, 4, 19, 0); break;
#define LDSST(U, SAUX)                                                           \
  hipLaunchKernelGGL((sum_ldsdma_st<U, SAUX>), dim3(blocks(nvec, 256 * U)), dim3(256), \
                     0, s, d, v, nvec)
    // store cache-policy bits (buffer stores)
    case 50: LDSST(4, 2); break;   // nt (= product policy, buffer form)
    case 51: LDSST(4, 16); break;  // sc1: write-through
    case 52: LDSST(4, 18); break;  // sc1 nt
    case 53: LDSST(4, 17); break;  // sc0 sc1
    case 54: LDSST(4, 19); break;  // sc0 sc1 nt
    case 55: LDSST(4, 0); break;   // plain
    case 56: LDSST(4, 1); break;   // sc0
    case 57: LDSST(4, 3); break;   // sc0 nt
    case 58: LDSDMA(4, 4, 16, 0); break;  // loads sc1 only, nt global stores
    case 59: LDSDMA(4, 4, 1, 0); break;   // loads sc0 only
#undef LDSST
#define LDSIL(W, U, SAUX)                                                        \
  hipLaunchKernelGGL((sum_ldsdma_il<W, U, SAUX>), dim3(blocks(nvec, W * 64 * U)),    \
                     dim3(W * 64), 0, s, d, v, nvec)
    // workgroup-interleaved tiles
    case 60: LDSIL(4, 4, 2); break;
    case 61: LDSIL(4, 4, 16); break;
    case 62: LDSIL(8, 2, 2); break;
    case 63: LDSIL(4, 2, 2); break;
#undef LDSIL
    default: return -LFA_EINVAL;
  }
#undef RUN
#undef LDSDMA
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

// ---------------------------------------------------------------------------
// the product kernels' alternative forms (lfa_kernels.hpp templates), timed
// against the product choice by bench.py --tune / --tune-tree
// ---------------------------------------------------------------------------
namespace lfa {

// Tree vector bodies the product does not ship: grid-stride plain loads (0),
// LDS-DMA with 4/2/1 waves (4-6), wave-contiguous U=2/4 (7-8), chunked sc1
// U=1/2 (9-10); anything else is the product's own choice.
struct TuneTreeBody {
  template <int OP, typename T, int NLEAF>
  static void launch(const TreeArgs &b, int nsrc, u32x4 *dst, size_t nvec,
                     hipStream_t s, int variant) {
    switch (variant) {
      case 0:
        hipLaunchKernelGGL((reduce_tree_vec<OP, T, NLEAF>),
                           dim3(grid_for(nvec, kBlock, 256 * 16)), dim3(kBlock), 0,
                           s, b, dst, nvec);
        return;
      case 4: return launch_tree_lds<OP, T, NLEAF, 4, 2>(b, nsrc, dst, nvec, s);
      case 5: return launch_tree_lds<OP, T, NLEAF, 2, 2>(b, nsrc, dst, nvec, s);
      case 6: return launch_tree_lds<OP, T, NLEAF, 1, 4>(b, nsrc, dst, nvec, s);
      case 7:
        hipLaunchKernelGGL((reduce_tree_wave<OP, T, NLEAF, 2>),
                           dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)),
                           dim3(kBlock), 0, s, b, dst, nvec);
        return;
      case 8:
        hipLaunchKernelGGL((reduce_tree_wave<OP, T, NLEAF, 4>),
                           dim3(grid_for(nvec, (size_t)kBlock * 4, 0x7fffffffu)),
                           dim3(kBlock), 0, s, b, dst, nvec);
        return;
      case 9:
        hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 1, kStoreSc1>),
                           dim3(grid_for(nvec, (size_t)kBlock, 0x7fffffffu)),
                           dim3(kBlock), 0, s, b, dst, nvec);
        return;
      case 10:
        hipLaunchKernelGGL((reduce_tree_chunk<OP, T, NLEAF, 2, kStoreSc1>),
                           dim3(grid_for(nvec, (size_t)kBlock * 2, 0x7fffffffu)),
                           dim3(kBlock), 0, s, b, dst, nvec);
        return;
      default:
        launch_tree_body<OP, T, NLEAF, true>(b, nsrc, dst, nvec, s, variant);
    }
  }
};

}  // namespace lfa

// Headline-kernel sweep (float SUM over nvec 16-B vectors).  -LFA_EINVAL for
// an unknown variant id.
extern "C" int lfa__tune_sum_f32(int variant, void *dst, const void *src,
                                 size_t nvec, void *stream) {
  using namespace lfa;
  hipStream_t s = (hipStream_t)stream;
  u32x4 *d = (u32x4 *)dst;
  const u32x4 *v = (const u32x4 *)src;
  auto chunk = [&](auto kern, int u) {
    hipLaunchKernelGGL(kern, dim3(grid_for(nvec, (size_t)kBlock * u, 0x7fffffffu)),
                       dim3(kBlock), 0, s, d, v, nvec);
  };
  auto gs = [&](auto kern, unsigned grid) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(kBlock), 0, s, d, v, nvec);
  };
  switch (variant) {
    case 0: chunk(combine_vec<OP_SUM, float, 4, true, true>, 4); break;
    case 30:  // the product launch itself
      return launch_write<OP_SUM, float>(dst, src, nvec * 4, s);
    case 1: chunk(combine_vec<OP_SUM, float, 1, true, true>, 1); break;
    case 2: chunk(combine_vec<OP_SUM, float, 2, true, true>, 2); break;
    case 3: chunk(combine_vec<OP_SUM, float, 8, true, true>, 8); break;
    case 4: chunk(combine_vec<OP_SUM, float, 4, false, false>, 4); break;
    case 5: chunk(combine_vec<OP_SUM, float, 4, true, false>, 4); break;
    case 6: chunk(combine_vec<OP_SUM, float, 4, false, true>, 4); break;
    case 7: gs(combine_vec_gs<OP_SUM, float, 4, true, true>, 2048); break;
    case 8: gs(combine_vec_gs<OP_SUM, float, 4, true, true>, 1024); break;
    case 9: gs(combine_vec_gs<OP_SUM, float, 2, true, true>, 4096); break;
    case 10: gs(combine_vec_gs<OP_SUM, float, 8, true, true>, 1024); break;
    case 11: chunk(combine_vec<OP_SUM, float, 8, false, false>, 8); break;
    default: return -LFA_EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

// Tree-kernel sweep: float SUM over `nsrc` device inputs; -1 = the product.
extern "C" int lfa__tune_tree_f32(int variant, void *dst, const void *const *srcs,
                                  int nsrc, size_t cnt, void *stream) {
  return lfa::launch_tree<lfa::OP_SUM, float, lfa::TuneTreeBody>(
      dst, srcs, nsrc, cnt, (hipStream_t)stream, variant);
}

// ---------------------------------------------------------------------------
// reduce_tree_put (LFA_ALGO_P2P kernel) forms, float SUM, vector body only:
// the product's loads/stores carry sc0 sc1 (system scope) for peer HBM over
// xGMI; these variants separate the cost of the scope bits from the tiling
// on LOCAL memory (bench.py --tune-treeput).  Not correct across GPUs unless
// they keep the product's scope bits.
// ---------------------------------------------------------------------------
namespace lfa {

template <int NLEAF, int U, int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void tp_tune(PutArgs a, size_t nvec) {
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t wbase = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP_SUM, float, u32x4, NLEAF>(a.t, [&](int k) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0, LAUX));
    });
  }
  for (int j = 0; j < a.nout; j++) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

// All loads of a wave's tile issued before any tree step (8 inputs, no
// leaf pairs: leaf k = input k, compile-time indices so the tiles stay in
// registers); the product evaluates input by input instead.
template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void tp_tune_pre(PutArgs a, size_t nvec) {
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t wbase = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 x[8][U];
#pragma unroll
  for (int k = 0; k < 8; k++) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      x[k][u] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(u * 64 + l) * 16, 0,
                                                       LAUX));
  }
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    auto f = [](u32x4 hi, u32x4 lo) { return apply_vec<OP_SUM, float>(hi, lo); };
    v[u] = f(f(f(x[7][u], x[6][u]), f(x[5][u], x[4][u])),
             f(f(x[3][u], x[2][u]), f(x[1][u], x[0][u])));
  }
  for (int j = 0; j < a.nout; j++) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

// Scalar wave index (the product's) with the outputs' stores paced: at 8
// outputs the round-2 body, whose divergent wave index put every store in a
// one-pass readfirstlane loop, ran 5 % faster than the product (round 3,
// 91.5 vs 96.4 us).  MODE 1: before output j >= 1, wait until at most
// output j-1's U stores are in flight; 2: until none are; 3: s_sleep 1
// between outputs; 4: u-major order (every output's u-th vector, then u+1).
template <int U, int LAUX, int SAUX, int MODE>
__global__ __launch_bounds__(kBlock) void tp_pace(PutArgs a, size_t nvec) {
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t wbase = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP_SUM, float, u32x4, 8>(a.t, [&](int k) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0, LAUX));
    });
  }
  if constexpr (MODE == 4) {
#pragma unroll
    for (int u = 0; u < U; u++)
      for (int j = 0; j < a.nout; j++)
        __builtin_amdgcn_raw_buffer_store_b128(
            __builtin_bit_cast(u32x4, v[u]), tile_rsrc((u32x4 *)a.out[j] + wbase, bytes),
            (unsigned)(u * 64 + l) * 16, 0, SAUX);
  } else {
    for (int j = 0; j < a.nout; j++) {
      if (j) {
        if constexpr (MODE == 1) wait_vmcnt<U>();
        if constexpr (MODE == 2) wait_vmcnt<0>();
        if constexpr (MODE == 3) __builtin_amdgcn_s_sleep(1);
      }
      __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                               (unsigned)(u * 64 + l) * 16, 0, SAUX);
    }
  }
}

// Round 4 forms of the 8 -> M push, product scope bits:
// STAGGER: wave g = 4·b + w writes the outputs starting at g mod M, so at
// any moment the waves' stores spread over every output stream instead of
// sweeping them in the same order.
template <int U, int LAUX, int SAUX, bool STAGGER>
__global__ __launch_bounds__(kBlock) void tp_r4(PutArgs a, size_t nvec) {
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t wbase = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP_SUM, float, u32x4, 8>(a.t, [&](int k) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0, LAUX));
    });
  }
  const int j0 = STAGGER ? (int)((blockIdx.x * (kBlock / 64) + w) % (unsigned)a.nout) : 0;
  for (int jj = 0; jj < a.nout; jj++) {
    int j = j0 + jj;
    if (j >= a.nout) j -= a.nout;
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

// Inputs through LDS-DMA (global_load_lds_dwordx4 with the loads' cache
// bits): the 8·U KiB of a wave's tile occupy no VGPRs while in flight, so
// more waves fit per SIMD; then the tree from LDS and the product's stores.
template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void tp_lds(PutArgs a, size_t nvec) {
  __shared__ u32x4 tl[8 * (kBlock / 64) * U * 64];  // [k][w][u][64]
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t wbase = (size_t)blockIdx.x * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  auto slot = [&](int k, int u) { return ((k * (kBlock / 64) + (int)w) * U + u) * 64; };
  u32x4 v[U];
  if (wbase + 64 * U <= nvec) {
#pragma unroll
    for (int k = 0; k < 8; k++)
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds(
            (const void *)((const u32x4 *)a.t.in[k] + wbase + u * 64 + l),
            (lds_void *)&tl[slot(k, u)], 16, 0, LAUX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int u = 0; u < U; u++)
      v[u] = tree_eval_with<OP_SUM, float, u32x4, 8>(
          a.t, [&](int k) { return tl[slot(k, u) + l]; });
  } else {
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = wbase + (size_t)u * 64 + l;
      v[u] = i < nvec ? tree_eval_with<OP_SUM, float, u32x4, 8>(
                            a.t, [&](int k) { return ((const u32x4 *)a.t.in[k])[i]; })
                      : u32x4{0, 0, 0, 0};
    }
  }
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  for (int j = 0; j < a.nout; j++) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

// Outputs split over the workgroup's waves: each wave reduces its own U-KiB
// tile as in the product and parks the result in LDS; after one barrier,
// wave w writes the WHOLE workgroup tile (4·U KiB, contiguous) to outputs
// w, w + 4, ...  Same bytes; each wave then has 2 output streams of
// 4·U KiB at 8 outputs instead of 8 streams of U KiB.
template <int U, int LAUX, int SAUX>
__global__ __launch_bounds__(kBlock) void tp_split(PutArgs a, size_t nvec) {
  constexpr int W = kBlock / 64;
  __shared__ u32x4 res[W * U * 64];
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t gbase = (size_t)blockIdx.x * (kBlock * U);
  const size_t wbase = gbase + (size_t)w * 64 * U;
  if (wbase < nvec) {
    const size_t left = nvec - wbase;
    const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const unsigned off = (unsigned)(u * 64 + l) * 16;
      res[(w * U + u) * 64 + l] = tree_eval_with<OP_SUM, float, u32x4, 8>(a.t, [&](int k) {
        return __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0, LAUX));
      });
    }
  }
  __syncthreads();
  if (gbase >= nvec) return;
  const size_t gleft = nvec - gbase;
  const unsigned gbytes = (unsigned)((gleft < (size_t)W * 64 * U ? gleft : (size_t)W * 64 * U) * 16);
  for (int j = (int)w; j < a.nout; j += W) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + gbase, gbytes);
#pragma unroll
    for (int t = 0; t < W * U; t++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, res[t * 64 + l]), r,
                                             (unsigned)(t * 64 + l) * 16, 0, SAUX);
  }
}

// Round 5 forms of the 8 -> M push, product body and scope
// bits.  XCD: workgroups are dispatched round-robin over the 8 XCDs, so by
// default XCD x streams tiles x, x + 8, ...; remapped, XCD x takes one
// contiguous run of tiles (a bijection for any grid), so each XCD's 16
// streams move through contiguous DRAM rows.  The occupancy cap (dynamic
// LDS that the body never touches, set at launch) bounds the workgroups per
// CU and so the bytes in flight: 136 VGPRs already allow 3 waves per SIMD
// (12 per CU, ~384 KiB of loads in flight per CU), far past what hides
// HBM latency, and fewer concurrent streams may keep more DRAM rows open.
template <int U, int LAUX, int SAUX, bool XCD, int NW = kBlock / 64>
__global__ __launch_bounds__(NW * 64) void tp_r5(PutArgs a, size_t nvec) {
  unsigned b = blockIdx.x;
  if constexpr (XCD) {
    const unsigned n = gridDim.x, q = n / 8, r = n % 8, x = b % 8;
    b = x * q + (x < r ? x : r) + b / 8;
  }
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t wbase = (size_t)b * (NW * 64 * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP_SUM, float, u32x4, 8>(a.t, [&](int k) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0, LAUX));
    });
  }
  for (int j = 0; j < a.nout; j++) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

// Round 6: the product's wide fan-out form (U = 2 KiB per input per wave,
// one workgroup per CU through the dynamic LDS it reserves, the product's
// cache policy) with a tapered tail: workgroups past `head` take 1-KiB tiles
// from vector `split` on, so the waves that end the launch are short — the
// form that gained ~1 % on the five-stream compare kernel (fetch_lds_taper).
template <int U>
__device__ __forceinline__ void tp_tile(const PutArgs &a, size_t wbase, size_t lim,
                                        unsigned l) {
  if (wbase >= lim) return;
  const size_t left = lim - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP_SUM, float, u32x4, 8>(a.t, [&](int k) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[k] + wbase, bytes), off, 0, kSysLoadAux));
    });
  }
  for (int j = 0; j < a.nout; j++) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, kSysAux);
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void tp_taper(PutArgs a, size_t nvec, size_t split,
                                                   unsigned head) {
  const unsigned b = blockIdx.x, w = wave_id<true>(), l = threadIdx.x % 64;
  if (b < head)
    tp_tile<U>(a, (size_t)b * (kBlock * U) + (size_t)w * 64 * U, split, l);
  else
    tp_tile<1>(a, split + (size_t)(b - head) * kBlock + (size_t)w * 64, nvec, l);
}

// Round 5: a resident grid whose waves walk tiles strided by the number of
// waves and keep the NEXT tile's loads in flight while they reduce and
// store the current one (two register buffers, ping-pong), so a wave's store
// phase no longer leaves HBM without reads; 8 inputs, the fixed
// ((7+6)+(5+4))+((3+2)+(1+0)) tree of a power-of-two member count.
template <int U>
__device__ __forceinline__ void tpp_load(u32x4 (&x)[8][U], const PutArgs &a, size_t tile,
                                         size_t nvec) {
  const size_t base = tile * (64 * U);
  const size_t left = nvec - base;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  const unsigned l = threadIdx.x % 64;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const __amdgpu_buffer_rsrc_t r = tile_rsrc((const u32x4 *)a.t.in[k] + base, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      x[k][u] = __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (unsigned)(u * 64 + l) * 16, 0,
                                                       kSysLoadAux));
  }
}

template <int U>
__device__ __forceinline__ void tpp_store(const u32x4 (&x)[8][U], const PutArgs &a,
                                          size_t tile, size_t nvec) {
  const size_t base = tile * (64 * U);
  const size_t left = nvec - base;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  const unsigned l = threadIdx.x % 64;
  auto f = [](u32x4 hi, u32x4 lo) { return apply_vec<OP_SUM, float>(hi, lo); };
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++)
    v[u] = f(f(f(x[7][u], x[6][u]), f(x[5][u], x[4][u])),
             f(f(x[3][u], x[2][u]), f(x[1][u], x[0][u])));
  for (int j = 0; j < a.nout; j++) {
    const __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + base, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(v[u], r, (unsigned)(u * 64 + l) * 16, 0, kSysAux);
  }
}

template <int U>
__global__ __launch_bounds__(kBlock) void tp_pipe(PutArgs a, size_t nvec) {
  const size_t nt = (nvec + 64 * U - 1) / (64 * U);
  const size_t step = (size_t)gridDim.x * (kBlock / 64);
  size_t t = (size_t)blockIdx.x * (kBlock / 64) + wave_id<true>();
  if (t >= nt) return;
  u32x4 A[8][U], B[8][U];
  tpp_load<U>(A, a, t, nvec);
  for (;;) {
    size_t t2 = t + step;
    if (t2 < nt) tpp_load<U>(B, a, t2, nvec);
    tpp_store<U>(A, a, t, nvec);
    if (t2 >= nt) break;
    t = t2;
    t2 = t + step;
    if (t2 < nt) tpp_load<U>(A, a, t2, nvec);
    tpp_store<U>(B, a, t, nvec);
    if (t2 >= nt) break;
    t = t2;
  }
}

// Round 5: the outputs split over G workgroups per tile, the G placed on ONE
// XCD back to back.  Workgroups are dispatched round-robin over the 8 XCDs
// (XCD = blockIdx mod 8), so XCD x's k-th workgroup is blockIdx x + 8k; it
// takes tile (k / G)·8 + x and outputs g, g + G, ... (g = k mod G).  Each
// tile's inputs are fetched from HBM by its first workgroup and from that
// XCD's L2 by the other G - 1; every workgroup drives nout / G output
// streams instead of nout.  HBM bytes stay 8 reads + nout writes.
template <int U, int LAUX, int SAUX, int G>
__global__ __launch_bounds__(kBlock) void tp_xsplit(PutArgs a, size_t nvec, unsigned ntile) {
  const unsigned b = blockIdx.x, x = b % 8, k = b / 8, g = k % G;
  const unsigned tile = (k / G) * 8 + x;
  if (tile >= ntile) return;
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t wbase = (size_t)tile * (kBlock * U) + (size_t)w * 64 * U;
  if (wbase >= nvec) return;
  const size_t left = nvec - wbase;
  const unsigned bytes = (unsigned)((left < 64 * U ? left : 64 * U) * 16);
  u32x4 v[U];
#pragma unroll
  for (int u = 0; u < U; u++) {
    const unsigned off = (unsigned)(u * 64 + l) * 16;
    v[u] = tree_eval_with<OP_SUM, float, u32x4, 8>(a.t, [&](int q) {
      return __builtin_bit_cast(
          u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                     tile_rsrc((const u32x4 *)a.t.in[q] + wbase, bytes), off, 0, LAUX));
    });
  }
  for (int j = (int)g; j < a.nout; j += G) {
    __amdgpu_buffer_rsrc_t r = tile_rsrc((u32x4 *)a.out[j] + wbase, bytes);
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[u]), r,
                                             (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

}  // namespace lfa

extern "C" int lfa__tune_treeput_f32(int variant, void *const *dsts, int ndst,
                                     const void *const *srcs, int nsrc, size_t cnt,
                                     void *stream) {
  using namespace lfa;
  hipStream_t s = (hipStream_t)stream;
  if (variant == 0)
    return launch_tree_put<OP_SUM, float>(dsts, ndst, srcs, nsrc, cnt, s);
  if (nsrc != 8 || ndst < 1 || ndst > kMaxPut || cnt % 4) return -LFA_EINVAL;
  PutArgs a;
  tree_leaves(a.t, srcs, nsrc);
  memset(a.out, 0, sizeof(a.out));
  a.nout = ndst;
  for (int j = 0; j < ndst; j++) a.out[j] = dsts[j];
  const size_t nvec = cnt / 4;
#define TP(U, L, S)                                                               \
  hipLaunchKernelGGL((tp_tune<8, U, L, S>), dim3(grid_for(nvec, (size_t)kBlock * U, \
                                                          0x7fffffffu)),           \
                     dim3(kBlock), 0, s, a, nvec)
#define TPP(U, L, S)                                                              \
  hipLaunchKernelGGL((tp_tune_pre<U, L, S>),                                       \
                     dim3(grid_for(nvec, (size_t)kBlock * U, 0x7fffffffu)),         \
                     dim3(kBlock), 0, s, a, nvec)
  switch (variant) {
    case 1: TP(2, 17, 17); break;   // the product body, through this harness
    case 2: TP(2, 2, 16); break;    // local policy: nt loads, sc1 stores
    case 3: TP(2, 16, 17); break;   // sc1 loads
    case 4: TP(4, 17, 17); break;
    case 5: TP(1, 17, 17); break;
    case 6: TP(2, 17, 16); break;   // sc1-only stores
    case 7: TP(4, 2, 16); break;
    case 8: TPP(2, 17, 17); break;  // every load before the tree
    case 9: TPP(1, 17, 17); break;
    case 10: TPP(2, 2, 16); break;
    case 11: TP(2, 0, 0); break;    // default policy both ways
    // system scope kept (sc0 sc1) + the nt streaming hint on loads / stores
    case 12: TP(2, 19, 17); break;
    case 13: TPP(2, 19, 17); break;
    case 14: TP(4, 19, 17); break;
    case 15: TP(2, 19, 19); break;
    case 16: TPP(2, 19, 19); break;
    case 17: TP(1, 19, 17); break;
#define TPM(M)                                                                       \
  hipLaunchKernelGGL((tp_pace<4, 19, 17, M>),                                        \
                     dim3(grid_for(nvec, (size_t)kBlock * 4, 0x7fffffffu)), dim3(kBlock), \
                     0, s, a, nvec)
    case 18: TPM(0); break;   // the product body through this harness
    case 19: TPM(1); break;
    case 20: TPM(2); break;
    case 21: TPM(3); break;
    case 22: TPM(4); break;
#undef TPM
#define TPG(K, U, ...)                                                              \
  hipLaunchKernelGGL((K<U, 19, 17, ##__VA_ARGS__>),                                  \
                     dim3(grid_for(nvec, (size_t)kBlock * U, 0x7fffffffu)), dim3(kBlock), \
                     0, s, a, nvec)
    case 23: TPG(tp_r4, 4, false); break;   // the product body, this harness
    case 24: TPG(tp_r4, 4, true); break;    // staggered output order
    case 25: TPG(tp_r4, 2, true); break;
    case 26: TPG(tp_lds, 2); break;         // LDS-DMA inputs, 64 KiB LDS / WG
    case 27: TPG(tp_lds, 1); break;
    case 28: TPG(tp_split, 4); break;       // outputs split over the waves
    case 29: TPG(tp_split, 2); break;
    case 30: TPG(tp_split, 1); break;
#undef TPG
#define TP5(U, XCD, LDS)                                                             \
  hipLaunchKernelGGL((tp_r5<U, 19, 17, XCD>),                                        \
                     dim3(grid_for(nvec, (size_t)kBlock * U, 0x7fffffffu)), dim3(kBlock), \
                     (LDS) << 10, s, a, nvec)
    case 31: TP5(4, false, 0); break;     // = the product body, this harness
    case 32: TP5(4, true, 0); break;      // XCD-contiguous tiles
    case 33: TP5(4, false, 41); break;    // <= 3 workgroups per CU (12 waves)
    case 34: TP5(4, false, 54); break;    // <= 2 workgroups per CU (8 waves)
    case 35: TP5(4, false, 81); break;    // 1 workgroup per CU (4 waves)
    case 36: TP5(4, true, 54); break;
    case 37: TP5(2, false, 54); break;
    case 38: TP5(2, true, 0); break;
    case 39: TP5(2, false, 81); break;    // U = 2, 1 workgroup per CU
    case 40: TP5(2, false, 41); break;    // U = 2, 3 workgroups per CU
    case 41: TP5(1, false, 54); break;
    case 42: TP5(1, false, 81); break;
#undef TP5
#define TPW(U, NW, LDS)                                                              \
  hipLaunchKernelGGL((tp_r5<U, 19, 17, false, NW>),                                  \
                     dim3(grid_for(nvec, (size_t)64 * NW * U, 0x7fffffffu)),           \
                     dim3(64 * NW), (LDS) << 10, s, a, nvec)
    case 43: TPW(2, 2, 41); break;        // 2-wave workgroups, 3 per CU (6 waves)
    case 44: TPW(2, 2, 54); break;        // 2-wave workgroups, 2 per CU (4 waves)
    case 45: TPW(2, 8, 81); break;        // 8-wave workgroups, 1 per CU
    case 46: TPW(4, 8, 81); break;
    case 47: TPW(2, 1, 27); break;        // 1-wave workgroups, 5 per CU
    case 48: TPW(2, 1, 20); break;        // 1-wave workgroups, 8 per CU
#undef TPW
#define TPQ(U, WGS, LDS)                                                              \
  do {                                                                               \
    int ncu = 256;                                                                   \
    hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);           \
    hipLaunchKernelGGL((tp_pipe<U>), dim3((unsigned)(ncu * (WGS))), dim3(kBlock),     \
                       (LDS) << 10, s, a, nvec);                                      \
  } while (0)
    case 59: TPQ(1, 1, 81); break;        // pipelined, 1 KiB tiles, 1 workgroup per CU
    case 60: TPQ(2, 1, 81); break;        // 2 KiB tiles
    case 61: TPQ(1, 2, 54); break;        // 2 workgroups per CU
    case 62: TPQ(2, 2, 54); break;
    case 63: TPQ(1, 3, 41); break;
#undef TPQ
#define TPX(U, L, G)                                                                 \
  do {                                                                               \
    const unsigned nt = grid_for(nvec, (size_t)kBlock * U, 0x7fffffffu);             \
    hipLaunchKernelGGL((tp_xsplit<U, L, 17, G>), dim3((nt + 7) / 8 * 8 * G), dim3(kBlock), \
                       0, s, a, nvec, nt);                                           \
  } while (0)
    case 49: TPX(4, 19, 2); break;        // outputs over 2 co-located workgroups
    case 50: TPX(4, 19, 4); break;
    case 51: TPX(2, 19, 2); break;
    case 52: TPX(4, 17, 2); break;        // loads without the nt hint (L2 reuse)
    case 53: TPX(4, 17, 4); break;
    case 54: TPX(4, 0, 2); break;         // default-policy loads
    case 55: TPX(4, 0, 4); break;
    case 56: TPX(2, 17, 4); break;
    case 57: TPX(4, 17, 8); break;
    case 58: TPX(4, 19, 1); break;        // G = 1: the remap alone
#undef TPX
    case 64: case 65: {                   // the wide form with a 1-KiB tail: 1/4, 1/8
      const size_t div = variant == 64 ? 4 : 8, hv = (size_t)kBlock * 2;
      size_t split = nvec - nvec / div;
      split -= split % hv;
      const unsigned head = (unsigned)(split / hv);
      const unsigned tail = (unsigned)((nvec - split + kBlock - 1) / kBlock);
      hipLaunchKernelGGL((tp_taper<2>), dim3(head + tail), dim3(kBlock), kPutNarrowLds, s, a,
                         nvec, split, head);
      break;
    }
    default: return -LFA_EINVAL;
  }
#undef TP
#undef TPP
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}
