// lfa_tune_b.hip — the second half of the tuning-only kernel forms
// (liblfa_tune.so; split out of lfa_tune.hip in round 6): the fetch / compare
// bodies, pure HBM streams, drained and dynamically scheduled combines,
// tapered and statically balanced grids, per-wave timestamps, and the solo
// copy's latency forms.  Not on the product path.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <errno.h>
#include <string.h>
#include <time.h>

#include "lfa_kernels.hpp"

// ---------------------------------------------------------------------------
// Compare body with its third input in registers: CSWAP's
// fetch_lds stages dst, src and cmp through LDS — 48 KiB per workgroup at
// U = 4, so 3 workgroups (12 waves, 144 KiB of loads in flight) per CU
// against the write body's 5 (160 KiB).  Here dst and src go HBM -> LDS and
// cmp into VGPRs (nt global loads issued right after), 32 KiB of LDS per
// workgroup: 5 per CU, 240 KiB in flight.  SAUX: the stores' cache policy.
namespace lfa {
template <int U, int SAUX, typename F>
__global__ __launch_bounds__(kLdsWaves * 64) void fetch_lds3r(F f, size_t nvec) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned w = wave_id(), l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (kLdsWaves * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U <= nvec) {
    u32x4 c[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      __builtin_amdgcn_global_load_lds((const void *)(f.dv + base + u * 64 + l),
                                       (lds_void *)&lds[0][w][u][0], 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void *)(f.sv + base + u * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    }
#pragma unroll
    for (int u = 0; u < U; u++) c[u] = ld<true>(f.cv + base + u * 64 + l);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t rr =
        __builtin_amdgcn_make_buffer_rsrc(f.rv + base, 0, 64 * U * 16, 0x00020000);
    const __amdgpu_buffer_rsrc_t rd =
        __builtin_amdgcn_make_buffer_rsrc(f.dv + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      const u32x4 a = lds[0][w][u][l], b = lds[1][w][u][l];
      const unsigned off = (unsigned)(u * 64 + l) * 16;
      if constexpr (SAUX == kStoreNt) {
        st<true>(f.rv + base + u * 64 + l, a);
        st<true>(f.dv + base + u * 64 + l, f.op(a, b, c[u]));
      } else {
        __builtin_amdgcn_raw_buffer_store_b128(a, rr, off, 0, SAUX);
        __builtin_amdgcn_raw_buffer_store_b128(f.op(a, b, c[u]), rd, off, 0, SAUX);
      }
    }
  } else {
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * 64 + l;
      if (i < nvec) f.vec(i);
    }
  }
}

}  // namespace lfa

// ---------------------------------------------------------------------------
// fetch / compare table bodies (tools/probe_fetch.py --tune): float SUM
// readwrite (swap = 0) or float CSWAP (swap = 1) over nvec co-aligned 16-B
// vectors.  0 = the round-1 register form (fetch_vec, 2 vectors per lane),
// 1..3 = fetch_lds U = 4 / 2 / 1 with nt stores, 4..5 = U = 4 / 2 with sc1
// write-through stores, 6 / 7 = U = 4 drained step by step (sc1 / nt),
// 12 / 13 drained nt U = 2 / 3, 14..17 drained nt U = 4 with a tapered tail.
// ---------------------------------------------------------------------------
extern "C" int lfa__tune_fetch_f32(int variant, int swap, void *dst, const void *src,
                                   const void *cmp, void *res, size_t nvec,
                                   void *stream) {
  using namespace lfa;
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto f) -> int {
    using FF = decltype(f);
    auto lds = [&](auto u, auto aux, auto drain) {
      constexpr int U = decltype(u)::value, A = decltype(aux)::value;
      constexpr bool D = decltype(drain)::value;
      hipLaunchKernelGGL((fetch_lds<U, A, FF, D>),
                         dim3(grid_for(nvec, (size_t)kLdsWaves * 64 * U, 0x7fffffffu)),
                         dim3(kLdsWaves * 64), 0, s, f, nvec);
    };
    using NO = std::false_type;
    using YES = std::true_type;
    using I4 = std::integral_constant<int, 4>;
    using I2 = std::integral_constant<int, 2>;
    using I1 = std::integral_constant<int, 1>;
    using NT = std::integral_constant<int, kStoreNt>;
    using SC1 = std::integral_constant<int, kStoreSc1>;
    switch (variant) {
      case 0:
        hipLaunchKernelGGL(fetch_vec<FF>,
                           dim3(grid_for(nvec, (size_t)kBlock * kFetchUnroll, 0x7fffffffu)),
                           dim3(kBlock), 0, s, f, nvec);
        break;
      case 1: lds(I4(), NT(), NO()); break;
      case 2: lds(I2(), NT(), NO()); break;
      case 3: lds(I1(), NT(), NO()); break;
      case 4: lds(I4(), SC1(), NO()); break;
      case 5: lds(I2(), SC1(), NO()); break;
      case 6: lds(I4(), SC1(), YES()); break;  // drained steps (combine_drain's scheme)
      case 7: lds(I4(), NT(), YES()); break;
      case 12: lds(I2(), NT(), YES()); break;   // drained nt, U = 2 / 3
      case 13: lds(std::integral_constant<int, 3>(), NT(), YES()); break;
      case 20: case 21: {
        // the write-through (sc1) body with a 1-KiB tapered tail, as the
        // combine has from 32 MiB: the last 1/8 (20) or 1/4 (21)
        const size_t div = variant == 20 ? 8 : 4;
        const size_t hv = (size_t)kLdsWaves * 64 * 4, tv = (size_t)kLdsWaves * 64;
        size_t split = nvec - nvec / div;
        split -= split % hv;
        const unsigned head = (unsigned)(split / hv);
        const unsigned tail = (unsigned)((nvec - split + tv - 1) / tv);
        hipLaunchKernelGGL((fetch_lds_taper<4, 1, kStoreSc1, FF>), dim3(head + tail),
                           dim3(kLdsWaves * 64), 0, s, f, nvec, split, head);
        break;
      }
      case 14: case 15: case 16: case 17: case 18: case 19: {
        // drained nt U = 4 with a tapered tail (fetch_lds_taper, lfa_k_fetch.hpp;
        // 17 is the product's form from kSc1Bytes since round 6): the last 1/div of the
        // vectors in UT-KiB tiles (14: UT 1, div 8; 15: UT 2, div 8;
        // 16: UT 1, div 16; 17: UT 1, div 4; 18: UT 1, div 2; 19: UT 2, div 4)
        const size_t div = variant == 16 ? 16 : variant == 17 || variant == 19 ? 4 :
                           variant == 18 ? 2 : 8;
        auto taper = [&](auto ut) {
          constexpr int UT = decltype(ut)::value;
          const size_t hv = (size_t)kLdsWaves * 64 * 4, tv = (size_t)kLdsWaves * 64 * UT;
          size_t split = nvec - nvec / div;
          split -= split % hv;
          const unsigned head = (unsigned)(split / hv);
          const unsigned tail = (unsigned)((nvec - split + tv - 1) / tv);
          hipLaunchKernelGGL((fetch_lds_taper<4, UT, kStoreNt, FF>), dim3(head + tail),
                             dim3(kLdsWaves * 64), 0, s, f, nvec, split, head);
        };
        if (variant == 15 || variant == 19) taper(I2());
        else taper(I1());
        break;
      }
      case 8: case 9: case 10: case 11:   // compare: cmp in registers
        if constexpr (FF::kIn == 3) {
          auto r3 = [&](auto u, auto aux) {
            constexpr int U = decltype(u)::value, A = decltype(aux)::value;
            hipLaunchKernelGGL((fetch_lds3r<U, A, FF>),
                               dim3(grid_for(nvec, (size_t)kLdsWaves * 64 * U, 0x7fffffffu)),
                               dim3(kLdsWaves * 64), 0, s, f, nvec);
          };
          if (variant == 8) r3(I4(), SC1());
          else if (variant == 9) r3(I4(), NT());
          else if (variant == 10) r3(I2(), SC1());
          else r3(I2(), NT());
          break;
        }
        return -LFA_EINVAL;
      default: return -LFA_EINVAL;
    }
    return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
  };
  if (swap)
    return go(SwapF<OP_CSWAP, float, true>{(char *)dst, (const char *)src,
                                           (const char *)cmp, (char *)res, (u32x4 *)dst,
                                           (const u32x4 *)src, (const u32x4 *)cmp,
                                           (u32x4 *)res});
  return go(RwF<OP_SUM, float, true>{(char *)dst, (const char *)src, (char *)res,
                                     (u32x4 *)dst, (const u32x4 *)src, (u32x4 *)res});
}

// ---------------------------------------------------------------------------
// Pure streams, to bound the combine by what HBM gives each access mix on
// this part (tools/probe_hbm.py): NIN inputs read HBM -> LDS with nt
// global_load_lds (the combine's load path, nothing stored but one vector
// per workgroup that no real data reaches), or a write-only stream of U KiB
// per wave with the combine's store policies.  Same tile shape as
// combine_lds: 4 waves per workgroup, U KiB per operand per wave.
// ---------------------------------------------------------------------------
namespace lfa_stream {
using lfa::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

template <int NIN, int U>
__global__ __launch_bounds__(256) void read_lds(const u32x4 *a, const u32x4 *b,
                                                u32x4 *sink, size_t nvec) {
  __shared__ u32x4 lds[NIN][4][U][64];
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (4 * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U > nvec) return;
#pragma unroll
  for (int k = 0; k < NIN; k++)
#pragma unroll
    for (int u = 0; u < U; u++)
      __builtin_amdgcn_global_load_lds((const void *)((k ? b : a) + base + u * 64 + l),
                                       (lds_void *)&lds[k][w][u][0], 16, 0, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const u32x4 x = lds[NIN - 1][w][U - 1][l];
  if (x.x == 0x9e3779b9u && x.y == 0x7f4a7c15u && x.z == 0x2545f491u && x.w == 1u)
    sink[blockIdx.x] = x;
}

template <int U, int SAUX>
__global__ __launch_bounds__(256) void write_only(u32x4 *dst, size_t nvec) {
  const unsigned w = threadIdx.x / 64, l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (4 * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U > nvec) return;
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
  const u32x4 v = {l, w, (unsigned)blockIdx.x, 0x3f800000u};
#pragma unroll
  for (int u = 0; u < U; u++)
    __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
}

// NIN inputs read in the shape of the product tree below 192 MiB of output
// (reduce_tree_chunk<U = 2>: each lane loads vectors t and t + 256 of every
// input with nt loads), XOR-folded so nothing is stored but one vector per
// workgroup that no real data reaches: the read side of the N -> 1 tree alone.
template <int NIN>
__global__ __launch_bounds__(256) void read_chunk(lfa::TreeArgs a, u32x4 *sink, size_t nvec) {
  const size_t base = (size_t)blockIdx.x * 512 + threadIdx.x;
  if (base + 256 >= nvec) return;
  u32x4 x = {0, 0, 0, 0};
#pragma unroll
  for (int k = 0; k < NIN; k++)
#pragma unroll
    for (int u = 0; u < 2; u++)
      x ^= __builtin_nontemporal_load((const u32x4 *)a.in[k] + base + u * 256);
  if (x.x == 0x9e3779b9u && x.y == 0x7f4a7c15u && x.z == 0x2545f491u && x.w == 1u)
    sink[blockIdx.x] = x;
}
}  // namespace lfa_stream

// The read side of the N-input tree (tools/probe_hbm.py --tree): nin in
// {2, 4, 8, 16} inputs of nvec 16-B vectors each, at the caller's addresses.
extern "C" int lfa__tune_read_n(const void *const *ins, int nin, void *sink, size_t nvec,
                                void *stream) {
  using namespace lfa_stream;
  hipStream_t s = (hipStream_t)stream;
  lfa::TreeArgs a;
  memset(&a, 0, sizeof(a));
  if (nin < 1 || nin > 16 || !nvec || nvec % 512) return -LFA_EINVAL;
  for (int k = 0; k < nin; k++) a.in[k] = ins[k];
  const dim3 grid((unsigned)(nvec / 512)), block(256);
  switch (nin) {
    case 2: hipLaunchKernelGGL((read_chunk<2>), grid, block, 0, s, a, (u32x4 *)sink, nvec); break;
    case 4: hipLaunchKernelGGL((read_chunk<4>), grid, block, 0, s, a, (u32x4 *)sink, nvec); break;
    case 8: hipLaunchKernelGGL((read_chunk<8>), grid, block, 0, s, a, (u32x4 *)sink, nvec); break;
    case 16: hipLaunchKernelGGL((read_chunk<16>), grid, block, 0, s, a, (u32x4 *)sink, nvec); break;
    default: return -LFA_EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

// kind 0: read a; 1: read a and b; 2: write dst, nt; 3: write dst, sc1.
// nvec 16-B vectors per operand, a multiple of the 16 KiB workgroup tile.
extern "C" int lfa__tune_stream(int kind, void *dst, const void *a, const void *b,
                                size_t nvec, void *stream) {
  using namespace lfa_stream;
  hipStream_t s = (hipStream_t)stream;
  const size_t tile = 4 * 64 * 4;
  if (!nvec || nvec % tile) return -LFA_EINVAL;
  const dim3 grid((unsigned)(nvec / tile)), block(256);
  switch (kind) {
    case 0:
      hipLaunchKernelGGL((read_lds<1, 4>), grid, block, 0, s, (const u32x4 *)a,
                         (const u32x4 *)a, (u32x4 *)dst, nvec);
      break;
    case 1:
      hipLaunchKernelGGL((read_lds<2, 4>), grid, block, 0, s, (const u32x4 *)a,
                         (const u32x4 *)b, (u32x4 *)dst, nvec);
      break;
    case 2:
      hipLaunchKernelGGL((write_only<4, lfa::kStoreNt>), grid, block, 0, s, (u32x4 *)dst, nvec);
      break;
    case 3:
      hipLaunchKernelGGL((write_only<4, lfa::kStoreSc1>), grid, block, 0, s, (u32x4 *)dst,
                         nvec);
      break;
    default:
      return -LFA_EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

// ---------------------------------------------------------------------------
// reduce_tree_put with a forced tile: the product picks
// U = 4 KiB per wave only up to 8 leaves of >= 4-byte lanes; this entry
// builds the other tiles for the narrow lanes so tools/probe_treeput_narrow.py
// can check them lane by lane against the oracle.  u in {1, 2, 4}.
// ---------------------------------------------------------------------------
extern "C" int lfa__tune_treeput_u(int u, int op, int dt, void *const *dsts, int ndst,
                                   const void *const *srcs, int nsrc, size_t cnt,
                                   void *stream) {
  using namespace lfa;
  hipStream_t s = (hipStream_t)stream;
  auto go = [&](auto opc, auto *tag) -> int {
    constexpr int O = decltype(opc)::value;
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    switch (u) {
      case 1: return launch_tree_put<O, T, 1>(dsts, ndst, srcs, nsrc, cnt, s);
      case 2: return launch_tree_put<O, T, 2>(dsts, ndst, srcs, nsrc, cnt, s);
      case 4: return launch_tree_put<O, T, 4>(dsts, ndst, srcs, nsrc, cnt, s);
      default: return -LFA_EINVAL;
    }
  };
  using SUM = std::integral_constant<int, OP_SUM>;
  using MIN = std::integral_constant<int, OP_MIN>;
  using PROD = std::integral_constant<int, OP_PROD>;
  using BXOR = std::integral_constant<int, OP_BXOR>;
  if (op == OP_SUM && dt == LFA_UINT8) return go(SUM(), (uint8_t *)0);
  if (op == OP_SUM && dt == LFA_INT8) return go(SUM(), (int8_t *)0);
  if (op == OP_SUM && dt == LFA_UINT16) return go(SUM(), (uint16_t *)0);
  if (op == OP_SUM && dt == LFA_INT16) return go(SUM(), (int16_t *)0);
  if (op == OP_MIN && dt == LFA_INT8) return go(MIN(), (int8_t *)0);
  if (op == OP_PROD && dt == LFA_UINT8) return go(PROD(), (uint8_t *)0);
  if (op == OP_BXOR && dt == LFA_UINT8) return go(BXOR(), (uint8_t *)0);
  if (op == OP_SUM && dt == LFA_FLOAT) return go(SUM(), (float *)0);
  return -LFA_EOPNOTSUPP;
}

// ---------------------------------------------------------------------------
// combine_lds with the wave's tile drained in steps: the
// loads of vector u of dst and src issue back to back (d0 s0 d1 s1 ...), and
// step u waits only until its own pair has landed — vmcnt counts loads,
// LDS-DMA and stores together in issue order, so before step u the
// 2(U-1-u) younger loads and the u stores already issued may stay in
// flight — then stores vector u while the later loads are still arriving.
// The product waits vmcnt(0) for the whole 2·U KiB before its first store.
// ---------------------------------------------------------------------------
namespace lfa_pipe {
using lfa::u32x4;
typedef __attribute__((address_space(3))) void lds_void;

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field is 6 bits");
  // gfx9 simm16: vmcnt[3:0] | expcnt[6:4] (7 = no wait) | lgkmcnt[11:8] (15) | vmcnt[5:4] << 14
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

template <int U, int W, int SAUX, int u>
__device__ __forceinline__ void drain_step(u32x4 (*lds)[W][U][64], unsigned w, unsigned l,
                                           u32x4 *dst, __amdgpu_buffer_rsrc_t r) {
  if constexpr (u < U) {
    wait_vm<2 * (U - 1 - u) + u>();
    const u32x4 v = lfa::apply_vec<lfa::OP_SUM, float>(lds[0][w][u][l], lds[1][w][u][l]);
    if constexpr (SAUX == lfa::kStoreNt)
      __builtin_nontemporal_store(v, dst + u * 64 + l);
    else
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
    drain_step<U, W, SAUX, u + 1>(lds, w, l, dst, r);
  }
}

template <int U, int W, int SAUX>
__global__ __launch_bounds__(W * 64) void sum_lds_drain(u32x4 *__restrict__ dst,
                                                        const u32x4 *__restrict__ src,
                                                        size_t nvec) {
  __shared__ u32x4 lds[2][W][U][64];
  const unsigned w = lfa::wave_id(), l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (W * 64 * U) + (size_t)w * 64 * U;
  if (base + 64 * U <= nvec) {
#pragma unroll
    for (int u = 0; u < U; u++) {
      __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                       (lds_void *)&lds[0][w][u][0], 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    }
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
    drain_step<U, W, SAUX, 0>(lds, w, l, dst + base, r);
  } else {
    for (int u = 0; u < U; u++) {
      const size_t i = base + (size_t)u * 64 + l;
      if (i < nvec)
        __builtin_nontemporal_store(
            lfa::apply_vec<lfa::OP_SUM, float>(__builtin_nontemporal_load(dst + i),
                                               __builtin_nontemporal_load(src + i)),
            dst + i);
    }
  }
}

// the product's store policy for the size: write-through below kSc1Bytes
template <int U, int W>
static void drain_auto(u32x4 *d, const u32x4 *v, size_t nvec, hipStream_t s) {
  const dim3 grid((unsigned)((nvec + W * 64 * U - 1) / (W * 64 * U))), block(W * 64);
  if (nvec * 16 < lfa::kSc1Bytes)
    hipLaunchKernelGGL((sum_lds_drain<U, W, lfa::kStoreSc1>), grid, block, 0, s, d, v, nvec);
  else
    hipLaunchKernelGGL((sum_lds_drain<U, W, lfa::kStoreNt>), grid, block, 0, s, d, v, nvec);
}
}  // namespace lfa_pipe

// 70.. : the drained-in-steps forms.  70 U=4 W=4 (the product's tile), 71
// U=8 W=4, 72 U=4 W=8, 73 U=2 W=8, 74 U=8 W=2, 75/76 U=4 with the store
// policy forced nt / sc1.  77: the round-2 product (combine_lds with the wave
// index divergent to the compiler, so its sc1 buffer stores ran in
// readfirstlane loops), with the product's store policy for the size.
// Dynamically scheduled combine (the per-wave stamps of
// tools/probe_ramp.py put one launch's fixed cost in its drain, with the
// XCDs finishing up to 0.9 us apart at 32 MiB per operand and 2 us at 64):
// a resident grid whose waves take 4 KiB-per-operand tiles from a global
// counter, so a slower XCD takes fewer tiles instead of finishing last.  The
// next tile's index is fetched while the current tile's loads are in flight
// (PF).  The last wave to leave resets the counters for the next launch.
// REJECTED (round 4, profiles/r04_tune_combine_dynamic.jsonl): 8-16x slower
// than the product at every size — the launch's time is the tile count times
// ~32 ns (32 MiB: 8,192 grabs 261 us, U=8's 4,096 grabs 132 us), i.e. one
// device-scope atomic on one address completes every ~32 ns however many
// waves ask.  Kept as the measured record.
namespace lfa {

template <int U, int SAUX, bool PF>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_dyn(u32x4 *__restrict__ dst,
                                                             const u32x4 *__restrict__ src,
                                                             size_t nvec, unsigned *ctr) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t ntiles = (nvec + 64 * U - 1) / (64 * U);
  auto grab = [&]() -> unsigned {
    unsigned v = 0;
    if (l == 0) v = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __builtin_amdgcn_readfirstlane(v);
  };
  unsigned t = grab();
  while (t < ntiles) {
    const size_t base = (size_t)t * 64 * U;
    unsigned next = 0;
    if (base + 64 * U <= nvec) {
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0, 2);
#pragma unroll
      for (int u = 0; u < U; u++)
        __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                         (lds_void *)&lds[1][w][u][0], 16, 0, 2);
      if constexpr (PF) next = grab();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const __amdgpu_buffer_rsrc_t r =
          __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
      for (int u = 0; u < U; u++) {
        u32x4 v = apply_vec<OP_SUM, float>(lds[0][w][u][l], lds[1][w][u][l]);
        if constexpr (SAUX == kStoreNt)
          st<true>(dst + base + u * 64 + l, v);
        else
          __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
      }
    } else {
      if constexpr (PF) next = grab();
      for (int u = 0; u < U; u++) {
        size_t i = base + (size_t)u * 64 + l;
        if (i < nvec)
          st<true>(dst + i, apply_vec<OP_SUM, float>(ld<true>(dst + i), ld<true>(src + i)));
      }
    }
    t = PF ? next : grab();
  }
  // every wave's last grab is behind it: the last one out resets both
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (l == 0) {
    const unsigned total = gridDim.x * kLdsWaves;
    if (__hip_atomic_fetch_add(ctr + 1, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1 ==
        total) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(ctr + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int U, int SAUX, bool PF>
static void launch_dyn(u32x4 *d, const u32x4 *v, size_t nvec, hipStream_t s) {
  static unsigned *ctr = nullptr;
  static int grid = 0;
  if (!ctr) {
    if (hipMalloc((void **)&ctr, 64) != hipSuccess || hipMemset(ctr, 0, 64) != hipSuccess)
      return;
  }
  int per_cu = 0, dev = 0, cus = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, combine_dyn<U, SAUX, PF>,
                                                   kLdsWaves * 64, 0) != hipSuccess ||
      hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
    return;
  grid = per_cu * cus;
  const size_t ntiles = (nvec + 64 * U - 1) / (64 * U);
  const size_t need = (ntiles + kLdsWaves - 1) / kLdsWaves;
  const unsigned g = (unsigned)(need < (size_t)grid ? need : (size_t)grid);
  hipLaunchKernelGGL((combine_dyn<U, SAUX, PF>), dim3(g), dim3(kLdsWaves * 64), 0, s, d, v,
                     nvec, ctr);
}

// Tapered tail: the per-wave stamps put a launch's fixed
// cost in its drain — the last round of waves, each living ~4.6 us, finishing
// over ~2.4 us at 32 MiB.  Here the last `tail` vectors go to workgroups
// whose waves own UT < UH KiB each, dispatched last (the highest block ids),
// so the waves still running at the end are shorter ones.
template <int UH, int UT, int SAUX>
__device__ __forceinline__ void taper_tile(u32x4 *__restrict__ dst,
                                           const u32x4 *__restrict__ src, size_t nvec,
                                           size_t base, u32x4 (*lds)[kLdsWaves][UH][64],
                                           unsigned w, unsigned l) {
  constexpr int U = UT;
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
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      u32x4 v = apply_vec<OP_SUM, float>(lds[0][w][u][l], lds[1][w][u][l]);
      if constexpr (SAUX == kStoreNt)
        st<true>(dst + base + u * 64 + l, v);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
    }
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * 64 + l;
      if (i < nvec)
        st<true>(dst + i, apply_vec<OP_SUM, float>(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
}

template <int UH, int UT, int SAUX>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_taper(u32x4 *__restrict__ dst,
                                                               const u32x4 *__restrict__ src,
                                                               size_t nvec, size_t split,
                                                               unsigned head_blocks) {
  __shared__ u32x4 lds[2][kLdsWaves][UH][64];
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const unsigned b = blockIdx.x;
  if (b < head_blocks)
    taper_tile<UH, UH, SAUX>(dst, src, split,
                             (size_t)b * (kLdsWaves * 64 * UH) + (size_t)w * 64 * UH, lds, w, l);
  else
    taper_tile<UH, UT, SAUX>(dst, src, nvec,
                             split + (size_t)(b - head_blocks) * (kLdsWaves * 64 * UT) +
                                 (size_t)w * 64 * UT,
                             lds, w, l);
}

template <int UH, int UT>
static void launch_taper(u32x4 *d, const u32x4 *v, size_t nvec, unsigned tail_div,
                         hipStream_t s) {
  const size_t hv = (size_t)kLdsWaves * 64 * UH, tv = (size_t)kLdsWaves * 64 * UT;
  size_t split = nvec - nvec / tail_div;
  split -= split % hv;
  const unsigned head = (unsigned)(split / hv);
  const unsigned tail = (unsigned)((nvec - split + tv - 1) / tv);
  if (nvec * 16 < kSc1Bytes)
    hipLaunchKernelGGL((combine_taper<UH, UT, kStoreSc1>), dim3(head + tail),
                       dim3(kLdsWaves * 64), 0, s, d, v, nvec, split, head);
  else
    hipLaunchKernelGGL((combine_taper<UH, UT, kStoreNt>), dim3(head + tail),
                       dim3(kLdsWaves * 64), 0, s, d, v, nvec, split, head);
}

// The product's drained nt body (combine_lds<..., DRAIN>) with a tapered tail
// (round 6): round 4's taper variants 85-89 ran their head tiles on the
// undrained body, so their +1 % at 256 MiB mixed two changes; the fetch
// kernel's drained head + 1-KiB tail at div 4 gained ~1 % (fetch_lds_taper).
template <int U, int SAUX>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_taper_drained(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec, size_t split,
    unsigned head_blocks) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const unsigned b = blockIdx.x;
  if (b < head_blocks) {
    const size_t base = (size_t)b * (kLdsWaves * 64 * U) + (size_t)w * 64 * U;
#pragma unroll
    for (int u = 0; u < U; u++) {
      __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                       (lds_void *)&lds[0][w][u][0], 16, 0, 2);
      __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                       (lds_void *)&lds[1][w][u][0], 16, 0, 2);
    }
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
    combine_drain<OP_SUM, float, U, SAUX, 0>(lds, w, l, dst + base, r);
    return;
  }
  taper_tile<U, 1, SAUX>(dst, src, nvec,
                         split + (size_t)(b - head_blocks) * (kLdsWaves * 64) + (size_t)w * 64,
                         lds, w, l);
}

static void launch_taper_drained(u32x4 *d, const u32x4 *v, size_t nvec, size_t div,
                                 hipStream_t s) {
  const size_t hv = (size_t)kLdsWaves * 64 * 4, tv = (size_t)kLdsWaves * 64;
  size_t split = nvec - nvec / div;
  split -= split % hv;
  const unsigned head = (unsigned)(split / hv);
  const unsigned tail = (unsigned)((nvec - split + tv - 1) / tv);
  if (nvec * 16 < kSc1Bytes)
    hipLaunchKernelGGL((combine_taper_drained<4, kStoreSc1>), dim3(head + tail),
                       dim3(kLdsWaves * 64), 0, s, d, v, nvec, split, head);
  else
    hipLaunchKernelGGL((combine_taper_drained<4, kStoreNt>), dim3(head + tail),
                       dim3(kLdsWaves * 64), 0, s, d, v, nvec, split, head);
}

// Statically balanced resident grid: exactly one round of
// workgroups (the occupancy limit per CU times the CUs, so the dispatcher
// gives every CU the same number), each wave owning a contiguous run of
// 1-KiB units (64 vectors) whose length differs by at most one unit between
// waves, walked U units per LDS-DMA step.  Every CU then carries the same
// bytes and no second, partial round of waves drains after the first — the
// fixed cost the per-wave stamps put at 2.37 us of a 32 MiB launch.  The
// last vectors past a whole unit go to the last wave's guarded path.
template <int U, int SAUX>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_static(u32x4 *__restrict__ dst,
                                                                const u32x4 *__restrict__ src,
                                                                size_t nvec) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t nw = (size_t)gridDim.x * kLdsWaves;
  const size_t gw = (size_t)blockIdx.x * kLdsWaves + w;
  const size_t units = nvec / 64;
  // balanced split: wave gw owns units [gw*units/nw, (gw+1)*units/nw)
  size_t ub = gw * units / nw;
  const size_t ue = (gw + 1) * units / nw;
  while (ub < ue) {
    const unsigned k = (unsigned)(ue - ub < (size_t)U ? ue - ub : (size_t)U);
    const size_t base = ub * 64;
#pragma unroll
    for (int u = 0; u < U; u++)
      if ((unsigned)u < k) {
        __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                         (lds_void *)&lds[0][w][u][0], 16, 0, 2);
        __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                         (lds_void *)&lds[1][w][u][0], 16, 0, 2);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++)
      if ((unsigned)u < k) {
        u32x4 v = apply_vec<OP_SUM, float>(lds[0][w][u][l], lds[1][w][u][l]);
        if constexpr (SAUX == kStoreNt)
          st<true>(dst + base + u * 64 + l, v);
        else
          __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
      }
    ub += k;
  }
  if (gw == nw - 1) {
    const size_t i = units * 64 + l;
    if (i < nvec)
      st<true>(dst + i, apply_vec<OP_SUM, float>(ld<true>(dst + i), ld<true>(src + i)));
  }
}

template <int U>
static void launch_static(u32x4 *d, const u32x4 *v, size_t nvec, int grid_mult,
                          hipStream_t s) {
  // the occupancy query once per store policy (round 6: variants 90-94 were
  // first measured with it on every launch)
  static int slots[2];
  const bool nt = nvec * 16 >= kSc1Bytes;
  if (!slots[nt]) {
    int per_cu = 0, dev = 0, cus = 0;
    if ((nt ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, combine_static<U, kStoreNt>,
                                                            kLdsWaves * 64, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, combine_static<U, kStoreSc1>,
                                                            kLdsWaves * 64, 0)) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return;
    slots[nt] = per_cu * cus;
  }
  size_t g = (size_t)slots[nt] * grid_mult;
  const size_t waves_needed = (nvec / 64 + 1 + kLdsWaves - 1) / kLdsWaves;
  if (g > waves_needed) g = waves_needed ? waves_needed : 1;
  if (nt)
    hipLaunchKernelGGL((combine_static<U, kStoreNt>), dim3((unsigned)g), dim3(kLdsWaves * 64), 0,
                       s, d, v, nvec);
  else
    hipLaunchKernelGGL((combine_static<U, kStoreSc1>), dim3((unsigned)g), dim3(kLdsWaves * 64), 0,
                       s, d, v, nvec);
}

// The static grid above, software-pipelined (round 6): each wave's steps of U
// units are double-buffered in LDS, and step j+1's LDS-DMA loads are issued
// before step j is combined and stored, so a wave always has a step's loads
// in flight — variants 90-94 waited vmcnt(0) between every step's loads and
// its stores, and lost 3-7 % to those serial phases.  LDS per wave equals the
// product's at U = 2 (2 buffers x 2 operands x 2 KiB = 8 KiB), so the same 5
// workgroups fit per CU.  vmcnt counts loads and stores together in issue
// order: with stores(j-1) and loads(j+1) behind loads(j), loads(j) have
// landed at vmcnt(3U) (2U at the first step, U at the last).  Buffer reuse:
// loads(j+1) overwrite the buffer step j-1 read, and are issued after step
// j-1's stores, which consumed those reads.  A wave's units past its last
// whole step take the guarded register path after the pipeline.
template <int U, int SAUX>
__device__ __forceinline__ void pipe_issue(const u32x4 *__restrict__ dst,
                                           const u32x4 *__restrict__ src, size_t base,
                                           u32x4 (*buf)[kLdsWaves][U][64], unsigned w,
                                           unsigned l) {
#pragma unroll
  for (int u = 0; u < U; u++) {
    __builtin_amdgcn_global_load_lds((const void *)(dst + base + u * 64 + l),
                                     (lds_void *)&buf[0][w][u][0], 16, 0, 2);
    __builtin_amdgcn_global_load_lds((const void *)(src + base + u * 64 + l),
                                     (lds_void *)&buf[1][w][u][0], 16, 0, 2);
  }
}

template <int U, int SAUX>
__device__ __forceinline__ void pipe_store(u32x4 *__restrict__ dst, size_t base,
                                           u32x4 (*buf)[kLdsWaves][U][64], unsigned w,
                                           unsigned l) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
  for (int u = 0; u < U; u++) {
    u32x4 v = apply_vec<OP_SUM, float>(buf[0][w][u][l], buf[1][w][u][l]);
    if constexpr (SAUX == kStoreNt)
      st<true>(dst + base + u * 64 + l, v);
    else
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
  }
}

template <int U, int SAUX>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_static_pipe(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec) {
  __shared__ u32x4 lds[2][2][kLdsWaves][U][64];  // [buffer][dst, src][wave][u][lane]
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t nw = (size_t)gridDim.x * kLdsWaves;
  const size_t gw = (size_t)blockIdx.x * kLdsWaves + w;
  const size_t units = nvec / 64;
  const size_t ub = gw * units / nw, ue = (gw + 1) * units / nw;
  const size_t nsteps = (ue - ub) / U;
  if (nsteps) {
    pipe_issue<U, SAUX>(dst, src, ub * 64, lds[0], w, l);
    if (nsteps > 1) {
      pipe_issue<U, SAUX>(dst, src, (ub + U) * 64, lds[1], w, l);
      wait_vmcnt<2 * U>();
    } else {
      wait_vmcnt<0>();
    }
    pipe_store<U, SAUX>(dst, ub * 64, lds[0], w, l);
    for (size_t j = 1; j < nsteps; j++) {
      const size_t base = (ub + j * U) * 64;
      if (j + 1 < nsteps) {
        pipe_issue<U, SAUX>(dst, src, base + U * 64, lds[(j + 1) & 1], w, l);
        wait_vmcnt<3 * U>();
      } else {
        wait_vmcnt<U>();
      }
      pipe_store<U, SAUX>(dst, base, lds[j & 1], w, l);
    }
  }
  // units past the last whole step, then the vectors past the last unit
  for (size_t i = (ub + nsteps * U) * 64 + l; i < ue * 64; i += 64)
    st<true>(dst + i, apply_vec<OP_SUM, float>(ld<true>(dst + i), ld<true>(src + i)));
  if (gw == nw - 1) {
    const size_t i = units * 64 + l;
    if (i < nvec)
      st<true>(dst + i, apply_vec<OP_SUM, float>(ld<true>(dst + i), ld<true>(src + i)));
  }
}

template <int U>
static void launch_static_pipe(u32x4 *d, const u32x4 *v, size_t nvec, int grid_mult,
                               hipStream_t s) {
  // one occupancy query per form and store policy (not one per launch: the
  // host must stay ahead of a 16 us kernel)
  static int slots[2];
  const bool nt = nvec * 16 >= kSc1Bytes;
  if (!slots[nt]) {
    int per_cu = 0, dev = 0, cus = 0;
    if ((nt ? hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &per_cu, combine_static_pipe<U, kStoreNt>, kLdsWaves * 64, 0)
            : hipOccupancyMaxActiveBlocksPerMultiprocessor(
                  &per_cu, combine_static_pipe<U, kStoreSc1>, kLdsWaves * 64, 0)) != hipSuccess ||
        hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return;
    slots[nt] = per_cu * cus;
  }
  size_t g = (size_t)slots[nt] * grid_mult;
  const size_t waves_needed = (nvec / 64 + 1 + kLdsWaves - 1) / kLdsWaves;
  if (g > waves_needed) g = waves_needed ? waves_needed : 1;
  if (nt)
    hipLaunchKernelGGL((combine_static_pipe<U, kStoreNt>), dim3((unsigned)g),
                       dim3(kLdsWaves * 64), 0, s, d, v, nvec);
  else
    hipLaunchKernelGGL((combine_static_pipe<U, kStoreSc1>), dim3((unsigned)g),
                       dim3(kLdsWaves * 64), 0, s, d, v, nvec);
}

}  // namespace lfa

extern "C" int lfa__tune3_sum_f32(int variant, void *dst, const void *src, size_t nvec,
                                  void *stream) {
  using namespace lfa_pipe;
  hipStream_t s = (hipStream_t)stream;
  u32x4 *d = (u32x4 *)dst;
  const u32x4 *v = (const u32x4 *)src;
  const dim3 g4((unsigned)((nvec + 1023) / 1024)), b4(256);
  switch (variant) {
    case 70: drain_auto<4, 4>(d, v, nvec, s); break;
    case 71: drain_auto<8, 4>(d, v, nvec, s); break;
    case 72: drain_auto<4, 8>(d, v, nvec, s); break;
    case 73: drain_auto<2, 8>(d, v, nvec, s); break;
    case 74: drain_auto<8, 2>(d, v, nvec, s); break;
    case 75:
      hipLaunchKernelGGL((sum_lds_drain<4, 4, lfa::kStoreNt>), g4, b4, 0, s, d, v, nvec);
      break;
    case 76:
      hipLaunchKernelGGL((sum_lds_drain<4, 4, lfa::kStoreSc1>), g4, b4, 0, s, d, v, nvec);
      break;
    case 80: lfa::launch_dyn<4, lfa::kStoreSc1, true>(d, v, nvec, s); break;
    case 81:
      if (nvec * 16 < lfa::kSc1Bytes) lfa::launch_dyn<4, lfa::kStoreSc1, true>(d, v, nvec, s);
      else lfa::launch_dyn<4, lfa::kStoreNt, true>(d, v, nvec, s);
      break;
    case 82: lfa::launch_dyn<2, lfa::kStoreSc1, true>(d, v, nvec, s); break;
    case 83: lfa::launch_dyn<4, lfa::kStoreSc1, false>(d, v, nvec, s); break;
    case 84: lfa::launch_dyn<8, lfa::kStoreSc1, true>(d, v, nvec, s); break;
    // tapered tail: head tiles 4 KiB per wave, the last 1/div of the data in
    // UT-KiB tiles
    // statically balanced resident grid: U-KiB steps, one (or two) rounds
    case 90: lfa::launch_static<4>(d, v, nvec, 1, s); break;
    case 91: lfa::launch_static<2>(d, v, nvec, 1, s); break;
    case 92: lfa::launch_static<8>(d, v, nvec, 1, s); break;
    case 93: lfa::launch_static<4>(d, v, nvec, 2, s); break;
    case 94: lfa::launch_static<1>(d, v, nvec, 1, s); break;
    // the same, software-pipelined (round 6): U = 2 / 4 / 1 KiB steps
    case 95: lfa::launch_static_pipe<2>(d, v, nvec, 1, s); break;
    case 96: lfa::launch_static_pipe<4>(d, v, nvec, 1, s); break;
    case 97: lfa::launch_static_pipe<1>(d, v, nvec, 1, s); break;
    // the drained body with a 1-KiB tapered tail: the last 1/4 (98), 1/8 (99)
    case 98: lfa::launch_taper_drained(d, v, nvec, 4, s); break;
    case 99: lfa::launch_taper_drained(d, v, nvec, 8, s); break;
    case 85: lfa::launch_taper<4, 2>(d, v, nvec, 8, s); break;
    case 86: lfa::launch_taper<4, 2>(d, v, nvec, 4, s); break;
    case 87: lfa::launch_taper<4, 1>(d, v, nvec, 8, s); break;
    case 88: lfa::launch_taper<4, 1>(d, v, nvec, 16, s); break;
    case 89: lfa::launch_taper<4, 2>(d, v, nvec, 16, s); break;
    case 78:  // the round-3 product: uniform 4-KiB tiles at every size
      if (nvec * 16 < lfa::kSc1Bytes)
        hipLaunchKernelGGL((lfa::combine_lds<lfa::OP_SUM, float, 4, lfa::kStoreSc1>), g4, b4, 0,
                           s, d, v, nvec);
      else
        hipLaunchKernelGGL((lfa::combine_lds<lfa::OP_SUM, float, 4, lfa::kStoreNt>), g4, b4, 0,
                           s, d, v, nvec);
      break;
    case 77:
      if (nvec * 16 < lfa::kSc1Bytes)
        hipLaunchKernelGGL((lfa::combine_lds<lfa::OP_SUM, float, 4, lfa::kStoreSc1, false>), g4,
                           b4, 0, s, d, v, nvec);
      else
        hipLaunchKernelGGL((lfa::combine_lds<lfa::OP_SUM, float, 4, lfa::kStoreNt, false>), g4,
                           b4, 0, s, d, v, nvec);
      break;
    default: return -LFA_EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

// ---------------------------------------------------------------------------
// Where a launch's fixed cost goes: the product combine body
// (float SUM, LDS-DMA staged, 4 KiB per operand per wave) with a timestamp
// pair per WAVE — s_memrealtime (the constant 100 MHz clock) when the wave
// starts and after its stores are acknowledged (vmcnt(0)) — and the XCC the
// wave ran on.  stamps[4·(4·b + w) ...] = {start, end, xcc, 0}.  Diagnostic
// build only: the stamps go to their own buffer, no output depends on them.
// ---------------------------------------------------------------------------
namespace lfa {

template <int U, int SAUX>
__global__ __launch_bounds__(kLdsWaves * 64) void combine_stamped(
    u32x4 *__restrict__ dst, const u32x4 *__restrict__ src, size_t nvec,
    unsigned long long *stamps) {
  __shared__ u32x4 lds[2][kLdsWaves][U][64];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  const unsigned w = wave_id<true>(), l = threadIdx.x % 64;
  const size_t base = (size_t)blockIdx.x * (kLdsWaves * 64 * U) + (size_t)w * 64 * U;
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
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + base, 0, 64 * U * 16, 0x00020000);
#pragma unroll
    for (int u = 0; u < U; u++) {
      u32x4 v = apply_vec<OP_SUM, float>(lds[0][w][u][l], lds[1][w][u][l]);
      if constexpr (SAUX == kStoreNt)
        st<true>(dst + base + u * 64 + l, v);
      else
        __builtin_amdgcn_raw_buffer_store_b128(v, r, (unsigned)(u * 64 + l) * 16, 0, SAUX);
    }
  } else {
    for (int u = 0; u < U; u++) {
      size_t i = base + (size_t)u * 64 + l;
      if (i < nvec)
        st<true>(dst + i, apply_vec<OP_SUM, float>(ld<true>(dst + i), ld<true>(src + i)));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  if (l == 0) {
    // HW_REG_XCC_ID (gfx940+): bits [3:0] the XCC this wave runs on
    const unsigned xcc = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (3 << 11)) & 0xf;
    unsigned long long *s = stamps + 4 * ((size_t)blockIdx.x * kLdsWaves + w);
    s[0] = t0;
    s[1] = t1;
    s[2] = xcc;
    s[3] = 0;
  }
}

}  // namespace lfa

extern "C" int lfa__tune_combine_stamped(void *dst, const void *src, size_t nvec,
                                         int sc1, void *stamps, void *stream) {
  using namespace lfa;
  const dim3 grid(grid_for(nvec, (size_t)kLdsWaves * 64 * kUnroll, 0x7fffffffu));
  if (sc1)
    hipLaunchKernelGGL((combine_stamped<kUnroll, kStoreSc1>), grid, dim3(kLdsWaves * 64), 0,
                       (hipStream_t)stream, (u32x4 *)dst, (const u32x4 *)src, nvec,
                       (unsigned long long *)stamps);
  else
    hipLaunchKernelGGL((combine_stamped<kUnroll, kStoreNt>), grid, dim3(kLdsWaves * 64), 0,
                       (hipStream_t)stream, (u32x4 *)dst, (const u32x4 *)src, nvec,
                       (unsigned long long *)stamps);
  return hipGetLastError() == hipSuccess ? (int)grid.x : -LFA_EIO;
}

// ---------------------------------------------------------------------------
// Where a small operation's time goes after the launch: a
// one-workgroup copy of `bytes` (<= 4 KiB) that ends in a host-mapped
// completion word, timed from the host (launch call -> word seen) in a loop.
//   mode 0  the product: the one-shot launcher with n = 1 (float FI_SUM over
//           one rank: a copy) and the word
//   mode 1  this file's copy of that body: stores, waitcnt, system release,
//           agent counter, system release, word
//   mode 2  the same without either system release (diagnostic only: the
//           data are not ordered before the word)
//   mode 3  write-through (sc0 sc1) data stores, then the releases
//   mode 4  no data: the counter and the word only, with the releases
//   mode 5  no data, no releases: the word alone
//   mode 6  lfa_solo_copy_async (liblfa.so): the product's world-1 path
// Returns the mean microseconds per operation in *us.
// ---------------------------------------------------------------------------
namespace lfa {

template <int MODE>
__global__ __launch_bounds__(kBlock) void solo_diag(const u32x4 *src, u32x4 *dst,
                                                    unsigned nvec, uint32_t *ctr,
                                                    uint64_t *word, uint64_t val) {
  const unsigned t = threadIdx.x;
  if constexpr (MODE <= 3) {
    if (t < nvec) {
      u32x4 v = src[t];
      if constexpr (MODE == 3)
        __builtin_amdgcn_raw_buffer_store_b128(
            v, __builtin_amdgcn_make_buffer_rsrc(dst, 0, (int)(nvec * 16), 0x00020000), t * 16,
            0, kSysAux);
      else
        dst[t] = v;
    }
  }
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t == 0) {
    if constexpr (MODE != 2 && MODE != 5) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const uint32_t seen =
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (seen + 1 == gridDim.x) {
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if constexpr (MODE != 2 && MODE != 5) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace lfa

extern "C" int lfa__tune_solo_latency(int mode, void *dst, const void *src, size_t bytes,
                                      int reps, double *us) {
  using namespace lfa;
  hipStream_t s;
  uint32_t *ctr = nullptr;
  uint64_t *word = nullptr;
  if (bytes > 4096 || bytes % 16 || reps <= 0 || !us) return -LFA_EINVAL;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -LFA_EIO;
  if (hipMalloc((void **)&ctr, 4) != hipSuccess ||
      hipHostMalloc((void **)&word, 8, hipHostMallocCoherent) != hipSuccess ||
      hipMemset(ctr, 0, 4) != hipSuccess) {
    hipStreamDestroy(s);
    return -LFA_EIO;
  }
  *(volatile uint64_t *)word = 0;
  struct lfa_direct *direct = nullptr;
  const unsigned nvec = (unsigned)(bytes / 16);
  struct lfa_oneshot a;
  memset(&a, 0, sizeof(a));
  a.send = src;
  a.result = dst;
  a.count = bytes / 4;
  a.mode = LFA_ONESHOT_ALL;
  a.n = 1;
  a.done_ctr = ctr;
  a.done_word = word;
  int rc = 0;
  double t0 = 0;
  for (int i = -50; i < reps && !rc; i++) {  // 50 untimed: code load, clocks
    if (i == 0) {
      struct timespec ts;
      clock_gettime(CLOCK_MONOTONIC, &ts);
      t0 = ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
    }
    const uint64_t val = (uint64_t)(i + 51);
    switch (mode) {
      case 0:
        a.done_val = val;
        rc = launch_oneshot<OP_SUM, float>(a, s);
        break;
#define SD(M) \
  hipLaunchKernelGGL((solo_diag<M>), dim3(1), dim3(kBlock), 0, s, (const u32x4 *)src, \
                     (u32x4 *)dst, nvec, ctr, word, val)
      case 1: SD(1); break;
      case 2: SD(2); break;
      case 3: SD(3); break;
      case 4: SD(4); break;
      case 5: SD(5); break;
#undef SD
      case 6:
        rc = lfa_solo_copy_async(dst, src, bytes, ctr, word, val, s);
        break;
      case 7:  // the same kernel through liblfa's own HSA queue (lfa_direct.cpp)
        if (!direct) {
          int dev = 0;
          hipGetDevice(&dev);
          direct = lfa_direct_open(dev);
          if (!direct) {
            rc = -LFA_ENOSYS;
            break;
          }
        }
        rc = lfa_direct_solo_copy(direct, dst, src, bytes, ctr, word, val);
        break;
      default: rc = -LFA_EINVAL;
    }
    // bounded: a word that never comes is an error, not a hang
    struct timespec w0, w1;
    clock_gettime(CLOCK_MONOTONIC, &w0);
    while (!rc && *(volatile uint64_t *)word < val) {
      clock_gettime(CLOCK_MONOTONIC, &w1);
      if (w1.tv_sec - w0.tv_sec > 2) rc = -ETIMEDOUT;
    }
  }
  if (direct) lfa_direct_close(direct);
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  *us = (ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3 - t0) / reps;
  hipStreamSynchronize(s);
  hipFree(ctr);
  hipHostFree(word);
  hipStreamDestroy(s);
  return rc;
}

// ---------------------------------------------------------------------------
// Round 5: the world-1 solo copy above one workgroup (4 KiB .. 1 MiB), launch
// -> completion word, by how each workgroup orders its stores before the
// counter.  The product (lfa_signal.hip solo_copy) gives every workgroup a
// system-scope release (an L2 write-back) and an agent-scope acq_rel counter
// add (another write-back and an invalidate), so 64 workgroups at 256 KiB
// queue 64 of each in the XCDs' L2s.
//   mode 0  lfa_solo_copy_async (the product, HIP launch)
//   mode 1  lfa_direct_solo_copy (the product, liblfa's HSA queue)
//   mode 2  solo_multi<0>: this file's copy of the product body (HIP launch)
//   mode 3  solo_multi<1>: a workgroup whose stores were all write-through
//           (sc0 sc1, acknowledged by its s_waitcnt) adds to the counter
//           relaxed with no fence; the last one acquires, releases at system
//           scope and stores the word (byte-wise tails keep the release)
//   mode 4  solo_multi<2>: as 3, the last one without the acquire
//   mode 5..7  solo_tile<2 / 4 / 8>: 8 / 16 / 32 KiB per workgroup, mode 3's
//           counter (16-B aligned operands only)
// ---------------------------------------------------------------------------
namespace lfa {

template <int MODE>
__global__ __launch_bounds__(256) void solo_multi(char *dst, const char *src, size_t bytes,
                                                  uint32_t *ctr, uint64_t *word, uint64_t val) {
  const unsigned t = threadIdx.x;
  const size_t lo = (size_t)blockIdx.x * 4096;
  const size_t hi = lo + 4096 < bytes ? lo + 4096 : bytes;
  const bool vec = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const size_t vhi = vec ? lo + ((hi - lo) & ~(size_t)15) : lo;
  if (lo + (size_t)t * 16 < vhi) {
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + lo, 0, 4096, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)(src + lo + (size_t)t * 16), r,
                                           t * 16, 0, kSysAux);
  }
  for (size_t o = vhi + t; o < hi; o += 256) dst[o] = src[o];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t != 0) return;
  if (gridDim.x == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  uint32_t seen;
  if constexpr (MODE == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    seen = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
  } else {
    if (vhi != hi) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");  // plain-store tail
    seen = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (seen + 1 == gridDim.x) {
    if constexpr (MODE == 1) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Larger workgroup tiles: K·4 KiB per workgroup, every load of the tile
// issued before its stores (K 16-B loads in flight per lane), then mode 3's
// counter.  Fewer workgroups, fewer counter adds, one deeper round trip.
template <int K>
__global__ __launch_bounds__(256) void solo_tile(char *dst, const char *src, size_t bytes,
                                                 uint32_t *ctr, uint64_t *word, uint64_t val) {
  const unsigned t = threadIdx.x;
  const size_t lo = (size_t)blockIdx.x * (4096 * K);
  const size_t hi = lo + 4096 * K < bytes ? lo + 4096 * K : bytes;
  const size_t vhi = lo + ((hi - lo) & ~(size_t)15);   // both pointers 16-B aligned here
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char *>(src) + lo, 0, (int)(vhi - lo), 0x00020000);
  const __amdgpu_buffer_rsrc_t rd =
      __builtin_amdgcn_make_buffer_rsrc(dst + lo, 0, (int)(vhi - lo), 0x00020000);
  u32x4 v[K];
#pragma unroll
  for (int k = 0; k < K; k++)
    v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                                         rs, (unsigned)(k * 4096 + t * 16), 0, 0));
#pragma unroll
  for (int k = 0; k < K; k++)
    __builtin_amdgcn_raw_buffer_store_b128(v[k], rd, (unsigned)(k * 4096 + t * 16), 0, kSysAux);
  for (size_t o = vhi + t; o < hi; o += 256) dst[o] = src[o];
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t != 0) return;
  if (gridDim.x == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return;
  }
  if (vhi != hi) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  const uint32_t seen = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (seen + 1 == gridDim.x) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

}  // namespace lfa

extern "C" int lfa__tune_solo_multi(int mode, void *dst, const void *src, size_t bytes,
                                    int reps, double *us) {
  using namespace lfa;
  hipStream_t s;
  uint32_t *ctr = nullptr;
  uint64_t *word = nullptr;
  if (!bytes || bytes > ((size_t)1 << 20) || reps <= 0 || !us || mode < 0 || mode > 7)
    return -LFA_EINVAL;
  if (mode >= 5 && (((uintptr_t)dst | (uintptr_t)src) & 15)) return -LFA_EINVAL;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -LFA_EIO;
  if (hipMalloc((void **)&ctr, 4) != hipSuccess ||
      hipHostMalloc((void **)&word, 8, hipHostMallocCoherent) != hipSuccess ||
      hipMemset(ctr, 0, 4) != hipSuccess) {
    hipStreamDestroy(s);
    return -LFA_EIO;
  }
  *(volatile uint64_t *)word = 0;
  struct lfa_direct *direct = nullptr;
  if (mode == 1) {
    int dev = 0;
    hipGetDevice(&dev);
    direct = lfa_direct_open(dev);
    if (!direct) {
      hipFree(ctr);
      hipHostFree(word);
      hipStreamDestroy(s);
      return -LFA_ENOSYS;
    }
  }
  const unsigned grid = (unsigned)((bytes + 4095) / 4096);
  int rc = 0;
  double t0 = 0;
  for (int i = -50; i < reps && !rc; i++) {
    if (i == 0) {
      struct timespec ts;
      clock_gettime(CLOCK_MONOTONIC, &ts);
      t0 = ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
    }
    const uint64_t val = (uint64_t)(i + 51);
    switch (mode) {
      case 0: rc = lfa_solo_copy_async(dst, src, bytes, ctr, word, val, s); break;
      case 1: rc = lfa_direct_solo_copy(direct, dst, src, bytes, ctr, word, val); break;
#define SM(M)                                                                          \
  hipLaunchKernelGGL((solo_multi<M>), dim3(grid), dim3(256), 0, s, (char *)dst,         \
                     (const char *)src, bytes, ctr, word, val);                          \
  rc = hipGetLastError() == hipSuccess ? 0 : -LFA_EIO
      case 2: SM(0); break;
      case 3: SM(1); break;
      case 4: SM(2); break;
#undef SM
#define ST(K)                                                                          \
  hipLaunchKernelGGL((solo_tile<K>), dim3((unsigned)((bytes + 4096 * K - 1) / (4096 * K))), \
                     dim3(256), 0, s, (char *)dst, (const char *)src, bytes, ctr, word, val); \
  rc = hipGetLastError() == hipSuccess ? 0 : -LFA_EIO
      case 5: ST(2); break;
      case 6: ST(4); break;
      case 7: ST(8); break;
#undef ST
    }
    struct timespec w0, w1;
    clock_gettime(CLOCK_MONOTONIC, &w0);
    while (!rc && *(volatile uint64_t *)word < val) {
      clock_gettime(CLOCK_MONOTONIC, &w1);
      if (w1.tv_sec - w0.tv_sec > 2) rc = -ETIMEDOUT;
    }
  }
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  *us = (ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3 - t0) / reps;
  hipStreamSynchronize(s);
  if (direct) lfa_direct_close(direct);
  hipFree(ctr);
  hipHostFree(word);
  hipStreamDestroy(s);
  return rc;
}
