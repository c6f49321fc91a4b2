// lfa_k_launch.hpp — the host-side launchers of every product kernel.
// Part of lfa_kernels.hpp (split in round 6); included by it, in order, after
// the shared helpers and the combine kernels.  Not included on its own.
#pragma once

namespace lfa {

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
    // From kSc1Bytes the last quarter of the vectors goes to 1-KiB tiles
    // (fetch_lds_taper, tune variant 17): 256 MiB float SUM readwrite
    // 167.0-167.3 -> 165.0-166.5 us, float CSWAP 215.6-215.9 -> 213.0-214.9 us,
    // three interleaved runs of 20 rounds on one box; UT 1 / 2 with the last
    // 1/16 .. 1/2 tapered measured within that (profiles/r06_tune_fetch_taper_*.jsonl).
    constexpr int U = 4;
    constexpr bool D = FF::kIn == 2;
    const dim3 grid(grid_for(nvec, (size_t)kLdsWaves * 64 * U, 0x7fffffffu));
    const bool nt = nvec * 16 >= kSc1Bytes;
    if (nt) {
      constexpr size_t hv = (size_t)kLdsWaves * 64 * U, tv = (size_t)kLdsWaves * 64;
      size_t split = nvec - nvec / 4;
      split -= split % hv;
      const unsigned nhead = (unsigned)(split / hv);
      const unsigned ntail = (unsigned)((nvec - split + tv - 1) / tv);
      hipLaunchKernelGGL((fetch_lds_taper<U, 1, kStoreNt, FF>), dim3(nhead + ntail),
                         dim3(kLdsWaves * 64), 0, s, f, nvec, split, nhead);
    }
    // Below kSc1Bytes the two-input readwrite takes the same tail from
    // kFetchTaperBytes, on its write-through drained body (tune variant 21 vs
    // 6: 64 MiB 39.1 / 38.6 -> 38.5 / 38.4 us, 128 MiB 83.0 -> 81.7 us); the
    // compare body keeps its undrained form there, which the tapered one
    // trailed at 64 MiB (48.5 vs 49.5-50.1 us) and tied at 128
    // (profiles/r06_tune_fetch_taper_sc1.jsonl).
    constexpr size_t kFetchTaperBytes = (size_t)64 << 20;
    if (nvec && !nt && FF::kIn == 2 && nvec * 16 >= kFetchTaperBytes) {
      constexpr size_t hv = (size_t)kLdsWaves * 64 * U, tv = (size_t)kLdsWaves * 64;
      size_t split = nvec - nvec / 4;
      split -= split % hv;
      const unsigned nhead = (unsigned)(split / hv);
      const unsigned ntail = (unsigned)((nvec - split + tv - 1) / tv);
      hipLaunchKernelGGL((fetch_lds_taper<U, 1, kStoreSc1, FF>), dim3(nhead + ntail),
                         dim3(kLdsWaves * 64), 0, s, f, nvec, split, nhead);
    } else if (nvec && !nt)
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
