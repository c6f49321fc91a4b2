// lfa_combine.hip — MI355X (gfx950) combine kernels + their C ABI (liblfa.so).
//
// What runs on the GPU for libfabric's L4 combine layer
// (ofi_atomic_write_handlers, prov/util/src/util_atomic.c:907-922, called by
// prov/coll's REDUCE items, prov/coll/src/coll_coll.c:758-768):
//
//   combine_lds    dst[i] = dst[i] OP src[i] over 16-byte vectors (the product
//                  body).  A pure HBM stream (2 reads + 1 write per element,
//                  ~0.1 op/B): no MFMA — the roofline is HBM.  Each
//                  wave DMAs 4 KiB of each operand into LDS (global_load_lds,
//                  nt), reads it back with ds_read_b128, applies OP and stores
//                  nt; every wave-instruction moves 1 KiB of consecutive bytes.
//   combine_vec    the register-staged form of the same (tuning reference,
//                  built only into liblfa_tune.so).
//   combine_elem   the same op for misaligned heads/tails and for buffers that
//                  are not co-aligned mod 16 (one element per lane, coalesced).
//   reduce_tree_*  N inputs → 1 output in ONE pass, in prov/coll's
//                  recursive-doubling association order (coll_coll.c:349-449):
//                  replaces log2(N) pairwise REDUCE+COPY items, traffic
//                  (N+1)·S instead of ~3·log2(N)·S.
//   reduce_tree_put the same tree with its result written to several
//                  outputs, every access system scope: the LFA_ALGO_P2P kernel
//                  that reads peers' HBM and pushes into it over xGMI.
//   fetch_vec/elem the fetch (readwrite) and compare-swap tables
//                  (util_atomic.c:924-980): res = old dst, then the update.
//
// Kernels and launchers: lfa_kernels.hpp.  Semantics: lfa_ops.hpp.  Build: hipcc --offload-arch=gfx950 -O3
// -ffp-contract=off -DLFA_OP=<op>, once per enum fi_op row (0..18; see
// libfabric_amd/build.py).
#include "lfa_kernels.hpp"

namespace lfa {

// ---------------------------------------------------------------------------
// per-op entry points
// ---------------------------------------------------------------------------
// This file is compiled once per write op (-DLFA_OP=<enum fi_op value>) so the
// ~100 (op, datatype) kernel families build in parallel; each object exports
//   lfa__write_op<N>(dt, dst, src, cnt, stream)
//   lfa__tree_op<N>(dt, dst, srcs, nsrc, cnt, stream)
// which lfa_capi.cpp dispatches to.  Return 0 or a negative LFA_E* code.
// Ops whose result bits do not depend on an integer's signedness: wrapping
// SUM / PROD (the low bits of a two's-complement sum or product), the
// bitwise and logical ops, READ / WRITE, CSWAP (bitwise compare), CSWAP_NE
// (integer != is sign-blind) and MSWAP.  A signed integer type runs its
// unsigned twin's kernels for them — the same bits, one kernel family
// instead of two (liblfa.so size).  MIN / MAX and the
// ordered compares keep their own.
template <int OP>
constexpr bool sign_blind() {
  return !(OP == OP_MIN || OP == OP_MAX || OP == OP_CSWAP_LE || OP == OP_CSWAP_LT ||
           OP == OP_CSWAP_GE || OP == OP_CSWAP_GT);
}

// the kernel type of a signed integer under OP: its unsigned twin when OP
// is sign-blind (if constexpr: the signed family is never instantiated)
template <int OP, typename S, typename U, typename F>
static int signed_case(F &&f) {
  if constexpr (sign_blind<OP>()) return f((U *)0);
  else return f((S *)0);
}

template <int OP, typename F>
static int by_type(int dt, F &&f) {
  switch (dt) {
    case LFA_INT8: return signed_case<OP, int8_t, uint8_t>(f);
    case LFA_UINT8: return f((uint8_t *)0);
    case LFA_INT16: return signed_case<OP, int16_t, uint16_t>(f);
    case LFA_UINT16: return f((uint16_t *)0);
    case LFA_INT32: return signed_case<OP, int32_t, uint32_t>(f);
    case LFA_UINT32: return f((uint32_t *)0);
    case LFA_INT64: return signed_case<OP, int64_t, uint64_t>(f);
    case LFA_UINT64: return f((uint64_t *)0);
    case LFA_FLOAT: return f((float *)0);
    case LFA_DOUBLE: return f((double *)0);
    case LFA_FLOAT_COMPLEX: return f((cf32 *)0);
    case LFA_INT128: return signed_case<OP, i128, u128>(f);
    case LFA_UINT128: return f((u128 *)0);
    default: return -LFA_EOPNOTSUPP;
  }
}

}  // namespace lfa

#ifndef LFA_OP
#error "compile with -DLFA_OP=<op>"
#endif

#define LFA_CAT2(a, b) a##b
#define LFA_CAT(a, b) LFA_CAT2(a, b)

#if LFA_OP <= 11
#if LFA_OP != 10
extern "C" int LFA_CAT(lfa__write_op, LFA_OP)(int dt, void *dst,
                                              const void *src, size_t cnt,
                                              void *stream) {
  // dt | LFA_WRITE_MAPPED: operands on their host mappings (lfa_capi.cpp)
  const bool mapped = (dt & LFA_WRITE_MAPPED) != 0;
  return lfa::by_type<LFA_OP>(dt & ~LFA_WRITE_MAPPED, [&](auto *tag) {
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    return lfa::launch_write<LFA_OP, T>(dst, src, cnt, (hipStream_t)stream, mapped);
  });
}
#endif

#if LFA_OP <= 9
extern "C" int LFA_CAT(lfa__tree_op, LFA_OP)(int dt, void *dst,
                                             const void *const *srcs, int nsrc,
                                             size_t cnt, void *stream) {
  return lfa::by_type<LFA_OP>(dt, [&](auto *tag) {
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    return lfa::launch_tree<LFA_OP, T>(dst, srcs, nsrc, cnt,
                                       (hipStream_t)stream);
  });
}

extern "C" int LFA_CAT(lfa__oneshot_op, LFA_OP)(int dt, const lfa_oneshot *a,
                                                void *stream) {
  return lfa::by_type<LFA_OP>(dt, [&](auto *tag) {
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    return lfa::launch_oneshot<LFA_OP, T>(*a, (hipStream_t)stream);
  });
}

extern "C" int LFA_CAT(lfa__treeput_op, LFA_OP)(int dt, void *const *dsts, int ndst,
                                                const void *const *srcs, int nsrc,
                                                size_t cnt, void *stream) {
  return lfa::by_type<LFA_OP>(dt, [&](auto *tag) {
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    return lfa::launch_tree_put<LFA_OP, T>(dsts, ndst, srcs, nsrc, cnt,
                                           (hipStream_t)stream);
  });
}
#endif

extern "C" int LFA_CAT(lfa__readwrite_op, LFA_OP)(int dt, void *dst,
                                                  const void *src, void *res,
                                                  size_t cnt, void *stream) {
  return lfa::by_type<LFA_OP>(dt, [&](auto *tag) {
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    return lfa::launch_readwrite<LFA_OP, T>(dst, src, res, cnt,
                                            (hipStream_t)stream);
  });
}
#else
extern "C" int LFA_CAT(lfa__swap_op, LFA_OP)(int dt, void *dst, const void *src,
                                             const void *cmp, void *res,
                                             size_t cnt, void *stream) {
  return lfa::by_type<LFA_OP>(dt, [&](auto *tag) {
    typedef typename std::remove_pointer<decltype(tag)>::type T;
    return lfa::launch_swap<LFA_OP, T>(dst, src, cmp, res, cnt,
                                       (hipStream_t)stream);
  });
}
#endif
