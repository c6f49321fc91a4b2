// lfa_host.cpp — the combine for HOST-resident buffers (liblfa.so).
//
// prov/coll hands its REDUCE items host memory (coll_coll.c:364 memcpy,
// :1058 calloc tmp, :758-768 the table call).  Device buffers always take the
// gfx950 kernels (lfa_combine.hip); this file serves the two places where the
// operands are host memory and moving them over PCIe would cost more than
// combining them where they are:
//   * the synchronous table (lfa_atomic_write_handlers) called with host
//     pointers on a bucket below LFA_HOST_SMALL_BYTES (SURVEY §7 "small-bucket
//     latency"); larger host buckets stream through HBM
//     (lfa_atomic_write_staged);
//   * endpoints opened on host memory with the owner's peer transport
//     (lfa_coll_domain_open_host), i.e. prov/coll's own configuration.
// The element semantics are lfa_ops.hpp — the SAME functors the kernels use —
// so host and device results are bit-identical by construction; both are
// pinned to the reference's fixtures (tests/test_host_combine.py,
// tests/test_combine_gpu.py).  Built with g++ -O3 -ffp-contract=off (no FMA
// contraction, IEEE denormals), like the reference's x86-64 build.
#include <stdint.h>
#include <string.h>

#include <type_traits>

#include "lfa_ops.hpp"
#include "../../include/lfa_atomic.h"

namespace lfa {
namespace {

template <typename T>
inline T load(const void *p, size_t i) {
  T v;
  memcpy(&v, (const char *)p + i * sizeof(T), sizeof(T));
  return v;
}

template <typename T>
inline void store(void *p, size_t i, T v) {
  memcpy((char *)p + i * sizeof(T), &v, sizeof(T));
}

template <int OP, typename T>
int host_write(void *dst, const void *src, size_t cnt) {
  if constexpr (!supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    if ((uintptr_t)dst % alignof(T) == 0 && (uintptr_t)src % alignof(T) == 0) {
      T *d = (T *)dst;
      const T *s = (const T *)src;
      for (size_t i = 0; i < cnt; i++) d[i] = apply<OP, T>(d[i], s[i]);
    } else {
      for (size_t i = 0; i < cnt; i++)
        store<T>(dst, i, apply<OP, T>(load<T>(dst, i), load<T>(src, i)));
    }
    return 0;
  }
}

// prov/coll's recursive-doubling association for nsrc ranks
// (coll_coll.c:349-449): leaves are (in[2k+1] OP in[2k]) for k < rem, then
// single inputs; partials merge pairwise, higher OP lower, level by level.
// Evaluated with a stack per block of elements (as the device tree does per
// lane), so only log2(leaves)+1 partial blocks are live.
constexpr int kHostBlock = 256;

template <int OP, typename T>
int host_tree(void *dst, const void *const *srcs, int nsrc, size_t cnt) {
  if constexpr (!supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    int pof2 = 1;
    while (pof2 * 2 <= nsrc) pof2 *= 2;
    const int rem = nsrc - pof2;
    T stack[7][kHostBlock];
    for (size_t b0 = 0; b0 < cnt; b0 += kHostBlock) {
      const size_t nb = cnt - b0 < (size_t)kHostBlock ? cnt - b0 : kHostBlock;
      int depth = 0;
      for (int k = 0; k < pof2; k++) {
        const int hi = k < rem ? 2 * k + 1 : k + rem;
        T *top = stack[depth++];
        for (size_t i = 0; i < nb; i++) top[i] = load<T>(srcs[hi], b0 + i);
        if (k < rem)
          for (size_t i = 0; i < nb; i++)
            top[i] = apply<OP, T>(top[i], load<T>(srcs[2 * k], b0 + i));
        for (int m = 1; m < pof2; m <<= 1) {
          if (((k + 1) & (2 * m - 1)) != 0) break;
          T *h = stack[depth - 1], *l = stack[depth - 2];
          for (size_t i = 0; i < nb; i++) l[i] = apply<OP, T>(h[i], l[i]);
          depth--;
        }
      }
      for (size_t i = 0; i < nb; i++) store<T>(dst, b0 + i, stack[0][i]);
    }
    return 0;
  }
}

// Fetch table: res = old dst, then dst = dst OP src (util_atomic.c:924-950).
template <int OP, typename T>
int host_readwrite(void *dst, const void *src, void *res, size_t cnt) {
  if constexpr (!rw_supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    for (size_t i = 0; i < cnt; i++) {
      T a = load<T>(dst, i);
      store<T>(res, i, a);
      if constexpr (OP != OP_READ) store<T>(dst, i, apply<OP, T>(a, load<T>(src, i)));
    }
    return 0;
  }
}

// Compare table: res = old dst, dst = src where the compare holds
// (util_atomic.c:952-980).
template <int OP, typename T>
int host_swap(void *dst, const void *src, const void *cmp, void *res, size_t cnt) {
  if constexpr (!swap_supported<OP, T>()) {
    return -LFA_EOPNOTSUPP;
  } else {
    for (size_t i = 0; i < cnt; i++) {
      T a = load<T>(dst, i);
      store<T>(res, i, a);
      store<T>(dst, i, swap_apply<OP, T>(a, load<T>(src, i), load<T>(cmp, i)));
    }
    return 0;
  }
}

template <typename F>
int by_type(int dt, F &&f) {
  switch (dt) {
    case LFA_INT8: return f((int8_t *)0);
    case LFA_UINT8: return f((uint8_t *)0);
    case LFA_INT16: return f((int16_t *)0);
    case LFA_UINT16: return f((uint16_t *)0);
    case LFA_INT32: return f((int32_t *)0);
    case LFA_UINT32: return f((uint32_t *)0);
    case LFA_INT64: return f((int64_t *)0);
    case LFA_UINT64: return f((uint64_t *)0);
    case LFA_FLOAT: return f((float *)0);
    case LFA_DOUBLE: return f((double *)0);
    case LFA_FLOAT_COMPLEX: return f((cf32 *)0);
    case LFA_INT128: return f((i128 *)0);
    case LFA_UINT128: return f((u128 *)0);
    default: return -LFA_EOPNOTSUPP;
  }
}

template <typename F>
int by_op(int op, F &&f) {
  switch (op) {
    case OP_MIN: return f(std::integral_constant<int, OP_MIN>());
    case OP_MAX: return f(std::integral_constant<int, OP_MAX>());
    case OP_SUM: return f(std::integral_constant<int, OP_SUM>());
    case OP_PROD: return f(std::integral_constant<int, OP_PROD>());
    case OP_LOR: return f(std::integral_constant<int, OP_LOR>());
    case OP_LAND: return f(std::integral_constant<int, OP_LAND>());
    case OP_BOR: return f(std::integral_constant<int, OP_BOR>());
    case OP_BAND: return f(std::integral_constant<int, OP_BAND>());
    case OP_LXOR: return f(std::integral_constant<int, OP_LXOR>());
    case OP_BXOR: return f(std::integral_constant<int, OP_BXOR>());
    case OP_READ: return f(std::integral_constant<int, OP_READ>());
    case OP_WRITE: return f(std::integral_constant<int, OP_WRITE>());
    default: return -LFA_EOPNOTSUPP;
  }
}

template <typename F>
int by_swap_op(int op, F &&f) {
  switch (op) {
    case OP_CSWAP: return f(std::integral_constant<int, OP_CSWAP>());
    case OP_CSWAP_NE: return f(std::integral_constant<int, OP_CSWAP_NE>());
    case OP_CSWAP_LE: return f(std::integral_constant<int, OP_CSWAP_LE>());
    case OP_CSWAP_LT: return f(std::integral_constant<int, OP_CSWAP_LT>());
    case OP_CSWAP_GE: return f(std::integral_constant<int, OP_CSWAP_GE>());
    case OP_CSWAP_GT: return f(std::integral_constant<int, OP_CSWAP_GT>());
    case OP_MSWAP: return f(std::integral_constant<int, OP_MSWAP>());
    default: return -LFA_EOPNOTSUPP;
  }
}

}  // namespace
}  // namespace lfa

extern "C" {

int lfa_host_write(enum lfa_op op, enum lfa_datatype dt, void *dst, const void *src,
                   size_t cnt) {
  if (lfa_atomic_valid(dt, op, 0)) return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !src)) return -LFA_EINVAL;
  return lfa::by_op(op, [&](auto opc) {
    constexpr int OP = decltype(opc)::value;
    if constexpr (OP == lfa::OP_READ) return -LFA_EOPNOTSUPP;
    else return lfa::by_type(dt, [&](auto *tag) {
      typedef typename std::remove_pointer<decltype(tag)>::type T;
      return lfa::host_write<OP, T>(dst, src, cnt);
    });
  });
}

int lfa_host_readwrite(enum lfa_op op, enum lfa_datatype dt, void *dst,
                       const void *src, void *res, size_t cnt) {
  if (lfa_atomic_valid(dt, op, LFA_FETCH_ATOMIC)) return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !res || (op != LFA_ATOMIC_READ && !src))) return -LFA_EINVAL;
  return lfa::by_op(op, [&](auto opc) {
    constexpr int OP = decltype(opc)::value;
    return lfa::by_type(dt, [&](auto *tag) {
      typedef typename std::remove_pointer<decltype(tag)>::type T;
      return lfa::host_readwrite<OP, T>(dst, src, res, cnt);
    });
  });
}

int lfa_host_swap(enum lfa_op op, enum lfa_datatype dt, void *dst, const void *src,
                  const void *cmp, void *res, size_t cnt) {
  if (lfa_atomic_valid(dt, op, LFA_COMPARE_ATOMIC)) return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !src || !cmp || !res)) return -LFA_EINVAL;
  return lfa::by_swap_op(op, [&](auto opc) {
    constexpr int OP = decltype(opc)::value;
    return lfa::by_type(dt, [&](auto *tag) {
      typedef typename std::remove_pointer<decltype(tag)>::type T;
      return lfa::host_swap<OP, T>(dst, src, cmp, res, cnt);
    });
  });
}

int lfa_host_reduce_tree(enum lfa_op op, enum lfa_datatype dt, void *dst,
                         const void *const *srcs, int nsrc, size_t cnt) {
  if ((unsigned)op > LFA_BXOR || lfa_atomic_valid(dt, op, 0)) return -LFA_EOPNOTSUPP;
  if (nsrc < 1 || nsrc > LFA_TREE_MAX || !srcs || (cnt && !dst)) return -LFA_EINVAL;
  for (int k = 0; k < nsrc; k++)
    if (cnt && !srcs[k]) return -LFA_EINVAL;
  if (!cnt) return 0;
  if (nsrc == 1) {
    if (dst != srcs[0]) memmove(dst, srcs[0], cnt * lfa_datatype_size(dt));
    return 0;
  }
  return lfa::by_op(op, [&](auto opc) {
    constexpr int OP = decltype(opc)::value;
    return lfa::by_type(dt, [&](auto *tag) {
      typedef typename std::remove_pointer<decltype(tag)>::type T;
      return lfa::host_tree<OP, T>(dst, srcs, nsrc, cnt);
    });
  });
}

}  // extern "C"
