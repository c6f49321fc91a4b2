// lfa_ops.hpp — element semantics of the combine tables, for gfx950 device code.
//
// One functor per libfabric write op, restating (not copying) the shipping
// handler semantics of prov/util/src/util_atomic.c:
//   MIN/MAX   util_atomic.c:71-72, 291-316  dst-biased compare: `if (d > s) d = s`
//             (NaN in dst stays, NaN in src is ignored, ties/±0 keep dst)
//   SUM/PROD  util_atomic.c:73-74, 266-289  integer arithmetic wraps mod 2^bits
//             (computed here in unsigned types: no UB); IEEE f32/f64, no FTZ
//   LOR/LAND/LXOR util_atomic.c:75-76, 82-83 → 0/1 in the element type
//   BOR/BAND/BXOR util_atomic.c:78-85       integers only
//   WRITE     util_atomic.c:86-87           d = s
//   float complex: include/unix/osd.h:241-271 (C99 arithmetic; the NaN+NaN·i
//             product recovery follows C11 Annex G / libgcc __mulsc3)
//
// Everything is compiled with -ffp-contract=off: a contracted FMA would change
// PROD/SUM chains and the complex product away from the reference's rounding.
//
// One source for both sides: hipcc compiles these functors for gfx950 (the
// kernels) and, through LFA_HD, for the host as well; g++ compiles them as
// plain inline host code for the product's host-memory loop (lfa_host.cpp).
#pragma once

#include <stdint.h>
#ifdef __HIPCC__
#include <hip/hip_runtime.h>
#define LFA_HD __host__ __device__ __forceinline__
#else
#define LFA_HD inline __attribute__((always_inline))
#endif

namespace lfa {

enum Op : int {
  OP_MIN = 0, OP_MAX, OP_SUM, OP_PROD, OP_LOR, OP_LAND, OP_BOR, OP_BAND,
  OP_LXOR, OP_BXOR, OP_READ, OP_WRITE
};

struct cf32 {  // ofi_complex_float: two IEEE floats, 8-byte aligned
  float re, im;
};

typedef __int128 i128;
typedef unsigned __int128 u128;

// Unsigned type wide enough to do wrapping arithmetic without promotion UB.
template <typename T> struct Wide { typedef T type; };
template <> struct Wide<int8_t> { typedef uint32_t type; };
template <> struct Wide<uint8_t> { typedef uint32_t type; };
template <> struct Wide<int16_t> { typedef uint32_t type; };
template <> struct Wide<uint16_t> { typedef uint32_t type; };
template <> struct Wide<int32_t> { typedef uint32_t type; };
template <> struct Wide<uint32_t> { typedef uint32_t type; };
template <> struct Wide<int64_t> { typedef uint64_t type; };
template <> struct Wide<uint64_t> { typedef uint64_t type; };
template <> struct Wide<i128> { typedef u128 type; };
template <> struct Wide<u128> { typedef u128 type; };

template <typename T> struct IsFloat { static constexpr bool value = false; };
template <> struct IsFloat<float> { static constexpr bool value = true; };
template <> struct IsFloat<double> { static constexpr bool value = true; };

template <typename T>
LFA_HD bool truth(T v) { return v != T(0); }
template <>
LFA_HD bool truth<cf32>(cf32 v) {
  return v.re != 0.0f || v.im != 0.0f;
}

template <typename T>
LFA_HD T from_bool(bool b) { return b ? T(1) : T(0); }
template <>
LFA_HD cf32 from_bool<cf32>(bool b) {
  return cf32{b ? 1.0f : 0.0f, 0.0f};
}

template <typename T>
LFA_HD T add(T a, T b) {
  if constexpr (IsFloat<T>::value) {
    return a + b;
  } else {
    typedef typename Wide<T>::type W;
    return (T)((W)a + (W)b);
  }
}

template <typename T>
LFA_HD T mul(T a, T b) {
  if constexpr (IsFloat<T>::value) {
    return a * b;
  } else {
    typedef typename Wide<T>::type W;
    return (T)((W)a * (W)b);
  }
}

template <>
LFA_HD cf32 add<cf32>(cf32 a, cf32 b) {
  return cf32{a.re + b.re, a.im + b.im};
}

LFA_HD float copysign0(float mag, float sgn) {
  return __builtin_copysignf(mag, sgn);
}

// (a + bi)(c + di) as gcc emits it on x86-64 (-O2, no FMA): the textbook
// formula with every product rounded, and the C11 Annex G recovery when both
// parts are NaN (libgcc __mulsc3).
template <>
LFA_HD cf32 mul<cf32>(cf32 x, cf32 y) {
#ifdef __clang__
#pragma clang fp contract(off)
#endif
  float a = x.re, b = x.im, c = y.re, d = y.im;
  float ac = a * c, bd = b * d, ad = a * d, bc = b * c;
  float re = ac - bd, im = ad + bc;
  if (__builtin_isnan(re) && __builtin_isnan(im)) {
    bool recalc = false;
    if (__builtin_isinf(a) || __builtin_isinf(b)) {
      a = copysign0(__builtin_isinf(a) ? 1.0f : 0.0f, a);
      b = copysign0(__builtin_isinf(b) ? 1.0f : 0.0f, b);
      if (__builtin_isnan(c)) c = copysign0(0.0f, c);
      if (__builtin_isnan(d)) d = copysign0(0.0f, d);
      recalc = true;
    }
    if (__builtin_isinf(c) || __builtin_isinf(d)) {
      c = copysign0(__builtin_isinf(c) ? 1.0f : 0.0f, c);
      d = copysign0(__builtin_isinf(d) ? 1.0f : 0.0f, d);
      if (__builtin_isnan(a)) a = copysign0(0.0f, a);
      if (__builtin_isnan(b)) b = copysign0(0.0f, b);
      recalc = true;
    }
    if (!recalc && (__builtin_isinf(ac) || __builtin_isinf(bd) ||
                    __builtin_isinf(ad) || __builtin_isinf(bc))) {
      if (__builtin_isnan(a)) a = copysign0(0.0f, a);
      if (__builtin_isnan(b)) b = copysign0(0.0f, b);
      if (__builtin_isnan(c)) c = copysign0(0.0f, c);
      if (__builtin_isnan(d)) d = copysign0(0.0f, d);
      recalc = true;
    }
    if (recalc) {
      re = __builtin_inff() * (a * c - b * d);
      im = __builtin_inff() * (a * d + b * c);
    }
  }
  return cf32{re, im};
}

// d OP s for one element.  OP is an enum fi_op value.
template <int OP, typename T>
LFA_HD T apply(T d, T s) {
  if constexpr (OP == OP_MIN) {
    return (d > s) ? s : d;
  } else if constexpr (OP == OP_MAX) {
    return (d < s) ? s : d;
  } else if constexpr (OP == OP_SUM) {
    return add<T>(d, s);
  } else if constexpr (OP == OP_PROD) {
    return mul<T>(d, s);
  } else if constexpr (OP == OP_LOR) {
    return from_bool<T>(truth(d) || truth(s));
  } else if constexpr (OP == OP_LAND) {
    return from_bool<T>(truth(d) && truth(s));
  } else if constexpr (OP == OP_LXOR) {
    return from_bool<T>((truth(d) && !truth(s)) || (!truth(d) && truth(s)));
  } else if constexpr (OP == OP_BOR) {
    return d | s;
  } else if constexpr (OP == OP_BAND) {
    return d & s;
  } else if constexpr (OP == OP_BXOR) {
    return d ^ s;
  } else {  // OP_WRITE
    return s;
  }
}

// Which (op, type) pairs the shipping table fills (util_atomic.c:907-922).
// Classes: REALNO (int8..double, int128) for MIN/MAX; ALL (+ float complex)
// for SUM/PROD/LOR/LAND/LXOR/WRITE; INT (int8..uint64, int128) for bitwise.
template <typename T> struct Class {
  static constexpr bool is_int = !IsFloat<T>::value;
  static constexpr bool is_complex = false;
};
template <> struct Class<cf32> {
  static constexpr bool is_int = false;
  static constexpr bool is_complex = true;
};

template <int OP, typename T>
constexpr bool supported() {
  if constexpr (OP == OP_READ) return false;
  if constexpr (OP == OP_MIN || OP == OP_MAX) return !Class<T>::is_complex;
  if constexpr (OP == OP_BOR || OP == OP_BAND || OP == OP_BXOR) return Class<T>::is_int;
  return true;
}

}  // namespace lfa

namespace lfa {

// ---------------------------------------------------------------------------
// fetch (readwrite) and compare-swap tables (util_atomic.c:345-760, 924-980)
// ---------------------------------------------------------------------------
enum SwapOp : int {
  OP_CSWAP = 12, OP_CSWAP_NE, OP_CSWAP_LE, OP_CSWAP_LT, OP_CSWAP_GE,
  OP_CSWAP_GT, OP_MSWAP
};

template <int N> struct Bits;
template <> struct Bits<1> { typedef uint8_t type; };
template <> struct Bits<2> { typedef uint16_t type; };
template <> struct Bits<4> { typedef uint32_t type; };
template <> struct Bits<8> { typedef uint64_t type; };
template <> struct Bits<16> { typedef u128 type; };

// __atomic_compare_exchange compares object representations, not values:
// the shipping CSWAP swaps on identical BITS (-0.0 != +0.0, NaN == same NaN).
template <typename T>
LFA_HD bool bits_eq(T a, T b) {
  typename Bits<sizeof(T)>::type x, y;
  __builtin_memcpy(&x, &a, sizeof(T));
  __builtin_memcpy(&y, &b, sizeof(T));
  return x == y;
}

template <typename T>
LFA_HD bool val_ne(T c, T d) { return c != d; }
template <>
LFA_HD bool val_ne<cf32>(cf32 c, cf32 d) {
  return !(c.re == d.re && c.im == d.im);
}

// new dst for the swap row OP given dst a, src b, compare c
template <int OP, typename T>
LFA_HD T swap_apply(T a, T b, T c) {
  if constexpr (OP == OP_CSWAP) {
    return bits_eq(a, c) ? b : a;
  } else if constexpr (OP == OP_CSWAP_NE) {
    return val_ne(c, a) ? b : a;
  } else if constexpr (OP == OP_CSWAP_LE) {
    return (c <= a) ? b : a;
  } else if constexpr (OP == OP_CSWAP_LT) {
    return (c < a) ? b : a;
  } else if constexpr (OP == OP_CSWAP_GE) {
    return (c >= a) ? b : a;
  } else if constexpr (OP == OP_CSWAP_GT) {
    return (c > a) ? b : a;
  } else {  // OP_MSWAP
    return (T)((b & c) | (a & ~c));
  }
}

template <int OP, typename T>
constexpr bool rw_supported() {
  if constexpr (OP == OP_READ) return true;  // ALL handlers
  else return supported<OP, T>();
}

template <int OP, typename T>
constexpr bool swap_supported() {
  if constexpr (OP == OP_CSWAP || OP == OP_CSWAP_NE) return true;
  else if constexpr (OP == OP_MSWAP) return Class<T>::is_int;
  else return !Class<T>::is_complex;
}

}  // namespace lfa
