// lfa_capi.cpp — the public C ABI of liblfa.so (include/lfa_atomic.h).
//
// Host-only C++: argument validation, the ofi_atomic_valid restatement, the
// synchronous [op][datatype] table, and dispatch to the per-op kernel
// objects built from lfa_combine.hip.  No CPU compute path exists: every
// combine runs on the GPU.
#include <hip/hip_runtime_api.h>
#include <errno.h>
#include <stdio.h>

#include "../../include/lfa_atomic.h"

extern "C" {
#define LFA_DECL(N)                                                            \
  int lfa__write_op##N(int, void *, const void *, size_t, void *);             \
  int lfa__tree_op##N(int, void *, const void *const *, int, size_t, void *);
LFA_DECL(0) LFA_DECL(1) LFA_DECL(2) LFA_DECL(3) LFA_DECL(4) LFA_DECL(5)
LFA_DECL(6) LFA_DECL(7) LFA_DECL(8) LFA_DECL(9) LFA_DECL(11)
#undef LFA_DECL
}

namespace {

typedef int (*write_launch_t)(int, void *, const void *, size_t, void *);
typedef int (*tree_launch_t)(int, void *, const void *const *, int, size_t,
                             void *);

const write_launch_t kWrite[LFA_WRITE_OP_CNT] = {
    lfa__write_op0, lfa__write_op1, lfa__write_op2, lfa__write_op3,
    lfa__write_op4, lfa__write_op5, lfa__write_op6, lfa__write_op7,
    lfa__write_op8, lfa__write_op9, nullptr,        lfa__write_op11};
const tree_launch_t kTree[LFA_BXOR + 1] = {
    lfa__tree_op0, lfa__tree_op1, lfa__tree_op2, lfa__tree_op3, lfa__tree_op4,
    lfa__tree_op5, lfa__tree_op6, lfa__tree_op7, lfa__tree_op8, lfa__tree_op9};

// Table membership (util_atomic.c:907-922, HAVE_BUILTIN_MM_ATOMICS build with
// 128-bit atomics): REALNO = int8..double + int128; ALL = REALNO + float
// complex; INT = int8..uint64 + int128.
constexpr bool in_table(int op, int dt) {
  const bool realno = dt <= LFA_DOUBLE || dt == LFA_INT128 || dt == LFA_UINT128;
  const bool all = realno || dt == LFA_FLOAT_COMPLEX;
  const bool ints = dt <= LFA_UINT64 || dt == LFA_INT128 || dt == LFA_UINT128;
  switch (op) {
    case LFA_MIN: case LFA_MAX: return realno;
    case LFA_SUM: case LFA_PROD: case LFA_LOR: case LFA_LAND: case LFA_LXOR:
    case LFA_ATOMIC_WRITE: return all;
    case LFA_BOR: case LFA_BAND: case LFA_BXOR: return ints;
    default: return false;
  }
}

template <int OP, int DT>
void sync_entry(void *dst, const void *src, size_t cnt) {
  int rc = kWrite[OP](DT, dst, src, cnt, nullptr);
  hipError_t e = hipStreamSynchronize(nullptr);
  if (rc || e != hipSuccess)
    fprintf(stderr, "lfa: combine op=%d dt=%d failed (%d, %s)\n", OP, DT, rc,
            hipGetErrorString(e));
}

template <int OP, int DT>
constexpr lfa_write_fn entry() {
  if constexpr (in_table(OP, DT)) return &sync_entry<OP, DT>;
  else return nullptr;
}

}  // namespace

#define LFA_ROW(OP)                                                        \
  { entry<OP, 0>(), entry<OP, 1>(), entry<OP, 2>(), entry<OP, 3>(),      \
    entry<OP, 4>(), entry<OP, 5>(), entry<OP, 6>(), entry<OP, 7>(),      \
    entry<OP, 8>(), entry<OP, 9>(), entry<OP, 10>(), entry<OP, 11>(),    \
    entry<OP, 12>(), entry<OP, 13>(), entry<OP, 14>(), entry<OP, 15>() }

extern "C" {

lfa_write_fn const lfa_atomic_write_handlers[LFA_WRITE_OP_CNT][LFA_DATATYPE_CNT] = {
    LFA_ROW(0), LFA_ROW(1), LFA_ROW(2), LFA_ROW(3), LFA_ROW(4),  LFA_ROW(5),
    LFA_ROW(6), LFA_ROW(7), LFA_ROW(8), LFA_ROW(9), LFA_ROW(10), LFA_ROW(11)};

size_t lfa_datatype_size(enum lfa_datatype dt) {
  static const size_t sz[LFA_DATATYPE_CNT] = {1, 1, 2, 2, 4, 4, 8, 8,
                                              4, 8, 8, 16, 16, 32, 16, 16};
  if ((unsigned)dt >= LFA_DATATYPE_CNT) {
    errno = EINVAL;
    return 0;
  }
  return sz[dt];
}

int lfa_atomic_valid(enum lfa_datatype dt, enum lfa_op op, uint64_t flags) {
  if (flags & LFA_TAGGED) {
    if (flags & (LFA_FETCH_ATOMIC | LFA_COMPARE_ATOMIC)) return -LFA_ENOSYS;
  } else if (flags & ~(LFA_FETCH_ATOMIC | LFA_COMPARE_ATOMIC)) {
    return -LFA_EBADFLAGS;
  } else if ((flags & LFA_FETCH_ATOMIC) && (flags & LFA_COMPARE_ATOMIC)) {
    return -LFA_EBADFLAGS;
  }
  if ((unsigned)dt >= LFA_DATATYPE_CNT) return -LFA_EOPNOTSUPP;
  if (flags & (LFA_FETCH_ATOMIC | LFA_COMPARE_ATOMIC))
    return -LFA_EOPNOTSUPP;  // fetch / compare tables are not provided
  if ((unsigned)op >= LFA_WRITE_OP_CNT || op == LFA_ATOMIC_READ)
    return -LFA_EOPNOTSUPP;
  return in_table(op, dt) ? 0 : -LFA_EOPNOTSUPP;
}

int lfa_atomic_write_async(enum lfa_op op, enum lfa_datatype dt, void *dst,
                           const void *src, size_t cnt, void *stream) {
  if ((unsigned)op >= LFA_WRITE_OP_CNT || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !src)) return -LFA_EINVAL;
  return kWrite[op](dt, dst, src, cnt, stream);
}

int lfa_reduce_tree_async(enum lfa_op op, enum lfa_datatype dt, void *dst,
                          const void *const *srcs, int nsrc, size_t cnt,
                          void *stream) {
  if ((unsigned)op > LFA_BXOR || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (nsrc < 1 || nsrc > LFA_TREE_MAX || !srcs || (cnt && !dst))
    return -LFA_EINVAL;
  for (int k = 0; k < nsrc; k++)
    if (cnt && !srcs[k]) return -LFA_EINVAL;
  return kTree[op](dt, dst, srcs, nsrc, cnt, stream);
}

const char *lfa_version(void) {
  return "lfa-combine 0.2 gfx950 (LDS-DMA staged, 4 KiB/operand/wave, nt loads/stores)";
}

}  // extern "C"
