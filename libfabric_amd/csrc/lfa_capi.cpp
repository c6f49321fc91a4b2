// lfa_capi.cpp — the public C ABI of liblfa.so (include/lfa_atomic.h).
//
// Host-only C++: argument validation, the ofi_atomic_valid restatement, the
// synchronous [op][datatype] tables (write, fetch, compare), and dispatch to
// the per-op kernel
// objects built from lfa_combine.hip.  No CPU compute path exists: every
// combine runs on the GPU.
#include <hip/hip_runtime_api.h>
#include <errno.h>
#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/lfa_atomic.h"
#include "lfa_signal.h"

extern "C" {
#define LFA_DECL_W(N)                                                          \
  int lfa__write_op##N(int, void *, const void *, size_t, void *);
#define LFA_DECL_T(N)                                                          \
  int lfa__tree_op##N(int, void *, const void *const *, int, size_t, void *);
#define LFA_DECL_TP(N)                                                         \
  int lfa__treeput_op##N(int, void *const *, int, const void *const *, int,    \
                         size_t, void *);
#define LFA_DECL_OS(N) int lfa__oneshot_op##N(int, const lfa_oneshot *, void *);
#define LFA_DECL_RW(N)                                                         \
  int lfa__readwrite_op##N(int, void *, const void *, void *, size_t, void *);
#define LFA_DECL_SW(N)                                                         \
  int lfa__swap_op##N(int, void *, const void *, const void *, void *, size_t, \
                      void *);
LFA_DECL_W(0) LFA_DECL_W(1) LFA_DECL_W(2) LFA_DECL_W(3) LFA_DECL_W(4)
LFA_DECL_W(5) LFA_DECL_W(6) LFA_DECL_W(7) LFA_DECL_W(8) LFA_DECL_W(9)
LFA_DECL_W(11)
LFA_DECL_T(0) LFA_DECL_T(1) LFA_DECL_T(2) LFA_DECL_T(3) LFA_DECL_T(4)
LFA_DECL_T(5) LFA_DECL_T(6) LFA_DECL_T(7) LFA_DECL_T(8) LFA_DECL_T(9)
LFA_DECL_TP(0) LFA_DECL_TP(1) LFA_DECL_TP(2) LFA_DECL_TP(3) LFA_DECL_TP(4)
LFA_DECL_TP(5) LFA_DECL_TP(6) LFA_DECL_TP(7) LFA_DECL_TP(8) LFA_DECL_TP(9)
LFA_DECL_OS(0) LFA_DECL_OS(1) LFA_DECL_OS(2) LFA_DECL_OS(3) LFA_DECL_OS(4)
LFA_DECL_OS(5) LFA_DECL_OS(6) LFA_DECL_OS(7) LFA_DECL_OS(8) LFA_DECL_OS(9)
LFA_DECL_RW(0) LFA_DECL_RW(1) LFA_DECL_RW(2) LFA_DECL_RW(3) LFA_DECL_RW(4)
LFA_DECL_RW(5) LFA_DECL_RW(6) LFA_DECL_RW(7) LFA_DECL_RW(8) LFA_DECL_RW(9)
LFA_DECL_RW(10) LFA_DECL_RW(11)
LFA_DECL_SW(12) LFA_DECL_SW(13) LFA_DECL_SW(14) LFA_DECL_SW(15)
LFA_DECL_SW(16) LFA_DECL_SW(17) LFA_DECL_SW(18)
#undef LFA_DECL_W
#undef LFA_DECL_T
#undef LFA_DECL_TP
#undef LFA_DECL_OS
#undef LFA_DECL_RW
#undef LFA_DECL_SW
}

namespace {

typedef int (*write_launch_t)(int, void *, const void *, size_t, void *);
typedef int (*tree_launch_t)(int, void *, const void *const *, int, size_t,
                             void *);

const write_launch_t kWrite[LFA_WRITE_OP_CNT] = {
    lfa__write_op0, lfa__write_op1, lfa__write_op2, lfa__write_op3,
    lfa__write_op4, lfa__write_op5, lfa__write_op6, lfa__write_op7,
    lfa__write_op8, lfa__write_op9, nullptr,        lfa__write_op11};
typedef int (*rw_launch_t)(int, void *, const void *, void *, size_t, void *);
typedef int (*swap_launch_t)(int, void *, const void *, const void *, void *,
                             size_t, void *);
const rw_launch_t kReadWrite[LFA_READWRITE_OP_CNT] = {
    lfa__readwrite_op0, lfa__readwrite_op1, lfa__readwrite_op2,
    lfa__readwrite_op3, lfa__readwrite_op4, lfa__readwrite_op5,
    lfa__readwrite_op6, lfa__readwrite_op7, lfa__readwrite_op8,
    lfa__readwrite_op9, lfa__readwrite_op10, lfa__readwrite_op11};
const swap_launch_t kSwap[LFA_SWAP_OP_CNT] = {
    lfa__swap_op12, lfa__swap_op13, lfa__swap_op14, lfa__swap_op15,
    lfa__swap_op16, lfa__swap_op17, lfa__swap_op18};

const tree_launch_t kTree[LFA_BXOR + 1] = {
    lfa__tree_op0, lfa__tree_op1, lfa__tree_op2, lfa__tree_op3, lfa__tree_op4,
    lfa__tree_op5, lfa__tree_op6, lfa__tree_op7, lfa__tree_op8, lfa__tree_op9};

typedef int (*treeput_launch_t)(int, void *const *, int, const void *const *, int,
                                size_t, void *);
const treeput_launch_t kTreePut[LFA_BXOR + 1] = {
    lfa__treeput_op0, lfa__treeput_op1, lfa__treeput_op2, lfa__treeput_op3,
    lfa__treeput_op4, lfa__treeput_op5, lfa__treeput_op6, lfa__treeput_op7,
    lfa__treeput_op8, lfa__treeput_op9};

typedef int (*oneshot_launch_t)(int, const lfa_oneshot *, void *);
const oneshot_launch_t kOneShot[LFA_BXOR + 1] = {
    lfa__oneshot_op0, lfa__oneshot_op1, lfa__oneshot_op2, lfa__oneshot_op3,
    lfa__oneshot_op4, lfa__oneshot_op5, lfa__oneshot_op6, lfa__oneshot_op7,
    lfa__oneshot_op8, lfa__oneshot_op9};

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

// Fetch table (util_atomic.c:924-950): the write rows plus an ALL-types
// ATOMIC_READ row; ATOMIC_WRITE is an exchange.
constexpr bool in_rw_table(int op, int dt) {
  return op == LFA_ATOMIC_READ ? in_table(LFA_ATOMIC_WRITE, dt) : in_table(op, dt);
}

// Compare table (util_atomic.c:952-980): CSWAP / CSWAP_NE over ALL types,
// LE/LT/GE/GT over REALNO, MSWAP over INT.
constexpr bool in_swap_table(int op, int dt) {
  switch (op) {
    case LFA_CSWAP: case LFA_CSWAP_NE: return in_table(LFA_SUM, dt);
    case LFA_CSWAP_LE: case LFA_CSWAP_LT: case LFA_CSWAP_GE: case LFA_CSWAP_GT:
      return in_table(LFA_MIN, dt);
    case LFA_MSWAP: return in_table(LFA_BOR, dt);
    default: return false;
  }
}

// Where an operand lives: the synchronous tables take what their caller has
// — prov/coll's REDUCE items hand over host memory (coll_coll.c:364, :1058),
// a GPU-resident caller device memory.  Pinned and registered host memory
// counts as host: a small bucket runs the host loop; above it
// lfa_atomic_write_staged combines it in place over PCIe (zero-copy).
enum { kDev = 1, kHost = 2 };

int ptr_kind(const void *p) {
  hipPointerAttribute_t a;
  if (!p) return kHost;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // unknown to HIP: plain host memory
    return kHost;
  }
  return (a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged) ? kDev : kHost;
}

// First failure of a synchronous table call on this thread (lfa_atomic_last_error).
thread_local int t_last_error = 0;

inline void note_error(int rc) {
  if (rc && !t_last_error) t_last_error = rc < 0 ? rc : -LFA_EIO;
}

template <int OP, int DT>
void sync_rw_entry(void *dst, const void *src, void *res, size_t cnt) {
  if (!cnt) return;  // the reference's loop over zero elements: nothing, no GPU call
  const int k = ptr_kind(dst) | ptr_kind(res) | (OP == LFA_ATOMIC_READ ? 0 : ptr_kind(src));
  if (k == kHost) {
    int rc = lfa_host_readwrite((lfa_op)OP, (lfa_datatype)DT, dst, src, res, cnt);
    if (rc) fprintf(stderr, "lfa: host fetch op=%d dt=%d failed (%d)\n", OP, DT, rc);
    note_error(rc);
    return;
  }
  if (k != kDev) {
    fprintf(stderr, "lfa: fetch op=%d dt=%d: mixed host/device operands\n", OP, DT);
    note_error(-LFA_EINVAL);
    return;
  }
  int rc = kReadWrite[OP](DT, dst, src, res, cnt, nullptr);
  hipError_t e = hipStreamSynchronize(nullptr);
  if (rc || e != hipSuccess)
    fprintf(stderr, "lfa: fetch op=%d dt=%d failed (%d, %s)\n", OP, DT, rc,
            hipGetErrorString(e));
  note_error(rc ? rc : e != hipSuccess ? -LFA_EIO : 0);
}

template <int OP, int DT>
void sync_swap_entry(void *dst, const void *src, const void *cmp, void *res,
                     size_t cnt) {
  if (!cnt) return;
  const int k = ptr_kind(dst) | ptr_kind(src) | ptr_kind(cmp) | ptr_kind(res);
  if (k == kHost) {
    int rc = lfa_host_swap((lfa_op)OP, (lfa_datatype)DT, dst, src, cmp, res, cnt);
    if (rc) fprintf(stderr, "lfa: host swap op=%d dt=%d failed (%d)\n", OP, DT, rc);
    note_error(rc);
    return;
  }
  if (k != kDev) {
    fprintf(stderr, "lfa: swap op=%d dt=%d: mixed host/device operands\n", OP, DT);
    note_error(-LFA_EINVAL);
    return;
  }
  int rc = kSwap[OP - LFA_CSWAP](DT, dst, src, cmp, res, cnt, nullptr);
  hipError_t e = hipStreamSynchronize(nullptr);
  if (rc || e != hipSuccess)
    fprintf(stderr, "lfa: swap op=%d dt=%d failed (%d, %s)\n", OP, DT, rc,
            hipGetErrorString(e));
  note_error(rc ? rc : e != hipSuccess ? -LFA_EIO : 0);
}

template <int OP, int DT>
constexpr lfa_readwrite_fn rw_entry() {
  if constexpr (in_rw_table(OP, DT)) return &sync_rw_entry<OP, DT>;
  else return nullptr;
}

template <int OP, int DT>
constexpr lfa_swap_fn swap_entry() {
  if constexpr (in_swap_table(OP, DT)) return &sync_swap_entry<OP, DT>;
  else return nullptr;
}

template <int OP, int DT>
void sync_entry(void *dst, const void *src, size_t cnt) {
  if (!cnt) return;
  const int k = ptr_kind(dst) | ptr_kind(src);
  if (k != kDev) {
    // host (or mixed) operands: the host loop for a small bucket, HBM
    // streaming above lfa_host_small_bytes() (SURVEY §7 small-bucket latency)
    int rc = k == kHost && cnt * lfa_datatype_size((lfa_datatype)DT) <= lfa_host_small_bytes()
                 ? lfa_host_write((lfa_op)OP, (lfa_datatype)DT, dst, src, cnt)
                 : lfa_atomic_write_staged((lfa_op)OP, (lfa_datatype)DT, dst, src, cnt, 0);
    if (rc) fprintf(stderr, "lfa: combine op=%d dt=%d (host operands) failed (%d)\n", OP, DT, rc);
    note_error(rc);
    return;
  }
  int rc = kWrite[OP](DT, dst, src, cnt, nullptr);
  hipError_t e = hipStreamSynchronize(nullptr);
  if (rc || e != hipSuccess)
    fprintf(stderr, "lfa: combine op=%d dt=%d failed (%d, %s)\n", OP, DT, rc,
            hipGetErrorString(e));
  note_error(rc ? rc : e != hipSuccess ? -LFA_EIO : 0);
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

#define LFA_RW_ROW(OP)                                                         \
  { rw_entry<OP, 0>(), rw_entry<OP, 1>(), rw_entry<OP, 2>(), rw_entry<OP, 3>(), \
    rw_entry<OP, 4>(), rw_entry<OP, 5>(), rw_entry<OP, 6>(), rw_entry<OP, 7>(), \
    rw_entry<OP, 8>(), rw_entry<OP, 9>(), rw_entry<OP, 10>(),                   \
    rw_entry<OP, 11>(), rw_entry<OP, 12>(), rw_entry<OP, 13>(),                 \
    rw_entry<OP, 14>(), rw_entry<OP, 15>() }
#define LFA_SW_ROW(OP)                                                         \
  { swap_entry<OP, 0>(), swap_entry<OP, 1>(), swap_entry<OP, 2>(),             \
    swap_entry<OP, 3>(), swap_entry<OP, 4>(), swap_entry<OP, 5>(),             \
    swap_entry<OP, 6>(), swap_entry<OP, 7>(), swap_entry<OP, 8>(),             \
    swap_entry<OP, 9>(), swap_entry<OP, 10>(), swap_entry<OP, 11>(),           \
    swap_entry<OP, 12>(), swap_entry<OP, 13>(), swap_entry<OP, 14>(),          \
    swap_entry<OP, 15>() }

extern "C" {

lfa_readwrite_fn const
    lfa_atomic_readwrite_handlers[LFA_READWRITE_OP_CNT][LFA_DATATYPE_CNT] = {
        LFA_RW_ROW(0), LFA_RW_ROW(1), LFA_RW_ROW(2), LFA_RW_ROW(3),
        LFA_RW_ROW(4), LFA_RW_ROW(5), LFA_RW_ROW(6), LFA_RW_ROW(7),
        LFA_RW_ROW(8), LFA_RW_ROW(9), LFA_RW_ROW(10), LFA_RW_ROW(11)};

lfa_swap_fn const lfa_atomic_swap_handlers[LFA_SWAP_OP_CNT][LFA_DATATYPE_CNT] = {
    LFA_SW_ROW(12), LFA_SW_ROW(13), LFA_SW_ROW(14), LFA_SW_ROW(15),
    LFA_SW_ROW(16), LFA_SW_ROW(17), LFA_SW_ROW(18)};

int lfa_atomic_readwrite_async(enum lfa_op op, enum lfa_datatype dt, void *dst,
                               const void *src, void *res, size_t cnt,
                               void *stream) {
  if ((unsigned)op >= LFA_READWRITE_OP_CNT || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_rw_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !res || (op != LFA_ATOMIC_READ && !src)))
    return -LFA_EINVAL;
  return kReadWrite[op](dt, dst, src, res, cnt, stream);
}

int lfa_atomic_swap_async(enum lfa_op op, enum lfa_datatype dt, void *dst,
                          const void *src, const void *cmp, void *res,
                          size_t cnt, void *stream) {
  if (op < LFA_CSWAP || op > LFA_MSWAP || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_swap_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !src || !cmp || !res)) return -LFA_EINVAL;
  return kSwap[op - LFA_CSWAP](dt, dst, src, cmp, res, cnt, stream);
}

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
  if (flags & LFA_FETCH_ATOMIC)
    return (unsigned)op < LFA_READWRITE_OP_CNT && in_rw_table(op, dt)
               ? 0 : -LFA_EOPNOTSUPP;
  if (flags & LFA_COMPARE_ATOMIC)
    return in_swap_table(op, dt) ? 0 : -LFA_EOPNOTSUPP;
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
  // One input is a copy (a one-member group's allreduce): from 16 MiB the
  // write table's ATOMIC_WRITE body beats hipMemcpyAsync D2D (83.3 vs 98.8 us
  // at 256 MiB, profiles/r02_probe_copy.log); below, the tree launcher's
  // hipMemcpyAsync stays.
  const size_t bytes = cnt * lfa_datatype_size(dt);
  if (nsrc == 1 && dst != srcs[0] && bytes >= ((size_t)16 << 20))
    return lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8, dst, srcs[0], bytes,
                                  stream);
  return kTree[op](dt, dst, srcs, nsrc, cnt, stream);
}

int lfa_reduce_tree_put_async(enum lfa_op op, enum lfa_datatype dt,
                              void *const *dsts, int ndst, const void *const *srcs,
                              int nsrc, size_t cnt, void *stream) {
  if ((unsigned)op > LFA_BXOR || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (nsrc < 1 || nsrc > LFA_TREE_MAX || !srcs || ndst < 1 || ndst > LFA_PUT_MAX ||
      !dsts)
    return -LFA_EINVAL;
  for (int k = 0; k < nsrc; k++)
    if (cnt && !srcs[k]) return -LFA_EINVAL;
  for (int j = 0; j < ndst; j++)
    if (cnt && !dsts[j]) return -LFA_EINVAL;
  return kTreePut[op](dt, dsts, ndst, srcs, nsrc, cnt, stream);
}

int lfa_atomic_last_error(void) {
  int rc = t_last_error;
  t_last_error = 0;
  return rc;
}

int lfa_oneshot_reduce_async(int op, int dt, const struct lfa_oneshot *a,
                                void *stream) {
  if ((unsigned)op > LFA_BXOR || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (!a) return -LFA_EINVAL;
  return kOneShot[op](dt, a, stream);
}

}  // extern "C"

namespace {
// Staging contexts for lfa_atomic_write_staged: two streams, the slot events
// and an HBM staging buffer that only grows.  kStageSlots per device, each
// with its own lock, so concurrent host-buffer callers on one device run at
// once instead of queueing behind one caller's PCIe transfer;
// a caller takes a free slot, and waits on one only when all are busy.
// Created on first use and kept for the life of the process (a hipMalloc +
// hipFree per call costs milliseconds and serialises the device).
struct StagingCtx {
  pthread_mutex_t lock = PTHREAD_MUTEX_INITIALIZER;
  hipStream_t s_in = nullptr, s_out = nullptr;
  hipEvent_t in_done[2] = {}, out_done[2] = {};
  char *dev = nullptr;
  size_t cap = 0;
};
constexpr int kMaxDevices = 64;
constexpr int kStageSlots = 4;
StagingCtx g_staging[kMaxDevices][kStageSlots];
unsigned g_stage_next[kMaxDevices];

// A staging slot of device `devno`, locked; staging_release unlocks it.
StagingCtx &staging_lock(int devno) {
  for (StagingCtx &c : g_staging[devno])
    if (!pthread_mutex_trylock(&c.lock)) return c;
  StagingCtx &c = g_staging[devno][__atomic_fetch_add(&g_stage_next[devno], 1u,
                                                      __ATOMIC_RELAXED) % kStageSlots];
  pthread_mutex_lock(&c.lock);
  return c;
}

int staging_acquire(StagingCtx &c, size_t bytes) {
  if (!c.s_in) {
    if (hipStreamCreateWithFlags(&c.s_in, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&c.s_out, hipStreamNonBlocking) != hipSuccess)
      return -LFA_ENOMEM;
    for (int i = 0; i < 2; i++)
      if (hipEventCreateWithFlags(&c.in_done[i], hipEventDisableTiming) != hipSuccess ||
          hipEventCreateWithFlags(&c.out_done[i], hipEventDisableTiming) != hipSuccess)
        return -LFA_ENOMEM;
  }
  if (c.cap < bytes) {
    if (c.dev) hipFree(c.dev);
    c.dev = nullptr;
    c.cap = 0;
    if (hipMalloc((void **)&c.dev, bytes) != hipSuccess) return -LFA_ENOMEM;
    c.cap = bytes;
  }
  return 0;
}

bool zero_copy_on() {
  const char *e = lfa_param("LFA_HOST_ZERO_COPY");
  return !e || strtol(e, nullptr, 0);
}

// Temporary registrations: pageable operands lfa_atomic_write_staged pins
// for one call (hipHostRegister), refcounted by exact (address, length) so
// callers combining the same buffer share one.  A registration's page range
// is in this table from before hipHostRegister until after hipHostUnregister
// (states PENDING -> READY -> DYING), and every classification checks the
// table first: a page range in it is never handed out as a zero-copy address
// (the call that made it may unregister it at any moment), and an operand
// overlapping another call's registration is staged.  g_reg_lock covers the
// table and the classifications — never a registration, a kernel or a
// stream synchronisation (holding it across the
// combine stalled every endpoint's submit for the whole PCIe transfer).
enum { kRegFree = 0, kRegPending, kRegReady, kRegDying };
struct TempReg {
  int state;
  uintptr_t lo, hi;  // the page range
  const void *p;
  size_t bytes;
  void *d;           // its device address once READY
  int refs;
};
constexpr int kTempRegs = 64;
TempReg g_temp[kTempRegs];
pthread_mutex_t g_reg_lock = PTHREAD_MUTEX_INITIALIZER;
constexpr uintptr_t kPage = 4096;

// The entry overlapping the pages of [p, p + bytes), or -1 (g_reg_lock held).
int temp_find(const void *p, size_t bytes) {
  const uintptr_t lo = (uintptr_t)p & ~(kPage - 1);
  const uintptr_t hi = ((uintptr_t)p + (bytes ? bytes : 1) + kPage - 1) & ~(kPage - 1);
  for (int i = 0; i < kTempRegs; i++)
    if (g_temp[i].state != kRegFree && g_temp[i].lo < hi && lo < g_temp[i].hi) return i;
  return -1;
}

// The address a kernel on device `devno` uses for operand p, or null when
// the operand must be staged: device memory of this device as it is, pinned
// or registered host memory through its device mapping (zero-copy: the
// combine reads and writes it over PCIe) — never a temporary registration.
// *pageable: p is host memory HIP does not know, which the caller may
// register for the call.  g_reg_lock held.
void *zero_copy_addr(const void *p, size_t bytes, int devno, bool *pageable) {
  hipPointerAttribute_t a;
  *pageable = false;
  if (temp_find(p, bytes) >= 0) return nullptr;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();
    *pageable = true;
    return nullptr;
  }
  if (a.type == hipMemoryTypeUnregistered) *pageable = true;
  if (a.type == hipMemoryTypeHost) return a.devicePointer;
  if (a.type == hipMemoryTypeDevice && a.device == devno) return const_cast<void *>(p);
  return nullptr;
}

// Pin pageable operand p (bytes long) for one call; its device address, or
// null if the runtime refuses (overlapping registrations, read-only pages):
// the caller then stages.
void *register_for_call(const void *p, size_t bytes) {
  void *d = nullptr;
  if (hipHostRegister(const_cast<void *>(p), bytes, hipHostRegisterMapped) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (hipHostGetDevicePointer(&d, const_cast<void *>(p), 0) != hipSuccess || !d) {
    (void)hipGetLastError();
    hipHostUnregister(const_cast<void *>(p));
    return nullptr;
  }
  return d;
}

// A temporary registration of exactly [p, p + bytes) for this call: a READY
// one shared (refs + 1), else a new one; its index and device address, or -1
// (the pages overlap another call's registration, another call holds one —
// `mine`, this call's other operand's, aside — or the runtime refused): the
// caller stages.
int temp_take(const void *p, size_t bytes, void **d, int mine) {
  pthread_mutex_lock(&g_reg_lock);
  int i = temp_find(p, bytes);
  if (i >= 0) {
    TempReg &t = g_temp[i];
    const bool share = t.state == kRegReady && t.p == p && t.bytes == bytes;
    if (share) {
      t.refs++;
      *d = t.d;
    }
    pthread_mutex_unlock(&g_reg_lock);
    return share ? i : -1;
  }
  // one call registers at a time: hipHostRegister / hipHostUnregister from
  // several threads at once slow each other down (4 threads of pageable
  // 2 MiB combines: 29x one call, against 3.7x when they stage;
  // profiles/r06_threads_probe_before.jsonl), so while another call holds or makes
  // a registration this one takes the staged pipeline, which overlaps
  int busy = 0;
  for (int k = 0; k < kTempRegs; k++) busy += k != mine && g_temp[k].state != kRegFree;
  for (i = 0; i < kTempRegs && g_temp[i].state != kRegFree; i++) {
  }
  if (busy || i == kTempRegs) {
    pthread_mutex_unlock(&g_reg_lock);
    return -1;
  }
  g_temp[i] = TempReg{kRegPending, (uintptr_t)p & ~(kPage - 1),
                      ((uintptr_t)p + bytes + kPage - 1) & ~(kPage - 1), p, bytes, nullptr, 1};
  pthread_mutex_unlock(&g_reg_lock);
  void *dp = register_for_call(p, bytes);  // outside the lock: milliseconds
  pthread_mutex_lock(&g_reg_lock);
  if (dp) {
    g_temp[i].state = kRegReady;
    g_temp[i].d = dp;
  } else {
    g_temp[i].state = kRegFree;
  }
  pthread_mutex_unlock(&g_reg_lock);
  *d = dp;
  return dp ? i : -1;
}

// Calls in the staged pipeline right now: a call does not register its
// pageable operands while any is (lfa_atomic_write_staged).
int g_staged_calls;

// Pageable buckets below this stage instead of registering for the call
// (LFA_HOST_REGISTER_BYTES, default 64 MiB): below it the gain is a few
// hundred microseconds, and a registration stalls concurrent callers.
size_t register_min_bytes() {
  // read per call (a call this size costs milliseconds): tests move it
  const char *e = lfa_param("LFA_HOST_REGISTER_BYTES");
  return e ? (size_t)strtoull(e, nullptr, 0) : (size_t)64 << 20;
}

// This call is done with registration i: the last user unregisters it (the
// pages stay in the table as DYING until hipHostUnregister has returned).
void temp_drop(int i) {
  if (i < 0) return;
  pthread_mutex_lock(&g_reg_lock);
  const bool last = --g_temp[i].refs == 0;
  if (last) g_temp[i].state = kRegDying;
  const void *p = g_temp[i].p;
  pthread_mutex_unlock(&g_reg_lock);
  if (!last) return;
  hipHostUnregister(const_cast<void *>(p));
  pthread_mutex_lock(&g_reg_lock);
  g_temp[i].state = kRegFree;
  pthread_mutex_unlock(&g_reg_lock);
}
}  // namespace

extern "C" {

int lfa_atomic_write_staged(enum lfa_op op, enum lfa_datatype dt, void *dst,
                            const void *src, size_t cnt, size_t chunk_bytes) {
  if ((unsigned)op >= LFA_WRITE_OP_CNT || (unsigned)dt >= LFA_DATATYPE_CNT ||
      !in_table(op, dt))
    return -LFA_EOPNOTSUPP;
  if (cnt && (!dst || !src)) return -LFA_EINVAL;
  if (!cnt) return 0;
  const size_t esz = lfa_datatype_size(dt);
  if (!chunk_bytes) chunk_bytes = 32u << 20;
  size_t per = chunk_bytes / esz;
  if (!per) per = 1;
  if (per > cnt) per = cnt;
  // chunk slots keep 256-byte alignment so the vector body applies
  const size_t slot = (per * esz + 255) & ~(size_t)255;
  int devno = 0;
  if (hipGetDevice(&devno) != hipSuccess || devno < 0 || devno >= kMaxDevices)
    return -LFA_EINVAL;
  const size_t bytes = cnt * esz;
  bool pd = false, ps = false;
  void *zd = nullptr, *zs = nullptr;
  int reg[2] = {-1, -1};
  if (zero_copy_on()) {
    pthread_mutex_lock(&g_reg_lock);
    zd = zero_copy_addr(dst, bytes, devno, &pd);
    zs = zero_copy_addr(src, bytes, devno, &ps);
    pthread_mutex_unlock(&g_reg_lock);
    if ((zd || pd) && (zs || ps) && (pd || ps) && bytes >= register_min_bytes() &&
        !__atomic_load_n(&g_staged_calls, __ATOMIC_RELAXED)) {
      // large pageable operands of a call that is alone are pinned for the
      // call: registration + the zero-copy combine beats the runtime's
      // staging of pageable memory (256 MiB 15.4 -> 11.5 ms,
      // profiles/r05_zero_copy_pageable.log).  Not below
      // LFA_HOST_REGISTER_BYTES, and not while another call is staging:
      // registering and unregistering stall every other caller's copies and
      // kernels (4 threads of 2 MiB: 29x one call registering, 3.7x
      // staging; profiles/r06_threads_probe_*.jsonl)
      if (pd) reg[0] = temp_take(dst, bytes, &zd, -1);
      if (ps && src == dst) zs = zd;
      else if (ps) reg[1] = temp_take(src, bytes, &zs, reg[0]);
    }
    if (!zd || !zs) {
      // stage instead
      zd = zs = nullptr;
      for (int &i : reg) temp_drop(i), i = -1;
    }
  }
  const bool staged = !(zd && zs);
  if (staged) __atomic_add_fetch(&g_staged_calls, 1, __ATOMIC_RELAXED);
  StagingCtx &c = staging_lock(devno);
  if (zd && zs) {
    // every operand reachable from the device: one combine over the mapped
    // buffers, no HBM round trip (256 MiB float SUM, both pinned: 9.96 ms
    // against 11.22 ms staged, profiles/r05_zero_copy.log)
    int ret = staging_acquire(c, 0);
    if (!ret) ret = kWrite[op](dt | LFA_WRITE_MAPPED, zd, zs, cnt, c.s_out);
    if (hipStreamSynchronize(c.s_out) != hipSuccess && !ret) ret = -LFA_EIO;
    pthread_mutex_unlock(&c.lock);
    for (int i : reg) temp_drop(i);
    return ret;
  }
  int ret = staging_acquire(c, 4 * slot);
  if (!ret) {
    for (int i = 0; i < 2; i++) hipEventRecord(c.out_done[i], c.s_out);
    for (size_t off = 0, k = 0; off < cnt && !ret; off += per, k ^= 1) {
      const size_t n = cnt - off < per ? cnt - off : per;
      char *dd = c.dev + k * 2 * slot, *ds = dd + slot;
      // slot reuse: the D2H of the chunk two back must have drained it
      hipStreamWaitEvent(c.s_in, c.out_done[k], 0);
      hipMemcpyAsync(dd, (char *)dst + off * esz, n * esz, hipMemcpyDefault, c.s_in);
      hipMemcpyAsync(ds, (const char *)src + off * esz, n * esz, hipMemcpyDefault,
                     c.s_in);
      hipEventRecord(c.in_done[k], c.s_in);
      hipStreamWaitEvent(c.s_out, c.in_done[k], 0);
      ret = kWrite[op](dt, dd, ds, n, c.s_out);
      hipMemcpyAsync((char *)dst + off * esz, dd, n * esz, hipMemcpyDefault, c.s_out);
      hipEventRecord(c.out_done[k], c.s_out);
    }
    if (hipStreamSynchronize(c.s_out) != hipSuccess && !ret) ret = -LFA_EIO;
    if (hipStreamSynchronize(c.s_in) != hipSuccess && !ret) ret = -LFA_EIO;
  }
  pthread_mutex_unlock(&c.lock);
  if (staged) __atomic_sub_fetch(&g_staged_calls, 1, __ATOMIC_RELAXED);
  return ret;
}

void *lfa_zero_copy_addr(const void *p, int device) {
  if (!p || !zero_copy_on()) return nullptr;
  bool pageable;
  pthread_mutex_lock(&g_reg_lock);
  void *r = zero_copy_addr(p, 1, device, &pageable);
  pthread_mutex_unlock(&g_reg_lock);
  return r;
}

int lfa__temp_registrations(void) {
  int n = 0;
  pthread_mutex_lock(&g_reg_lock);
  for (const TempReg &t : g_temp) n += t.state != kRegFree;
  pthread_mutex_unlock(&g_reg_lock);
  return n;
}

size_t lfa_host_small_bytes(void) {
  static size_t v = [] {
    const char *e = lfa_param("LFA_HOST_SMALL_BYTES");
    return e ? (size_t)strtoull(e, nullptr, 0) : (size_t)LFA_HOST_SMALL_DEFAULT;
  }();
  return v;
}

namespace {
constexpr int kParams = 64;
constexpr size_t kParamValueMax = 80;
// A value, once set, is never written again: a new value of the same name
// is a new string and the old one is kept (a caller may still be parsing it
// on another thread), so every pointer lfa_param returned stays valid and
// unchanged for the life of the process.  Sets are rare (provider init,
// tests), so what is kept stays small.
struct ParamSlot {
  char name[48];
  const char *value;  // null: not set (the environment shows through)
};
ParamSlot g_params[kParams];
pthread_mutex_t g_param_lock = PTHREAD_MUTEX_INITIALIZER;
}  // namespace

const char *lfa_param(const char *name) {
  if (!name) return nullptr;
  const char *v = nullptr;
  pthread_mutex_lock(&g_param_lock);
  for (const ParamSlot &p : g_params)
    if (p.value && !strcmp(p.name, name)) v = p.value;
  pthread_mutex_unlock(&g_param_lock);
  return v ? v : getenv(name);
}

int lfa_param_set(const char *name, const char *value) {
  if (!name || !*name || strlen(name) >= sizeof(ParamSlot::name) ||
      (value && strlen(value) >= kParamValueMax))
    return -LFA_EINVAL;
  char *copy = value ? strdup(value) : nullptr;
  if (value && !copy) return -LFA_ENOMEM;
  int ret = -LFA_ENOMEM;
  pthread_mutex_lock(&g_param_lock);
  ParamSlot *slot = nullptr;
  for (ParamSlot &p : g_params)
    if (p.name[0] && !strcmp(p.name, name)) slot = &p;
  if (!slot)
    for (ParamSlot &p : g_params)
      if (!p.name[0]) {
        slot = &p;
        strcpy(p.name, name);
        break;
      }
  if (slot) {
    slot->value = copy;  // the previous string, if any, is kept (above)
    copy = nullptr;
    ret = 0;
  }
  pthread_mutex_unlock(&g_param_lock);
  free(copy);
  return ret;
}

const char *lfa_version(void) {
  return "lfa-combine 0.2 gfx950 (LDS-DMA staged, 4 KiB/operand/wave, nt loads/stores)";
}

}  // extern "C"
