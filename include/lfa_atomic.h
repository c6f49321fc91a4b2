/*
 * lfa_atomic.h — C ABI of the MI355X combine kernels (liblfa.so).
 *
 * Drop-in for libfabric's element-wise combine tables, the L4 layer that
 * prov/coll's REDUCE work items call (prov/coll/src/coll_coll.c:758-768):
 *
 *   lfa_datatype_size()          replaces ofi_datatype_size()
 *                                  prov/util/src/util_atomic.c:58-64,
 *                                  include/ofi_atomic.h:45
 *   lfa_atomic_valid()           replaces ofi_atomic_valid() (write table)
 *                                  prov/util/src/util_atomic.c:1088-1140
 *   lfa_atomic_write_handlers    replaces ofi_atomic_write_handlers[op][dt]
 *                                  prov/util/src/util_atomic.c:907-922,
 *                                  include/ofi_atomic.h:73-82
 *                                (same signature; synchronous; dst/src are
 *                                 device OR host pointers, classified per
 *                                 call — see "The synchronous tables" below:
 *                                 device operands run the gfx950 kernels
 *                                 on the null stream, host operands the
 *                                 host loop or the staged HBM stream)
 *   lfa_atomic_write_async()     the GPU form: same semantics, enqueued on a
 *                                  HIP stream, returns 0 / negative errno
 *   lfa_atomic_readwrite_handlers / lfa_atomic_readwrite_async
 *                                replace ofi_atomic_readwrite_handlers
 *                                  (util_atomic.c:924-950)
 *   lfa_atomic_swap_handlers / lfa_atomic_swap_async
 *                                replace ofi_atomic_swap_handlers
 *                                  (util_atomic.c:952-980)
 *   lfa_reduce_tree_async()      N-input fused combine in prov/coll's
 *                                  recursive-doubling association order
 *                                  (coll_coll.c:349-449), one pass over HBM
 *   lfa_reduce_tree_put_async()  the same tree, result written to several
 *                                  outputs, system-scope accesses (peer HBM
 *                                  over xGMI; the LFA_ALGO_P2P kernel)
 *
 * Semantics are the shipping (HAVE_BUILTIN_MM_ATOMICS) table's, bit-exact:
 * dst-biased MIN/MAX, wrapping integer SUM/PROD, IEEE float/double with no
 * denormal flush, 0/1 logical results, bitwise ops on integers only, int128
 * columns as built with HAVE_BUILTIN_MM_INT128_ATOMICS.
 *
 * Buffers: any alignment (16-byte co-aligned buffers take the vector path),
 * dst updated in place, src read-only, no allocation.  Streams are passed as
 * `void *` (a hipStream_t; NULL = the null stream), so this header needs no
 * HIP include.
 */
#ifndef LFA_ATOMIC_H
#define LFA_ATOMIC_H

#include "lfa_fabric.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef void (*lfa_write_fn)(void *dst, const void *src, size_t cnt);

/* 0 and errno = EINVAL for datatype >= LFA_DATATYPE_CNT. */
size_t lfa_datatype_size(enum lfa_datatype datatype);

/* 0, -LFA_EOPNOTSUPP, -LFA_EBADFLAGS or -LFA_ENOSYS, as ofi_atomic_valid
 * (write table; LFA_FETCH_ATOMIC → fetch table; LFA_COMPARE_ATOMIC → compare
 * table). */
int lfa_atomic_valid(enum lfa_datatype datatype, enum lfa_op op, uint64_t flags);

/* Synchronous table form: [op][datatype], NULL where unsupported. */
extern lfa_write_fn const lfa_atomic_write_handlers[LFA_WRITE_OP_CNT][LFA_DATATYPE_CNT];

/*
 * The synchronous tables keep the reference's void signature, which has no
 * way to fail on the CPU.  On the GPU a call can (a HIP error, operands
 * mixing host and device memory): the first failure since the last call of
 * this function is kept per thread and returned here (a negative LFA_E*
 * code; -LFA_EIO for a HIP error, also named on stderr), and cleared.  0 when
 * every table call of this thread since then succeeded.
 */
int lfa_atomic_last_error(void);

/*
 * dst[i] = dst[i] OP src[i] for i < cnt, on `stream`.
 * Returns 0, -LFA_EOPNOTSUPP (no handler), -LFA_EINVAL (bad pointer/args),
 * -LFA_EIO (launch failure).
 */
int lfa_atomic_write_async(enum lfa_op op, enum lfa_datatype datatype,
			   void *dst, const void *src, size_t cnt, void *stream);

/*
 * dst[i] = tree(srcs[0][i], …, srcs[nsrc-1][i]) where tree is prov/coll's
 * recursive-doubling association for nsrc ranks (every pairwise step is
 * `higher-rank partial OP lower-rank partial`).  `srcs` is a HOST array of
 * DEVICE pointers; dst may alias any srcs[k].  1 <= nsrc <= LFA_TREE_MAX.
 * Any byte offset: operands not aligned to the element are moved byte-wise.
 */
#define LFA_TREE_MAX 32
int lfa_reduce_tree_async(enum lfa_op op, enum lfa_datatype datatype,
			  void *dst, const void *const *srcs, int nsrc,
			  size_t cnt, void *stream);

/*
 * The same tree, its result written to each of dsts[0..ndst).  Inputs and
 * outputs may be other GPUs' memory mapped over IPC (xGMI): every load and
 * store is system scope (sc0 sc1), so a peer ordered after this kernel (e.g.
 * by a stream-ordered barrier) reads the stored bytes.  `dsts`/`srcs` are
 * HOST arrays of device pointers; outputs must not alias inputs.
 * 1 <= nsrc <= LFA_TREE_MAX, 1 <= ndst <= LFA_PUT_MAX.  An operand not aligned
 * to the element is moved byte-wise with ordinary (device-scope) accesses, so
 * it must be this GPU's own memory — in the P2P schedules only the caller's
 * buffers can be; the peers' workspace slots are 256-B aligned.
 */
#define LFA_PUT_MAX 32
int lfa_reduce_tree_put_async(enum lfa_op op, enum lfa_datatype datatype,
			      void *const *dsts, int ndst, const void *const *srcs,
			      int nsrc, size_t cnt, void *stream);

/*
 * Fetch table — replaces ofi_atomic_readwrite_handlers (util_atomic.c:924-950):
 * res[i] = dst[i], then dst[i] = dst[i] OP src[i] (ATOMIC_READ: load only,
 * ATOMIC_WRITE: exchange).
 */
typedef void (*lfa_readwrite_fn)(void *dst, const void *src, void *res,
				 size_t cnt);
extern lfa_readwrite_fn const
	lfa_atomic_readwrite_handlers[LFA_READWRITE_OP_CNT][LFA_DATATYPE_CNT];
int lfa_atomic_readwrite_async(enum lfa_op op, enum lfa_datatype datatype,
			       void *dst, const void *src, void *res,
			       size_t cnt, void *stream);

/*
 * Compare table — replaces ofi_atomic_swap_handlers (util_atomic.c:952-980),
 * indexed [op - LFA_CSWAP][datatype]: res[i] = dst[i]; dst[i] = src[i] when
 * the compare holds.  LFA_CSWAP compares BITS, as the shipping
 * __atomic_compare_exchange does (-0.0 != +0.0; a NaN equals its own bits);
 * CSWAP_NE/LE/LT/GE/GT compare values (cmp OP dst); MSWAP writes
 * (src & cmp) | (dst & ~cmp).
 */
typedef void (*lfa_swap_fn)(void *dst, const void *src, const void *cmp,
			    void *res, size_t cnt);
extern lfa_swap_fn const
	lfa_atomic_swap_handlers[LFA_SWAP_OP_CNT][LFA_DATATYPE_CNT];
int lfa_atomic_swap_async(enum lfa_op op, enum lfa_datatype datatype,
			  void *dst, const void *src, const void *cmp,
			  void *res, size_t cnt, void *stream);

/*
 * Host-resident buffers (what prov/coll's REDUCE items see, coll_coll.c:763):
 * dst/src are streamed through HBM in `chunk_bytes` pieces (0 = 32 MiB) on
 * two HIP streams — chunk c+1's H2D overlaps chunk c's combine and D2H — and
 * the call returns when dst is updated.  When every operand is reachable
 * from the device — pinned (hipHostMalloc / hipHostRegister) host memory or
 * this device's memory — there is no staging: one combine runs on the mapped
 * buffers and reads / writes host memory over PCIe (zero-copy).  Pageable
 * operands are registered for the duration of the call and combined the same
 * way; if the runtime refuses the registration (e.g. dst and src share
 * pages) they are staged.  LFA_HOST_ZERO_COPY=0 forces the staged pipeline.
 * Returns 0 or a negative LFA_E* code.
 */
int lfa_atomic_write_staged(enum lfa_op op, enum lfa_datatype datatype,
			    void *dst, const void *src, size_t cnt,
			    size_t chunk_bytes);

/*
 * Host-memory forms (no GPU involved): the same element semantics as the
 * kernels — one functor source, lfa_ops.hpp — for operands that live in host
 * memory: the synchronous table's small host buckets and endpoints opened with
 * lfa_coll_domain_open_host.  Device pointers must not be passed here.
 * lfa_host_write:       dst[i] = dst[i] OP src[i]  (ofi_atomic_write_handler
 *                       argument order, util_atomic.c:907-922)
 * lfa_host_reduce_tree: dst = prov/coll's recursive-doubling tree of srcs
 *                       (coll_coll.c:349-449), 1 <= nsrc <= LFA_TREE_MAX
 * Return 0, -LFA_EOPNOTSUPP or -LFA_EINVAL.
 */
int lfa_host_write(enum lfa_op op, enum lfa_datatype datatype, void *dst,
		   const void *src, size_t cnt);
int lfa_host_reduce_tree(enum lfa_op op, enum lfa_datatype datatype, void *dst,
			 const void *const *srcs, int nsrc, size_t cnt);
/* Fetch and compare tables on host memory (res = old dst, as the
 * readwrite / swap handlers, util_atomic.c:924-980). */
int lfa_host_readwrite(enum lfa_op op, enum lfa_datatype datatype, void *dst,
		       const void *src, void *res, size_t cnt);
int lfa_host_swap(enum lfa_op op, enum lfa_datatype datatype, void *dst,
		  const void *src, const void *cmp, void *res, size_t cnt);

/*
 * The synchronous tables (lfa_atomic_write_handlers and the fetch / compare
 * tables) accept DEVICE or HOST pointers, classified per call with
 * hipPointerGetAttributes: device operands run the gfx950 kernels on the null
 * stream; host operands — what prov/coll's REDUCE items hand over
 * (coll_coll.c:758-768) — run the host loop while the bucket is at most
 * lfa_host_small_bytes() (env LFA_HOST_SMALL_BYTES, default below), and are
 * streamed through HBM (lfa_atomic_write_staged) above it.  Mixed write
 * operands also take the staged path.
 */
#define LFA_HOST_SMALL_DEFAULT (1u << 20)
size_t lfa_host_small_bytes(void);

/* Version string of the kernel library (build id, target arch). */
const char *lfa_version(void);

/*
 * Tuning parameters.  Every knob of liblfa.so and liblfa_coll.so (LFA_*,
 * DESIGN.md §5b's table) is read through lfa_param(name): a value set with
 * lfa_param_set, else the environment variable of that name.  The off_lfa
 * provider registers the deployer-facing ones with libfabric's parameter
 * system (fi_param_define, src/var.c:188-231) as FI_OFF_LFA_<NAME> — so they
 * show in `fi_info -e` — and hands what fi_param_get returns to
 * lfa_param_set before it opens a domain.  Most knobs are read once, at first
 * use: set them before the first collective of the process.
 * lfa_param_set: value NULL removes the setting; 0 or -LFA_EINVAL / -LFA_ENOMEM.
 * Both are thread-safe; a string lfa_param returned from a set value is never
 * changed or freed (a later set of the same name makes a new one).
 */
const char *lfa_param(const char *name);
int lfa_param_set(const char *name, const char *value);

#ifdef __cplusplus
}
#endif

#endif /* LFA_ATOMIC_H */
