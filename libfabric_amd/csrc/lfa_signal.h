/*
 * lfa_signal.h — device-side synchronisation over the LFA_ALGO_P2P symmetric
 * workspace (liblfa.so; called by liblfa_coll.so, not installed).
 *
 * Every member's workspace ends in a flag area of LFA_SIG_AREA_BYTES that its
 * peers map over IPC.  Word k of the barrier row is written only by group rank
 * k, with a per-group epoch that grows by one per barrier, so a rank waits on
 * its OWN memory (local polling) while its peers post into it over xGMI.
 * prov/coll's barrier is a zero-byte allreduce through the work queue
 * (coll_coll.c:997-1038); on device buffers the same ordering point is this
 * one-wave kernel on the endpoint stream instead of an RCCL collective.
 */
#ifndef LFA_SIGNAL_H
#define LFA_SIGNAL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LFA_SIG_MAX 32                  /* ranks (= LFA_TREE_MAX) */
#define LFA_SIG_AREA_BYTES (1u << 20)   /* flag area after the two regions */
#define LFA_SIG_BAR_OFF 0               /* barrier row: uint32[LFA_SIG_MAX] */
/* one-shot rows: uint32[LFA_SIG_OS_CHUNKS][LFA_SIG_MAX], word [b][k] written
 * by rank k's workgroup b */
#define LFA_SIG_OS_OFF 256
#define LFA_SIG_OS_CHUNKS 128
/* identity word: a value the owner writes before exporting the workspace
 * and sends with its handle, read back by every peer through its mapping
 * (lfa_coll.c sym_open) */
#define LFA_SIG_ID_OFF (LFA_SIG_AREA_BYTES - 64u)
#define LFA_OS_MAX_RANKS 8              /* one-shot groups: 1..8 members */
/*
 * LL one-shot (parts of at most LFA_OS_LL_BYTES): every 4 bytes of a part
 * travel as one 8-byte word {data, flag} with flag = 2·epoch + 1, written
 * and read whole, so the data's arrival is its own signal — no separate
 * flag, no acknowledgement wait before it, no second read.  The words live in
 * the flag area (zeroed at every workspace growth, never holding raw data):
 * per parity (epoch & 1) LFA_OS_MAX_RANKS slots of LFA_SIG_LL_SLOT bytes, the
 * slot of rank k holding what rank k sent.  A word left in a slot matches a
 * later operation's flag only 2^31 one-shots later at the same position (the
 * parity halves alternate, so consecutive uses differ by 2 epochs).  It relies
 * on an aligned 8-byte store reaching a peer whole, over xGMI as on one GPU.
 * Allreduce and reduce_scatter only, and only with LFA_OS_LL=1 in the
 * environment (the same on every member): measured slower than the flagged
 * kernel on one GPU (lfa_kernels.hpp ll_enabled).
 */
#define LFA_OS_LL_BYTES (16u << 10)
#define LFA_SIG_LL_SLOT (2u * LFA_OS_LL_BYTES)
#define LFA_SIG_LL_PARITY (LFA_OS_MAX_RANKS * LFA_SIG_LL_SLOT)
#define LFA_SIG_LL_OFF (64u << 10)
#if LFA_SIG_LL_OFF + 2 * LFA_SIG_LL_PARITY > LFA_SIG_ID_OFF || \
    LFA_SIG_OS_OFF + 4 * LFA_SIG_OS_CHUNKS * LFA_SIG_MAX > LFA_SIG_LL_OFF
#error "flag area layout"
#endif

/*
 * Timed-out waits.  *status is one host-mapped word per group holding the
 * lowest `ticket` (the group's P2P operation number, from 1) whose wait gave
 * up, LFA_SIG_NONE while none has.  Both are 64-bit, so no group ever hands
 * out a ticket equal to LFA_SIG_NONE or wraps to 0 (a 32-bit
 * ticket met 0xffffffff after 2^32 P2P operations and failed that one).  A kernel that times out lowers it to its
 * own ticket — the group's kernels run in stream order, so no two race on it
 * — and the host fails that operation and every later P2P operation of the
 * group, while the earlier ones complete normally.
 */
#define LFA_SIG_NONE 0xffffffffffffffffull	/* 64-bit: never reached by a ticket */

/*
 * Enqueue a barrier on `stream`: after the steps before it on every member's
 * stream, before the steps after it.  post[k] (k != rank) = this rank's word
 * in peer k's barrier row (IPC-mapped); wait = this rank's own barrier row.
 * A peer that has not posted `epoch` within timeout_us makes the kernel lower
 * *status to `ticket` and return.  0 or -LFA_E*.
 */
int lfa_flag_barrier_async(uint32_t *const *post, const uint32_t *wait, int n,
			   int rank, uint32_t epoch, uint64_t *status, uint64_t ticket,
			   uint64_t timeout_us, void *stream);

/*
 * One-shot reduction (LFA_STEP_ONESHOT) of `count` elements, ONE kernel:
 * workgroup b pushes chunk b of the part of this rank's input that member k
 * reduces into slot `rank` of member k's SYM_IN (system-scope stores over
 * xGMI), posts `epoch` into row b of every peer's one-shot rows, waits for
 * every peer's post in its own row b, then reduces chunk b of its own part
 * over all ranks' inputs — its own slots, its own input for itself — in
 * prov/coll's association order into `result`.  The part of member k: the
 * whole vector (mode LFA_ONESHOT_ALL, allreduce), block k of
 * lfa_coll_block's partition (LFA_ONESHOT_SCATTER, reduce_scatter: result
 * receives this rank's block), or the whole vector for k == mode only
 * (reduce to root `mode`).  n = 1 is the degenerate group: no pushes, no
 * flags, no workspace (sym and status may be NULL) — the part is copied into
 * `result` in one launch, the small-bucket path of a one-member group.
 * Slots are double-buffered by epoch parity in two
 * FIXED halves of SYM_IN: member j holds rank k's part of epoch e at
 * sym[j] + (e & 1)·parity_off + k·slot_bytes, so a peer one operation ahead
 * never overwrites a slot still being read.  The halves must not move with
 * the slot size: with a parity-p base of p·n·slot_bytes, a small operation
 * after a large one put its odd slots inside the large one's even slots,
 * which the slower members were still reading (wrong results in the mixed
 * in-flight test, round 3).  Needs n·slot_bytes <= parity_off.
 */
#ifndef LFA_ONESHOT_ALL                 /* also in lfa_coll.h */
#define LFA_ONESHOT_ALL (-1)
#define LFA_ONESHOT_SCATTER (-2)
#endif
struct lfa_oneshot {
	const void *send;       /* this rank's input, count elements */
	void *result;           /* this rank's part of the result */
	size_t count;
	int mode;               /* LFA_ONESHOT_ALL / _SCATTER / root */
	char *const *sym;       /* [n]: every member's workspace as mapped here */
	size_t slot_bytes;      /* one slot: the largest part, rounded up to 256 */
	size_t parity_off;      /* odd epochs' slots: this far above the even ones */
	size_t flag_off;        /* the flag area's offset in a workspace */
	int n, rank;            /* 1 <= n <= LFA_OS_MAX_RANKS */
	uint32_t epoch;         /* this group's one-shot operations so far + 1 */
	uint64_t *status;       /* host-mapped; lowered to ticket on a timeout */
	uint64_t ticket;        /* this P2P operation's number in the group */
	uint64_t timeout_us;
	/* Completion word, optional (done_word NULL: none):
	 * every workgroup, its result stores acknowledged and released at
	 * system scope, counts itself in *done_ctr (device memory, 0 at rest);
	 * the last one resets it and stores done_val into *done_word
	 * (host-mapped), so the host sees the operation complete with one
	 * memory read, without an event record / query per operation. */
	uint32_t *done_ctr;
	uint64_t *done_word;
	uint64_t done_val;
};
int lfa_oneshot_reduce_async(int op, int datatype, const struct lfa_oneshot *a,
				void *stream);

/* The address device `device`'s kernels use for p without staging (liblfa,
 * lfa_capi.cpp): pinned or registered host memory through its device mapping,
 * that device's own memory as it is; NULL for pageable memory, another
 * device's, or LFA_HOST_ZERO_COPY=0.  Never a registration lfa_atomic_write_staged
 * made for one call of its own. */
void *lfa_zero_copy_addr(const void *p, int device);
/* Flag on the datatype argument of liblfa's internal per-op write entries
 * (lfa__write_op<N>): the operands are host memory on its device mapping. */
#define LFA_WRITE_MAPPED 0x10000
/* Temporary registrations lfa_atomic_write_staged holds right now (tests:
 * 0 once every call has returned). */
int lfa__temp_registrations(void);

/*
 * A one-member group's small reducing collective (allreduce, reduce and
 * reduce_scatter of one rank are each a copy of the input): `bytes` from
 * send to result in one launch of a few workgroups that ends in the
 * completion word, as struct lfa_oneshot's done_* fields describe.  The
 * same result as the one-shot kernel with n = 1 for every (op, datatype),
 * with 48 bytes of kernel arguments instead of ~700 (about
 * 1 us of launch-to-word latency).  Any alignment.  0 or -LFA_E*.
 */
int lfa_solo_copy_async(void *result, const void *send, size_t bytes, uint32_t *done_ctr,
			uint64_t *done_word, uint64_t done_val, void *stream);

/* The solo copy's workgroup count (lfa_solo_body.hpp): 16 KiB per workgroup
 * when both pointers are 16-B aligned, 4 KiB otherwise. */
static inline uint32_t lfa_solo_blocks(const void *result, const void *send, size_t bytes)
{
	const size_t tile = (((uintptr_t)result | (uintptr_t)send) & 15) ? 4096 : 16384;

	return (uint32_t)((bytes + tile - 1) / tile);
}

#ifdef __HIPCC__
/* A wait of operation `ticket` gave up: lower the group's status word to it
 * (plain system-scope load and store: the group's kernels are stream-ordered,
 * and every lane of one kernel that times out stores the same ticket). */
static __device__ __forceinline__ void lfa_sig_note_timeout(uint64_t *status,
							     uint64_t ticket)
{
	if (__hip_atomic_load(status, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) > ticket)
		__hip_atomic_store(status, ticket, __ATOMIC_RELAXED,
				   __HIP_MEMORY_SCOPE_SYSTEM);
}
#endif

/*
 * Direct dispatch (lfa_direct.cpp): lfa_solo_copy_async's kernel launched
 * with this library's own AQL packet on its own HSA queue of `device` instead
 * of a HIP stream — no ordering with any stream; kernels on the queue run in
 * order.  open returns NULL where the queue cannot be set up (the caller keeps
 * the HIP launch).  done_ctr must not be shared with kernels on other queues.
 */
struct lfa_direct;
struct lfa_direct *lfa_direct_open(int device);
/* 0, -LFA_EINVAL, or -LFA_EIO: the queue has failed (a runtime queue error,
 * or a full ring that did not drain within LFA_SIG_TIMEOUT_MS); nothing was
 * enqueued, and the caller launches through HIP instead. */
int lfa_direct_solo_copy(struct lfa_direct *d, void *result, const void *send, size_t bytes,
			 uint32_t *done_ctr, uint64_t *done_word, uint64_t done_val);
/* Nonzero once the queue has failed: the words its packets owe may never
 * come (the provider fails those operations with EIO). */
int lfa_direct_failed(const struct lfa_direct *d);
void lfa_direct_close(struct lfa_direct *d);
/* Test hooks: mark a queue failed; a stub queue without HSA whose read index
 * is *read_index and whose ring bound is timeout_ms (CPU tests), and the
 * packets written to it. */
void lfa__direct_mark_failed(struct lfa_direct *d);
struct lfa_direct *lfa__direct_stub_open(const volatile uint64_t *read_index,
					 uint64_t timeout_ms);
uint64_t lfa__direct_stub_written(const struct lfa_direct *d);

/* GPU wall-clock ticks per microsecond (the kernels' timeout unit). */
uint64_t lfa__wallclock_ticks_per_us(void);
/* LFA_SIG_AREA_BYTES, for callers that build a workspace by hand (tests). */
size_t lfa__sig_area_bytes(void);

#ifdef __cplusplus
}
#endif

#endif
