/*
 * lfa_coll.h — C ABI of the MI355X collective provider (liblfa_coll.so).
 *
 * The host side of libfabric's software-collective path (prov/coll), in C,
 * driving RCCL over xGMI for transport and the gfx950 combine kernels of
 * liblfa.so (include/lfa_atomic.h) for every reduction.
 *
 * Reference interfaces each entry point replaces:
 *
 *   lfa_barrier / lfa_broadcast / lfa_allreduce / lfa_allgather /
 *   lfa_reduce_scatter / lfa_reduce
 *       struct fi_ops_collective slots, include/rdma/fi_collective.h:92-139;
 *       prov/coll implementations coll_ep_barrier (coll_coll.c:1035),
 *       coll_ep_allreduce (:1040-1085), coll_ep_allgather (:1087),
 *       coll_ep_broadcast (:1158-1216); reduce / reduce_scatter are
 *       fi_coll_no_* in the reference (coll_ep.c:75-76) — new here, with the
 *       semantics of man/fi_collective.3.md:354-404.
 *   lfa_query_collective   coll_query_collective, coll_coll.c:1267-1318
 *   lfa_join_collective    coll_join_collective, coll_coll.c:912-995
 *                          (group id = lowest common free id of the 256-bit
 *                          cid masks, agreed by a UINT8 BAND allreduce)
 *   lfa_cq_read / lfa_cq_readerr / lfa_eq_read
 *                          the completions the reference writes to the peer
 *                          CQ (coll_collective_comp, :722-756) and EQ
 *                          (coll_join_comp, :690-720)
 *   lfa_coll_plan          the schedule builder (coll_do_allreduce,
 *                          :349-449, and friends): a rank's work queue of
 *                          SEND/RECV/REDUCE/TREE/COPY items, as data
 *
 * Argument meaning and errors follow libfabric: calls return 0 (work queued,
 * completion reported later through lfa_cq_read with the caller's context)
 * or a negative LFA_E* errno; -LFA_EAGAIN is retryable.
 *
 * Buffers: `buf`/`result` may be device memory (hipMalloc, the data path of
 * this provider) or host memory (staged through HBM in pipelined chunks).
 * `desc`/`result_desc` are accepted and ignored, as in prov/coll.
 */
#ifndef LFA_COLL_H
#define LFA_COLL_H

#include <sys/types.h>
#include "lfa_fabric.h"

#ifdef __cplusplus
extern "C" {
#endif

struct lfa_coll_domain;
struct lfa_coll_ep;
struct lfa_coll_mc;

/* Algorithms for reducing collectives. */
enum lfa_coll_algo {
	/* default: per-rank block exchange over RCCL grouped send/recv, ONE
	 * fused N-input combine kernel per block in prov/coll's
	 * recursive-doubling association order, then block all-gather.
	 * Bit-identical to the reference for every op and datatype. */
	LFA_ALGO_TREE = 0,
	/* the reference's own schedule (coll_coll.c:349-449): log2(N)
	 * full-buffer pairwise exchanges, each followed by the binary combine
	 * kernel (and COPY), exactly as prov/coll orders its work items. */
	LFA_ALGO_RD = 1,
	/* RCCL's own reduction (ncclAllReduce / ncclReduceScatter /
	 * ncclReduce) for SUM/PROD/MIN/MAX on RCCL datatypes: fastest, but
	 * ring association order (float results within the documented
	 * tolerance, not bit-identical); other ops fall back to TREE. */
	LFA_ALGO_RCCL = 2,
	/* LFA_ALGO_TREE with the block exchange and the block all-gather done
	 * by RCCL's own ncclAllToAll / in-place ncclAllGather instead of
	 * grouped ncclSend/ncclRecv (when count divides evenly over the
	 * group), and small allreduces gathering every input with one
	 * ncclAllGather; otherwise identical to LFA_ALGO_TREE.  Same bits. */
	LFA_ALGO_TREE_COLL = 3,
	/* direct xGMI peer access, same tree and bits as LFA_ALGO_TREE: each
	 * rank stages its input in a symmetric workspace whose peers map it
	 * over IPC (hipIpcOpenMemHandle); rank r's kernel reads block r of
	 * every rank's input straight from peer HBM, reduces it and writes
	 * (pushes) the result block into every rank's workspace in the same
	 * pass; two stream-ordered barriers per operation, each a one-wave
	 * flag kernel on the workspace (no RCCL collective).  Small buckets
	 * (allreduce / reduce <= 2 MiB over all members, reduce_scatter <=
	 * 4 MiB per member, 2..8 members; LFA_OS_AG_BYTES / LFA_OS_RS_BYTES,
	 * FI_OFF_LFA_ONESHOT_*) are ONE kernel: push into the peers' slots,
	 * flags, tree.  No intermediate transport copies, xGMI in and out
	 * directions busy at once. */
	LFA_ALGO_P2P = 4,
	/* the default on device domains: per operation, LFA_ALGO_P2P's
	 * one-kernel path for small buckets (allreduce / reduce of <= 2 MiB
	 * summed over the members, reduce_scatter of <= 4 MiB, 2..8 members)
	 * and, above them, LFA_ALGO_P2P's two-barrier schedule for groups of
	 * 2..32 (since round 6; lfa_coll_auto_bulk, LFA_AUTO_BULK=tree for
	 * LFA_ALGO_TREE as in rounds 3-5).  The choice depends only on
	 * (collective, count, members, datatype size) — lfa_coll_auto_algo —
	 * and on the group's P2P state, itself agreed by every member: the
	 * first P2P operation sets up the IPC workspaces with a MIN agreement
	 * over the members, and if any member cannot map a peer's workspace
	 * every member runs TREE from then on.  Same bits either way.  Peer
	 * domains run LFA_ALGO_TREE. */
	LFA_ALGO_AUTO = 5,
};

/* LFA_ALGO_AUTO's choice for one operation: LFA_ALGO_P2P or LFA_ALGO_TREE.
 * p2p_ok: the group's agreed P2P state (0 once the workspace agreement
 * failed).  Pure; every member computes the same (LFA_AUTO_BULK must agree
 * across the members, as every knob that shapes a schedule). */
int lfa_coll_auto_algo(enum lfa_collective_op coll, size_t count, int nranks,
		       size_t esz, int p2p_ok);
/* AUTO's choice above the one-shot bounds: LFA_ALGO_P2P (default) or
 * LFA_ALGO_TREE (LFA_AUTO_BULK=tree, FI_OFF_LFA_AUTO_BULK). */
int lfa_coll_auto_bulk(void);

/* ---- bootstrap (replaces fi_getinfo/fi_fabric/fi_domain/fi_endpoint
 *      and AV insertion for this path) ---------------------------------- */

/* Bytes of the opaque unique id rank 0 creates and every rank passes in. */
#define LFA_UNIQUE_ID_BYTES 128
int lfa_coll_get_unique_id(void *id, size_t len);

int lfa_coll_domain_open(int device, int rank, int nranks, const void *id,
			 size_t id_len, struct lfa_coll_domain **domain);

/*
 * Peer transfer: a domain whose buffers are HOST memory and whose transport
 * is the owner provider's tagged messaging — prov/coll's own configuration,
 * where SEND/RECV work items become fi_tsendmsg / fi_trecvmsg(FI_PEER_TRANSFER)
 * on the host provider's endpoint (coll_coll.c:770-814) and completions come
 * back through peer_ops->complete (coll_coll.c:1218-1241).
 *
 * send / recv post one transfer of `bytes` to / from domain rank `peer` with
 * prov/coll's tag (coll_form_tag, coll_coll.c:37-45: the operation's cid
 * (group_id << 16 | seq) | the SENDING group rank << 32) and store a handle
 * in *req; messages between one pair with one tag match in posting order.
 * test returns 1 once the transfer behind `req` has completed (the handle is
 * then released), 0 while pending, or a negative LFA_E* code.
 *
 * Endpoints of such a domain run each collective's schedule on the host:
 * transfers through these callbacks, REDUCE / TREE items through
 * lfa_host_write / lfa_host_reduce_tree (include/lfa_atomic.h), progressed by
 * lfa_cq_read as prov/coll progresses in fi_cq_read.  LFA_ALGO_RCCL runs as
 * LFA_ALGO_TREE, and so does LFA_ALGO_P2P on a domain without a GPU (on a
 * GPU peer domain it keeps its schedule, see lfa_coll_domain_open_peer);
 * LFA_ALGO_TREE_COLL's collective items become grouped sends/receives.
 */
struct lfa_peer_xfer_ops {
	int (*send)(void *ctx, int peer, const void *buf, size_t bytes,
		    uint64_t tag, void **req);
	int (*recv)(void *ctx, int peer, void *buf, size_t bytes, uint64_t tag,
		    void **req);
	int (*test)(void *ctx, void *req);
};
int lfa_coll_domain_open_host(int rank, int nranks,
			      const struct lfa_peer_xfer_ops *ops, void *ctx,
			      struct lfa_coll_domain **domain);
/* The same on GPU `device` (< 0: lfa_coll_domain_open_host): collectives
 * whose buffers are device memory then run the same schedule with the local
 * items as the gfx950 kernels on the endpoint's stream, and every transfer
 * staged through host memory (device -> host before a send, host -> device
 * after a receive), so the owner only ever moves host bytes — prov/coll over
 * an owner without FI_HMEM.  Host buffers keep the host combine.  A buffer
 * pair must be both device or both host memory (-LFA_EINVAL otherwise);
 * members may differ from one another.  LFA_ALGO_P2P keeps its schedule
 * here: the members map each other's symmetric workspaces over IPC (the
 * handshake runs from progress calls), its barriers and small buckets are
 * GPU-side flag kernels on those workspaces (no owner transfers), a
 * host-buffer member is staged through device copies, and a P2P
 * operation starts once the endpoint's earlier operations have finished. */
int lfa_coll_domain_open_peer(int device, int rank, int nranks,
			      const struct lfa_peer_xfer_ops *ops, void *ctx,
			      struct lfa_coll_domain **domain);
/* Ranks in the RCCL communicator of a device domain (ncclCommCount): what
 * RCCL itself sees, beside the rank count the caller passed.  0,
 * -LFA_EINVAL, -LFA_EOPNOTSUPP (peer-transfer domain), -LFA_EIO. */
int lfa_coll_domain_comm_count(struct lfa_coll_domain *d, int *count);
int lfa_coll_domain_close(struct lfa_coll_domain *domain);

/* An endpoint owns one HIP stream (its progress context), a work-item
 * workspace in HBM and a completion queue. */
int lfa_coll_ep_open(struct lfa_coll_domain *domain, struct lfa_coll_ep **ep);
int lfa_coll_ep_close(struct lfa_coll_ep *ep);
/* The endpoint's HIP stream (hipStream_t), for callers that order work. */
void *lfa_coll_ep_stream(struct lfa_coll_ep *ep);
/* The algorithm picks the schedule, so every member of a group must use the
 * same one when it issues a collective (as every rank of an RCCL
 * communicator issues the same calls); the buffers' memory type and the
 * chunk size need not agree.  LFA_ALGO_P2P on peer domains also needs every
 * member's domain on a GPU (lfa_coll_domain_open_peer with a device): a
 * domain without one runs it as LFA_ALGO_TREE, a different schedule. */
int lfa_coll_ep_set_algo(struct lfa_coll_ep *ep, enum lfa_coll_algo algo);
/* Host-staging chunk size in bytes (0 = default 32 MiB) of a ONE-member
 * group: H2D, collective and D2H of consecutive chunks overlap. */
int lfa_coll_ep_set_chunk(struct lfa_coll_ep *ep, size_t bytes);
/* The GROUP chunk, in bytes: LFA_GROUP_CHUNK_AUTO (the default), 0 = off,
 * or a size (also read from LFA_GROUP_CHUNK_BYTES at endpoint open).  AUTO
 * is lfa_coll_group_chunk's rule, a function of the operation's byte count
 * alone, so every member derives the same chunk.  A chunked member issues one
 * device collective per chunk, so in a group of N > 1 chunking must be a
 * group-wide choice: with a group chunk set — the SAME value on every
 * member, like the collectives themselves — every member, whatever memory
 * its buffers are in, splits allreduce / reduce / broadcast / equal-block
 * reduce_scatter of more than one chunk into the same chunks
 * (lfa_coll_member_chunk): host members pipeline H2D / collective / D2H
 * across them, device members run the chunks back to back on their buffers
 * (reduce_scatter's 2-D chunks staged on the device).  Every element meets
 * the same schedule as unchunked, so results are bit-identical.  Off, a
 * group of N > 1 stages host buffers whole (one chunk).  The result the
 * reference defines stays the same: prov/coll copies host buffers whole
 * (coll_coll.c:364, 1058). */
int lfa_coll_ep_set_group_chunk(struct lfa_coll_ep *ep, size_t bytes);
#define LFA_GROUP_CHUNK_AUTO ((size_t)-1)
/* The group chunk an operation of `bytes` (count × datatype size, the
 * per-member input) runs with in a group of `nranks` under the setting
 * `group_chunk` (0 = none): AUTO gives LFA_AUTO_CHUNK_BYTES (32 MiB) to
 * operations of at least twice that in groups of N > 1, none otherwise; a
 * size is used as it is.  Pure: the same on every member. */
#define LFA_AUTO_CHUNK_BYTES ((size_t)32 << 20)
size_t lfa_coll_group_chunk(size_t group_chunk, int nranks, size_t bytes);
/* The chunk, in bytes, a member stages an operation with (0 = one chunk,
 * the whole buffer): the group chunk when there is one (every member; pass
 * lfa_coll_group_chunk's result), otherwise the local chunk for a host
 * member of a one-member group, otherwise 0.  Pure: what
 * tests/test_coll_plan.py replays for mixed members. */
size_t lfa_coll_member_chunk(int nranks, int host, size_t group_chunk,
			     size_t local_chunk);

/* ---- groups (fi_join_collective) -------------------------------------- */

/* Form a group from the parent `coll_addr` (LFA_ADDR_NOTAVAIL = the world
 * group).  `ranks` (`nmembers` distinct parent ranks, in any order) selects
 * the members and numbers them: ranks[i] becomes group rank i — prov/coll's
 * local_rank is the member's index in the joined av_set's address array
 * (coll_find_local_rank, coll_coll.c:669-689), so a set built as stride
 * {0, 2, 4} plus an inserted 1 numbers parent rank 1 as group rank 3.  Group
 * ranks decide the block order of allgather / scatter / reduce_scatter, the
 * tree's association order and what a root_addr names.  NULL = all, in parent
 * order.  EVERY parent rank calls it with the same list — the
 * group id is agreed by a UINT8 BAND allreduce of the free-id masks over the
 * parent, as coll_join_collective does (coll_coll.c:969-973).  Non-members
 * get a handle too, but collectives on it return -LFA_EINVAL.
 * Completion: an LFA_JOIN_COMPLETE event on lfa_eq_read. */
#define LFA_JOIN_COMPLETE 6
int lfa_join_collective(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
			const int *ranks, size_t nmembers, uint64_t flags,
			struct lfa_coll_mc **mc, void *context);
/* The same group formed by its MEMBERS ONLY: prov/coll's join whose parent is
 * the av_set's own address (coll_av_set_addr, coll_av_set.c:166-175, taken as
 * the parent at coll_coll.c:939-941), so the free-id BAND runs over the new
 * group itself and the rest of `coll_addr`'s group does not call anything
 * (fabtests core_coll.c:138-178, the stride test).  `ranks` are distinct ranks
 * of `coll_addr`'s group in group-rank order, as above, and must include the
 * caller.  The agreement travels
 * under group id 256 (outside the 0..255 ids a join hands out), so it cannot
 * meet a joined group's traffic.  On a device domain a strict subset gets an
 * RCCL communicator of its own (the first member's unique id sent to the
 * others point-to-point over the parent's communicator, then
 * ncclCommInitRank among the members); the whole group splits as usual. */
int lfa_join_members(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
		     const int *ranks, size_t nmembers, uint64_t flags,
		     struct lfa_coll_mc **mc, void *context);
lfa_addr_t lfa_mc_addr(struct lfa_coll_mc *mc);
/* The group id the join agreed on (util_coll_mc.group_id, ofi_util.h:849-856;
 * the world group is 0), or -LFA_EAGAIN before the join completed. */
int lfa_mc_group_id(struct lfa_coll_mc *mc);
int lfa_mc_close(struct lfa_coll_mc *mc);
/* The world group, usable without a join (the reference's av_set coll_mc). */
lfa_addr_t lfa_coll_world_addr(struct lfa_coll_ep *ep);

/* What the group's LFA_ALGO_P2P operations ran on this member so far
 * (prov/coll keeps no collective counters; these let a caller see which
 * path a bucket took): one-shot kernels (small buckets in one launch),
 * flag barriers, and P2P operations in total.  timed_out is 1 once a wait
 * of the group gave up (the group then refuses P2P operations). */
struct lfa_mc_counters {
	uint64_t p2p_ops;
	uint64_t oneshot;
	uint64_t flag_barriers;
	int timed_out;
};
int lfa_mc_counters(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
		    struct lfa_mc_counters *out);
/* Test entry: the group's P2P ticket count continues from `ticket` (every
 * member must seed the same value before the group's next P2P operation).
 * Tickets and the timed-out status word are 64-bit; this lets a test run
 * operations across 2^32 without issuing 4 billion of them.  0 or
 * -LFA_EINVAL (unknown group, or operations of the group in flight). */
int lfa_mc_seed_ticket(struct lfa_coll_ep *ep, lfa_addr_t coll_addr, uint64_t ticket);
/* Test entry for the completion-word error path.  Small operations complete
 * through a host-mapped word instead of an event; one whose word does not
 * come within the bound (LFA_SIG_TIMEOUT_MS, default 20 s) completes once, in
 * error, through lfa_cq_readerr (err ETIMEDOUT; EIO when the queue owing it
 * failed).  drop_next: the next drop_next word operations wait for a value
 * their word never reaches; timeout_ms > 0: this endpoint's bound;
 * fail_direct: mark the endpoint's direct queue failed (as a runtime queue
 * error would).  0 or -LFA_EINVAL. */
int lfa_coll_ep_test_word(struct lfa_coll_ep *ep, int drop_next, long timeout_ms,
			  int fail_direct);
/* Test entry: a one-member group's reducing collectives of at most
 * max_bytes run as the solo copy (default LFA_SOLO_BYTES, 4 MiB); 0 sends
 * them through the schedule of the endpoint's algorithm instead — under
 * LFA_ALGO_P2P the one-shot kernel at n = 1 and its completion word, the
 * device-domain one-shot path that otherwise needs two GPUs.  0 or
 * -LFA_EINVAL. */
int lfa_coll_ep_test_solo(struct lfa_coll_ep *ep, size_t max_bytes);
/* 1 when the endpoint's one-member small operations go through the direct
 * queue, 2 when that queue has failed (they take the HIP launch), 0 when it
 * was never opened (diagnostics, tests). */
int lfa_coll_ep_uses_direct(struct lfa_coll_ep *ep);
/* Operations of the endpoint reaped through a completion word rather than
 * an event (diagnostics: which completion path small buckets took). */
uint64_t lfa_coll_ep_word_ops(struct lfa_coll_ep *ep);

/* ---- fi_ops_collective ------------------------------------------------ */

ssize_t lfa_barrier(struct lfa_coll_ep *ep, lfa_addr_t coll_addr, void *context);
ssize_t lfa_broadcast(struct lfa_coll_ep *ep, void *buf, size_t count,
		      void *desc, lfa_addr_t coll_addr, lfa_addr_t root_addr,
		      enum lfa_datatype datatype, uint64_t flags, void *context);
ssize_t lfa_allreduce(struct lfa_coll_ep *ep, const void *buf, size_t count,
		      void *desc, void *result, void *result_desc,
		      lfa_addr_t coll_addr, enum lfa_datatype datatype,
		      enum lfa_op op, uint64_t flags, void *context);
ssize_t lfa_allgather(struct lfa_coll_ep *ep, const void *buf, size_t count,
		      void *desc, void *result, void *result_desc,
		      lfa_addr_t coll_addr, enum lfa_datatype datatype,
		      uint64_t flags, void *context);
/* `count` = elements each rank contributes; rank r receives the block
 * [off(r), off(r+1)) of the reduced vector, off() splitting `count` into
 * nranks contiguous blocks, the first count % nranks one element longer
 * (lfa_coll_block). */
ssize_t lfa_reduce_scatter(struct lfa_coll_ep *ep, const void *buf,
			   size_t count, void *desc, void *result,
			   void *result_desc, lfa_addr_t coll_addr,
			   enum lfa_datatype datatype, enum lfa_op op,
			   uint64_t flags, void *context);
/* Full reduced vector lands in `result` at root_addr (a group rank) only. */
ssize_t lfa_reduce(struct lfa_coll_ep *ep, const void *buf, size_t count,
		   void *desc, void *result, void *result_desc,
		   lfa_addr_t coll_addr, lfa_addr_t root_addr,
		   enum lfa_datatype datatype, enum lfa_op op, uint64_t flags,
		   void *context);
/* coll_ep_scatter (prov/coll/src/coll_coll.c:1121-1156): root's buf holds
 * nranks blocks of `count` elements; block r lands in rank r's result. */
ssize_t lfa_scatter(struct lfa_coll_ep *ep, const void *buf, size_t count,
		    void *desc, void *result, void *result_desc,
		    lfa_addr_t coll_addr, lfa_addr_t root_addr,
		    enum lfa_datatype datatype, uint64_t flags, void *context);

int lfa_query_collective(struct lfa_coll_domain *domain,
			 enum lfa_collective_op coll,
			 struct lfa_collective_attr *attr, uint64_t flags);

/* ---- completions ------------------------------------------------------ */

/* Mirrors struct fi_cq_data_entry (include/rdma/fi_eq.h:215-222). */
struct lfa_cq_entry {
	void *op_context;
	uint64_t flags;      /* LFA_COLLECTIVE */
	size_t len;
	void *buf;
	uint64_t data;
};
struct lfa_cq_err_entry {
	void *op_context;
	uint64_t flags;
	int err;             /* positive LFA_E* */
	int prov_errno;      /* hipError_t / ncclResult_t */
};
struct lfa_eq_entry {        /* mirrors struct fi_eq_entry */
	void *fid;           /* the lfa_coll_mc */
	void *context;
	uint64_t data;
};

/* Progresses the endpoint and returns completed entries (>0), or
 * -LFA_EAGAIN when none are ready, or -LFA_EIO when an error entry waits
 * (read it with lfa_cq_readerr). */
ssize_t lfa_cq_read(struct lfa_coll_ep *ep, struct lfa_cq_entry *buf,
		    size_t count);
ssize_t lfa_cq_readerr(struct lfa_coll_ep *ep, struct lfa_cq_err_entry *buf);
ssize_t lfa_eq_read(struct lfa_coll_ep *ep, uint32_t *event,
		    struct lfa_eq_entry *entry);
/* Blocks until every queued operation has completed (convenience); on a GPU
 * peer domain it also frees the idle staging buffers. */
int lfa_coll_ep_flush(struct lfa_coll_ep *ep);
/* Device bytes a GPU peer domain's staging pool holds (busy and idle):
 * bounded by what operations in flight use plus 1 GiB kept idle, and 0 idle
 * after lfa_coll_ep_flush (diagnostics, tests). */
size_t lfa_coll_ep_stage_bytes(struct lfa_coll_ep *ep);
/* Device bytes of released P2P workspaces this process keeps for reuse
 * (LFA_WS_CACHE_BYTES, default 4 GiB; 0 frees them).  While a GPU domain is
 * open, an exported workspace is never handed back to the allocator below
 * the cache and quarantine caps: a fresh allocation at a once-exported
 * address may be refused an export, or exported as the earlier memory
 * (DESIGN.md §12).  0 after the process's last GPU domain closes.
 * Diagnostics, tests. */
size_t lfa_coll_ws_cached_bytes(void);
/* Device bytes of released P2P workspaces held but never reused: those of
 * groups whose P2P wait timed out (a stalled peer may still post into them),
 * and those evicted above the cache's cap (LFA_WS_QUARANTINE_BYTES, default
 * 4 GiB).  Both kinds are freed when the process's last GPU domain closes.
 * Diagnostics, tests. */
size_t lfa_coll_ws_quarantined_bytes(void);
/* The allocation flags P2P workspaces are made with (LFA_WS_MEM, read once
 * per process): hipDeviceMallocUncached (3, the default),
 * hipDeviceMallocFinegrained (1) or hipDeviceMallocDefault (0, coarse).
 * Every byte of a workspace is written by peers over xGMI while its owner's
 * kernels run. */
int lfa_coll_ws_mem(void);
/* A group's P2P workspaces as this member maps them (diagnostics, tests):
 * the kind they were allocated with, the region size (0: none yet), and
 * hipPointerGetAttributes' allocationFlags of each member's workspace as
 * mapped here (its own allocation at this rank, the IPC mappings of the
 * others).  0 or -LFA_E*. */
struct lfa_ws_info {
	int mem;
	int mapped;                     /* workspaces mapped here, own included */
	size_t region;
	unsigned alloc_flags[32];       /* [group rank] */
};
int lfa_mc_ws_info(struct lfa_coll_ep *ep, lfa_addr_t coll_addr, struct lfa_ws_info *out);

/* ---- schedules as data ------------------------------------------------ */

enum lfa_step_type {
	LFA_STEP_SEND = 0,     /* bytes from src to peer                     */
	LFA_STEP_RECV = 1,     /* bytes from peer into dst                   */
	LFA_STEP_GROUP_END = 2,/* the SEND/RECVs since the last GROUP_END run
				  concurrently (one RCCL group)              */
	LFA_STEP_REDUCE = 3,   /* dst[i] = dst[i] OP src[i], count elements  */
	LFA_STEP_TREE = 4,     /* dst = tree(refs[first..first+nsrc)), count */
	LFA_STEP_COPY = 5,     /* bytes from src to dst                      */
	LFA_STEP_ALLTOALL = 6, /* count bytes per rank: block p of src goes to
				  rank p, block q of dst comes from rank q    */
	LFA_STEP_ALLGATHER = 7,/* count bytes: src (this rank's block) to
				  block r of dst on every rank                */
	LFA_STEP_BARRIER = 8,  /* every rank's earlier steps (its own stream)
				  complete before any rank's later steps run  */
	LFA_STEP_TREE_PUT = 9, /* TREE whose result also goes to `peer` more
				  destinations: refs[first+nsrc ..
				  first+nsrc+peer) (LFA_ALGO_P2P pushes)      */
	LFA_STEP_ONESHOT = 10, /* ONE kernel for a small reducing collective
				  over `count` elements of src, rank order:
				  peer = LFA_ONESHOT_ALL: dst = the whole
				  result (allreduce); LFA_ONESHOT_SCATTER:
				  dst = block `rank` (reduce_scatter); root
				  >= 0: dst = the whole result on the root
				  only (reduce).  Each rank's part for member
				  k goes to slot `rank` of k's SYM_IN (slots
				  double-buffered by the group's one-shot
				  count), flags in the workspace order it.
				  Same result as COPY src -> own SYM_IN,
				  BARRIER, TREE of the part over every rank's
				  SYM_IN, BARRIER.  LFA_ALGO_P2P, 2..8
				  members.                                   */
};
#define LFA_ONESHOT_ALL (-1)
#define LFA_ONESHOT_SCATTER (-2)
/* SYM_IN / SYM_OUT: the symmetric workspace of group rank `ref.rank`, two
 * regions of count·esz bytes each (input staging, gathered result), mapped
 * into every member's address space; offsets mirror SEND / RESULT. */
enum lfa_buf_id { LFA_BUF_SEND = 0, LFA_BUF_RESULT = 1, LFA_BUF_TMP = 2,
		  LFA_BUF_SYM_IN = 3, LFA_BUF_SYM_OUT = 4 };

struct lfa_ref {
	int32_t buf;           /* enum lfa_buf_id */
	uint32_t rank;         /* SYM_IN/SYM_OUT: owning group rank */
	uint64_t off;          /* byte offset */
};
struct lfa_step {
	int32_t type;          /* enum lfa_step_type */
	int32_t peer;          /* SEND/RECV: group rank; TREE_PUT: extra
				  destinations */
	uint64_t count;        /* bytes (SEND/RECV/COPY) or elements */
	struct lfa_ref dst;
	struct lfa_ref src;
	uint32_t first;        /* TREE: first index into the refs array */
	uint32_t nsrc;         /* TREE: number of inputs (rank order) */
};

/*
 * Build rank `rank`'s schedule for one collective of `count` elements of
 * `esz` bytes in an `nranks` group (root: group rank, or -1).  Writes up to
 * *nsteps steps / *nrefs refs and returns the counts in them, and the HBM
 * workspace the schedule needs in *tmp_bytes.  Host-only, no GPU needed.
 * Returns 0, -LFA_EINVAL, -LFA_ENOSYS (collective/algo not planned) or
 * -LFA_ETOOSMALL (arrays too short; *nsteps and *nrefs = sizes needed).
 */
#define LFA_ETOOSMALL 257
int lfa_coll_plan(enum lfa_collective_op coll, enum lfa_coll_algo algo,
		  int rank, int nranks, int root, size_t count, size_t esz,
		  struct lfa_step *steps, size_t *nsteps,
		  struct lfa_ref *refs, size_t *nrefs, size_t *tmp_bytes);

/* Block [off, off + len) of rank r when `count` splits over `nranks`. */
void lfa_coll_block(size_t count, int nranks, int r, size_t *off, size_t *len);

/*
 * Host-buffer staging plan: chunk `idx` of a collective of `count` elements
 * of `esz` bytes over `nranks`, staged `chunk_bytes` at a time (the geometry
 * lfa_allreduce & co. use for host memory).  Chunk idx copies `height` rows
 * of `width` bytes, `src_pitch` apart, from buf + src_off into a dense
 * staging area, runs the device collective on `dev_count` elements of it and
 * copies `width` bytes back to result + dst_off.  Returns 1 and fills *c for
 * an existing chunk, 0 past the last one, -LFA_EINVAL for a collective the
 * pipeline does not chunk (ragged reduce_scatter, allgather, scatter).
 * Host-only, no GPU needed.
 */
/* Staging geometry: chunk idx of an operation staged `chunk_bytes` at a time
 * (0 = one chunk), for allreduce / reduce / broadcast (contiguous chunks) and
 * reduce_scatter with count % nranks == 0 (chunk j gathers elements
 * [j, j+w) of every rank's block: height nranks, pitch = one block).
 * Returns 1 and fills *c, 0 past the last chunk, -LFA_EINVAL for other
 * collectives and ragged reduce_scatter (staged whole). */
struct lfa_host_chunk {
	size_t src_off, src_pitch, width, height, dev_count, dst_off;
};
int lfa_coll_host_chunk(enum lfa_collective_op coll, size_t count, int nranks,
			size_t esz, size_t chunk_bytes, size_t idx,
			struct lfa_host_chunk *c);

/*
 * Single-GPU multi-rank execution of the schedules: runs the plans of all
 * `nranks` ranks on this device, matching every SEND with its RECV by a
 * device-to-device copy, with the real combine kernels.  send[r]/result[r]
 * are device pointers.  For testing the schedule+kernel data path at N>1 on
 * one GPU; the RCCL transport is used by lfa_allreduce & co.
 */
int lfa_coll_loopback(enum lfa_collective_op coll, enum lfa_coll_algo algo,
		      int nranks, int root, enum lfa_datatype datatype,
		      enum lfa_op op, size_t count, void *const *send,
		      void *const *result, void *stream);

#ifdef __cplusplus
}
#endif

#endif /* LFA_COLL_H */
