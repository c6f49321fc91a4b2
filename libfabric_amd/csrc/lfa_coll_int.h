/*
 * lfa_coll_int.h — internal types shared by the collective provider's
 * translation units (liblfa_coll.so): the domain / endpoint / group state
 * (lfa_coll.c), the executor and its transports (lfa_coll_exec.c) and the
 * single-GPU loopback (lfa_coll_loopback.c).  Not installed.
 */
#ifndef LFA_COLL_INT_H
#define LFA_COLL_INT_H

#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>
#include <rccl/rccl.h>

#include "lfa_atomic.h"
#include "lfa_coll.h"
#include "lfa_coll_plan.h"
#include "lfa_signal.h"

#define LFA_MAX_GROUP_ID 256            /* OFI_MAX_GROUP_ID, ofi_coll.h:44 */
#define LFA_CID_BYTES (LFA_MAX_GROUP_ID / 8)
/* Bytes of one P2P handle-exchange record (struct sym_rec, lfa_coll.c). */
#define LFA_SYM_REC_BYTES 80
#define LFA_STAGE_POOL 128              /* peer-domain staging buffers kept */
#define LFA_BOUNCE_POOL 8               /* pinned host bounce blocks kept */
#define LFA_BOUNCE_BYTES (1u << 20)     /* per operand: the largest operation of a
					 * pageable host member copied through one */
#define LFA_EXPORT_TRIES 4              /* workspace allocations per growth
					 * whose IPC export may be refused */
/* idle staging bytes the pool keeps by default (the endpoint's
 * stage_cap, LFA_STAGE_POOL_BYTES at open): a buffer returned above it is
 * freed, and lfa_coll_ep_flush frees every idle one */
#define LFA_STAGE_POOL_BYTES ((size_t)1 << 30)

/* Where a plan's refs point for one execution: the operation's buffers and,
 * for LFA_ALGO_P2P, every group rank's symmetric workspace as mapped here
 * (IN region at 0, OUT region at `region`, flag area at 2·region). */
struct xctx {
	void *base[3];          /* SEND, RESULT, TMP */
	char *const *sym;       /* [group rank] */
	size_t region;
	uint64_t ticket;        /* the group's P2P operation number (timeouts) */
	/* completion word (lfa_signal.h struct lfa_oneshot): set by the caller
	 * when the plan's one step is the one-shot kernel; the launch takes
	 * its value from *done_seq (stream order) and reports it in done_val */
	uint32_t *done_ctr;
	uint64_t *done_word;
	uint64_t *done_seq;
	uint64_t done_val;
};

/* ====================================================================== */
/* domain / endpoint                                                       */
/* ====================================================================== */

struct lfa_coll_mc {
	struct lfa_coll_ep *ep;
	ncclComm_t comm;
	int owns_comm;
	int rank, size;
	uint16_t group_id;
	uint16_t seq;
	int is_world;
	/* host (peer-transfer) domains: group rank -> domain rank, NULL for
	 * the world group (prov/coll's av_set fi_addr_array) */
	int *members;
	/* join in flight */
	uint8_t *mask_host;     /* pinned result of the cid-mask BAND */
	void *join_context;
	/* LFA_ALGO_P2P symmetric workspace: `sym_local` (2 regions + the flag
	 * area, hipMalloc, IPC-exported) and every member's as mapped here
	 * (sym[rank] = local) */
	char *sym_local;
	char **sym;
	size_t sym_region;
	/* flag barriers enqueued on this group so far (the epoch of the next
	 * is one more; equal on every member, collectives being ordered) */
	uint32_t bar_epoch;
	uint32_t os_epoch;      /* one-shot operations, likewise */
	/* timed-out P2P waits of this group (lfa_signal.h): the host-mapped
	 * status word (lowest failing ticket, LFA_SIG_NONE), the last ticket
	 * handed out, and whether a failure was reaped — the members' epochs
	 * then disagree, so the group refuses P2P operations (other groups of
	 * the endpoint are unaffected) */
	uint64_t *sig_word;
	uint64_t p2p_ticket;
	int sig_failed;
	uint64_t n_oneshot, n_barrier;  /* lfa_mc_counters */
	/* LFA_ALGO_AUTO: 0 not tried, 1 the workspace agreement held, -1 it
	 * failed on some member (every member then runs TREE) */
	int p2p_state;
};

struct lfa_coll_domain {
	int device, rank, nranks;
	ncclComm_t comm;
	int host;                       /* peer-transfer domain (host memory) */
	struct lfa_peer_xfer_ops xops;
	void *xctx;
};

struct hop;

struct pending {
	hipEvent_t ev;          /* device domains */
	struct hop *hop;        /* host domains: the operation's state */
	void *context;
	int kind;               /* 0 collective, 1 join, 2 join of a closed mc,
				 * 3 a non-final chunk of a collective (no entry) */
	struct lfa_coll_mc *mc;
	/* the group the operation's P2P kernels ran on and its highest ticket
	 * (0: none); timed_out: found failed when that group was closed */
	struct lfa_coll_mc *pmc;
	uint64_t ticket;
	int timed_out;
	/* device domains: completes when the endpoint's completion word reaches
	 * done_val (the one-shot kernel wrote it; no event), 0: the event;
	 * done_w: that word (NULL: the endpoint's done_word) */
	uint64_t done_val;
	const uint64_t *done_w;
	/* word operations: when the operation fails if its word has not come,
	 * and when the queue or stream owing it was last asked for an error
	 * (lfa_coll.c word_overdue); armed: the bound runs from the first poll
	 * that finds the operation at the head of the queue, so an operation
	 * queued behind a long one is not charged for its wait */
	struct word_wait {
		uint64_t deadline_ns, checked_ns;
		int armed;
	} ww;
	/* device domains: a one-member group's operation on pageable host
	 * buffers run through a pinned bounce block (ep->bounce); its result is
	 * copied to bounce_user when the operation is reaped */
	void *bounce, *bounce_out, *bounce_user;
	size_t bounce_bytes;
	/* the chunks of one chunked operation (peer_submit_chunked) share a
	 * nonzero chain id: the operation posts ONE completion — the first
	 * chunk's error, or the last chunk's success */
	uint64_t chain;
};

struct lfa_coll_ep {
	struct lfa_coll_domain *dom;
	pthread_mutex_t lock;       /* queue, CQ/EQ, stream enqueue order */
	pthread_mutex_t comm_lock;  /* communicator management (split/destroy,
				     * P2P workspace exchange), in call order */
	hipStream_t stream;         /* executor stream (RCCL + kernels) */
	hipStream_t copy_stream;    /* host staging copies, H2D */
	hipStream_t d2h_stream;     /* host staging copies, D2H (the other
				     * PCIe direction runs concurrently) */
	enum lfa_coll_algo algo;
	uint64_t next_chain;        /* chain ids of chunked operations */
	uint64_t failed_chain;      /* the chain whose error was reported: its
				     * remaining chunks reap silently */
	size_t chunk;               /* one-member groups: host staging chunk */
	size_t group_chunk;         /* every member, any N (0 = off) */
	void *ws;                   /* device workspace */
	size_t ws_size;
	void *hs[2];                /* device staging for host buffers */
	size_t hs_size;
	/* peer domains: device staging of host buffers (LFA_ALGO_P2P) and the
	 * device hops' TMP, kept across operations — a hipMalloc / hipFree pair
	 * of 256 MiB per operation cost more than its PCIe copies */
	struct stage_buf {
		void *p;
		size_t bytes;
		int busy;
		uint64_t used;      /* stage_clock at the last stage_get */
	} stage[LFA_STAGE_POOL];
	uint64_t stage_clock;
	/* peer domains: pinned host blocks (input half, output half) that a
	 * pageable host member's small P2P operation is copied through on the
	 * CPU, so its kernels run on the block's mapping instead of staging the
	 * buffers through HBM; allocated on first use, freed at close */
	struct bounce_buf {
		void *p;
		int busy;
	} bounce[LFA_BOUNCE_POOL];
	int bounce_retired;         /* blocks kept out after failed operations */
	size_t stage_cap;           /* idle staging bytes kept */
	int stage_trim_due;         /* idle bytes passed the cap: trim when the
				     * queue has drained */
	uint64_t *barrier_host;     /* pinned ~rank for barrier */
	void *barrier_dev;          /* 2 x uint64 */
	void *ctl_dev;              /* P2P handle exchange, nranks records */
	void *ctl_host;
	uint8_t cid_mask[LFA_CID_BYTES];
	struct lfa_coll_mc world;
	hipEvent_t evpool[64];      /* recycled completion events */
	/* the completion word of small operations: the last
	 * workgroup of a one-shot kernel on ep->stream counts in done_ctr and
	 * stores the launch's value (done_seq, in stream order) into done_word,
	 * which the host reads instead of querying an event */
	uint32_t *done_ctr;         /* device, 0 at rest */
	uint64_t *done_word;        /* host-mapped */
	uint64_t done_seq;
	uint64_t op_done_val;       /* run_device's last launch's value, or 0 */
	const uint64_t *op_done_w;  /* ... and its word (NULL: done_word) */
	/* direct dispatch (lfa_signal.h lfa_direct_*): a one-member group's
	 * small reducing collective as liblfa's own AQL packet on its own HSA
	 * queue (one per device and process, shared by its endpoints), with its
	 * own counter and word (kernels there are not ordered with ep->stream).
	 * Taken at first use; LFA_DIRECT=0 keeps the HIP
	 * launch.  allow_direct: set by submit around a caller's operation (the
	 * barrier's own staging copy is stream-ordered, so it never goes direct) */
	struct lfa_direct *direct;
	int direct_tried, allow_direct;
	uint32_t *ddone_ctr;
	uint64_t *ddone_word;
	uint64_t ddone_seq;
	/* bound on a word operation's wait (LFA_SIG_TIMEOUT_MS at open, as every
	 * GPU wait of the provider), and the test knob that makes the next
	 * drop_words words unreachable (lfa_coll_ep_test_word) */
	uint64_t word_timeout_ns;
	int drop_words;
	/* a one-member group's reducing collectives of at most this many bytes
	 * run as the solo copy (LFA_SOLO_BYTES at open; lfa_coll_ep_test_solo) */
	size_t solo_max;
	uint64_t word_ops;          /* operations reaped through a word */
	int nev;
	struct plan_cache {         /* last schedules built, keyed by shape */
		int valid, coll, algo, rank, n, root;
		size_t count, esz;
		struct plan pl;
	} pc[8];
	unsigned pc_next;
	struct pending *q;          /* FIFO ring of in-flight ops */
	size_t qcap, qhead, qlen;
	struct lfa_cq_err_entry err;
	int have_err;
	struct { uint32_t event; struct lfa_eq_entry entry; } eq[64];
	size_t eqh, eqn;
};

/* group rank -> domain rank (host domains; identity for the world) */
static inline int world_rank(const struct lfa_coll_mc *mc, int grank)
{
	return mc->members ? mc->members[grank] : grank;
}

/* ---------------------------------------------------------------------- */
/* host (peer-transfer) executor                                          */
/* ---------------------------------------------------------------------- */

/*
 * The executor.  A schedule (struct plan) runs through ONE loop,
 * xrun_advance, whatever carries its transfers; a transport table (xport)
 * supplies the transfers and the local items:
 *   xport_rccl  device buffers: SEND/RECV groups are RCCL grouped
 *               ncclSend/ncclRecv, ALLTOALL/ALLGATHER/BARRIER RCCL
 *               collectives, REDUCE/TREE/TREE_PUT/COPY gfx950 kernels — all
 *               enqueued on the endpoint's stream, so a group "completes" as
 *               soon as it is posted and one call runs the whole schedule;
 *   xport_peer  host buffers of a peer-transfer domain: SEND/RECV are the
 *               owner's tagged transfers (lfa_peer_xfer_ops), REDUCE/TREE the
 *               host combine; a group is waited on with test() and the run
 *               resumes there on the next progress call (prov/coll's fenced
 *               work queue, coll_coll.c:153-227, 816-890).
 * The multi-process CPU tests (tests/test_coll_host.py) therefore run this
 * same loop, planner and tag scheme that the GPU endpoints run.
 */
struct xrun;
struct xport {
	int (*group_start)(struct xrun *r);
	int (*post)(struct xrun *r, const struct lfa_step *st, void **req);
	int (*group_end)(struct xrun *r);
	int (*test)(struct xrun *r, void *req);       /* NULL: stream-ordered */
	int (*local)(struct xrun *r, const struct lfa_step *st);
	int (*coll)(struct xrun *r, const struct lfa_step *st);
};

struct xrun {
	const struct xport *xp;
	const struct plan *pl;
	struct xctx x;
	struct lfa_coll_mc *mc;
	enum lfa_op op;
	enum lfa_datatype dt;
	hipStream_t stream;     /* xport_rccl */
	uint64_t cid;           /* xport_peer tags: group_id << 16 | seq */
	size_t pc;
	void **reqs;            /* the current group's transfers; NULL = done */
	size_t nreq, creq;      /* nreq = steps of the group posted so far */
	int hip_err;            /* first failing HIP call's code (prov_errno) */
};

/*
 * A HIP call of an operation failed: keep the first code (it becomes the
 * completion's prov_errno, fi_cq_err_entry's provider-specific error) and,
 * with LFA_DEBUG set, name the call on stderr.  Returns the call's result.
 */
/* LFA_TRACE=1: one stderr line per hop state change (diagnostics). */
static int lfa_trace_on __attribute__((unused)) = -1;
#define LFA_TRACE(...)                                                        \
	do {                                                                  \
		if (lfa_trace_on < 0)                                         \
			lfa_trace_on = lfa_param("LFA_TRACE") != NULL;            \
		if (lfa_trace_on) {                                           \
			struct timespec ts_;                                  \
			clock_gettime(CLOCK_MONOTONIC, &ts_);                 \
			fprintf(stderr, "lfa-trace %ld.%06ld pid %d: ",      \
				(long)ts_.tv_sec, ts_.tv_nsec / 1000,         \
				(int)getpid());                               \
			fprintf(stderr, __VA_ARGS__);                         \
			fputc('\n', stderr);                                  \
		}                                                             \
	} while (0)

LFA_INTERNAL hipError_t lfa_hip_note(int *slot, hipError_t e, const char *what);

/* lfa_coll_exec.c */
LFA_INTERNAL void *resolve(const struct xctx *x, struct lfa_ref r);
/* Non-communication step on `stream`. */
LFA_INTERNAL int run_local(const struct lfa_step *s, const struct lfa_ref *refs,
			   const struct xctx *x, enum lfa_op op, enum lfa_datatype dt,
			   hipStream_t stream);
LFA_INTERNAL int plan_uses_sym(const struct lfa_step *st, size_t nsteps);
LFA_INTERNAL size_t sym_region(size_t count, size_t esz);
/* Bytes per workspace region the plan needs (ONESHOT: 2·n slots). */
LFA_INTERNAL size_t plan_sym_need(const struct lfa_step *st, size_t nsteps, int n,
				  size_t count, size_t esz);
LFA_INTERNAL int xrun_advance(struct xrun *r);
/* BARRIER of a plan on the symmetric workspace: the flag-barrier kernel. */
LFA_INTERNAL int sig_barrier(struct xrun *r);
/* ONESHOT step: the one-kernel small allreduce (lfa_signal.h). */
LFA_INTERNAL int sig_oneshot(struct xrun *r, const struct lfa_step *st);
/* x->done_val receives the one-shot launch's completion-word value (0: the
 * operation completes through an event). */
LFA_INTERNAL int exec_plan(struct lfa_coll_mc *mc, const struct plan *pl,
			   struct xctx *x, enum lfa_op op, enum lfa_datatype dt,
			   hipStream_t s);
LFA_INTERNAL extern const struct xport xport_peer, xport_peer_dev;

/* lfa_coll.c */
LFA_INTERNAL int check_reduce_args(enum lfa_datatype dt, enum lfa_op op);

/* One member's record in the P2P workspace handshake (lfa_coll_ws.c): its
 * export succeeded, the IPC handle, the workspace's identity word. */
struct sym_rec {
	int32_t ok;
	int32_t pad;
	hipIpcMemHandle_t h;
	uint64_t id;            /* the workspace's identity word (LFA_SIG_ID_OFF) */
};


/*
 * One collective on a host domain: prov/coll's util_coll_operation and its
 * work queue (ofi_coll.h:146-163) — the schedule, its own TMP, and the run.
 */
struct hop {
	struct xrun r;
	struct plan pl;
	void *tmp;              /* host, or device memory for a device hop */
	int done, err;
	int dev;                /* device buffers (xport_peer_dev) */
	hipEvent_t fin;         /* device hop: the stream reached the end */
	/* host buffers run as a device hop (LFA_ALGO_P2P on a GPU peer domain:
	 * every member must follow the one schedule): staged copies, H2D on the
	 * endpoint's copy stream (in_ev: the run's first item waits for it), D2H
	 * on its d2h stream after the run (out_ev ends the hop) */
	void *st_in, *st_out, *user_out;
	size_t out_bytes;
	hipEvent_t in_ev, out_ev;
	int in_waited;
	/* pageable host buffers of a small operation: a pinned bounce block
	 * (ep->bounce) holds the input and the result; the result is copied to
	 * bounce_user on the CPU when the hop completes (bounce_finish) */
	void *bounce, *bounce_out, *bounce_user;
	size_t bounce_bytes;
	/* a device hop whose every item is on the stream: a later P2P hop may
	 * enqueue behind it (stream order) without waiting for it to finish */
	int issued;
	struct word_wait ww;    /* a hop ending in the completion word */
	/* LFA_ALGO_P2P prologue (hop_prologue): wait for the earlier operations
	 * (they share the symmetric workspace), then grow it if needed through
	 * two handshake collectives on the reserved seqs sub_seq, sub_seq + 1 */
	int phase;
	size_t sym_need, sym_size;
	struct hop *sub;
	uint16_t sub_seq;
	int32_t agree_in, agree_out;
	unsigned char mine[LFA_SYM_REC_BYTES];
	uint64_t scratch[2];    /* barrier word and its result */
	struct lfa_coll_ep *ep;
};

enum { HOP_RUN, HOP_WAIT_PRIOR, HOP_SYM_GATHER, HOP_SYM_AGREE };

/* host-buffer chunk (bench.py --only-extra host_rs, 256 MiB float allreduce:
 * 8 MiB 9.49 ms, 16 MiB 6.57, 32 MiB 6.49, 64 MiB 6.81, 128 MiB 7.63) */
#define LFA_DEFAULT_CHUNK (32u << 20)

/* Internal entry points shared by the provider's translation units. */
/* lfa_coll.c */
LFA_INTERNAL struct lfa_coll_mc *mc_of(struct lfa_coll_ep *ep, lfa_addr_t a);
LFA_INTERNAL void release_event(struct lfa_coll_ep *ep, hipEvent_t ev);
LFA_INTERNAL hipEvent_t event_get(struct lfa_coll_ep *ep);
LFA_INTERNAL int queue_reserve(struct lfa_coll_ep *ep, size_t n);
LFA_INTERNAL struct pending *queue_slot(struct lfa_coll_ep *ep);
LFA_INTERNAL int enqueue_completion(struct lfa_coll_ep *ep, hipStream_t s,
			      void *context, int kind, struct lfa_coll_mc *mc,
			      uint64_t done_val, const uint64_t *done_w);
LFA_INTERNAL int run_device(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
		      enum lfa_collective_op coll, const void *buf, void *result,
		      size_t count, int root, enum lfa_datatype dt,
		      enum lfa_op op, hipStream_t s, enum lfa_coll_algo algo);
LFA_INTERNAL int mc_member(const struct lfa_coll_mc *mc);
/* lfa_coll_word.c */
LFA_INTERNAL int word_overdue(const struct lfa_coll_ep *ep, const uint64_t *w, hipStream_t s,
			struct word_wait *ww, int *perr);
LFA_INTERNAL int done_word_init(struct lfa_coll_ep *ep);
LFA_INTERNAL void done_word_free(struct lfa_coll_ep *ep, int stream_ok);
LFA_INTERNAL size_t solo_bytes(void);
LFA_INTERNAL int run_solo(struct lfa_coll_ep *ep, const void *buf, void *result, size_t count,
		    enum lfa_datatype dt);
/* lfa_coll_ws.c */
LFA_INTERNAL void sig_word_free(struct lfa_coll_mc *mc);
LFA_INTERNAL int sig_ready(struct lfa_coll_mc *mc);
LFA_INTERNAL void tag_p2p(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc, uint64_t t0);
LFA_INTERNAL int p2p_timed_out(const struct pending *p);
LFA_INTERNAL void ws_domain_ref(int delta);
LFA_INTERNAL void p2p_release(struct lfa_coll_mc *mc);
LFA_INTERNAL size_t sym_grow(const struct lfa_coll_mc *mc, size_t region);
LFA_INTERNAL void sym_prepare(struct lfa_coll_mc *mc, size_t region, int ok,
			struct sym_rec *mine, int *why);
LFA_INTERNAL int sym_open(struct lfa_coll_mc *mc, const struct sym_rec *recs, size_t region,
		    int *why);
LFA_INTERNAL int p2p_ensure(struct lfa_coll_mc *mc, size_t region);
/* lfa_coll_host.c */
LFA_INTERNAL int is_device_ptr(const void *p);
LFA_INTERNAL void *zero_copy_of(const void *p, int dev);
LFA_INTERNAL int grow_staging(struct lfa_coll_ep *ep, size_t need);
LFA_INTERNAL void stage_trim(struct lfa_coll_ep *ep, size_t keep);
LFA_INTERNAL void *bounce_get(struct lfa_coll_ep *ep);
LFA_INTERNAL void bounce_put(struct lfa_coll_ep *ep, void *p);
LFA_INTERNAL void bounce_retire(struct lfa_coll_ep *ep, void *p);
LFA_INTERNAL void bounce_free_all(struct lfa_coll_ep *ep, int drained);
LFA_INTERNAL void hop_free(struct hop *h);
LFA_INTERNAL void host_progress_all(struct lfa_coll_ep *ep);
LFA_INTERNAL int enqueue_host(struct lfa_coll_ep *ep, struct hop *h, void *context,
			int kind, struct lfa_coll_mc *mc);
LFA_INTERNAL int run_host_chunked(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			    enum lfa_collective_op coll, const void *buf,
			    void *result, size_t count, int root,
			    enum lfa_datatype dt, enum lfa_op op, size_t chunk);
LFA_INTERNAL int run_device_chunked(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			      enum lfa_collective_op coll, const void *buf,
			      void *result, size_t count, int root,
			      enum lfa_datatype dt, enum lfa_op op, size_t chunk);
LFA_INTERNAL int run_host_whole(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			  enum lfa_collective_op coll, const void *buf,
			  size_t in_bytes, void *result, size_t out_bytes,
			  size_t count, int root, enum lfa_datatype dt,
			  enum lfa_op op);
LFA_INTERNAL int host_start(struct lfa_coll_ep *ep, struct hop *h,
		      struct lfa_coll_mc *mc, enum lfa_collective_op coll,
		      const void *buf, void *result, size_t count, int root,
		      enum lfa_datatype dt, enum lfa_op op, int dev,
		      enum lfa_coll_algo algo);
LFA_INTERNAL int host_submit(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
		       enum lfa_collective_op coll, const void *buf,
		       void *result, size_t count, int root,
		       enum lfa_datatype dt, enum lfa_op op, void *context,
		       int kind, struct lfa_coll_mc *jmc, int dev,
		       enum lfa_coll_algo algo);
LFA_INTERNAL size_t peer_chunked(const struct lfa_coll_ep *ep, const struct lfa_coll_mc *mc,
			   enum lfa_collective_op coll, size_t count, size_t esz);
LFA_INTERNAL int peer_submit_chunked(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			       enum lfa_collective_op coll, const void *buf,
			       void *result, size_t count, int root,
			       enum lfa_datatype dt, enum lfa_op op, void *context,
			       int dev, size_t chunk);
/* lfa_coll_group.c */
LFA_INTERNAL void join_finish(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc);

#endif
