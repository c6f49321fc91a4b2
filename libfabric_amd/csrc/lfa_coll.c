/*
 * lfa_coll.c — MI355X collective provider: the host side of libfabric's
 * software-collective path (prov/coll), in C.
 *
 * Reference structure this restates (not copies):
 *   prov/coll builds, per operation, a work queue of SEND / RECV / REDUCE /
 *   COPY / COMP items (include/ofi_coll.h:64-119, coll_coll.c:229-343) and
 *   drains it from the application's progress thread (coll_ep_progress,
 *   coll_coll.c:816-890), with transport delegated to the host provider
 *   through FI_PEER_TRANSFER tagged messages (coll_coll.c:770-814) and every
 *   REDUCE item calling ofi_atomic_write_handler (coll_coll.c:758-768).
 *
 * The MI355X design keeps that split — schedule / transport / combine — but:
 *   - the schedule is built once per call as an array of lfa_step items
 *     (lfa_coll_plan, host-only, testable on CPU);
 *   - the executor enqueues the whole schedule on the endpoint's HIP stream:
 *     SEND/RECV groups become RCCL grouped ncclSend/ncclRecv over xGMI,
 *     REDUCE / TREE items launch the gfx950 combine kernels (liblfa.so),
 *     COPY items are D2D copies; nothing blocks the host;
 *   - completion is a HIP event per operation, reaped by lfa_cq_read (the
 *     progress call, like fi_cq_read driving coll_ep_progress).
 *
 * Default algorithm (LFA_ALGO_TREE): rank r receives block r of every
 * rank's input (one grouped exchange, (N-1)/N·S bytes out per rank), reduces
 * the N blocks in ONE fused kernel in the reference's recursive-doubling
 * association order — so every rank's result is bit-identical to prov/coll's
 * — and all-gathers the reduced blocks.  Bandwidth-optimal like RS+AG, and
 * valid for every op including the bitwise/logical ones RCCL lacks.
 */
#define _GNU_SOURCE
#include <dirent.h>
#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "lfa_coll_int.h"


int lfa_coll_get_unique_id(void *id, size_t len)
{
	ncclUniqueId uid;

	if (!id || len < sizeof(uid) || sizeof(uid) > LFA_UNIQUE_ID_BYTES)
		return -LFA_EINVAL;
	if (ncclGetUniqueId(&uid) != ncclSuccess)
		return -LFA_EIO;
	memset(id, 0, len);
	memcpy(id, &uid, sizeof(uid));
	return 0;
}

int lfa_coll_domain_open(int device, int rank, int nranks, const void *id,
			 size_t id_len, struct lfa_coll_domain **domain)
{
	struct lfa_coll_domain *d;
	ncclUniqueId uid;

	if (!domain || !id || id_len < sizeof(uid) || nranks < 1 || rank < 0 ||
	    rank >= nranks)
		return -LFA_EINVAL;
	if (hipSetDevice(device) != hipSuccess)
		return -LFA_EINVAL;
	d = calloc(1, sizeof(*d));
	if (!d)
		return -LFA_ENOMEM;
	memcpy(&uid, id, sizeof(uid));
	d->device = device;
	d->rank = rank;
	d->nranks = nranks;
	if (ncclCommInitRank(&d->comm, nranks, uid, rank) != ncclSuccess) {
		free(d);
		return -LFA_EIO;
	}
	ws_domain_ref(1);
	*domain = d;
	return 0;
}

int lfa_coll_domain_open_host(int rank, int nranks,
			      const struct lfa_peer_xfer_ops *ops, void *ctx,
			      struct lfa_coll_domain **domain)
{
	return lfa_coll_domain_open_peer(-1, rank, nranks, ops, ctx, domain);
}

int lfa_coll_domain_open_peer(int device, int rank, int nranks,
			      const struct lfa_peer_xfer_ops *ops, void *ctx,
			      struct lfa_coll_domain **domain)
{
	struct lfa_coll_domain *d;

	if (!domain || !ops || !ops->send || !ops->recv || !ops->test ||
	    nranks < 1 || rank < 0 || rank >= nranks)
		return -LFA_EINVAL;
	if (device >= 0 && hipSetDevice(device) != hipSuccess)
		return -LFA_EINVAL;
	d = calloc(1, sizeof(*d));
	if (!d)
		return -LFA_ENOMEM;
	d->device = device < 0 ? -1 : device;
	d->rank = rank;
	d->nranks = nranks;
	d->host = 1;
	d->xops = *ops;
	d->xctx = ctx;
	if (d->device >= 0)
		ws_domain_ref(1);
	*domain = d;
	return 0;
}

int lfa_coll_domain_comm_count(struct lfa_coll_domain *d, int *count)
{
	if (!d || !count)
		return -LFA_EINVAL;
	if (d->host)
		return -LFA_EOPNOTSUPP;
	return ncclCommCount(d->comm, count) == ncclSuccess ? 0 : -LFA_EIO;
}

int lfa_coll_domain_close(struct lfa_coll_domain *d)
{
	if (!d)
		return -LFA_EINVAL;
	if (!d->host)
		ncclCommDestroy(d->comm);
	if (d->device >= 0)
		ws_domain_ref(-1);
	free(d);
	return 0;
}

/* Frees whatever lfa_coll_ep_open managed to create (open's error path). */
static void ep_release(struct lfa_coll_ep *ep)
{
	done_word_free(ep, 1);
	if (ep->barrier_dev)
		hipFree(ep->barrier_dev);
	if (ep->ctl_dev)
		hipFree(ep->ctl_dev);
	if (ep->barrier_host)
		hipHostFree(ep->barrier_host);
	if (ep->copy_stream)
		hipStreamDestroy(ep->copy_stream);
	if (ep->d2h_stream)
		hipStreamDestroy(ep->d2h_stream);
	if (ep->stream)
		hipStreamDestroy(ep->stream);
	free(ep->ctl_host);
	free(ep->q);
	pthread_mutex_destroy(&ep->lock);
	pthread_mutex_destroy(&ep->comm_lock);
	free(ep);
}

int lfa_coll_ep_open(struct lfa_coll_domain *d, struct lfa_coll_ep **out)
{
	struct lfa_coll_ep *ep;
	size_t ctl;

	if (!d || !out)
		return -LFA_EINVAL;
	ep = calloc(1, sizeof(*ep));
	if (!ep)
		return -LFA_ENOMEM;
	ep->dom = d;
	pthread_mutex_init(&ep->lock, NULL);
	pthread_mutex_init(&ep->comm_lock, NULL);
	/* device domains choose per bucket; peer domains run the tree */
	ep->algo = d->host ? LFA_ALGO_TREE : LFA_ALGO_AUTO;
	ep->chunk = LFA_DEFAULT_CHUNK;
	ep->solo_max = solo_bytes();
	{
		const char *e = lfa_param("LFA_SIG_TIMEOUT_MS");
		const long ms = e ? atol(e) : 0;

		ep->word_timeout_ns = (uint64_t)(ms > 0 ? ms : 20000) * 1000000ull;
	}
	{
		const char *e = lfa_param("LFA_GROUP_CHUNK_BYTES");

		ep->group_chunk = e ? (size_t)strtoull(e, NULL, 0) : LFA_GROUP_CHUNK_AUTO;
		e = lfa_param("LFA_STAGE_POOL_BYTES");
		ep->stage_cap = e ? (size_t)strtoull(e, NULL, 0) : LFA_STAGE_POOL_BYTES;
	}
	/* the P2P workspace exchange needs these on every member even when a
	 * local allocation fails later, so they exist up front */
	ctl = (size_t)d->nranks * LFA_SYM_REC_BYTES;
	if (!d->host) {
		hipSetDevice(d->device);
		if (hipStreamCreateWithFlags(&ep->stream, hipStreamNonBlocking) != hipSuccess ||
		    hipStreamCreateWithFlags(&ep->copy_stream, hipStreamNonBlocking) != hipSuccess ||
		    hipStreamCreateWithFlags(&ep->d2h_stream, hipStreamNonBlocking) != hipSuccess ||
		    hipHostMalloc((void **)&ep->barrier_host, 2 * sizeof(uint64_t), 0) != hipSuccess ||
		    hipMalloc(&ep->barrier_dev, 4 * sizeof(uint64_t)) != hipSuccess ||
		    hipMalloc(&ep->ctl_dev, ctl) != hipSuccess ||
		    !(ep->ctl_host = calloc(1, ctl)) || done_word_init(ep)) {
			ep_release(ep);
			return -LFA_EIO;
		}
		ep->barrier_host[0] = ~(uint64_t)d->rank;   /* coll_ep_barrier2 :1011 */
	} else if (d->device >= 0) {
		/* device buffers on a peer-transfer domain: the local items' kernels
		 * run on this stream, staged host buffers' H2D / D2H on the two copy
		 * streams (so chunks pipeline); ctl_host holds the P2P handshake
		 * records */
		hipSetDevice(d->device);
		if (hipStreamCreateWithFlags(&ep->stream, hipStreamNonBlocking) != hipSuccess ||
		    hipStreamCreateWithFlags(&ep->copy_stream, hipStreamNonBlocking) != hipSuccess ||
		    hipStreamCreateWithFlags(&ep->d2h_stream, hipStreamNonBlocking) != hipSuccess ||
		    !(ep->ctl_host = calloc(1, ctl)) || done_word_init(ep)) {
			ep_release(ep);
			return -LFA_EIO;
		}
	}
	memset(ep->cid_mask, 0xff, sizeof(ep->cid_mask));
	ep->cid_mask[0] &= (uint8_t)~1u;            /* world group id 0 taken */
	ep->world.ep = ep;
	ep->world.comm = d->comm;
	ep->world.rank = d->rank;
	ep->world.size = d->nranks;
	ep->world.is_world = 1;
	ep->qcap = 256;
	ep->q = calloc(ep->qcap, sizeof(*ep->q));
	if (!ep->q) {
		ep_release(ep);
		return -LFA_ENOMEM;
	}
	*out = ep;
	return 0;
}

int lfa_coll_ep_close(struct lfa_coll_ep *ep)
{
	int drained;

	if (!ep)
		return -LFA_EINVAL;
	drained = lfa_coll_ep_flush(ep) == 0;
	if (ep->dom->host) {
		for (size_t i = 0; i < ep->qlen; i++)
			hop_free(ep->q[(ep->qhead + i) % ep->qcap].hop);
		p2p_release(&ep->world);
		sig_word_free(&ep->world);
		if (ep->stream)
			hipStreamDestroy(ep->stream);
		if (ep->copy_stream)
			hipStreamDestroy(ep->copy_stream);
		if (ep->d2h_stream)
			hipStreamDestroy(ep->d2h_stream);
		for (int i = 0; i < LFA_STAGE_POOL; i++)
			if (ep->stage[i].p)
				hipFree(ep->stage[i].p);
		bounce_free_all(ep, drained);
		for (int i = 0; i < ep->nev; i++)
			hipEventDestroy(ep->evpool[i]);
		done_word_free(ep, drained);
		free(ep->ctl_host);
		free(ep->q);
		pthread_mutex_destroy(&ep->lock);
		pthread_mutex_destroy(&ep->comm_lock);
		free(ep);
		return 0;
	}
	/* every P2P operation ended in a barrier: no peer touches it now */
	p2p_release(&ep->world);
	sig_word_free(&ep->world);
	for (size_t i = 0; i < ep->qlen; i++)
		if (ep->q[(ep->qhead + i) % ep->qcap].ev)
			hipEventDestroy(ep->q[(ep->qhead + i) % ep->qcap].ev);
	for (size_t i = 0; i < ep->qlen; i++)
		bounce_put(ep, ep->q[(ep->qhead + i) % ep->qcap].bounce);
	bounce_free_all(ep, drained);
	for (int i = 0; i < ep->nev; i++)
		hipEventDestroy(ep->evpool[i]);
	done_word_free(ep, drained);
	for (int i = 0; i < 8; i++)
		if (ep->pc[i].valid)
			plan_free(&ep->pc[i].pl);
	free(ep->q);
	if (ep->ws)
		hipFree(ep->ws);
	for (int i = 0; i < 2; i++)
		if (ep->hs[i])
			hipFree(ep->hs[i]);
	hipFree(ep->barrier_dev);
	hipFree(ep->ctl_dev);
	free(ep->ctl_host);
	hipHostFree(ep->barrier_host);
	hipStreamDestroy(ep->stream);
	hipStreamDestroy(ep->copy_stream);
	hipStreamDestroy(ep->d2h_stream);
	pthread_mutex_destroy(&ep->lock);
	pthread_mutex_destroy(&ep->comm_lock);
	free(ep);
	return 0;
}

void *lfa_coll_ep_stream(struct lfa_coll_ep *ep)
{
	return ep ? (void *)ep->stream : NULL;
}

int lfa_coll_ep_set_algo(struct lfa_coll_ep *ep, enum lfa_coll_algo algo)
{
	if (!ep || (algo != LFA_ALGO_TREE && algo != LFA_ALGO_RD &&
		    algo != LFA_ALGO_RCCL && algo != LFA_ALGO_TREE_COLL &&
		    algo != LFA_ALGO_P2P && algo != LFA_ALGO_AUTO))
		return -LFA_EINVAL;
	ep->algo = algo;
	return 0;
}

int lfa_coll_ep_set_chunk(struct lfa_coll_ep *ep, size_t bytes)
{
	if (!ep)
		return -LFA_EINVAL;
	ep->chunk = bytes ? bytes : LFA_DEFAULT_CHUNK;
	return 0;
}

int lfa_coll_ep_set_group_chunk(struct lfa_coll_ep *ep, size_t bytes)
{
	if (!ep)
		return -LFA_EINVAL;
	ep->group_chunk = bytes;
	return 0;
}

size_t lfa_coll_group_chunk(size_t group_chunk, int nranks, size_t bytes)
{
	if (group_chunk != LFA_GROUP_CHUNK_AUTO)
		return group_chunk;
	/* host members of a group pipeline H2D / collective / D2H per chunk
	 * (2 processes, 256 MiB: 20.4 ms whole, 13.1 ms in 32 MiB chunks,
	 * DESIGN.md §3); below two chunks there is nothing to overlap */
	return nranks > 1 && bytes >= 2 * LFA_AUTO_CHUNK_BYTES ? LFA_AUTO_CHUNK_BYTES : 0;
}

size_t lfa_coll_member_chunk(int nranks, int host, size_t group_chunk,
			     size_t local_chunk)
{
	if (group_chunk)
		return group_chunk;
	return host && nranks == 1 ? local_chunk : 0;
}

lfa_addr_t lfa_coll_world_addr(struct lfa_coll_ep *ep)
{
	return ep ? (lfa_addr_t)(uintptr_t)&ep->world : LFA_ADDR_NOTAVAIL;
}

lfa_addr_t lfa_mc_addr(struct lfa_coll_mc *mc)
{
	return (lfa_addr_t)(uintptr_t)mc;
}

int lfa_mc_group_id(struct lfa_coll_mc *mc)
{
	if (!mc)
		return -LFA_EINVAL;
	return mc->group_id < LFA_MAX_GROUP_ID ? (int)mc->group_id : -LFA_EAGAIN;
}

LFA_INTERNAL struct lfa_coll_mc *mc_of(struct lfa_coll_ep *ep, lfa_addr_t a)
{
	if (a == LFA_ADDR_NOTAVAIL || a == 0)
		return &ep->world;
	return (struct lfa_coll_mc *)(uintptr_t)a;
}

int lfa_mc_counters(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
		    struct lfa_mc_counters *out)
{
	struct lfa_coll_mc *mc;

	if (!ep || !out)
		return -LFA_EINVAL;
	mc = mc_of(ep, coll_addr);
	if (!mc)
		return -LFA_EINVAL;
	pthread_mutex_lock(&ep->lock);
	out->p2p_ops = mc->p2p_ticket;
	out->oneshot = mc->n_oneshot;
	out->flag_barriers = mc->n_barrier;
	out->timed_out = mc->sig_failed ||
			 (mc->sig_word && *(volatile uint64_t *)mc->sig_word != LFA_SIG_NONE);
	pthread_mutex_unlock(&ep->lock);
	return 0;
}

/* Grow-only device buffer, stream-ordered so in-flight users stay valid. */
static int grow(void **buf, size_t *size, size_t need, hipStream_t s)
{
	void *nb;

	if (need <= *size)
		return 0;
	need = (need + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
	if (hipMallocAsync(&nb, need, s) != hipSuccess)
		return -LFA_ENOMEM;
	if (*buf)
		hipFreeAsync(*buf, s);
	*buf = nb;
	*size = need;
	return 0;
}

/* ---------------------------------------------------------------------- */
/* completion queue                                                        */
/* ---------------------------------------------------------------------- */

LFA_INTERNAL void release_event(struct lfa_coll_ep *ep, hipEvent_t ev)
{
	if (ep->nev < (int)(sizeof(ep->evpool) / sizeof(ep->evpool[0])))
		ep->evpool[ep->nev++] = ev;
	else
		hipEventDestroy(ev);
}

/* A completion event from the endpoint's pool (ep->lock held): creating
 * one costs a runtime call per operation otherwise.  NULL on failure. */
LFA_INTERNAL hipEvent_t event_get(struct lfa_coll_ep *ep)
{
	hipEvent_t ev;

	if (ep->nev)
		return ep->evpool[--ep->nev];
	return hipEventCreateWithFlags(&ev, hipEventDisableTiming) == hipSuccess ? ev : NULL;
}

/* Room for `n` more operations in the FIFO of in-flight operations (the
 * ring doubles as needed): 0 or -LFA_ENOMEM. */
LFA_INTERNAL int queue_reserve(struct lfa_coll_ep *ep, size_t n)
{
	size_t cap = ep->qcap;

	while (cap - ep->qlen < n)
		cap *= 2;
	if (cap != ep->qcap) {
		struct pending *nq = calloc(cap, sizeof(*nq));

		if (!nq)
			return -LFA_ENOMEM;
		for (size_t i = 0; i < ep->qlen; i++)
			nq[i] = ep->q[(ep->qhead + i) % ep->qcap];
		free(ep->q);
		ep->q = nq;
		ep->qhead = 0;
		ep->qcap = cap;
	}
	return 0;
}

/* A free slot at the tail of the FIFO of in-flight operations. */
LFA_INTERNAL struct pending *queue_slot(struct lfa_coll_ep *ep)
{
	if (queue_reserve(ep, 1))
		return NULL;
	return &ep->q[(ep->qhead + ep->qlen) % ep->qcap];
}

LFA_INTERNAL int enqueue_completion(struct lfa_coll_ep *ep, hipStream_t s,
			      void *context, int kind, struct lfa_coll_mc *mc,
			      uint64_t done_val, const uint64_t *done_w)
{
	struct pending *p = queue_slot(ep);

	if (!p)
		return -LFA_ENOMEM;
	memset(p, 0, sizeof(*p));
	if (done_val) {
		/* the one-shot kernel stores done_val into the completion word:
		 * no event to record or query */
		p->done_val = done_val;
		p->done_w = done_w;
		/* p->ww stays unarmed: its bound starts at the head of the queue */
		if (ep->drop_words > 0) {
			/* test knob: a value the word never reaches */
			ep->drop_words--;
			p->done_val |= 1ull << 62;
		}
		p->context = context;
		p->kind = kind;
		p->mc = mc;
		ep->qlen++;
		return 0;
	}
	if (ep->nev)
		p->ev = ep->evpool[--ep->nev];
	else if (hipEventCreateWithFlags(&p->ev, hipEventDisableTiming) != hipSuccess)
		return -LFA_EIO;
	if (hipEventRecord(p->ev, s) != hipSuccess) {
		release_event(ep, p->ev);
		return -LFA_EIO;
	}
	p->context = context;
	p->kind = kind;
	p->mc = mc;
	ep->qlen++;
	return 0;
}

/* Completion state of a queued operation: 0 done, 1 pending, <0 / hip error
 * code (>0 in *perr) failed. */
static int pending_state(const struct lfa_coll_ep *ep, struct pending *p,
			 int *perr)
{
	if (p->hop) {
		if (p->hop->err) {
			/* the failing HIP call's code when there was one */
			*perr = p->hop->r.hip_err ? p->hop->r.hip_err : -p->hop->err;
			return -1;
		}
		return p->hop->done ? 0 : 1;
	}
	if (p->done_val) {
		const uint64_t *w = p->done_w ? p->done_w : ep->done_word;

		if (*(const volatile uint64_t *)w >= p->done_val)
			return 0;
		return word_overdue(ep, w, ep->stream, &p->ww, perr);
	}
	hipError_t e = hipEventQuery(p->ev);

	if (e == hipErrorNotReady)
		return 1;
	if (e != hipSuccess) {
		*perr = (int)e;
		return -1;
	}
	return 0;
}

/* failed: the operation was reaped in error (a word timeout, a failed queue
 * or stream) — its kernel may still run later and read or write its bounce
 * block, so the block leaves the pool for good instead of going back to be
 * refilled by the next submit (done_word_free keeps owed words
 * the same way).  A hop's own free synchronises its stream first. */
static void pending_release(struct lfa_coll_ep *ep, struct pending *p, int failed)
{
	if (p->hop)
		hop_free(p->hop);
	else if (p->ev)
		release_event(ep, p->ev);
	if (failed && !p->hop)
		bounce_retire(ep, p->bounce);
	else
		bounce_put(ep, p->bounce);
	p->hop = NULL;
	p->ev = NULL;
	p->bounce = NULL;
}

/* Reap completed operations in issue order. */
static void progress(struct lfa_coll_ep *ep, struct lfa_cq_entry *out,
		     size_t count, size_t *nout)
{
	*nout = 0;
	if (ep->dom->host)
		host_progress_all(ep);
	while (ep->qlen && !ep->have_err) {
		struct pending *p = &ep->q[ep->qhead];
		int perr = 0, st = pending_state(ep, p, &perr);

		if (st > 0)
			break;
		if (st == 0 && p2p_timed_out(p)) {
			/* a flag barrier or one-shot wait of this operation, or of
			 * an earlier one of its group, gave up waiting for a member
			 * (lfa_signal.h): this one and every later P2P operation of
			 * the group fail; the earlier ones completed normally */
			if (p->pmc)
				p->pmc->sig_failed = 1;
			st = -1;
			perr = ETIMEDOUT;
		} else if (st < 0 && p->pmc) {
			/* a P2P operation reaped as failed for another cause (its
			 * word's bound, a failed queue or stream): its kernel may
			 * still run and post into the workspace, so the group takes
			 * no further P2P operation and its workspace goes to the
			 * quarantine at close, as after a timed-out wait */
			p->pmc->sig_failed = 1;
		}
		if (st == 0 && p->bounce_bytes) {
			/* a bounced operation's result to the caller's buffer */
			memcpy(p->bounce_user, p->bounce_out, p->bounce_bytes);
			p->bounce_bytes = 0;
		}
		if (p->chain && p->chain == ep->failed_chain) {
			/* a chunk of an operation whose error was already
			 * reported: its outcome is that error, no second entry */
		} else if (p->kind == 0 && st == 0 && *nout >= count) {
			break;
		} else if (st < 0) {
			ep->err.op_context = p->context;
			ep->err.flags = LFA_COLLECTIVE;
			/* a word operation's own cause (ETIMEDOUT / EIO), else EIO
			 * with the HIP code as prov_errno */
			ep->err.err = p->hop || (p->done_val && (perr == ETIMEDOUT || perr == EIO))
				      ? perr : LFA_EIO;
			ep->err.prov_errno = perr;
			ep->have_err = 1;
			if (p->chain)
				ep->failed_chain = p->chain;
		} else if (p->kind == 1) {
			join_finish(ep, p->mc);
		} else if (p->kind == 2) {
			/* join of a handle closed before it completed */
		} else if (p->kind == 3) {
			/* a chunk of a larger operation (peer_chunked): its last
			 * chunk completes it */
		} else {
			struct lfa_cq_entry *c = &out[(*nout)++];

			memset(c, 0, sizeof(*c));
			c->op_context = p->context;
			c->flags = LFA_COLLECTIVE;
		}
		if (st == 0 && p->done_val)
			ep->word_ops++;
		pending_release(ep, p, st < 0);
		ep->qhead = (ep->qhead + 1) % ep->qcap;
		ep->qlen--;
	}
	if (ep->stage_trim_due && !ep->qlen) {
		stage_trim(ep, ep->stage_cap);
		ep->stage_trim_due = 0;
	}
}

ssize_t lfa_cq_read(struct lfa_coll_ep *ep, struct lfa_cq_entry *buf,
		    size_t count)
{
	size_t n;
	int have_err;
	ncclResult_t async;

	if (!ep || (!buf && count))
		return -LFA_EINVAL;
	pthread_mutex_lock(&ep->lock);
	progress(ep, buf, count, &n);
	if (!n && !ep->have_err && !ep->dom->host &&
	    ncclCommGetAsyncError(ep->dom->comm, &async) == ncclSuccess &&
	    async != ncclSuccess && async != ncclInProgress) {
		ep->err.op_context = ep->qlen ? ep->q[ep->qhead].context : NULL;
		ep->err.flags = LFA_COLLECTIVE;
		ep->err.err = LFA_EIO;
		ep->err.prov_errno = (int)async;
		ep->have_err = 1;
	}
	have_err = ep->have_err;
	pthread_mutex_unlock(&ep->lock);
	if (n)
		return (ssize_t)n;
	return have_err ? -LFA_EIO : -LFA_EAGAIN;
}

ssize_t lfa_cq_readerr(struct lfa_coll_ep *ep, struct lfa_cq_err_entry *buf)
{
	ssize_t ret = -LFA_EAGAIN;

	if (!ep || !buf)
		return -LFA_EINVAL;
	pthread_mutex_lock(&ep->lock);
	if (ep->have_err) {
		*buf = ep->err;
		ep->have_err = 0;
		ret = 1;
	}
	pthread_mutex_unlock(&ep->lock);
	return ret;
}

ssize_t lfa_eq_read(struct lfa_coll_ep *ep, uint32_t *event,
		    struct lfa_eq_entry *entry)
{
	struct lfa_cq_entry tmp[1];
	size_t n;
	ssize_t ret = -LFA_EAGAIN;

	if (!ep || !event || !entry)
		return -LFA_EINVAL;
	pthread_mutex_lock(&ep->lock);
	/* progress joins only up to the first collective completion */
	while (ep->qlen && ep->q[ep->qhead].kind == 1 && !ep->have_err) {
		int perr;

		progress(ep, tmp, 0, &n);
		if (ep->qlen && ep->q[ep->qhead].kind == 1 &&
		    pending_state(ep, &ep->q[ep->qhead], &perr) > 0)
			break;
	}
	if (ep->dom->host && !(ep->qlen && ep->q[ep->qhead].kind == 1))
		host_progress_all(ep);
	if (ep->eqn) {
		*event = ep->eq[ep->eqh].event;
		*entry = ep->eq[ep->eqh].entry;
		ep->eqh = (ep->eqh + 1) % 64;
		ep->eqn--;
		ret = (ssize_t)sizeof(*entry);
	}
	pthread_mutex_unlock(&ep->lock);
	return ret;
}

int lfa_coll_ep_flush(struct lfa_coll_ep *ep)
{
	if (!ep)
		return -LFA_EINVAL;
	if (ep->dom->host) {
		/* drive the transfers until every queued operation finished */
		for (;;) {
			int busy = 0, err = 0;

			pthread_mutex_lock(&ep->lock);
			host_progress_all(ep);
			for (size_t i = 0; i < ep->qlen; i++) {
				struct hop *h = ep->q[(ep->qhead + i) % ep->qcap].hop;

				if (h && h->err)
					err = h->err;
				else if (h && !h->done)
					busy = 1;
			}
			if (!busy && !err)
				stage_trim(ep, 0);
			pthread_mutex_unlock(&ep->lock);
			if (err)
				return err;
			if (!busy)
				return 0;
			sched_yield();
		}
	}
	return hipStreamSynchronize(ep->stream) == hipSuccess &&
	       hipStreamSynchronize(ep->copy_stream) == hipSuccess &&
	       hipStreamSynchronize(ep->d2h_stream) == hipSuccess ? 0 : -LFA_EIO;
}

static int rccl_type(enum lfa_datatype dt, ncclDataType_t *t)
{
	switch (dt) {
	case LFA_INT8: *t = ncclInt8; return 1;
	case LFA_UINT8: *t = ncclUint8; return 1;
	case LFA_INT32: *t = ncclInt32; return 1;
	case LFA_UINT32: *t = ncclUint32; return 1;
	case LFA_INT64: *t = ncclInt64; return 1;
	case LFA_UINT64: *t = ncclUint64; return 1;
	case LFA_FLOAT: *t = ncclFloat32; return 1;
	case LFA_DOUBLE: *t = ncclFloat64; return 1;
	default: return 0;
	}
}

static int rccl_op(enum lfa_op op, ncclRedOp_t *o)
{
	switch (op) {
	case LFA_SUM: *o = ncclSum; return 1;
	case LFA_PROD: *o = ncclProd; return 1;
	case LFA_MIN: *o = ncclMin; return 1;
	case LFA_MAX: *o = ncclMax; return 1;
	default: return 0;
	}
}

/*
 * LFA_ALGO_AUTO above the one-shot bounds (LFA_AUTO_BULK, round 6): the P2P
 * two-barrier schedule (default) or the tree.  A device domain's members sit
 * on distinct GPUs (RCCL takes one rank per device), here the 8 of an xGMI
 * mesh: the P2P schedule pulls every other member's block of the input and
 * pushes the reduced block back, about 2·S/n over each link, where the tree
 * (prov/coll's recursive doubling) sends the whole S over one link in each
 * of its log2(n) rounds — and both reduce in the same order, bit for bit
 * (DESIGN.md §6b).  Provisional until the driver's 8-GPU run prices it:
 * LFA_AUTO_BULK=tree restores the rounds-3-5 choice.
 */
int lfa_coll_auto_bulk(void)
{
	static int v = -1;

	if (v < 0) {
		const char *e = lfa_param("LFA_AUTO_BULK");

		v = e && !strcmp(e, "tree") ? LFA_ALGO_TREE : LFA_ALGO_P2P;
	}
	return v;
}

int lfa_coll_auto_algo(enum lfa_collective_op coll, size_t count, int nranks,
		       size_t esz, int p2p_ok)
{
	const size_t bytes = count * esz;
	const int os = nranks <= LFA_OS_MAX_RANKS;
	int bulk;

	if (!p2p_ok || nranks < 2 || nranks > LFA_SIG_MAX || !count)
		return LFA_ALGO_TREE;
	bulk = lfa_coll_auto_bulk();
	switch (coll) {
	case LFA_ALLREDUCE:
	case LFA_REDUCE:
		/* the planner's one-shot rule (plan_p2p): one kernel */
		return os && bytes * (size_t)nranks <= lfa_os_ag_bytes() ? LFA_ALGO_P2P : bulk;
	case LFA_REDUCE_SCATTER:
		return os && bytes <= lfa_os_rs_bytes() ? LFA_ALGO_P2P : bulk;
	default:
		return LFA_ALGO_TREE;
	}
}

/* LFA_ALGO_RCCL for one device-resident operation; 1 = handled. */
static int try_rccl(struct lfa_coll_mc *mc, enum lfa_collective_op coll,
		    const void *buf, void *result, size_t count, int root,
		    enum lfa_datatype dt, enum lfa_op op, hipStream_t s, int *ret)
{
	ncclDataType_t t;
	ncclRedOp_t o;
	ncclResult_t r;

	if (!rccl_type(dt, &t) || !rccl_op(op, &o))
		return 0;
	/* float MIN/MAX: RCCL's NaN and signed-zero rules are its own, not
	 * libfabric's dst-biased compare (util_atomic.c:291-316); the tree
	 * keeps the reference's bits */
	if ((op == LFA_MIN || op == LFA_MAX) &&
	    (dt == LFA_FLOAT || dt == LFA_DOUBLE))
		return 0;
	switch (coll) {
	case LFA_ALLREDUCE:
		r = ncclAllReduce(buf, result, count, t, o, mc->comm, s);
		break;
	case LFA_REDUCE_SCATTER:
		if (count % (size_t)mc->size)
			return 0;   /* ragged blocks: use the tree schedule */
		r = ncclReduceScatter(buf, result, count / (size_t)mc->size, t, o,
				      mc->comm, s);
		break;
	case LFA_REDUCE:
		r = ncclReduce(buf, result, count, t, o, root, mc->comm, s);
		break;
	default:
		return 0;
	}
	*ret = r == ncclSuccess ? 0 : -LFA_EIO;
	return 1;
}

/* Schedules depend only on shape: reuse the last few (repeated collectives
 * of one size are the common case, and building one allocates). */
static int cached_plan(struct lfa_coll_ep *ep, const struct plan **out,
		       enum lfa_collective_op coll, enum lfa_coll_algo algo,
		       int rank, int n, int root, size_t count, size_t esz)
{
	struct plan_cache *c;
	int ret;

	for (int i = 0; i < 8; i++) {
		c = &ep->pc[i];
		if (c->valid && c->coll == (int)coll && c->algo == (int)algo &&
		    c->rank == rank && c->n == n && c->root == root &&
		    c->count == count && c->esz == esz) {
			*out = &c->pl;
			return 0;
		}
	}
	c = &ep->pc[ep->pc_next++ % 8];
	if (c->valid)
		plan_free(&c->pl);
	c->valid = 0;
	ret = plan_make(&c->pl, coll, algo, rank, n, root, count, esz);
	if (ret)
		return ret;
	c->valid = 1;
	c->coll = (int)coll;
	c->algo = (int)algo;
	c->rank = rank;
	c->n = n;
	c->root = root;
	c->count = count;
	c->esz = esz;
	*out = &c->pl;
	return 0;
}

/*
 * One operation on device buffers, enqueued on ep->stream.
 */
LFA_INTERNAL int run_device(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
		      enum lfa_collective_op coll, const void *buf, void *result,
		      size_t count, int root, enum lfa_datatype dt,
		      enum lfa_op op, hipStream_t s, enum lfa_coll_algo algo)
{
	const struct plan *pl;
	size_t esz = lfa_datatype_size(dt);
	const enum lfa_coll_algo asked = algo;
	struct xctx x;
	int ret;

	ep->op_done_val = 0;
	ep->op_done_w = NULL;
	if (algo == LFA_ALGO_RCCL && mc->size > 1 &&
	    try_rccl(mc, coll, buf, result, count, root, dt, op, s, &ret))
		return ret;
	if (mc->size == 1 && s == ep->stream && ep->done_word &&
	    (coll == LFA_ALLREDUCE || coll == LFA_REDUCE || coll == LFA_REDUCE_SCATTER) &&
	    count * esz <= ep->solo_max)
		return run_solo(ep, buf, result, count, dt);
	if (algo == LFA_ALGO_AUTO)
		algo = (enum lfa_coll_algo)lfa_coll_auto_algo(coll, count, mc->size, esz,
							       mc->p2p_state >= 0);
replan:
	ret = cached_plan(ep, &pl, coll, algo, mc->rank, mc->size, root,
			  count, esz);
	if (ret)
		return ret;
	memset(&x, 0, sizeof(x));
	if (plan_uses_sym(pl->steps, pl->nsteps)) {
		ret = sig_ready(mc);
		if (ret)
			return ret;
		ret = p2p_ensure(mc, plan_sym_need(pl->steps, pl->nsteps, mc->size,
						   count, esz));
		if (ret && asked == LFA_ALGO_AUTO && mc->p2p_state == 0) {
			/* the members agreed (MIN over their flags, p2p_ensure)
			 * that some member cannot map a peer's workspace: every
			 * one of them runs the tree from now on */
			mc->p2p_state = -1;
			algo = LFA_ALGO_TREE;
			goto replan;
		}
		if (ret)
			return ret;
		mc->p2p_state = 1;
		x.ticket = ++mc->p2p_ticket;
		x.sym = mc->sym;
		x.region = mc->sym_region;
		if (pl->nsteps == 1 && pl->steps[0].type == LFA_STEP_ONESHOT &&
		    s == ep->stream && ep->done_word) {
			/* the small bucket is one kernel: it ends in the
			 * completion word, no event */
			x.done_ctr = ep->done_ctr;
			x.done_word = ep->done_word;
			x.done_seq = &ep->done_seq;
		}
	}
	ret = grow(&ep->ws, &ep->ws_size, pl->tmp, s);
	if (!ret) {
		x.base[LFA_BUF_SEND] = (void *)buf;
		x.base[LFA_BUF_RESULT] = result;
		x.base[LFA_BUF_TMP] = ep->ws;
		ret = exec_plan(mc, pl, &x, op, dt, s);
	}
	if (!ret)
		ep->op_done_val = x.done_val;
	return ret;
}

LFA_INTERNAL int check_reduce_args(enum lfa_datatype dt, enum lfa_op op)
{
	if (op < LFA_MIN || op > LFA_BXOR)
		return -LFA_ENOSYS;   /* coll_process_reduce_item :760-761 */
	if (lfa_atomic_valid(dt, op, 0))
		return -LFA_EOPNOTSUPP;
	return 0;
}

static int group_rank(struct lfa_coll_mc *mc, lfa_addr_t a)
{
	/* root_addr is a group rank (the reference indexes fi_addr_array by
	 * rank, coll_coll.c:782) */
	if (a >= (lfa_addr_t)mc->size)
		return -1;
	return (int)a;
}

/* Can this rank issue collectives on the group? */
LFA_INTERNAL int mc_member(const struct lfa_coll_mc *mc)
{
	return mc->rank >= 0 && (mc->ep->dom->host || mc->comm);
}

static ssize_t submit(struct lfa_coll_ep *ep, enum lfa_collective_op coll,
		      const void *buf, size_t count, void *result,
		      lfa_addr_t coll_addr, lfa_addr_t root_addr,
		      enum lfa_datatype dt, enum lfa_op op, void *context)
{
	struct lfa_coll_mc *mc;
	size_t esz, chunk;
	uint64_t t0, done_val = 0;
	const uint64_t *done_w = NULL;
	int root = -1, ret, host, chunkable, zc1 = 0;
	void *zb = NULL, *zr = NULL, *bnc = NULL;

	if (!ep)
		return -LFA_EINVAL;
	mc = mc_of(ep, coll_addr);
	if (!mc || !mc_member(mc))
		return -LFA_EINVAL;   /* not a member of this group */
	esz = lfa_datatype_size(dt);
	if (!esz)
		return -LFA_EINVAL;
	if (coll == LFA_REDUCE || coll == LFA_BROADCAST || coll == LFA_SCATTER) {
		root = group_rank(mc, root_addr);
		if (root < 0)
			return -LFA_EINVAL;
	}
	if (coll == LFA_ALLREDUCE || coll == LFA_REDUCE ||
	    coll == LFA_REDUCE_SCATTER) {
		ret = check_reduce_args(dt, op);
		if (ret)
			return ret;
	}
	if (ep->dom->host) {
		/* device buffers (a peer domain opened on a GPU): both must be
		 * device memory — the kernels read and write them in place */
		const void *in = coll == LFA_SCATTER && mc->rank != root ? NULL : buf;
		const void *out = coll == LFA_REDUCE && mc->rank != root ? NULL : result;
		int din = ep->dom->device >= 0 && in && count && is_device_ptr(in);
		int dout = ep->dom->device >= 0 && out && count && is_device_ptr(out);
		int dev = din || dout;

		if (dev && ((in && count && !din) || (out && count && !dout)))
			return -LFA_EINVAL;
		/* LFA_ALGO_P2P on a GPU peer domain: host buffers follow the
		 * device schedule too (staged), so members may still mix */
		if (!dev && ep->dom->device >= 0 && ep->algo == LFA_ALGO_P2P && count &&
		    mc->size > 1 && mc->size <= LFA_TREE_MAX && mc->size <= LFA_PUT_MAX &&
		    (coll == LFA_ALLREDUCE || coll == LFA_REDUCE_SCATTER ||
		     coll == LFA_REDUCE))
			dev = 2;
		pthread_mutex_lock(&ep->lock);
		if (dev && (chunk = peer_chunked(ep, mc, coll, count, esz)))
			ret = peer_submit_chunked(ep, mc, coll, buf, result, count, root, dt,
						  op, context, dev, chunk);
		else
			ret = host_submit(ep, mc, coll, buf, result, count, root, dt, op,
					  context, 0, NULL, dev, ep->algo);
		pthread_mutex_unlock(&ep->lock);
		return ret;
	}
	pthread_mutex_lock(&ep->lock);
	hipSetDevice(ep->dom->device);
	mc->seq++;                              /* coll_get_next_id :48-52 */
	t0 = mc->p2p_ticket;
	host = (buf && count && !is_device_ptr(buf)) ||
	       (result && count && !is_device_ptr(result));
	chunkable = coll == LFA_ALLREDUCE || coll == LFA_BROADCAST ||
		    coll == LFA_REDUCE ||
		    (coll == LFA_REDUCE_SCATTER && !(count % mc->size));
	/* the chunk this member stages with: a group chunk applies to every
	 * member alike, a local one only to a one-member group's host buffers
	 * (lfa_coll_member_chunk), so every member issues the same device
	 * collectives whatever memory its buffers are in */
	chunk = lfa_coll_member_chunk(mc->size, host,
				      lfa_coll_group_chunk(ep->group_chunk, mc->size,
							   count * esz),
				      ep->chunk);
	if (count && host && mc->size == 1 &&
	    (coll == LFA_ALLREDUCE || coll == LFA_REDUCE || coll == LFA_REDUCE_SCATTER)) {
		zb = zero_copy_of(buf, ep->dom->device);
		zr = zero_copy_of(result, ep->dom->device);
		if (zb && zr) {
			zc1 = 1;
		} else if (count * esz <= LFA_BOUNCE_BYTES && buf && result && !is_device_ptr(buf) &&
			   !is_device_ptr(result) && (bnc = bounce_get(ep))) {
			zb = zero_copy_of(bnc, ep->dom->device);
			zr = zero_copy_of((char *)bnc + LFA_BOUNCE_BYTES, ep->dom->device);
			if (zb && zr) {
				memcpy(bnc, buf, count * esz);
				zc1 = 2;
			} else {
				bounce_put(ep, bnc);
				bnc = NULL;
			}
		}
	}
	if (!count) {
		ret = 0;
	} else if (!host && chunk && chunkable &&
		   count * esz > chunk) {
		ret = run_device_chunked(ep, mc, coll, buf, result, count, root, dt, op,
					 chunk);
	} else if (!host) {
		/* a small bucket's one-shot kernel ends in the completion word */
		ep->op_done_val = 0;
		ep->op_done_w = NULL;
		ep->allow_direct = 1;
		ret = run_device(ep, mc, coll, buf, result, count, root, dt, op,
				 ep->stream, ep->algo);
		ep->allow_direct = 0;
		done_val = ep->op_done_val;
		done_w = ep->op_done_w;
	} else if (zc1) {
		/* a one-member group's reducing collective is a copy; with
		 * pinned host buffers it runs on their mappings over PCIe, no
		 * staging (32 MiB 1.35 -> 0.93 ms);
		 * pageable ones of at most LFA_BOUNCE_BYTES through a pinned
		 * bounce block (copied in here, out when reaped) */
		if (count * esz <= ep->solo_max) {
			ep->op_done_val = 0;
			ep->op_done_w = NULL;
			ret = run_solo(ep, zb, zr, count, dt);
			done_val = ep->op_done_val;
			done_w = ep->op_done_w;
		} else {
			ret = lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8, zr, zb,
						     count * esz, ep->stream);
		}
	} else if (chunkable) {
		ret = run_host_chunked(ep, mc, coll, buf, result, count, root, dt,
				       op, chunk);
	} else {
		size_t moff, mlen, in_b = count * esz, out_b = count * esz;

		lfa_coll_block(count, mc->size, mc->rank, &moff, &mlen);
		if (coll == LFA_REDUCE_SCATTER)
			out_b = mlen * esz;
		else if (coll == LFA_ALLGATHER)
			out_b = (size_t)mc->size * count * esz;
		else if (coll == LFA_SCATTER)
			in_b = mc->rank == root ? (size_t)mc->size * count * esz : 0;
		else if (coll == LFA_REDUCE && mc->rank != root)
			out_b = 0;
		ret = run_host_whole(ep, mc, coll, buf, in_b, result, out_b, count,
				     root, dt, op);
	}
	if (!ret)
		ret = enqueue_completion(ep, ep->stream, context, 0, NULL, done_val, done_w);
	if (!ret && bnc) {
		struct pending *p = &ep->q[(ep->qhead + ep->qlen - 1) % ep->qcap];

		p->bounce = bnc;
		p->bounce_out = (char *)bnc + LFA_BOUNCE_BYTES;
		p->bounce_user = result;
		p->bounce_bytes = count * esz;   /* one member: its block is everything */
	} else if (bnc) {
		/* the copy may be on the stream: wait before reusing the block */
		hipStreamSynchronize(ep->stream);
		bounce_put(ep, bnc);
	}
	if (!ret)
		tag_p2p(ep, mc, t0);
	pthread_mutex_unlock(&ep->lock);
	return ret;
}

ssize_t lfa_allreduce(struct lfa_coll_ep *ep, const void *buf, size_t count,
		      void *desc, void *result, void *result_desc,
		      lfa_addr_t coll_addr, enum lfa_datatype datatype,
		      enum lfa_op op, uint64_t flags, void *context)
{
	(void)desc; (void)result_desc; (void)flags;
	if (count && (!buf || !result))
		return -LFA_EINVAL;
	return submit(ep, LFA_ALLREDUCE, buf, count, result, coll_addr, 0,
		      datatype, op, context);
}

ssize_t lfa_reduce_scatter(struct lfa_coll_ep *ep, const void *buf,
			   size_t count, void *desc, void *result,
			   void *result_desc, lfa_addr_t coll_addr,
			   enum lfa_datatype datatype, enum lfa_op op,
			   uint64_t flags, void *context)
{
	(void)desc; (void)result_desc; (void)flags;
	if (count && (!buf || !result))
		return -LFA_EINVAL;
	return submit(ep, LFA_REDUCE_SCATTER, buf, count, result, coll_addr, 0,
		      datatype, op, context);
}

ssize_t lfa_reduce(struct lfa_coll_ep *ep, const void *buf, size_t count,
		   void *desc, void *result, void *result_desc,
		   lfa_addr_t coll_addr, lfa_addr_t root_addr,
		   enum lfa_datatype datatype, enum lfa_op op, uint64_t flags,
		   void *context)
{
	(void)desc; (void)result_desc; (void)flags;
	if (count && !buf)
		return -LFA_EINVAL;
	return submit(ep, LFA_REDUCE, buf, count, result, coll_addr, root_addr,
		      datatype, op, context);
}

ssize_t lfa_allgather(struct lfa_coll_ep *ep, const void *buf, size_t count,
		      void *desc, void *result, void *result_desc,
		      lfa_addr_t coll_addr, enum lfa_datatype datatype,
		      uint64_t flags, void *context)
{
	(void)desc; (void)result_desc; (void)flags;
	if (count && (!buf || !result))
		return -LFA_EINVAL;
	return submit(ep, LFA_ALLGATHER, buf, count, result, coll_addr, 0,
		      datatype, LFA_NOOP, context);
}

/* coll_ep_scatter (coll_coll.c:1121-1156): root's buf holds nranks blocks
 * of `count` elements, block r lands in rank r's result. */
ssize_t lfa_scatter(struct lfa_coll_ep *ep, const void *buf, size_t count,
		    void *desc, void *result, void *result_desc,
		    lfa_addr_t coll_addr, lfa_addr_t root_addr,
		    enum lfa_datatype datatype, uint64_t flags, void *context)
{
	(void)desc; (void)result_desc; (void)flags;
	if (count && !result)
		return -LFA_EINVAL;
	return submit(ep, LFA_SCATTER, buf, count, result, coll_addr, root_addr,
		      datatype, LFA_NOOP, context);
}

ssize_t lfa_broadcast(struct lfa_coll_ep *ep, void *buf, size_t count,
		      void *desc, lfa_addr_t coll_addr, lfa_addr_t root_addr,
		      enum lfa_datatype datatype, uint64_t flags, void *context)
{
	(void)desc; (void)flags;
	if (count && !buf)
		return -LFA_EINVAL;
	return submit(ep, LFA_BROADCAST, buf, count, buf, coll_addr, root_addr,
		      datatype, LFA_NOOP, context);
}

ssize_t lfa_barrier(struct lfa_coll_ep *ep, lfa_addr_t coll_addr, void *context)
{
	/* coll_ep_barrier2 (coll_coll.c:997-1033): an allreduce of ~rank with
	 * FI_BAND over one uint64. */
	struct lfa_coll_mc *mc;
	uint64_t t0;
	int ret;

	if (!ep)
		return -LFA_EINVAL;
	mc = mc_of(ep, coll_addr);
	if (!mc_member(mc))
		return -LFA_EINVAL;
	pthread_mutex_lock(&ep->lock);
	if (ep->dom->host) {
		struct hop *h = calloc(1, sizeof(*h));

		ret = h ? 0 : -LFA_ENOMEM;
		if (!ret) {
			h->scratch[0] = ~(uint64_t)mc->rank;
			mc->seq++;
			ret = host_start(ep, h, mc, LFA_ALLREDUCE, &h->scratch[0],
					 &h->scratch[1], 1, -1, LFA_UINT64, LFA_BAND, 0, ep->algo);
			if (!ret)
				ret = enqueue_host(ep, h, context, 0, NULL);
			if (ret)
				hop_free(h);
		}
		pthread_mutex_unlock(&ep->lock);
		return ret;
	}
	hipSetDevice(ep->dom->device);
	t0 = mc->p2p_ticket;
	ep->op_done_val = 0;
	ep->barrier_host[0] = ~(uint64_t)mc->rank;
	ret = hipMemcpyAsync(ep->barrier_dev, ep->barrier_host, sizeof(uint64_t),
			     hipMemcpyHostToDevice, ep->stream) == hipSuccess ?
	      0 : -LFA_EIO;
	if (!ret)
		ret = run_device(ep, mc, LFA_ALLREDUCE, ep->barrier_dev,
				 (uint64_t *)ep->barrier_dev + 1, 1, -1, LFA_UINT64,
				 LFA_BAND, ep->stream, ep->algo);
	if (!ret)
		ret = enqueue_completion(ep, ep->stream, context, 0, NULL, ep->op_done_val,
					 ep->op_done_w);
	if (!ret)
		tag_p2p(ep, mc, t0);
	pthread_mutex_unlock(&ep->lock);
	return ret;
}

/* ---------------------------------------------------------------------- */
/* query (coll_query_collective, coll_coll.c:1267-1318)                     */
/* ---------------------------------------------------------------------- */

int lfa_query_collective(struct lfa_coll_domain *domain,
			 enum lfa_collective_op coll,
			 struct lfa_collective_attr *attr, uint64_t flags)
{
	int ret;
	size_t esz;

	(void)domain;
	if (!attr || attr->mode != 0)
		return -LFA_EINVAL;
	switch (coll) {
	case LFA_BARRIER:
	case LFA_ALLGATHER:
	case LFA_SCATTER:
	case LFA_BROADCAST:
		ret = 0;
		break;
	case LFA_ALLREDUCE:
	case LFA_REDUCE_SCATTER:   /* new here: -FI_ENOSYS in the reference */
	case LFA_REDUCE:
		if (attr->op < LFA_MIN || attr->op > LFA_BXOR)
			return -LFA_ENOSYS;
		if (flags & LFA_TAGGED)
			return -LFA_EINVAL;          /* rxm_atomic.c:505-509 */
		ret = lfa_atomic_valid(attr->datatype, attr->op, flags);
		if (ret)
			return ret;
		esz = lfa_datatype_size(attr->datatype);
		attr->datatype_attr.size = esz;
		/* limited by HBM, not by an eager buffer: 64 GiB per buffer */
		attr->datatype_attr.count = (size_t)(64ULL << 30) / esz;
		break;
	case LFA_ALLTOALL:
	case LFA_GATHER:
	default:
		return -LFA_ENOSYS;
	}
	attr->max_members = ~(0x80000000u);
	return 0;
}
