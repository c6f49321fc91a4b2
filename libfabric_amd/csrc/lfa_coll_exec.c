/*
 * lfa_coll_exec.c — the collective provider's executor: ONE loop
 * (xrun_advance) runs a schedule whatever carries its transfers, over three
 * transport tables — xport_rccl (RCCL + the gfx950 kernels on the
 * endpoint stream), xport_peer (the owner provider's tagged transfers + the
 * host combine) and xport_peer_dev (the owner's transfers staged through
 * host bounce buffers + the kernels).  prov/coll's counterpart is the work
 * queue drained by coll_ep_progress (coll_coll.c:816-890) with its
 * FI_PEER_TRANSFER sends and receives (coll_coll.c:770-814).
 */
#define _GNU_SOURCE
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "lfa_coll_int.h"

LFA_INTERNAL hipError_t lfa_hip_note(int *slot, hipError_t e, const char *what)
{
	if (e != hipSuccess) {
		/* handled here: consume the thread's sticky HIP error, so the
		 * caller's next framework call (a torch launch check, say) does
		 * not report this failure as its own */
		(void)hipGetLastError();
		if (slot && !*slot)
			*slot = (int)e;
		if (lfa_param("LFA_DEBUG"))
			fprintf(stderr, "lfa: %s failed: %s (%d)\n", what,
				hipGetErrorString(e), (int)e);
	}
	return e;
}

LFA_INTERNAL void *resolve(const struct xctx *x, struct lfa_ref r)
{
	if (r.buf == LFA_BUF_SYM_IN)
		return x->sym[r.rank] + r.off;
	if (r.buf == LFA_BUF_SYM_OUT)
		return x->sym[r.rank] + x->region + r.off;
	return (char *)x->base[r.buf] + r.off;
}

#define LFA_COPY_KERNEL_BYTES ((size_t)16 << 20)

/* Non-communication step on `stream`. */
LFA_INTERNAL int run_local(const struct lfa_step *s, const struct lfa_ref *refs,
		     const struct xctx *x, enum lfa_op op,
		     enum lfa_datatype dt, hipStream_t stream)
{
	switch (s->type) {
	case LFA_STEP_REDUCE:
		return lfa_atomic_write_async(op, dt, resolve(x, s->dst),
					      resolve(x, s->src), s->count,
					      stream);
	case LFA_STEP_TREE: {
		const void *srcs[LFA_TREE_MAX];

		if (s->nsrc > LFA_TREE_MAX)
			return -LFA_EINVAL;
		for (uint32_t k = 0; k < s->nsrc; k++)
			srcs[k] = resolve(x, refs[s->first + k]);
		return lfa_reduce_tree_async(op, dt, resolve(x, s->dst), srcs,
					     (int)s->nsrc, s->count, stream);
	}
	case LFA_STEP_TREE_PUT: {
		const void *srcs[LFA_TREE_MAX];
		void *dsts[LFA_PUT_MAX];

		if (s->nsrc > LFA_TREE_MAX || s->peer < 0 || s->peer + 1 > LFA_PUT_MAX)
			return -LFA_EINVAL;
		for (uint32_t k = 0; k < s->nsrc; k++)
			srcs[k] = resolve(x, refs[s->first + k]);
		dsts[0] = resolve(x, s->dst);
		for (int j = 0; j < s->peer; j++)
			dsts[1 + j] = resolve(x, refs[s->first + s->nsrc + (uint32_t)j]);
		return lfa_reduce_tree_put_async(op, dt, dsts, 1 + s->peer, srcs,
						 (int)s->nsrc, s->count, stream);
	}
	case LFA_STEP_COPY:
		if (s->src.buf == LFA_BUF_SYM_IN || s->src.buf == LFA_BUF_SYM_OUT ||
		    s->dst.buf == LFA_BUF_SYM_IN || s->dst.buf == LFA_BUF_SYM_OUT) {
			/* the symmetric workspace, either way, through the P2P
			 * kernel: system-scope loads for bytes peers pushed into it
			 * (the unstage), and WRITE-THROUGH stores for bytes this
			 * rank stages into it.  A plain-store copy (hipMemcpyAsync's
			 * blit, the nt body) leaves the lines valid in this GPU's L2
			 * slices; peers later overwrite the same bytes — one-shot
			 * slots share SYM_IN with the staging area — through their
			 * IPC mappings, which do not invalidate them, and this rank's
			 * next one-shot read them stale (DESIGN.md §6b, round 3:
			 * the first one-shot after a two-barrier allreduce, 4+
			 * members).  sc0 sc1 stores drop the line instead. */
			void *d = resolve(x, s->dst);
			const void *sp = resolve(x, s->src);

			return lfa_reduce_tree_put_async(LFA_BOR, LFA_UINT8, &d, 1, &sp, 1,
							 s->count, stream);
		}
		/* large copies through the write table's ATOMIC_WRITE row (the
		 * LDS-DMA body, no dst read): 83.3 vs 98.8 us at 256 MiB and 12.3
		 * vs 14.5 us at 32 MiB against hipMemcpyAsync D2D, which stays
		 * ahead below (4.95 vs 5.43 us at 4 MiB; tools/probe_copy.py,
		 * profiles/r02_probe_copy.log).  COPY items never touch a peer's
		 * memory (the planner's copies stay in this rank's buffers). */
		if (s->count >= LFA_COPY_KERNEL_BYTES)
			return lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8,
						      resolve(x, s->dst), resolve(x, s->src),
						      s->count, stream);
		return hipMemcpyAsync(resolve(x, s->dst), resolve(x, s->src),
				      s->count, hipMemcpyDeviceToDevice,
				      stream) == hipSuccess ? 0 : -LFA_EIO;
	default:
		return -LFA_EINVAL;
	}
}

/* Does the plan address the symmetric workspace? */
LFA_INTERNAL int plan_uses_sym(const struct lfa_step *st, size_t nsteps)
{
	for (size_t i = 0; i < nsteps; i++)
		if (st[i].type == LFA_STEP_BARRIER || st[i].type == LFA_STEP_TREE_PUT ||
		    st[i].type == LFA_STEP_ONESHOT)
			return 1;
	return 0;
}

/* Bytes of one symmetric-workspace region for `count` elements. */
LFA_INTERNAL size_t sym_region(size_t count, size_t esz)
{
	return (count * esz + 255) & ~(size_t)255;
}

/* One ONESHOT slot: the largest part any member reduces. */
static size_t os_slot(const struct lfa_step *st, int n, size_t esz)
{
	size_t part = st->count;

	if (st->peer == LFA_ONESHOT_SCATTER)
		part = (st->count + (size_t)n - 1) / (size_t)n;
	return sym_region(part, esz);
}

LFA_INTERNAL size_t plan_sym_need(const struct lfa_step *st, size_t nsteps, int n,
				  size_t count, size_t esz)
{
	size_t need = sym_region(count, esz);

	for (size_t i = 0; i < nsteps; i++)
		if (st[i].type == LFA_STEP_ONESHOT &&
		    2 * (size_t)n * os_slot(&st[i], n, esz) > need)
			need = 2 * (size_t)n * os_slot(&st[i], n, esz);
	return need;
}


/* How long a flag barrier waits for a member before failing the operation
 * (LFA_SIG_TIMEOUT_MS, default 20 s). */
static uint64_t sig_timeout_us(void)
{
	static uint64_t us;

	if (!us) {
		const char *e = lfa_param("LFA_SIG_TIMEOUT_MS");
		long ms = e ? atol(e) : 0;

		us = (uint64_t)(ms > 0 ? ms : 20000) * 1000;
	}
	return us;
}

/*
 * BARRIER of a plan on the symmetric workspace, stream-ordered: the one-wave
 * flag kernel (lfa_signal.hip) posts this group's next epoch into every
 * peer's barrier row and waits for theirs in its own — no RCCL collective,
 * no host round trip.  The peers' rows are the IPC mappings the workspace
 * handshake set up, so it runs wherever the P2P kernels do (RCCL device
 * domains and GPU peer domains alike).
 */
LFA_INTERNAL int sig_barrier(struct xrun *r)
{
	struct lfa_coll_mc *mc = r->mc;
	const size_t row = 2 * r->x.region + LFA_SIG_BAR_OFF;
	uint32_t *post[LFA_SIG_MAX];
	int ret;

	if (!r->x.sym || mc->size > LFA_SIG_MAX || !mc->sig_word)
		return -LFA_EINVAL;
	for (int k = 0; k < mc->size; k++)
		post[k] = k == mc->rank ? NULL :
			  (uint32_t *)(r->x.sym[k] + row) + mc->rank;
	ret = lfa_flag_barrier_async(post, (const uint32_t *)(r->x.sym[mc->rank] + row),
				     mc->size, mc->rank, mc->bar_epoch + 1,
				     mc->sig_word, r->x.ticket, sig_timeout_us(), r->stream);
	if (!ret) {
		mc->bar_epoch++;
		mc->n_barrier++;
	}
	return ret;
}

LFA_INTERNAL int sig_oneshot(struct xrun *r, const struct lfa_step *st)
{
	struct lfa_coll_mc *mc = r->mc;
	size_t esz = lfa_datatype_size(r->dt);
	struct lfa_oneshot a;
	int ret;

	if (!r->x.sym || !mc->sig_word || !esz || (int)st->nsrc != mc->size ||
	    2 * (size_t)mc->size * os_slot(st, mc->size, esz) > r->x.region)
		return -LFA_EINVAL;
	memset(&a, 0, sizeof(a));
	a.send = resolve(&r->x, st->src);
	/* reduce: a non-root has no result */
	a.result = st->peer >= 0 && st->peer != mc->rank ? NULL : resolve(&r->x, st->dst);
	a.count = st->count;
	a.mode = st->peer;
	a.sym = r->x.sym;
	a.slot_bytes = os_slot(st, mc->size, esz);
	a.parity_off = (r->x.region / 2) & ~(size_t)255;   /* the same on every member */
	a.flag_off = 2 * r->x.region;
	a.n = mc->size;
	a.rank = mc->rank;
	a.epoch = mc->os_epoch + 1;
	a.status = mc->sig_word;
	a.ticket = r->x.ticket;
	a.timeout_us = sig_timeout_us();
	if (r->x.done_word && r->x.done_seq) {
		a.done_ctr = r->x.done_ctr;
		a.done_word = r->x.done_word;
		a.done_val = *r->x.done_seq + 1;
	}
	ret = lfa_oneshot_reduce_async(r->op, r->dt, &a, r->stream);
	if (!ret && a.done_word)
		r->x.done_val = ++*r->x.done_seq;
	LFA_TRACE("cid %#x one-shot launched (epoch %u, rc %d)", (unsigned)r->cid, a.epoch, ret);
	if (!ret) {
		mc->os_epoch++;
		mc->n_oneshot++;
	}
	return ret;
}

/* Run the schedule as far as it goes: 1 done, 0 waiting on transfers, <0.
 * A post that returns -LFA_EAGAIN (the owner's queue is full: prov/coll
 * requeues such items, coll_coll.c:845-852) is retried on the next call. */
LFA_INTERNAL int xrun_advance(struct xrun *r)
{
	const struct plan *pl = r->pl;
	int ret;

	while (r->pc < pl->nsteps) {
		const struct lfa_step *st = &pl->steps[r->pc];
		size_t end;
		int pending = 0;

		switch (st->type) {
		case LFA_STEP_GROUP_END:
			r->pc++;
			continue;
		case LFA_STEP_SEND:
		case LFA_STEP_RECV:
			break;
		case LFA_STEP_ALLTOALL:
		case LFA_STEP_ALLGATHER:
		case LFA_STEP_BARRIER:
			ret = r->xp->coll(r, st);
			if (ret)
				return ret;
			r->pc++;
			continue;
		default:
			ret = r->xp->local(r, st);
			if (ret)
				return ret;
			r->pc++;
			continue;
		}
		for (end = r->pc; end < pl->nsteps &&
		     pl->steps[end].type != LFA_STEP_GROUP_END; end++)
			;
		if (r->nreq < end - r->pc) {
			size_t need = end - r->pc;

			if (r->xp->test && need > r->creq) {
				void **nr = realloc(r->reqs, need * sizeof(*nr));

				if (!nr)
					return -LFA_ENOMEM;
				r->reqs = nr;
				r->creq = need;
			}
			ret = r->xp->group_start(r);
			while (!ret && r->nreq < need) {
				void *req = NULL;

				ret = r->xp->post(r, &pl->steps[r->pc + r->nreq], &req);
				if (!ret && r->xp->test)
					r->reqs[r->nreq] = req;
				if (!ret)
					r->nreq++;
			}
			if (r->xp->group_end(r) && !ret)
				ret = -LFA_EIO;
			if (ret == -LFA_EAGAIN)
				pending = 1;
			else if (ret)
				return ret;
		}
		for (size_t i = 0; r->xp->test && i < r->nreq; i++) {
			if (!r->reqs[i])
				continue;
			ret = r->xp->test(r, r->reqs[i]);
			if (ret < 0)
				return ret;
			if (ret)
				r->reqs[i] = NULL;
			else
				pending = 1;
		}
		if (pending)
			return 0;
		r->nreq = 0;
		r->pc = end < pl->nsteps ? end + 1 : end;
	}
	return 1;
}


/* ---- xport_peer: the owner's tagged transfers + the host combine ------ */

static int peer_nop(struct xrun *r)
{
	return 0;
}

static int peer_post(struct xrun *r, const struct lfa_step *st, void **req)
{
	const struct lfa_coll_domain *d = r->mc->ep->dom;

	/* coll_form_tag (coll_coll.c:37-45): cid | the SENDING rank << 32 */
	if (st->type == LFA_STEP_SEND)
		return d->xops.send(d->xctx, world_rank(r->mc, st->peer),
				    resolve(&r->x, st->src), st->count,
				    r->cid | (uint64_t)r->mc->rank << 32, req);
	return d->xops.recv(d->xctx, world_rank(r->mc, st->peer),
			    resolve(&r->x, st->dst), st->count,
			    r->cid | (uint64_t)st->peer << 32, req);
}

static int peer_test(struct xrun *r, void *req)
{
	const struct lfa_coll_domain *d = r->mc->ep->dom;

	return d->xops.test(d->xctx, req);
}

static int peer_local(struct xrun *r, const struct lfa_step *st)
{
	switch (st->type) {
	case LFA_STEP_REDUCE:
		return lfa_host_write(r->op, r->dt, resolve(&r->x, st->dst),
				      resolve(&r->x, st->src), st->count);
	case LFA_STEP_TREE: {
		const void *srcs[LFA_TREE_MAX];

		if (st->nsrc > LFA_TREE_MAX)
			return -LFA_EINVAL;
		for (uint32_t k = 0; k < st->nsrc; k++)
			srcs[k] = resolve(&r->x, r->pl->refs[st->first + k]);
		return lfa_host_reduce_tree(r->op, r->dt, resolve(&r->x, st->dst),
					    srcs, (int)st->nsrc, st->count);
	}
	case LFA_STEP_COPY:
		memmove(resolve(&r->x, st->dst), resolve(&r->x, st->src), st->count);
		return 0;
	default:
		return -LFA_EINVAL;     /* TREE_PUT: P2P plans are not used here */
	}
}

static int peer_coll(struct xrun *r, const struct lfa_step *st)
{
	return -LFA_EINVAL;             /* lowered to SEND/RECV by host_start */
}

LFA_INTERNAL const struct xport xport_peer = {
	peer_nop, peer_post, peer_nop, peer_test, peer_local, peer_coll,
};

/* device hops: a P2P plan's BARRIER is the flag kernel (host_start keeps it
 * unlowered); ALLTOALL / ALLGATHER were lowered to transfers */
static int pdev_coll(struct xrun *r, const struct lfa_step *st)
{
	if (st->type != LFA_STEP_BARRIER)
		return -LFA_EINVAL;
	return sig_barrier(r);
}

/*
 * ---- xport_peer_dev: device buffers over the owner's transfers ----------
 * The owner moves host bytes only (an FI_HMEM-less rxm), so every transfer
 * is staged: a SEND copies its device bytes — as the endpoint stream has
 * them after the items enqueued before it — into a host bounce buffer and
 * sends that; a RECV lands in a bounce buffer and is copied to the device
 * on the stream before the group counts as done.  REDUCE / TREE / COPY are
 * the gfx950 kernels on the endpoint stream.  The schedule (and so every
 * tag and size) is the host form's, so members may mix host and device
 * buffers freely.
 */
struct stg {
	void *inner;            /* the owner's request */
	char *bounce;
	void *dst;              /* RECV: device destination */
	size_t n;
};

static int pdev_post(struct xrun *r, const struct lfa_step *st, void **req)
{
	const struct lfa_coll_domain *d = r->mc->ep->dom;
	struct stg *g = calloc(1, sizeof(*g));
	int ret;

	if (!g || !(g->bounce = malloc(st->count ? st->count : 1))) {
		free(g);
		return -LFA_ENOMEM;
	}
	g->n = st->count;
	if (st->type == LFA_STEP_SEND) {
		/* the stream first: a zero-byte send is a barrier arrival and
		 * must leave only after this rank's earlier items completed */
		LFA_TRACE("cid %#x send to %d: stream sync", (unsigned)r->cid, st->peer);
		if (lfa_hip_note(&r->hip_err, hipStreamSynchronize(r->stream),
				 "send: stream sync") != hipSuccess ||
		    (st->count &&
		     (lfa_hip_note(&r->hip_err,
				   hipMemcpyAsync(g->bounce, resolve(&r->x, st->src), st->count,
						  hipMemcpyDeviceToHost, r->stream),
				   "send: D2H staging") != hipSuccess ||
		      lfa_hip_note(&r->hip_err, hipStreamSynchronize(r->stream),
				   "send: stream sync after D2H") != hipSuccess)))
			ret = -LFA_EIO;
		else
			ret = d->xops.send(d->xctx, world_rank(r->mc, st->peer), g->bounce,
					   st->count, r->cid | (uint64_t)r->mc->rank << 32,
					   &g->inner);
	} else {
		g->dst = st->count ? resolve(&r->x, st->dst) : NULL;
		ret = d->xops.recv(d->xctx, world_rank(r->mc, st->peer), g->bounce,
				   st->count, r->cid | (uint64_t)st->peer << 32, &g->inner);
	}
	if (ret) {
		free(g->bounce);
		free(g);
		return ret;
	}
	*req = g;
	return 0;
}

static int pdev_test(struct xrun *r, void *req)
{
	const struct lfa_coll_domain *d = r->mc->ep->dom;
	struct stg *g = req;
	int ret = d->xops.test(d->xctx, g->inner);

	if (ret == 0)
		return 0;
	if (ret > 0 && g->dst &&
	    (lfa_hip_note(&r->hip_err,
			  hipMemcpyAsync(g->dst, g->bounce, g->n, hipMemcpyHostToDevice,
					 r->stream), "recv: H2D staging") != hipSuccess ||
	     lfa_hip_note(&r->hip_err, hipStreamSynchronize(r->stream),
			  "recv: stream sync after H2D") != hipSuccess))
		ret = -LFA_EIO;
	free(g->bounce);
	free(g);
	return ret;
}

static int pdev_local(struct xrun *r, const struct lfa_step *st)
{
	if (st->type == LFA_STEP_ONESHOT)
		return sig_oneshot(r, st);
	return run_local(st, r->pl->refs, &r->x, r->op, r->dt, r->stream);
}

LFA_INTERNAL const struct xport xport_peer_dev = {
	peer_nop, pdev_post, peer_nop, pdev_test, pdev_local, pdev_coll,
};

/* ---------------------------------------------------------------------- */
/* executor: schedule -> RCCL + kernels on the endpoint stream             */
/* ---------------------------------------------------------------------- */

/* ---- xport_rccl: RCCL over xGMI + the gfx950 kernels, stream-ordered -- */

static int rccl_group_start(struct xrun *r)
{
	return ncclGroupStart() == ncclSuccess ? 0 : -LFA_EIO;
}

static int rccl_group_end(struct xrun *r)
{
	return ncclGroupEnd() == ncclSuccess ? 0 : -LFA_EIO;
}

static int rccl_post(struct xrun *r, const struct lfa_step *st, void **req)
{
	ncclResult_t e;

	if (st->type == LFA_STEP_SEND)
		e = ncclSend(resolve(&r->x, st->src), st->count, ncclUint8, st->peer,
			     r->mc->comm, r->stream);
	else
		e = ncclRecv(resolve(&r->x, st->dst), st->count, ncclUint8, st->peer,
			     r->mc->comm, r->stream);
	return e == ncclSuccess ? 0 : -LFA_EIO;
}

static int rccl_local(struct xrun *r, const struct lfa_step *st)
{
	if (st->type == LFA_STEP_ONESHOT)
		return sig_oneshot(r, st);
	return run_local(st, r->pl->refs, &r->x, r->op, r->dt, r->stream);
}

static int rccl_coll(struct xrun *r, const struct lfa_step *st)
{
	ncclComm_t c = r->mc->comm;
	ncclResult_t e;

	switch (st->type) {
	case LFA_STEP_ALLTOALL:
		e = ncclAllToAll(resolve(&r->x, st->src), resolve(&r->x, st->dst),
				 st->count, ncclUint8, c, r->stream);
		break;
	case LFA_STEP_ALLGATHER:
		e = ncclAllGather(resolve(&r->x, st->src), resolve(&r->x, st->dst),
				  st->count, ncclUint8, c, r->stream);
		break;
	default: {
		/* BARRIER, stream-ordered.  On the symmetric workspace (P2P
		 * plans): the flag kernel.  Otherwise a one-word allreduce,
		 * which completes on a rank only after every member's stream
		 * has reached it. */
		uint64_t *w = (uint64_t *)r->mc->ep->barrier_dev + 2;

		if (r->x.sym)
			return sig_barrier(r);
		e = ncclAllReduce(w, w, 1, ncclUint64, ncclSum, c, r->stream);
	}
	}
	return e == ncclSuccess ? 0 : -LFA_EIO;
}

static const struct xport xport_rccl = {
	rccl_group_start, rccl_post, rccl_group_end, NULL, rccl_local, rccl_coll,
};

/* Enqueue a whole schedule on `s` (one xrun_advance pass runs it all). */
LFA_INTERNAL int exec_plan(struct lfa_coll_mc *mc, const struct plan *pl,
		     struct xctx *x, enum lfa_op op, enum lfa_datatype dt,
		     hipStream_t s)
{
	struct xrun r;
	int ret;

	memset(&r, 0, sizeof(r));
	r.xp = &xport_rccl;
	r.pl = pl;
	r.x = *x;
	r.mc = mc;
	r.op = op;
	r.dt = dt;
	r.stream = s;
	ret = xrun_advance(&r);
	/* sig_oneshot reports the word value in the run's copy (the
	 * caller's stayed 0, so device-domain one-shots completed by event) */
	x->done_val = r.x.done_val;
	return ret == 1 ? 0 : ret ? ret : -LFA_EIO;
}
