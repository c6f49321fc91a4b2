/*
 * lfa_coll_host.c — host buffers and host (peer-transfer) operations of the
 * collective provider (liblfa_coll.so; split out of lfa_coll.c in round 6):
 * a hop (one operation of a peer domain, prov/coll's util_coll_operation and
 * work queue, ofi_coll.h:146-163) and its progress, the P2P prologue run
 * from progress, the peer domain's staging pool and pinned bounce blocks,
 * zero-copy classification, and the device domains' pipelined staging of
 * host buffers.
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

LFA_INTERNAL int is_device_ptr(const void *p)
{
	hipPointerAttribute_t a;

	if (!p)
		return 0;
	if (hipPointerGetAttributes(&a, p) != hipSuccess) {
		(void)hipGetLastError();
		return 0;
	}
	return a.type == hipMemoryTypeDevice || a.type == hipMemoryTypeManaged;
}

/* Zero-copy operand address (lfa_zero_copy_addr, liblfa: pinned or
 * registered host memory through its mapping, `dev`'s memory as it is), or
 * NULL: stage. */
LFA_INTERNAL void *zero_copy_of(const void *p, int dev)
{
	return lfa_zero_copy_addr(p, dev);
}

/* Both host-staging slots, always the same size. */
LFA_INTERNAL int grow_staging(struct lfa_coll_ep *ep, size_t need)
{
	void *nb[2];

	if (need <= ep->hs_size)
		return 0;
	need = (need + (1u << 20) - 1) & ~(size_t)((1u << 20) - 1);
	for (int i = 0; i < 2; i++) {
		if (hipMallocAsync(&nb[i], need, ep->stream) != hipSuccess) {
			if (i)
				hipFreeAsync(nb[0], ep->stream);
			return -LFA_ENOMEM;
		}
	}
	for (int i = 0; i < 2; i++) {
		if (ep->hs[i])
			hipFreeAsync(ep->hs[i], ep->stream);
		ep->hs[i] = nb[i];
	}
	ep->hs_size = need;
	return 0;
}

/* A device buffer of at least `bytes` from the endpoint's staging pool (the
 * smallest free one that fits and is at most twice the size, else a free
 * slot (re)allocated to `bytes`), or a plain hipMalloc when every slot is
 * busy; NULL on failure.  ep->lock held.  stage_put returns it.  (Without
 * the factor-2 bound, 32 MiB chunks took the idle 64 MiB buffers of an
 * earlier size first and allocated the rest, so every operation passed the
 * cap and the trim churned: 13.1 -> 19.3 ms for 32 MiB chunks after 64.) */
static void *stage_get(struct lfa_coll_ep *ep, size_t bytes)
{
	struct stage_buf *fit = NULL, *spare = NULL;
	void *p;

	if (!bytes)
		bytes = 1;
	for (int i = 0; i < LFA_STAGE_POOL; i++) {
		struct stage_buf *b = &ep->stage[i];

		if (b->busy)
			continue;
		if (b->p && b->bytes >= bytes && b->bytes / 2 <= bytes &&
		    (!fit || b->bytes < fit->bytes))
			fit = b;
		else if (!spare || (spare->p && !b->p))
			spare = b;      /* prefer an empty slot */
	}
	if (fit) {
		fit->busy = 1;
		fit->used = ++ep->stage_clock;
		return fit->p;
	}
	if (spare) {
		if (spare->p)
			hipFree(spare->p);
		spare->p = NULL;
		spare->bytes = 0;
		if (hipMalloc(&spare->p, bytes) != hipSuccess) {
			spare->p = NULL;
			return NULL;
		}
		spare->bytes = bytes;
		spare->busy = 1;
		spare->used = ++ep->stage_clock;
		return spare->p;
	}
	return hipMalloc(&p, bytes) == hipSuccess ? p : NULL;
}

/* Idle bytes in the staging pool (ep->lock held). */
static size_t stage_idle(const struct lfa_coll_ep *ep)
{
	size_t idle = 0;

	for (int i = 0; i < LFA_STAGE_POOL; i++)
		if (ep->stage[i].p && !ep->stage[i].busy)
			idle += ep->stage[i].bytes;
	return idle;
}

/* Free idle staging buffers, least recently used first, until at most `keep`
 * idle bytes remain (ep->lock held).  hipFree waits for the device, so this
 * runs only where nothing of the endpoint is in flight.  (Largest-first
 * evicted the buffers the current operation size had just allocated, so a
 * size sweep reallocated on every operation: 256 MiB whole 20.3 -> 28.9 ms.) */
LFA_INTERNAL void stage_trim(struct lfa_coll_ep *ep, size_t keep)
{
	while (stage_idle(ep) > keep) {
		struct stage_buf *old = NULL;

		for (int i = 0; i < LFA_STAGE_POOL; i++) {
			struct stage_buf *b = &ep->stage[i];

			if (b->p && !b->busy && (!old || b->used < old->used))
				old = b;
		}
		if (!old)
			break;
		hipFree(old->p);
		old->p = NULL;
		old->bytes = 0;
	}
}

/* Back to the pool.  When the pool's idle bytes pass the cap
 * (LFA_STAGE_POOL_BYTES; ADVICE r3: a sweep of sizes or many chunks in
 * flight otherwise pinned the sum of every buffer until close) the excess
 * is freed once the endpoint's queue has drained (progress), not here: a
 * hipFree in the middle of a pipelined operation would stall it (a first
 * form freed here and doubled a 2-process 256 MiB host allreduce in 16 MiB
 * chunks, 13.1 -> 25.7 ms). */
static void stage_put(struct lfa_coll_ep *ep, void *p)
{
	if (!p)
		return;
	for (int i = 0; i < LFA_STAGE_POOL; i++)
		if (ep->stage[i].p == p) {
			ep->stage[i].busy = 0;
			if (stage_idle(ep) > ep->stage_cap)
				ep->stage_trim_due = 1;
			return;
		}
	hipFree(p);
}

size_t lfa_coll_ep_stage_bytes(struct lfa_coll_ep *ep)
{
	size_t n = 0;

	if (!ep)
		return 0;
	pthread_mutex_lock(&ep->lock);
	for (int i = 0; i < LFA_STAGE_POOL; i++)
		if (ep->stage[i].p)
			n += ep->stage[i].bytes;
	pthread_mutex_unlock(&ep->lock);
	return n;
}

/* A free pinned bounce block (2 x LFA_BOUNCE_BYTES), or NULL when all are
 * busy or none can be allocated (ep->lock held). */
LFA_INTERNAL void *bounce_get(struct lfa_coll_ep *ep)
{
	for (int i = 0; i < LFA_BOUNCE_POOL; i++) {
		struct bounce_buf *b = &ep->bounce[i];

		if (b->busy)
			continue;
		if (!b->p && hipHostMalloc(&b->p, 2 * (size_t)LFA_BOUNCE_BYTES, 0) != hipSuccess) {
			(void)hipGetLastError();
			b->p = NULL;
			return NULL;
		}
		b->busy = 1;
		return b->p;
	}
	return NULL;
}

LFA_INTERNAL void bounce_put(struct lfa_coll_ep *ep, void *p)
{
	for (int i = 0; p && i < LFA_BOUNCE_POOL; i++)
		if (ep->bounce[i].p == p)
			ep->bounce[i].busy = 0;
}

/* A block a failed operation's kernel may still touch: out of the pool for
 * good (its pinned memory is left allocated, with a line on stderr). */
LFA_INTERNAL void bounce_retire(struct lfa_coll_ep *ep, void *p)
{
	for (int i = 0; p && i < LFA_BOUNCE_POOL; i++)
		if (ep->bounce[i].p == p) {
			ep->bounce[i].p = NULL;
			ep->bounce[i].busy = 0;
			ep->bounce_retired++;
			fprintf(stderr, "lfa: a failed operation's bounce block (%p) is kept "
				"out of the pool: its kernel may still run\n", p);
		}
}

/* Endpoint close: the pinned bounce blocks back to the runtime, or, when
 * the endpoint did not drain (a kernel may still write one), kept. */
LFA_INTERNAL void bounce_free_all(struct lfa_coll_ep *ep, int drained)
{
	for (int i = 0; i < LFA_BOUNCE_POOL; i++) {
		if (ep->bounce[i].p && drained)
			hipHostFree(ep->bounce[i].p);
		ep->bounce[i].p = NULL;
	}
}

/* A completed hop's result to the caller's pageable buffer (the kernels
 * wrote it to the bounce block's mapping; the completion word or event
 * that ended the hop made it visible to the host). */
static void bounce_finish(struct hop *h)
{
	if (h->bounce_bytes)
		memcpy(h->bounce_user, h->bounce_out, h->bounce_bytes);
	h->bounce_bytes = 0;
}

LFA_INTERNAL void hop_free(struct hop *h)
{
	if (!h)
		return;
	hop_free(h->sub);
	plan_free(&h->pl);
	if (h->dev) {
		/* a failed run may have left items on the stream that use tmp, and
		 * staging copies in flight on the copy streams; a finished one
		 * has passed its events already */
		if (!h->done)
			hipStreamSynchronize(h->r.stream);
		if (h->in_ev) {
			if (!h->done)
				hipEventSynchronize(h->in_ev);
			release_event(h->ep, h->in_ev);
		}
		if (h->out_ev) {
			if (!h->done)
				hipEventSynchronize(h->out_ev);
			release_event(h->ep, h->out_ev);
		}
		stage_put(h->ep, h->tmp);
		stage_put(h->ep, h->st_in);
		stage_put(h->ep, h->st_out);
		if (h->fin)
			release_event(h->ep, h->fin);
	} else {
		free(h->tmp);
	}
	/* after the stream sync above when the hop had not finished (a hop
	 * that failed before it became a device hop never launched) */
	bounce_put(h->ep, h->bounce);
	free(h->r.reqs);
	free(h);
}

static int hop_prologue(struct lfa_coll_ep *ep, struct hop *h, size_t idx);

/* Advance every in-flight host operation (ep->lock held). */
LFA_INTERNAL void host_progress_all(struct lfa_coll_ep *ep)
{
	/* device hops issue HIP calls from whichever thread progresses (e.g.
	 * off_lfa's progress thread): make the domain's GPU current there */
	if (ep->dom->device >= 0 && ep->qlen)
		hipSetDevice(ep->dom->device);
	for (size_t i = 0; i < ep->qlen; i++) {
		struct hop *h = ep->q[(ep->qhead + i) % ep->qcap].hop;
		int ret;

		if (!h || h->done || h->err)
			continue;
		if (h->phase != HOP_RUN) {
			ret = hop_prologue(ep, h, i);
			if (ret < 0)
				h->err = ret;
			if (h->phase != HOP_RUN || h->err)
				continue;
		}
		if (h->in_ev && !h->in_waited) {
			/* the staged input's H2D (copy stream) before the first item */
			if (lfa_hip_note(&h->r.hip_err, hipStreamWaitEvent(h->r.stream, h->in_ev, 0),
					 "staged input wait") != hipSuccess) {
				h->err = -LFA_EIO;
				continue;
			}
			h->in_waited = 1;
		}
		ret = h->issued ? 1 : xrun_advance(&h->r);
		if (ret < 0) {
			h->err = ret;
		} else if (ret && h->dev) {
			/* done once the stream has run the last local items (and, for
			 * staged host buffers, the D2H behind them) */
			hipEvent_t last;
			hipError_t e;

			if (!h->issued && h->r.x.done_val) {
				h->issued = 1;
				h->ww.armed = 0;    /* armed at the head of the queue */
				if (ep->drop_words > 0) {
					ep->drop_words--;
					h->r.x.done_val |= 1ull << 62;
				}
				LFA_TRACE("hop cid %#x issued (completion word %llu)",
					  (unsigned)h->r.cid, (unsigned long long)h->r.x.done_val);
			}
			if (!h->issued) {
				if (!(h->fin = event_get(ep)) ||
				    lfa_hip_note(&h->r.hip_err, hipEventRecord(h->fin, h->r.stream),
						 "completion event record") != hipSuccess) {
					h->err = -LFA_EIO;
					continue;
				}
				if (h->out_bytes &&
				    (!(h->out_ev = event_get(ep)) ||
				     lfa_hip_note(&h->r.hip_err,
						  hipStreamWaitEvent(ep->d2h_stream, h->fin, 0),
						  "staged result wait") != hipSuccess ||
				     lfa_hip_note(&h->r.hip_err,
						  hipMemcpyAsync(h->user_out, h->st_out, h->out_bytes,
								 hipMemcpyDeviceToHost, ep->d2h_stream),
						  "staged result D2H") != hipSuccess ||
				     lfa_hip_note(&h->r.hip_err, hipEventRecord(h->out_ev, ep->d2h_stream),
						  "staged result event record") != hipSuccess)) {
					h->err = -LFA_EIO;
					continue;
				}
				h->issued = 1;
				LFA_TRACE("hop cid %#x issued", (unsigned)h->r.cid);
			}
			if (h->r.x.done_val) {
				int werr = 0;

				if (*(volatile uint64_t *)ep->done_word >= h->r.x.done_val) {
					ep->word_ops++;
					bounce_finish(h);
					h->done = 1;
					LFA_TRACE("hop cid %#x done", (unsigned)h->r.cid);
				} else if (i == 0 &&    /* only the head's bound runs */
					   word_overdue(ep, ep->done_word, h->r.stream, &h->ww,
							&werr) < 0) {
					/* ETIMEDOUT / EIO as the error entry's err;
					 * a stream's HIP code as its prov_errno */
					if (werr != ETIMEDOUT && werr != EIO)
						h->r.hip_err = werr;
					h->err = werr == ETIMEDOUT ? -ETIMEDOUT : -LFA_EIO;
					LFA_TRACE("hop cid %#x word overdue (%d)", (unsigned)h->r.cid, werr);
				}
				continue;
			}
			last = h->out_ev ? h->out_ev : h->fin;
			e = hipEventQuery(last);
			if (e == hipSuccess) {
				bounce_finish(h);
				h->done = 1;
				LFA_TRACE("hop cid %#x done", (unsigned)h->r.cid);
			} else if (e != hipErrorNotReady &&
				 lfa_hip_note(&h->r.hip_err, e, "completion event query"))
				h->err = -LFA_EIO;
		} else if (ret) {
			h->done = 1;
		}
	}
}

LFA_INTERNAL int enqueue_host(struct lfa_coll_ep *ep, struct hop *h, void *context,
			int kind, struct lfa_coll_mc *mc)
{
	struct pending *p = queue_slot(ep);

	if (!p)
		return -LFA_ENOMEM;
	memset(p, 0, sizeof(*p));
	p->hop = h;
	p->context = context;
	p->kind = kind;
	p->mc = mc;
	ep->qlen++;
	/* kick: run up to the first transfer now (coll_progress_work) */
	host_progress_all(ep);
	return 0;
}

/* A handshake collective of hop `h` on its reserved seq (host buffers). */
static int sub_start(struct lfa_coll_ep *ep, struct hop *h, enum lfa_collective_op coll,
		     const void *buf, void *result, size_t count,
		     enum lfa_datatype dt, enum lfa_op op, uint16_t seq)
{
	struct lfa_coll_mc *mc = h->r.mc;
	int ret;

	h->sub = calloc(1, sizeof(*h->sub));
	if (!h->sub)
		return -LFA_ENOMEM;
	/* a fixed schedule: the handshake starts from progress, at a different
	 * point of each member's calls, so the endpoint's algorithm then (the
	 * caller may have selected another for later operations) can differ
	 * between members */
	ret = host_start(ep, h->sub, mc, coll, buf, result, count, -1, dt, op, 0,
			 LFA_ALGO_TREE);
	h->sub->r.cid = (uint64_t)mc->group_id << 16 | seq;
	LFA_TRACE("hop cid %#x handshake %d on cid %#x (mc seq now %u)", (unsigned)h->r.cid,
		  (int)coll, (unsigned)h->sub->r.cid, (unsigned)mc->seq);
	return ret;
}

/* Run the current handshake collective: 1 done, 0 pending, <0 failed. */
static int sub_advance(struct hop *h)
{
	int ret = xrun_advance(&h->sub->r);

	if (ret) {
		hop_free(h->sub);
		h->sub = NULL;
	}
	return ret;
}

/*
 * The P2P prologue of a peer-domain hop, driven from progress calls like the
 * rest of it (nothing blocks inside a submit: the owner's transfers may only
 * move when the application drives progress).  WAIT_PRIOR: the operations
 * queued before this one share the symmetric workspace, so they finish
 * first — each ends with a barrier, so no peer still reads or writes it.
 * Then, if the workspace must grow, p2p_ensure's two agreements run as host
 * collectives on the seqs reserved at submit.
 */
static int hop_prologue(struct lfa_coll_ep *ep, struct hop *h, size_t idx)
{
	struct lfa_coll_mc *mc = h->r.mc;
	struct sym_rec *recs = ep->ctl_host;
	int ret;

	switch (h->phase) {
	case HOP_WAIT_PRIOR:
		for (size_t j = 0; j < idx; j++) {
			struct hop *p = ep->q[(ep->qhead + j) % ep->qcap].hop;

			if (p && p->err)
				return p->err;
			/* a device hop with every item on the stream is far enough:
			 * this one's items queue behind it (a growth below first
			 * synchronises the stream) */
			if (p && !p->done && !p->issued)
				return 0;
		}
		LFA_TRACE("hop cid %#x prologue: prior hops done or issued, need %zu have %zu",
			  (unsigned)h->r.cid, h->sym_need, mc->sym_region);
		if (h->sym_need <= mc->sym_region)
			break;
		h->sym_size = sym_grow(mc, h->sym_need);
		sym_prepare(mc, h->sym_size,
			    lfa_hip_note(&h->r.hip_err, hipStreamSynchronize(ep->stream),
					 "P2P prologue stream sync") == hipSuccess,
			    (struct sym_rec *)h->mine, &h->r.hip_err);
		if (mc->size == 1) {
			h->agree_in = h->agree_out = ((struct sym_rec *)h->mine)->ok;
			recs[0] = *(struct sym_rec *)h->mine;
			h->agree_out = h->agree_out &&
				       sym_open(mc, recs, h->sym_size, &h->r.hip_err) == 0;
			goto agreed;
		}
		ret = sub_start(ep, h, LFA_ALLGATHER, h->mine, recs, sizeof(struct sym_rec),
				LFA_UINT8, LFA_NOOP, h->sub_seq);
		if (ret)
			return ret;
		h->phase = HOP_SYM_GATHER;
		LFA_TRACE("hop cid %#x workspace gather started (seq %u)", (unsigned)h->r.cid,
			  (unsigned)h->sub_seq);
		return 0;
	case HOP_SYM_GATHER:
		ret = sub_advance(h);
		if (ret <= 0)
			return ret;
		h->agree_in = sym_open(mc, recs, h->sym_size, &h->r.hip_err) == 0;
		ret = sub_start(ep, h, LFA_ALLREDUCE, &h->agree_in, &h->agree_out, 1,
				LFA_INT32, LFA_MIN, (uint16_t)(h->sub_seq + 1));
		if (ret)
			return ret;
		h->phase = HOP_SYM_AGREE;
		LFA_TRACE("hop cid %#x workspace gathered, mapped=%d", (unsigned)h->r.cid,
			  (int)h->agree_in);
		return 0;
	case HOP_SYM_AGREE:
		ret = sub_advance(h);
		if (ret <= 0)
			return ret;
agreed:
		if (!h->agree_out) {
			p2p_release(mc);
			return -LFA_EIO;
		}
		mc->sym_region = h->sym_size;
		break;
	default:
		return 0;
	}
	h->r.x.sym = mc->sym;
	h->r.x.region = mc->sym_region;
	h->phase = HOP_RUN;
	LFA_TRACE("hop cid %#x runs on the workspace (%zu B)", (unsigned)h->r.cid,
		  mc->sym_region);
	return 0;
}

int lfa_coll_host_chunk(enum lfa_collective_op coll, size_t count, int nranks,
			size_t esz, size_t chunk_bytes, size_t idx,
			struct lfa_host_chunk *c)
{
	const int rs = coll == LFA_REDUCE_SCATTER;
	size_t nb, span, per, off;

	if (!c || !esz || nranks < 1 ||
	    !(coll == LFA_ALLREDUCE || coll == LFA_BROADCAST ||
	      coll == LFA_REDUCE || rs) ||
	    (rs && count % (size_t)nranks))
		return -LFA_EINVAL;
	nb = rs ? (size_t)nranks : 1;       /* blocks gathered per chunk */
	span = count / nb;                  /* elements per block */
	/* chunk_bytes 0: one chunk, the whole buffer.  Which chunk a member
	 * uses is lfa_coll_member_chunk's rule: in a group of N > 1 only a
	 * group-wide chunk, so every member issues the same device schedule
	 * whatever its memory type (chunking is otherwise a local
	 * choice the peers cannot see) */
	per = chunk_bytes ? chunk_bytes / esz / nb : span;
	if (!per)
		per = 1;
	if (per > span)
		per = span;
	if (!per || idx >= (span + per - 1) / per)
		return 0;
	off = idx * per;
	c->src_off = off * esz;
	c->src_pitch = span * esz;
	c->width = (span - off < per ? span - off : per) * esz;
	c->height = nb;
	c->dev_count = nb * (c->width / esz);
	c->dst_off = off * esz;
	return 1;
}

/*
 * Host buffers: stream chunks through HBM on three streams: chunk c+1's H2D
 * (copy stream), chunk c's collective (executor stream) and chunk c-1's D2H
 * (d2h stream) run together, so both PCIe directions are busy at once; two
 * staging slots, ordered with events.  Valid for the element-wise collectives
 * (allreduce, reduce, broadcast), where chunks are independent, and for
 * reduce_scatter with equal blocks (count % N == 0): chunk c holds elements
 * [j, j+n) of EVERY rank's block (one 2-D H2D, height N), so the device
 * reduce_scatter of those N·n elements hands rank r elements [j, j+n) of its
 * own block.  Every element meets the same schedule as unchunked, so the
 * result is bit-identical to the whole-buffer form.
 */
LFA_INTERNAL int run_host_chunked(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			    enum lfa_collective_op coll, const void *buf,
			    void *result, size_t count, int root,
			    enum lfa_datatype dt, enum lfa_op op, size_t chunk)
{
	size_t esz = lfa_datatype_size(dt), in_slot, idx;
	struct lfa_host_chunk c0, c;
	hipEvent_t h2d[2], comp[2], done[2];
	int ret, slot = 0;
	const int out = coll != LFA_REDUCE || mc->rank == root;

	ret = lfa_coll_host_chunk(coll, count, mc->size, esz, chunk, 0, &c0);
	if (ret <= 0)
		return ret < 0 ? ret : 0;
	/* chunk 0 is the widest; the output half starts 256-byte aligned
	 * (vector body of the kernels) */
	in_slot = (c0.height * c0.width + 255) & ~(size_t)255;
	if (grow_staging(ep, in_slot + c0.width))
		return -LFA_ENOMEM;
	ret = 0;
	for (int i = 0; i < 2; i++) {
		hipEventCreateWithFlags(&h2d[i], hipEventDisableTiming);
		hipEventCreateWithFlags(&comp[i], hipEventDisableTiming);
		hipEventCreateWithFlags(&done[i], hipEventDisableTiming);
		hipEventRecord(done[i], ep->stream);
	}
	for (idx = 0; !ret &&
	     lfa_coll_host_chunk(coll, count, mc->size, esz, chunk, idx, &c) == 1;
	     idx++) {
		char *din = ep->hs[slot], *dout = din + in_slot;

		/* slot reuse: wait until chunk c-2's D2H finished */
		hipStreamWaitEvent(ep->copy_stream, done[slot], 0);
		if (c.height > 1)
			hipMemcpy2DAsync(din, c.width, (const char *)buf + c.src_off,
					 c.src_pitch, c.width, c.height,
					 hipMemcpyDefault, ep->copy_stream);
		else if (coll != LFA_BROADCAST || mc->rank == root)
			hipMemcpyAsync(din, (const char *)buf + c.src_off, c.width,
				       hipMemcpyDefault, ep->copy_stream);
		hipEventRecord(h2d[slot], ep->copy_stream);
		hipStreamWaitEvent(ep->stream, h2d[slot], 0);
		ret = run_device(ep, mc, coll, din,
				 coll == LFA_BROADCAST ? din : dout, c.dev_count,
				 root, dt, op, ep->stream, ep->algo);
		hipEventRecord(comp[slot], ep->stream);
		hipStreamWaitEvent(ep->d2h_stream, comp[slot], 0);
		if (out)
			hipMemcpyAsync((char *)result + c.dst_off,
				       coll == LFA_BROADCAST ? din : dout,
				       c.width, hipMemcpyDefault, ep->d2h_stream);
		hipEventRecord(done[slot], ep->d2h_stream);
		slot ^= 1;
	}
	/* the operation completes when the last D2H lands */
	hipStreamWaitEvent(ep->stream, done[slot ^ 1], 0);
	for (int i = 0; i < 2; i++) {
		hipEventDestroy(h2d[i]);
		hipEventDestroy(comp[i]);
		hipEventDestroy(done[i]);
	}
	return ret;
}

/*
 * Device buffers under a group chunk: the chunks lfa_coll_host_chunk gives
 * the host members, run back to back on the caller's buffers — contiguous
 * chunks in place, reduce_scatter's 2-D chunks (elements [j, j+w) of every
 * block) through the staging pipeline, which moves them device to device.
 */
LFA_INTERNAL int run_device_chunked(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			      enum lfa_collective_op coll, const void *buf,
			      void *result, size_t count, int root,
			      enum lfa_datatype dt, enum lfa_op op, size_t chunk)
{
	struct lfa_host_chunk c;
	int ret = 0;

	if (coll == LFA_REDUCE_SCATTER)
		return run_host_chunked(ep, mc, coll, buf, result, count, root, dt, op,
					chunk);
	for (size_t idx = 0; !ret &&
	     lfa_coll_host_chunk(coll, count, mc->size, lfa_datatype_size(dt), chunk, idx,
				 &c) == 1; idx++)
		ret = run_device(ep, mc, coll, buf ? (const char *)buf + c.src_off : NULL,
				 result ? (char *)result + c.dst_off : NULL, c.dev_count,
				 root, dt, op, ep->stream, ep->algo);
	return ret;
}

/* Host buffers for non-elementwise collectives: whole-buffer staging.
 * (Staging copies use hipMemcpyDefault: one side may be device memory when
 * the caller mixes a device buf with a host result.) */
LFA_INTERNAL int run_host_whole(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			  enum lfa_collective_op coll, const void *buf,
			  size_t in_bytes, void *result, size_t out_bytes,
			  size_t count, int root, enum lfa_datatype dt,
			  enum lfa_op op)
{
	char *din, *dout;
	int ret;

	if (grow_staging(ep, in_bytes + out_bytes + 32))
		return -LFA_ENOMEM;
	din = ep->hs[0];
	dout = din + ((in_bytes + 15) & ~(size_t)15);
	if (buf && in_bytes)
		hipMemcpyAsync(din, buf, in_bytes, hipMemcpyDefault, ep->stream);
	ret = run_device(ep, mc, coll, din, dout, count, root, dt, op, ep->stream, ep->algo);
	if (!ret && result && out_bytes)
		hipMemcpyAsync(result, dout, out_bytes, hipMemcpyDefault,
			       ep->stream);
	return ret;
}

/* Schedule `h` for one collective on a host domain: the algorithm's plan
 * (P2P / RCCL run as TREE; TREE_COLL's collective items lowered to grouped
 * sends/receives) and its own TMP, so operations may overlap. */
LFA_INTERNAL int host_start(struct lfa_coll_ep *ep, struct hop *h,
		      struct lfa_coll_mc *mc, enum lfa_collective_op coll,
		      const void *buf, void *result, size_t count, int root,
		      enum lfa_datatype dt, enum lfa_op op, int dev,
		      enum lfa_coll_algo algo)
{
	size_t esz = lfa_datatype_size(dt);
	/* this operation's sequence number, taken before a P2P handshake below
	 * draws the next ones */
	const uint16_t seq = (uint16_t)(mc->seq - 1);
	struct plan raw;
	int ret, sym;

	h->ep = ep;
	if (dev == 2) {
		/* host buffers the GPU reaches (pinned, registered): the device
		 * schedule runs on their mappings — this member's kernels alone
		 * touch its buf and result (peers only see the symmetric
		 * workspaces), so nothing is staged */
		void *zb = buf ? zero_copy_of(buf, ep->dom->device) : NULL;
		void *zr = result ? zero_copy_of(result, ep->dom->device) : NULL;

		if ((!buf || zb) && (!result || zr)) {
			buf = zb;
			result = zr;
			dev = 1;
		} else if (count * esz <= LFA_BOUNCE_BYTES && (h->bounce = bounce_get(ep))) {
			/* pageable buffers of a small operation: the input copied
			 * into a pinned bounce block on the CPU, the schedule run on
			 * the block's mapping, the result copied back when the hop
			 * completes — no H2D / D2H copies and their events (2
			 * processes, 4 KiB: DESIGN.md §7 round 5) */
			char *bin = h->bounce, *bout = bin + LFA_BOUNCE_BYTES;
			size_t moff, mlen;

			lfa_coll_block(count, mc->size, mc->rank, &moff, &mlen);
			/* a non-root member of a reduce has no result: the kernels never
			 * write the block's output half, so nothing is copied back
			 * (the half still held an earlier operation's bytes,
			 * and an in-place caller's input was overwritten with them) —
			 * the staged path's out_bytes rule below */
			if (coll == LFA_REDUCE && mc->rank != root)
				result = NULL;
			h->bounce_out = bout;
			h->bounce_user = result;
			h->bounce_bytes = !result ? 0 : coll == LFA_REDUCE_SCATTER ? mlen * esz :
					  count * esz;
			zb = zero_copy_of(bin, ep->dom->device);
			zr = zero_copy_of(bout, ep->dom->device);
			if (!zb || !zr) {
				bounce_put(ep, h->bounce);
				h->bounce = NULL;
				h->bounce_bytes = 0;
			} else {
				memcpy(bin, buf, count * esz);
				buf = zb;
				result = result ? zr : NULL;
				dev = 1;
			}
		}
	}
	/* P2P keeps its schedule on device buffers (the peers' symmetric
	 * workspaces are IPC-mapped device memory; its barriers become zero-byte
	 * messages); host buffers and RCCL run as TREE */
	if ((algo == LFA_ALGO_P2P && !dev) || algo == LFA_ALGO_RCCL ||
	    algo == LFA_ALGO_AUTO)
		algo = LFA_ALGO_TREE;
	ret = plan_make(&raw, coll, algo, mc->rank, mc->size, root, count, esz);
	if (ret)
		return ret;
	sym = plan_uses_sym(raw.steps, raw.nsteps);
	if (sym && dev) {
		ret = sig_ready(mc);
		if (ret) {
			plan_free(&raw);
			return ret;     /* epochs disagree since a timed-out wait */
		}
		h->r.x.ticket = ++mc->p2p_ticket;
	}
	/* a device hop's BARRIER stays: the flag kernel (sig_barrier) */
	ret = lower_plan(&raw, mc->rank, mc->size, esz, &h->pl, sym && !dev, !dev);
	plan_free(&raw);
	if (ret)
		return ret;
	if (sym) {
		/* the workspace is set up by hop_prologue, from progress; its two
		 * possible handshakes get the next two seqs on every member */
		h->phase = HOP_WAIT_PRIOR;
		h->sym_need = plan_sym_need(h->pl.steps, h->pl.nsteps, mc->size,
					    count, esz);
		h->sub_seq = mc->seq;
		mc->seq += 2;
	}
	h->dev = dev != 0;
	h->r.stream = ep->stream;
	if (dev == 1 && sym && h->pl.nsteps == 1 && h->pl.steps[0].type == LFA_STEP_ONESHOT &&
	    ep->done_word) {
		/* one kernel in place on device buffers: it ends in the
		 * completion word, no event */
		h->r.x.done_ctr = ep->done_ctr;
		h->r.x.done_word = ep->done_word;
		h->r.x.done_seq = &ep->done_seq;
	}
	if (dev) {
		hipSetDevice(ep->dom->device);
		if (h->pl.tmp && !(h->tmp = stage_get(ep, h->pl.tmp)))
			return -LFA_ENOMEM;
	} else if (h->pl.tmp && !(h->tmp = malloc(h->pl.tmp))) {
		return -LFA_ENOMEM;
	}
	if (dev == 2) {
		/* host buffers through device copies (reducing collectives) */
		size_t moff, mlen, in_b = count * esz;

		lfa_coll_block(count, mc->size, mc->rank, &moff, &mlen);
		h->out_bytes = coll == LFA_REDUCE_SCATTER ? mlen * esz :
			       coll == LFA_REDUCE && mc->rank != root ? 0 : count * esz;
		h->user_out = result;
		if (!(h->st_in = stage_get(ep, in_b)) ||
		    !(h->st_out = stage_get(ep, h->out_bytes)))
			return -LFA_ENOMEM;     /* hop_free releases what was made */
		/* H2D on the copy stream now: a chunked operation's later chunks
		 * upload while the earlier ones reduce (host_progress_all makes
		 * the run wait for in_ev) */
		if (!(h->in_ev = event_get(ep)))
			return -LFA_EIO;
		if (hipMemcpyAsync(h->st_in, buf, in_b, hipMemcpyHostToDevice,
				   ep->copy_stream) != hipSuccess ||
		    hipEventRecord(h->in_ev, ep->copy_stream) != hipSuccess)
			return -LFA_EIO;
		buf = h->st_in;
		result = h->st_out;
	}
	h->r.xp = dev ? &xport_peer_dev : &xport_peer;
	h->r.pl = &h->pl;
	h->r.mc = mc;
	h->r.op = op;
	h->r.dt = dt;
	h->r.cid = (uint64_t)mc->group_id << 16 | seq;
	h->r.x.base[LFA_BUF_SEND] = coll == LFA_BROADCAST ? result : (void *)buf;
	h->r.x.base[LFA_BUF_RESULT] = result;
	h->r.x.base[LFA_BUF_TMP] = h->tmp;
	return 0;
}

LFA_INTERNAL int host_submit(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
		       enum lfa_collective_op coll, const void *buf,
		       void *result, size_t count, int root,
		       enum lfa_datatype dt, enum lfa_op op, void *context,
		       int kind, struct lfa_coll_mc *jmc, int dev,
		       enum lfa_coll_algo algo)
{
	struct hop *h = calloc(1, sizeof(*h));
	const uint64_t t0 = mc->p2p_ticket;
	int ret;

	if (!h)
		return -LFA_ENOMEM;
	mc->seq++;                              /* coll_get_next_id :48-52 */
	ret = host_start(ep, h, mc, coll, buf, result, count, root, dt, op, dev, algo);
	LFA_TRACE("submit cid %#x coll %d count %zu dev %d algo %d phase %d sub_seq %u -> %d",
		  (unsigned)h->r.cid, (int)coll, count, dev, (int)algo, h->phase,
		  (unsigned)h->sub_seq, ret);
	if (!ret)
		ret = enqueue_host(ep, h, context, kind, jmc);
	if (ret)
		hop_free(h);
	else
		tag_p2p(ep, mc, t0);
	return ret;
}

/*
 * The group chunk on a GPU peer domain.  Under LFA_ALGO_P2P
 * every member — host buffers staged, device buffers in place — runs the
 * one device schedule, so a group chunk splits an allreduce or reduce into
 * the same ⌈count / chunk⌉ P2P operations on every member: a rule of
 * (algorithm, collective, count, n, esz, chunk) only, never of the member's
 * buffer type.  Host members' chunks then pipeline: chunk c+1's H2D (copy
 * stream) and chunk c-1's D2H (d2h stream) overlap chunk c's kernels.
 * reduce_scatter keeps one operation (its chunks are 2-D).
 */
LFA_INTERNAL size_t peer_chunked(const struct lfa_coll_ep *ep, const struct lfa_coll_mc *mc,
			   enum lfa_collective_op coll, size_t count, size_t esz)
{
	const size_t g = lfa_coll_group_chunk(ep->group_chunk, mc->size, count * esz);

	return ep->algo == LFA_ALGO_P2P && g && ep->dom->device >= 0 &&
	       mc->size > 1 && mc->size <= LFA_TREE_MAX && mc->size <= LFA_PUT_MAX &&
	       (coll == LFA_ALLREDUCE || coll == LFA_REDUCE) &&
	       count * esz > g ? g : 0;
}

LFA_INTERNAL int peer_submit_chunked(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc,
			       enum lfa_collective_op coll, const void *buf,
			       void *result, size_t count, int root,
			       enum lfa_datatype dt, enum lfa_op op, void *context,
			       int dev, size_t chunk)
{
	const size_t esz = lfa_datatype_size(dt);
	const uint64_t chain = ++ep->next_chain;
	size_t per = chunk / esz;
	int ret;

	if (!per)
		per = 1;
	/* every chunk's queue slot before the first chunk is posted (ADVICE
	 * r4): a full ring can then not stop the operation partway, which
	 * would leave the members with different operations on the group */
	ret = queue_reserve(ep, (count + per - 1) / per);
	if (ret)
		return ret;
	for (size_t off = 0; off < count; off += per) {
		const size_t n = count - off < per ? count - off : per;
		const int last = off + n == count;
		void *r = result ? (char *)result + off * esz : NULL;

		ret = host_submit(ep, mc, coll, (const char *)buf + off * esz, r, n, root,
				  dt, op, context, last ? 0 : 3, NULL, dev, ep->algo);

		if (ret) {
			/* the caller is told the operation never started: the
			 * chunks already queued still run (their peers wait for
			 * them) but reap silently.  The members have now issued
			 * different operations on the group, so its later
			 * collectives fail (P2P waits time out): close and
			 * re-join it (lfa_coll.h) */
			if (off)
				ep->failed_chain = chain;
			return ret;
		}
		ep->q[(ep->qhead + ep->qlen - 1) % ep->qcap].chain = chain;
	}
	return 0;
}
