/*
 * lfa_coll_plan.c — the schedule builder of the collective provider: a
 * collective becomes an array of lfa_step items for one rank (lfa_coll_plan,
 * include/lfa_coll.h), host-only and testable on CPU.  prov/coll builds the
 * same thing as a work queue per operation (include/ofi_coll.h:64-119,
 * coll_coll.c:229-343); the executor that runs these schedules over RCCL or
 * the owner's transfers is lfa_coll_exec.c.
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "lfa_atomic.h"
#include "lfa_coll.h"
#include "lfa_coll_plan.h"
#include "lfa_signal.h"

/* ====================================================================== */
/* schedule builder                                                        */
/* ====================================================================== */

void lfa_coll_block(size_t count, int nranks, int r, size_t *off, size_t *len)
{
	size_t base = count / (size_t)nranks, extra = count % (size_t)nranks;
	size_t rr = (size_t)r;

	*len = base + (rr < extra ? 1 : 0);
	*off = rr * base + (rr < extra ? rr : extra);
}

struct planner {
	struct lfa_step *steps;
	size_t cap, n;
	struct lfa_ref *refs;
	size_t rcap, nr;
	int pending_comm;       /* SEND/RECV since the last GROUP_END */
	uint64_t tmp_base;      /* TMP bytes the schedule itself uses */
	uint64_t tmp_extra;     /* + partials of split trees (p_tree_any) */
};

static struct lfa_ref ref(int buf, uint64_t off)
{
	struct lfa_ref r;

	r.buf = buf;
	r.rank = 0;
	r.off = off;
	return r;
}

/* A ref into group rank `rank`'s symmetric workspace (LFA_ALGO_P2P). */
static struct lfa_ref sref(int buf, int rank, uint64_t off)
{
	struct lfa_ref r = ref(buf, off);

	r.rank = (uint32_t)rank;
	return r;
}

static struct lfa_step *push(struct planner *p, int type)
{
	struct lfa_step *s;

	if (p->n < p->cap) {
		s = &p->steps[p->n];
		memset(s, 0, sizeof(*s));
		s->type = type;
	} else {
		s = NULL;
	}
	p->n++;
	return s;
}

static void p_xfer(struct planner *p, int type, int peer, struct lfa_ref r,
		   uint64_t bytes)
{
	struct lfa_step *s;

	if (!bytes)
		return;
	s = push(p, type);
	if (s) {
		s->peer = peer;
		s->count = bytes;
		if (type == LFA_STEP_SEND)
			s->src = r;
		else
			s->dst = r;
	}
	p->pending_comm = 1;
}

static void p_group_end(struct planner *p)
{
	if (!p->pending_comm)
		return;
	push(p, LFA_STEP_GROUP_END);
	p->pending_comm = 0;
}

static void p_reduce(struct planner *p, struct lfa_ref dst, struct lfa_ref src,
		     uint64_t count)
{
	struct lfa_step *s;

	p_group_end(p);
	if (!count)
		return;
	s = push(p, LFA_STEP_REDUCE);
	if (s) {
		s->dst = dst;
		s->src = src;
		s->count = count;
	}
}

static void p_copy(struct planner *p, struct lfa_ref dst, struct lfa_ref src,
		   uint64_t bytes)
{
	struct lfa_step *s;

	p_group_end(p);
	if (!bytes || (dst.buf == src.buf && dst.off == src.off))
		return;
	s = push(p, LFA_STEP_COPY);
	if (s) {
		s->dst = dst;
		s->src = src;
		s->count = bytes;
	}
}

/* TREE over refs pushed by the caller with p_tree_src() right before. */
static uint32_t p_tree_begin(struct planner *p)
{
	p_group_end(p);
	return (uint32_t)p->nr;
}

static void p_tree_src(struct planner *p, struct lfa_ref r)
{
	if (p->nr < p->rcap)
		p->refs[p->nr] = r;
	p->nr++;
}

static void p_tree_end(struct planner *p, uint32_t first, struct lfa_ref dst,
		       uint64_t count)
{
	struct lfa_step *s;

	if (!count)
		return;
	s = push(p, LFA_STEP_TREE);
	if (s) {
		s->dst = dst;
		s->first = first;
		s->nsrc = (uint32_t)(p->nr - first);
		s->count = count;
	}
}

/* TREE_PUT: inputs pushed with p_tree_src() since `first`, then `nput`
 * extra destinations pushed after them. */
static void p_tree_put_end(struct planner *p, uint32_t first, uint32_t nsrc,
			   struct lfa_ref dst, uint64_t count)
{
	struct lfa_step *s;

	if (!count)
		return;
	s = push(p, LFA_STEP_TREE_PUT);
	if (s) {
		s->dst = dst;
		s->first = first;
		s->nsrc = nsrc;
		s->peer = (int32_t)(p->nr - first - nsrc);
		s->count = count;
	}
}

static void p_oneshot(struct planner *p, int mode, int n, uint64_t count)
{
	struct lfa_step *s;

	p_group_end(p);
	if (!count)
		return;
	s = push(p, LFA_STEP_ONESHOT);
	if (s) {
		s->dst = ref(LFA_BUF_RESULT, 0);
		s->src = ref(LFA_BUF_SEND, 0);
		s->peer = mode;
		s->nsrc = (uint32_t)n;
		s->count = count;
	}
}

static void p_barrier(struct planner *p)
{
	p_group_end(p);
	push(p, LFA_STEP_BARRIER);
}

static void p_coll(struct planner *p, int type, struct lfa_ref dst,
		   struct lfa_ref src, uint64_t bytes)
{
	struct lfa_step *s;

	p_group_end(p);
	if (!bytes)
		return;
	s = push(p, type);
	if (s) {
		s->dst = dst;
		s->src = src;
		s->count = bytes;
	}
}

static uint64_t pof2_floor(uint64_t v)
{
	uint64_t q = 1;

	while (q * 2 <= v)
		q *= 2;
	return q;
}

/*
 * Tree algorithm, phase 1: rank r collects block r of every rank's input.
 * TMP slot p (block-r sized) receives rank p's block; rank r's own block is
 * read in place from SEND.  Returns the ref list start for the TREE item.
 */
/*
 * Distance between the gathered blocks in TMP.  The tree kernel reads all N
 * blocks at the same offset at once; blocks exactly B apart put those N
 * streams on the same HBM channels, and the 8 x 32 MiB tree drops from
 * 71 % to 68 % of peak.  Skewing block k by k x 6 KiB lifts it to 73 %
 * (bench.py --tune-tree-layout, profiles/r01_tune_tree_layout.log).  Small
 * blocks keep the dense layout.
 */
#define LFA_TREE_SKEW_MIN (1u << 20)
#define LFA_TREE_SKEW 6144u

static uint64_t blk_stride(size_t mlen, size_t esz)
{
	uint64_t b = (uint64_t)mlen * esz;

	if (b < LFA_TREE_SKEW_MIN)
		return b;
	return ((b + 255) & ~(uint64_t)255) + LFA_TREE_SKEW;
}

static void plan_gather_blocks(struct planner *p, int r, int n, size_t count,
			       size_t esz)
{
	size_t off, len, moff, mlen;

	lfa_coll_block(count, n, r, &moff, &mlen);
	for (int k = 1; k < n; k++) {
		/* pairwise order (r+k, r-k) spreads the peers over xGMI links */
		int to = (r + k) % n, from = (r - k + n) % n;

		lfa_coll_block(count, n, to, &off, &len);
		p_xfer(p, LFA_STEP_SEND, to, ref(LFA_BUF_SEND, off * esz), len * esz);
		p_xfer(p, LFA_STEP_RECV, from,
		       ref(LFA_BUF_TMP, (uint64_t)from * blk_stride(mlen, esz)),
		       mlen * esz);
	}
	p_group_end(p);
}

/*
 * A tree over n inputs of any size.  Up to LFA_TREE_MAX inputs it is ONE
 * TREE item (one fused kernel).  Above that it is split into whole subtrees
 * of prov/coll's recursive-doubling tree, so the bits do not change:
 * virtual rank v < pof2 is the leaf pair (in[2v+1] OP in[2v]) for v < rem
 * and in[v + rem] otherwise (coll_coll.c:366-389); aligned runs of 16
 * virtual ranks are subtrees of at most 32 inputs, each reduced into a TMP
 * partial, and the pof2/16 partials are combined by the same rule
 * (recursively, for groups above 512 ranks).  A run with k < 16 pairs is
 * the kernel's own tree for 16 + k inputs (pairs first, as in the kernel); a
 * run of 16 pairs is its plain 32-input tree, whose first level is exactly
 * the pairs.
 */
struct tree_in {
	int kind;               /* 0: rank order, `own` in place, the rest TMP
				   slots k*stride; 1: TMP run at base + k*stride */
	int own;
	struct lfa_ref own_ref;
	uint64_t base, stride;
};

static struct lfa_ref tree_in_ref(const struct tree_in *t, int k)
{
	if (t->kind == 0 && k == t->own)
		return t->own_ref;
	return ref(LFA_BUF_TMP, t->base + (uint64_t)k * t->stride);
}

#define LFA_TREE_GROUP 16       /* virtual ranks per split subtree */

static void p_tree_any(struct planner *p, const struct tree_in *in, int lo,
		       int n, struct lfa_ref dst, uint64_t count, size_t esz)
{
	uint64_t pof2 = pof2_floor((uint64_t)n), rem = (uint64_t)n - pof2;
	uint64_t ngrp, pstride, pbase;
	struct tree_in parts;
	uint32_t first;

	if (n <= LFA_TREE_MAX) {
		first = p_tree_begin(p);
		for (int k = 0; k < n; k++)
			p_tree_src(p, tree_in_ref(in, lo + k));
		p_tree_end(p, first, dst, count);
		return;
	}
	ngrp = pof2 / LFA_TREE_GROUP;
	pstride = ((uint64_t)count * esz + 255) & ~(uint64_t)255;
	pbase = (p->tmp_base + p->tmp_extra + 255) & ~(uint64_t)255;
	p->tmp_extra = pbase + ngrp * pstride - p->tmp_base;
	for (uint64_t g = 0; g < ngrp; g++) {
		uint64_t v0 = g * LFA_TREE_GROUP, v1 = v0 + LFA_TREE_GROUP;
		uint64_t s0 = v0 < rem ? 2 * v0 : v0 + rem;
		uint64_t s1 = v1 < rem ? 2 * v1 : v1 + rem;

		first = p_tree_begin(p);
		for (uint64_t k = s0; k < s1; k++)
			p_tree_src(p, tree_in_ref(in, lo + (int)k));
		p_tree_end(p, first, ref(LFA_BUF_TMP, pbase + g * pstride), count);
	}
	parts.kind = 1;
	parts.own = -1;
	parts.base = pbase;
	parts.stride = pstride;
	p_tree_any(p, &parts, 0, (int)ngrp, dst, count, esz);
}

static void plan_tree_block(struct planner *p, int r, int n, size_t count,
			    size_t esz, struct lfa_ref dst)
{
	size_t moff, mlen;
	struct tree_in in;

	lfa_coll_block(count, n, r, &moff, &mlen);
	in.kind = 0;
	in.own = r;
	in.own_ref = ref(LFA_BUF_SEND, moff * esz);
	in.base = 0;
	in.stride = blk_stride(mlen, esz);
	p->tmp_base = n > 1 ? (uint64_t)n * blk_stride(mlen, esz) : 0;
	p_tree_any(p, &in, 0, n, dst, mlen, esz);
}

static void plan_allgather_blocks(struct planner *p, int r, int n,
				  size_t count, size_t esz)
{
	size_t off, len, moff, mlen;

	lfa_coll_block(count, n, r, &moff, &mlen);
	for (int k = 1; k < n; k++) {
		int to = (r + k) % n, from = (r - k + n) % n;

		lfa_coll_block(count, n, from, &off, &len);
		p_xfer(p, LFA_STEP_SEND, to, ref(LFA_BUF_RESULT, moff * esz),
		       mlen * esz);
		p_xfer(p, LFA_STEP_RECV, from, ref(LFA_BUF_RESULT, off * esz),
		       len * esz);
	}
	p_group_end(p);
}

/* Small messages: everyone gets everyone's full input, one tree per rank.
 * One exchange phase instead of two; TMP holds N full inputs. */
static void plan_allreduce_small(struct planner *p, int r, int n, size_t count,
				 size_t esz, struct lfa_ref dst)
{
	struct tree_in in;

	for (int k = 1; k < n; k++) {
		int to = (r + k) % n, from = (r - k + n) % n;

		p_xfer(p, LFA_STEP_SEND, to, ref(LFA_BUF_SEND, 0), count * esz);
		p_xfer(p, LFA_STEP_RECV, from,
		       ref(LFA_BUF_TMP, (uint64_t)from * count * esz), count * esz);
	}
	p_group_end(p);
	in.kind = 0;
	in.own = r;
	in.own_ref = ref(LFA_BUF_SEND, 0);
	in.base = 0;
	in.stride = (uint64_t)count * esz;
	p->tmp_base = (uint64_t)n * count * esz;
	p_tree_any(p, &in, 0, n, dst, count, esz);
}

/*
 * The reference's recursive-doubling schedule, item for item
 * (coll_do_allreduce, coll_coll.c:349-449), into `res` with `tmp` scratch.
 */
static void plan_rd_allreduce(struct planner *p, uint64_t local, uint64_t n,
			      size_t count, size_t esz, struct lfa_ref res,
			      struct lfa_ref tmp)
{
	uint64_t pof2 = pof2_floor(n), rem = n - pof2, newid, mask;
	uint64_t bytes = (uint64_t)count * esz;

	p_copy(p, res, ref(LFA_BUF_SEND, 0), bytes);        /* :364 memcpy */
	if (local < 2 * rem) {
		if (local % 2 == 0) {
			p_xfer(p, LFA_STEP_SEND, (int)local + 1, res, bytes);
			p_group_end(p);
			newid = (uint64_t)-1;
		} else {
			p_xfer(p, LFA_STEP_RECV, (int)local - 1, tmp, bytes);
			p_group_end(p);
			p_reduce(p, res, tmp, count);       /* result = result OP tmp */
			newid = local / 2;
		}
	} else {
		newid = local - rem;
	}
	if (newid != (uint64_t)-1) {
		for (mask = 1; mask < pof2; mask <<= 1) {
			uint64_t nr = newid ^ mask;
			uint64_t remote = nr < rem ? nr * 2 + 1 : nr + rem;

			p_xfer(p, LFA_STEP_RECV, (int)remote, tmp, bytes);
			p_xfer(p, LFA_STEP_SEND, (int)remote, res, bytes);
			p_group_end(p);
			if (remote < local) {
				p_reduce(p, res, tmp, count);
			} else {
				p_reduce(p, tmp, res, count);
				p_copy(p, res, tmp, bytes);
			}
		}
	}
	if (local < 2 * rem) {
		if (local % 2)
			p_xfer(p, LFA_STEP_SEND, (int)local - 1, res, bytes);
		else
			p_xfer(p, LFA_STEP_RECV, (int)local + 1, res, bytes);
		p_group_end(p);
	}
}

/*
 * LFA_ALGO_P2P.  Every rank stages the blocks the others need in its own
 * SYM_IN region (rank r's block is read in place from SEND), then, after a
 * barrier, reduces block r of all inputs straight out of the peers' SYM_IN
 * over xGMI and writes the result to `outs` (local result and/or peers'
 * SYM_OUT).  A closing barrier guarantees no peer still reads or writes this
 * rank's workspace once its operation completes (so the next operation may
 * overwrite it, and close may free it).
 */
static void p2p_stage_input(struct planner *p, int r, int n, size_t count,
			    size_t esz)
{
	/* ONE copy of the whole input: block r itself is read in place from
	 * SEND, but copying it too (1/n more local bytes) saves the second
	 * launch the two ranges around it would need */
	(void)n;
	p_copy(p, sref(LFA_BUF_SYM_IN, r, 0), ref(LFA_BUF_SEND, 0), count * esz);
	p_barrier(p);
}

/* Tree of block r over all ranks' inputs; result to dst, and with push_all
 * also into every peer's SYM_OUT at the block's offset. */
static void p2p_tree_block(struct planner *p, int r, int n, size_t count,
			   size_t esz, struct lfa_ref dst, int push_all)
{
	size_t moff, mlen;
	uint32_t first;

	lfa_coll_block(count, n, r, &moff, &mlen);
	first = p_tree_begin(p);
	for (int k = 0; k < n; k++)
		p_tree_src(p, k == r ? ref(LFA_BUF_SEND, moff * esz) :
			   sref(LFA_BUF_SYM_IN, k, moff * esz));
	if (push_all) {
		/* in the order r+1, r+2, …: each block's pushes start on a
		 * different link */
		for (int k = 1; k < n; k++)
			p_tree_src(p, sref(LFA_BUF_SYM_OUT, (r + k) % n, moff * esz));
	}
	p_tree_put_end(p, first, (uint32_t)n, dst, mlen);
}

/* Copy the whole gathered result from rank r's SYM_OUT: its own block was
 * written there by its own tree, so one launch covers every block. */
static void p2p_unstage_output(struct planner *p, int r, size_t count, size_t esz)
{
	p_copy(p, ref(LFA_BUF_RESULT, 0), sref(LFA_BUF_SYM_OUT, r, 0), count * esz);
}

size_t lfa_os_ag_bytes(void)
{
	static long long v = -1;

	if (v < 0) {
		const char *e = lfa_param("LFA_OS_AG_BYTES");
		const long long x = e ? atoll(e) : 0;

		v = x > 0 && x <= (1ll << 30) ? x : (long long)LFA_OS_AG_BYTES_DEFAULT;
	}
	return (size_t)v;
}

size_t lfa_os_rs_bytes(void)
{
	static long long v = -1;

	if (v < 0) {
		const char *e = lfa_param("LFA_OS_RS_BYTES");
		const long long x = e ? atoll(e) : 0;

		v = x > 0 && x <= (1ll << 30) ? x : (long long)LFA_OS_RS_BYTES;
	}
	return (size_t)v;
}

static int plan_p2p(struct planner *p, enum lfa_collective_op coll, int r,
		    int n, int root, size_t count, size_t esz)
{
	size_t moff, mlen, bytes = count * esz;
	uint32_t first;

	lfa_coll_block(count, n, r, &moff, &mlen);
	switch (coll) {
	case LFA_ALLREDUCE:
		if (bytes * (size_t)n <= lfa_os_ag_bytes() && n <= LFA_OS_MAX_RANKS) {
			/* one kernel: push into the peers' slots, flags, tree */
			p_oneshot(p, LFA_ONESHOT_ALL, n, count);
			return 0;
		}
		if (bytes * (size_t)n <= LFA_SMALL_AG_BYTES) {
			/* one phase: every rank reduces the whole vector */
			p_copy(p, sref(LFA_BUF_SYM_IN, r, 0), ref(LFA_BUF_SEND, 0),
			       bytes);
			p_barrier(p);
			first = p_tree_begin(p);
			for (int k = 0; k < n; k++)
				p_tree_src(p, k == r ? ref(LFA_BUF_SEND, 0) :
					   sref(LFA_BUF_SYM_IN, k, 0));
			p_tree_put_end(p, first, (uint32_t)n, ref(LFA_BUF_RESULT, 0),
				       count);
			p_barrier(p);
			return 0;
		}
		p2p_stage_input(p, r, n, count, esz);
		p2p_tree_block(p, r, n, count, esz, sref(LFA_BUF_SYM_OUT, r, moff * esz),
			       1);
		p_barrier(p);
		p2p_unstage_output(p, r, count, esz);
		return 0;
	case LFA_REDUCE_SCATTER:
		if (bytes <= lfa_os_rs_bytes() && n <= LFA_OS_MAX_RANKS) {
			p_oneshot(p, LFA_ONESHOT_SCATTER, n, count);
			return 0;
		}
		p2p_stage_input(p, r, n, count, esz);
		p2p_tree_block(p, r, n, count, esz, ref(LFA_BUF_RESULT, 0), 0);
		p_barrier(p);
		return 0;
	case LFA_REDUCE:
		if (bytes * (size_t)n <= lfa_os_ag_bytes() && n <= LFA_OS_MAX_RANKS) {
			p_oneshot(p, root, n, count);
			return 0;
		}
		p2p_stage_input(p, r, n, count, esz);
		p2p_tree_block(p, r, n, count, esz, sref(LFA_BUF_SYM_OUT, root, moff * esz),
			       0);
		p_barrier(p);
		if (r == root)
			p2p_unstage_output(p, r, count, esz);
		return 0;
	default:
		return -LFA_ENOSYS;
	}
}

int lfa_coll_plan(enum lfa_collective_op coll, enum lfa_coll_algo algo,
		  int rank, int nranks, int root, size_t count, size_t esz,
		  struct lfa_step *steps, size_t *nsteps, struct lfa_ref *refs,
		  size_t *nrefs, size_t *tmp_bytes)
{
	struct planner p;
	size_t moff, mlen, bytes = count * esz;
	int r = rank, n = nranks;

	if (!nsteps || !nrefs || !tmp_bytes || n < 1 || r < 0 || r >= n || !esz)
		return -LFA_EINVAL;
	if ((coll == LFA_REDUCE || coll == LFA_BROADCAST || coll == LFA_SCATTER) &&
	    (root < 0 || root >= n))
		return -LFA_EINVAL;
	memset(&p, 0, sizeof(p));
	p.steps = steps;
	p.cap = steps ? *nsteps : 0;
	p.refs = refs;
	p.rcap = refs ? *nrefs : 0;
	*tmp_bytes = 0;
	lfa_coll_block(count, n, r, &moff, &mlen);

	if (algo == LFA_ALGO_RCCL)
		algo = LFA_ALGO_TREE;   /* the RCCL algo is not a schedule */
	if (algo == LFA_ALGO_P2P) {
		/* reducing collectives over the symmetric workspace; the rest
		 * (pure transport) keep the RCCL schedules */
		/* n = 1: only a one-shot-sized bucket — the one-shot kernel's
		 * degenerate group, one copy launch ending in the completion
		 * word (a one-member endpoint runs it when its solo copy is
		 * turned off, lfa_coll_ep_test_solo) */
		const int os1 = n == 1 &&
				(coll == LFA_REDUCE_SCATTER ? bytes <= lfa_os_rs_bytes() :
							       bytes <= lfa_os_ag_bytes());

		if ((n > 1 || os1) && n <= LFA_TREE_MAX && n <= LFA_PUT_MAX &&
		    (coll == LFA_ALLREDUCE || coll == LFA_REDUCE_SCATTER ||
		     coll == LFA_REDUCE)) {
			int ret = plan_p2p(&p, coll, r, n, root, count, esz);

			if (ret)
				return ret;
			*nsteps = p.n;
			*nrefs = p.nr;
			if (!steps || !refs)
				return 0;
			return (p.n > p.cap || p.nr > p.rcap) ? -LFA_ETOOSMALL : 0;
		}
		algo = LFA_ALGO_TREE;
	}
	if (algo == LFA_ALGO_TREE_COLL) {
		/* collective transport only for even blocks of the big path */
		int even = count % (size_t)n == 0 && n <= LFA_TREE_MAX &&
			   !(coll == LFA_ALLREDUCE &&
			     bytes * (size_t)n <= LFA_SMALL_AG_BYTES);

		if (coll == LFA_ALLREDUCE && n > 1 && n <= LFA_TREE_MAX &&
		    bytes * (size_t)n <= LFA_SMALL_AG_BYTES) {
			uint32_t first;

			/* small: every rank's whole input through ONE RCCL
			 * allgather (TMP slot k <- rank k), then the tree over the
			 * slots in rank order — the grouped-send form's bits */
			p_coll(&p, LFA_STEP_ALLGATHER, ref(LFA_BUF_TMP, 0),
			       ref(LFA_BUF_SEND, 0), bytes);
			first = p_tree_begin(&p);
			for (int k = 0; k < n; k++)
				p_tree_src(&p, ref(LFA_BUF_TMP, (uint64_t)k * bytes));
			p_tree_end(&p, first, ref(LFA_BUF_RESULT, 0), count);
			*tmp_bytes = (size_t)n * bytes;
			*nsteps = p.n;
			*nrefs = p.nr;
			if (!steps || !refs)
				return 0;
			return (p.n > p.cap || p.nr > p.rcap) ? -LFA_ETOOSMALL : 0;
		}

		if (even && (coll == LFA_ALLREDUCE || coll == LFA_REDUCE_SCATTER)) {
			uint32_t first;

			/* TMP slot q <- block r of rank q (own block too) */
			p_coll(&p, LFA_STEP_ALLTOALL, ref(LFA_BUF_TMP, 0),
			       ref(LFA_BUF_SEND, 0), mlen * esz);
			first = p_tree_begin(&p);
			for (int k = 0; k < n; k++)
				p_tree_src(&p, ref(LFA_BUF_TMP, (uint64_t)k * mlen * esz));
			p_tree_end(&p, first, coll == LFA_ALLREDUCE ?
				   ref(LFA_BUF_RESULT, moff * esz) :
				   ref(LFA_BUF_RESULT, 0), mlen);
			if (coll == LFA_ALLREDUCE)
				p_coll(&p, LFA_STEP_ALLGATHER, ref(LFA_BUF_RESULT, 0),
				       ref(LFA_BUF_RESULT, moff * esz), mlen * esz);
			*tmp_bytes = (size_t)n * mlen * esz;
			*nsteps = p.n;
			*nrefs = p.nr;
			if (!steps || !refs)
				return 0;
			return (p.n > p.cap || p.nr > p.rcap) ? -LFA_ETOOSMALL : 0;
		}
		algo = LFA_ALGO_TREE;
	}
	if (algo != LFA_ALGO_TREE && algo != LFA_ALGO_RD)
		return -LFA_ENOSYS;

	switch (coll) {
	case LFA_ALLREDUCE:
		if (algo == LFA_ALGO_RD) {
			plan_rd_allreduce(&p, (uint64_t)r, (uint64_t)n, count, esz,
					  ref(LFA_BUF_RESULT, 0), ref(LFA_BUF_TMP, 0));
			*tmp_bytes = n > 1 ? bytes : 0;
		} else if (n > 1 && bytes * (size_t)n <= LFA_SMALL_AG_BYTES) {
			plan_allreduce_small(&p, r, n, count, esz,
					     ref(LFA_BUF_RESULT, 0));
			*tmp_bytes = (size_t)n * bytes;
		} else {
			plan_gather_blocks(&p, r, n, count, esz);
			plan_tree_block(&p, r, n, count, esz,
					ref(LFA_BUF_RESULT, moff * esz));
			plan_allgather_blocks(&p, r, n, count, esz);
			*tmp_bytes = n > 1 ? (size_t)n * blk_stride(mlen, esz) : 0;
		}
		break;
	case LFA_REDUCE_SCATTER:
		if (algo == LFA_ALGO_RD) {
			plan_rd_allreduce(&p, (uint64_t)r, (uint64_t)n, count, esz,
					  ref(LFA_BUF_TMP, bytes), ref(LFA_BUF_TMP, 0));
			p_copy(&p, ref(LFA_BUF_RESULT, 0),
			       ref(LFA_BUF_TMP, bytes + moff * esz), mlen * esz);
			*tmp_bytes = 2 * bytes;
		} else {
			plan_gather_blocks(&p, r, n, count, esz);
			plan_tree_block(&p, r, n, count, esz, ref(LFA_BUF_RESULT, 0));
			*tmp_bytes = n > 1 ? (size_t)n * blk_stride(mlen, esz) : 0;
		}
		break;
	case LFA_REDUCE:
		if (algo == LFA_ALGO_RD) {
			plan_rd_allreduce(&p, (uint64_t)r, (uint64_t)n, count, esz,
					  ref(LFA_BUF_TMP, bytes), ref(LFA_BUF_TMP, 0));
			if (r == root)
				p_copy(&p, ref(LFA_BUF_RESULT, 0),
				       ref(LFA_BUF_TMP, bytes), bytes);
			*tmp_bytes = 2 * bytes;
		} else {
			size_t off, len;

			plan_gather_blocks(&p, r, n, count, esz);
			plan_tree_block(&p, r, n, count, esz,
					r == root ? ref(LFA_BUF_RESULT, moff * esz) :
					ref(LFA_BUF_TMP, (uint64_t)r * blk_stride(mlen, esz)));
			if (r != root) {
				p_xfer(&p, LFA_STEP_SEND, root,
				       ref(LFA_BUF_TMP, (uint64_t)r * blk_stride(mlen, esz)),
				       mlen * esz);
			} else {
				for (int k = 0; k < n; k++) {
					if (k == root)
						continue;
					lfa_coll_block(count, n, k, &off, &len);
					p_xfer(&p, LFA_STEP_RECV, k,
					       ref(LFA_BUF_RESULT, off * esz), len * esz);
				}
			}
			p_group_end(&p);
			*tmp_bytes = n > 1 ? (size_t)n * blk_stride(mlen, esz) : 0;
		}
		break;
	case LFA_ALLGATHER:
		for (int k = 1; k < n; k++) {
			int to = (r + k) % n, from = (r - k + n) % n;

			p_xfer(&p, LFA_STEP_SEND, to, ref(LFA_BUF_SEND, 0), bytes);
			p_xfer(&p, LFA_STEP_RECV, from,
			       ref(LFA_BUF_RESULT, (uint64_t)from * bytes), bytes);
		}
		p_group_end(&p);
		p_copy(&p, ref(LFA_BUF_RESULT, (uint64_t)r * bytes),
		       ref(LFA_BUF_SEND, 0), bytes);
		break;
	case LFA_BROADCAST:
		/* buf is in/out: the executor binds SEND and RESULT to it */
		if (r == root) {
			for (int k = 1; k < n; k++)
				p_xfer(&p, LFA_STEP_SEND, (root + k) % n,
				       ref(LFA_BUF_RESULT, 0), bytes);
		} else {
			p_xfer(&p, LFA_STEP_RECV, root, ref(LFA_BUF_RESULT, 0), bytes);
		}
		p_group_end(&p);
		break;
	case LFA_SCATTER: {
		/* root's buf holds n blocks of `count`; everyone gets block r */
		if (r == root) {
			for (int k = 1; k < n; k++) {
				int to = (root + k) % n;

				p_xfer(&p, LFA_STEP_SEND, to,
				       ref(LFA_BUF_SEND, (uint64_t)to * bytes), bytes);
			}
		} else {
			p_xfer(&p, LFA_STEP_RECV, root, ref(LFA_BUF_RESULT, 0), bytes);
		}
		p_group_end(&p);
		if (r == root)
			p_copy(&p, ref(LFA_BUF_RESULT, 0),
			       ref(LFA_BUF_SEND, (uint64_t)r * bytes), bytes);
		break;
	}
	default:
		return -LFA_ENOSYS;
	}
	p_group_end(&p);
	*tmp_bytes += p.tmp_extra;      /* partials of trees over > 32 ranks */

	*nsteps = p.n;
	*nrefs = p.nr;
	if (!steps || !refs)
		return 0;               /* size query */
	if (p.n > p.cap || p.nr > p.rcap)
		return -LFA_ETOOSMALL;
	return 0;
}

LFA_INTERNAL void plan_free(struct plan *pl)
{
	free(pl->steps);
	free(pl->refs);
	memset(pl, 0, sizeof(*pl));
}

LFA_INTERNAL int plan_make(struct plan *pl, enum lfa_collective_op coll,
			   enum lfa_coll_algo algo, int rank, int n, int root,
			   size_t count, size_t esz)
{
	size_t ns = 0, nr = 0;
	int ret;

	memset(pl, 0, sizeof(*pl));
	ret = lfa_coll_plan(coll, algo, rank, n, root, count, esz, NULL, &ns,
			    NULL, &nr, &pl->tmp);
	if (ret)
		return ret;
	pl->steps = calloc(ns ? ns : 1, sizeof(*pl->steps));
	pl->refs = calloc(nr ? nr : 1, sizeof(*pl->refs));
	if (!pl->steps || !pl->refs) {
		plan_free(pl);
		return -LFA_ENOMEM;
	}
	pl->nsteps = ns;
	pl->nrefs = nr;
	ret = lfa_coll_plan(coll, algo, rank, n, root, count, esz, pl->steps,
			    &pl->nsteps, pl->refs, &pl->nrefs, &pl->tmp);
	if (ret)
		plan_free(pl);
	return ret;
}

/* Collective items -> grouped SEND/RECV items (transports without
 * collectives).  lower_barrier: BARRIER -> a ring of zero-byte messages,
 * every rank to every other (peer transports, whose sends leave only after
 * the rank's earlier items have completed).  lower_oneshot: ONESHOT -> the
 * items it is defined by (COPY src -> own SYM_IN, BARRIER, TREE over every
 * rank's SYM_IN, BARRIER), for executors that run all ranks on one stream
 * (the loopback), where one rank's kernel cannot wait for another's. */
LFA_INTERNAL int lower_plan(const struct plan *in, int r, int n, size_t esz,
			    struct plan *out, int lower_barrier, int lower_oneshot)
{
	size_t cap = in->nsteps + 1, rcap = in->nrefs + 1;

	for (size_t i = 0; i < in->nsteps; i++) {
		if (in->steps[i].type == LFA_STEP_ALLTOALL ||
		    in->steps[i].type == LFA_STEP_ALLGATHER ||
		    (lower_barrier && in->steps[i].type == LFA_STEP_BARRIER))
			cap += 2 * (size_t)n + 2;
		if (lower_oneshot && in->steps[i].type == LFA_STEP_ONESHOT) {
			cap += 4;
			rcap += (size_t)n;
		}
	}
	memset(out, 0, sizeof(*out));
	out->steps = calloc(cap, sizeof(*out->steps));
	out->refs = calloc(rcap, sizeof(*out->refs));
	if (!out->steps || !out->refs) {
		plan_free(out);
		return -LFA_ENOMEM;
	}
	memcpy(out->refs, in->refs, in->nrefs * sizeof(*in->refs));
	out->nrefs = in->nrefs;
	out->tmp = in->tmp;
	for (size_t i = 0; i < in->nsteps; i++) {
		const struct lfa_step *st = &in->steps[i];
		int a2a = st->type == LFA_STEP_ALLTOALL;
		struct lfa_step *o;

		if (lower_oneshot && st->type == LFA_STEP_ONESHOT) {
			/* this rank's part: [moff, moff + mlen) of the vector */
			size_t moff = 0, mlen = st->count;

			if (st->peer == LFA_ONESHOT_SCATTER)
				lfa_coll_block(st->count, n, r, &moff, &mlen);
			else if (st->peer >= 0 && st->peer != r)
				mlen = 0;
			o = &out->steps[out->nsteps++];
			memset(o, 0, sizeof(*o));
			o->type = LFA_STEP_COPY;
			o->dst = sref(LFA_BUF_SYM_IN, r, 0);
			o->src = st->src;
			o->count = st->count * esz;     /* COPY counts bytes */
			o = &out->steps[out->nsteps++];
			memset(o, 0, sizeof(*o));
			o->type = LFA_STEP_BARRIER;
			if (mlen) {
				o = &out->steps[out->nsteps++];
				memset(o, 0, sizeof(*o));
				o->type = LFA_STEP_TREE;
				o->dst = st->dst;
				o->first = (uint32_t)out->nrefs;
				o->nsrc = st->nsrc;
				o->count = mlen;
				for (int k = 0; k < (int)st->nsrc; k++) {
					struct lfa_ref in = k == r ? st->src :
							    sref(LFA_BUF_SYM_IN, k, 0);

					in.off += moff * esz;
					out->refs[out->nrefs++] = in;
				}
			}
			o = &out->steps[out->nsteps++];
			memset(o, 0, sizeof(*o));
			o->type = LFA_STEP_BARRIER;
			continue;
		}

		if (lower_barrier && st->type == LFA_STEP_BARRIER) {
			for (int k = 1; k < n; k++) {
				o = &out->steps[out->nsteps++];
				memset(o, 0, sizeof(*o));
				o->type = LFA_STEP_SEND;
				o->peer = (r + k) % n;
				o = &out->steps[out->nsteps++];
				memset(o, 0, sizeof(*o));
				o->type = LFA_STEP_RECV;
				o->peer = (r - k + n) % n;
			}
			if (n > 1) {
				o = &out->steps[out->nsteps++];
				memset(o, 0, sizeof(*o));
				o->type = LFA_STEP_GROUP_END;
			}
			continue;
		}
		if (!a2a && st->type != LFA_STEP_ALLGATHER) {
			out->steps[out->nsteps++] = *st;
			continue;
		}
		for (int k = 1; k < n; k++) {
			int to = (r + k) % n, from = (r - k + n) % n;

			o = &out->steps[out->nsteps++];
			memset(o, 0, sizeof(*o));
			o->type = LFA_STEP_SEND;
			o->peer = to;
			o->count = st->count;
			o->src = st->src;
			if (a2a)
				o->src.off += (uint64_t)to * st->count;
			o = &out->steps[out->nsteps++];
			memset(o, 0, sizeof(*o));
			o->type = LFA_STEP_RECV;
			o->peer = from;
			o->count = st->count;
			o->dst = st->dst;
			o->dst.off += (uint64_t)from * st->count;
		}
		if (n > 1) {
			o = &out->steps[out->nsteps++];
			memset(o, 0, sizeof(*o));
			o->type = LFA_STEP_GROUP_END;
		}
		o = &out->steps[out->nsteps++];
		memset(o, 0, sizeof(*o));
		o->type = LFA_STEP_COPY;
		o->count = st->count;
		o->dst = st->dst;
		o->dst.off += (uint64_t)r * st->count;
		o->src = st->src;
		if (a2a)
			o->src.off += (uint64_t)r * st->count;
		if (o->dst.buf == o->src.buf && o->dst.off == o->src.off)
			out->nsteps--;
	}
	return 0;
}
