/*
 * lfa_coll_loopback.c — every rank of an N-rank schedule on ONE GPU: the
 * planner's SEND/RECV groups become device copies through per-pair
 * mailboxes, the local items the real gfx950 kernels (run_local).  Used by
 * the tests and the bench to execute N = 2..64-rank schedules on one MI355X
 * against the oracle (prov/coll's coll_do_allreduce order,
 * coll_coll.c:349-449).
 */
#include <stdlib.h>

#include "lfa_coll_int.h"

/* ====================================================================== */
/* single-GPU multi-rank executor (loopback transport)                     */
/* ====================================================================== */

struct lb_msg {
	struct lb_msg *next;
	void *data;
	size_t bytes;
};

int lfa_coll_loopback(enum lfa_collective_op coll, enum lfa_coll_algo algo,
		      int n, int root, enum lfa_datatype dt, enum lfa_op op,
		      size_t count, void *const *send, void *const *result,
		      void *stream)
{
	hipStream_t s = (hipStream_t)stream;
	size_t esz = lfa_datatype_size(dt);
	struct plan *pl = NULL;
	size_t *pc = NULL, *arrived = NULL, region = sym_region(count, esz);
	void **tmp = NULL;
	char **sym = NULL;
	struct lb_msg **box = NULL;
	int ret = 0, done, progressed;

	if (n < 1 || n > 64 || !send || !result || !esz)
		return -LFA_EINVAL;
	if ((coll == LFA_ALLREDUCE || coll == LFA_REDUCE ||
	     coll == LFA_REDUCE_SCATTER) && (ret = check_reduce_args(dt, op)))
		return ret;
	if (algo == LFA_ALGO_RCCL)
		algo = LFA_ALGO_TREE;
	if (algo != LFA_ALGO_TREE && algo != LFA_ALGO_RD &&
	    algo != LFA_ALGO_TREE_COLL && algo != LFA_ALGO_P2P)
		return -LFA_EINVAL;
	pl = calloc((size_t)n, sizeof(*pl));
	pc = calloc((size_t)n, sizeof(*pc));
	arrived = calloc((size_t)n, sizeof(*arrived));
	tmp = calloc((size_t)n, sizeof(*tmp));
	sym = calloc((size_t)n, sizeof(*sym));
	box = calloc((size_t)n * (size_t)n, sizeof(*box));
	if (!pl || !pc || !arrived || !tmp || !sym || !box) {
		ret = -LFA_ENOMEM;
		goto out;
	}
	for (int r = 0; r < n && !ret; r++) {
		struct plan raw;

		ret = plan_make(&raw, coll, algo, r, n, root, count, esz);
		if (ret)
			break;
		ret = lower_plan(&raw, r, n, esz, &pl[r], 0, 1);
		plan_free(&raw);
		if (!ret && pl[r].tmp &&
		    hipMallocAsync(&tmp[r], pl[r].tmp, s) != hipSuccess)
			ret = -LFA_ENOMEM;
		/* P2P: every rank's symmetric workspace, plain pointers here */
		if (!ret && plan_uses_sym(pl[r].steps, pl[r].nsteps) &&
		    hipMallocAsync((void **)&sym[r], 2 * region, s) != hipSuccess)
			ret = -LFA_ENOMEM;
	}
	/*
	 * Lockstep: a rank runs local steps freely; at a comm group it posts
	 * all its SENDs (snapshot copies) and completes once every RECV of the
	 * group has a message waiting — RCCL group semantics.
	 */
	do {
		done = 1;
		progressed = 0;
		for (int r = 0; r < n && !ret; r++) {
			struct xctx xc = { .base = { send[r], result[r], tmp[r] }, .sym = sym,
					   .region = region };

			if (coll == LFA_BROADCAST)
				xc.base[LFA_BUF_SEND] = result[r];
			while (pc[r] < pl[r].nsteps && !ret) {
				struct lfa_step *st = &pl[r].steps[pc[r]];

				if (st->type == LFA_STEP_BARRIER) {
					/* one stream: a rank passes barrier b once every
					 * rank has enqueued everything before its b-th */
					int all = 1;

					if (!(arrived[r] & 1)) {
						arrived[r] += 3;   /* count in bits 1.., flag 1 */
						progressed = 1;
					}
					for (int q = 0; q < n; q++)
						if ((arrived[q] >> 1) < (arrived[r] >> 1))
							all = 0;
					if (!all)
						break;
					arrived[r] &= ~(size_t)1;
					pc[r]++;
					progressed = 1;
					continue;
				}
				if (st->type != LFA_STEP_SEND && st->type != LFA_STEP_RECV &&
				    st->type != LFA_STEP_GROUP_END) {
					ret = run_local(st, pl[r].refs, &xc, op, dt, s);
					pc[r]++;
					progressed = 1;
					continue;
				}
				/* a group: [pc, end) up to GROUP_END */
				size_t end = pc[r];
				int ready = 1;

				while (end < pl[r].nsteps &&
				       pl[r].steps[end].type != LFA_STEP_GROUP_END)
					end++;
				/* post sends once (mark by negating peer) */
				for (size_t i = pc[r]; i < end; i++) {
					struct lfa_step *x = &pl[r].steps[i];

					if (x->type != LFA_STEP_SEND || x->peer < 0)
						continue;
					struct lb_msg *m = calloc(1, sizeof(*m)), **t;

					if (!m || hipMallocAsync(&m->data, x->count, s) != hipSuccess) {
						free(m);
						ret = -LFA_ENOMEM;
						break;
					}
					m->bytes = x->count;
					hipMemcpyAsync(m->data, resolve(&xc, x->src), x->count,
						       hipMemcpyDeviceToDevice, s);
					t = &box[(size_t)r * n + x->peer];
					while (*t)
						t = &(*t)->next;
					*t = m;
					x->peer = -x->peer - 1;
					progressed = 1;
				}
				/* every recv matched? (count per peer in order) */
				for (size_t i = pc[r]; i < end && ready; i++) {
					struct lfa_step *x = &pl[r].steps[i];
					int need = 0;

					if (x->type != LFA_STEP_RECV)
						continue;
					for (size_t j = pc[r]; j <= i; j++)
						if (pl[r].steps[j].type == LFA_STEP_RECV &&
						    pl[r].steps[j].peer == x->peer)
							need++;
					struct lb_msg *m = box[(size_t)x->peer * n + r];

					while (m && --need)
						m = m->next;
					if (!m)
						ready = 0;
				}
				if (!ready || ret)
					break;
				for (size_t i = pc[r]; i < end; i++) {
					struct lfa_step *x = &pl[r].steps[i];
					struct lb_msg *m;

					if (x->type == LFA_STEP_SEND) {
						x->peer = -x->peer - 1;  /* restore */
						continue;
					}
					m = box[(size_t)x->peer * n + r];
					box[(size_t)x->peer * n + r] = m->next;
					if (m->bytes != x->count)
						ret = -LFA_EIO;
					hipMemcpyAsync(resolve(&xc, x->dst), m->data, x->count,
						       hipMemcpyDeviceToDevice, s);
					hipFreeAsync(m->data, s);
					free(m);
				}
				pc[r] = end < pl[r].nsteps ? end + 1 : end;
				progressed = 1;
			}
			if (pc[r] < pl[r].nsteps)
				done = 0;
		}
		if (!done && !progressed && !ret)
			ret = -LFA_EIO;   /* schedule deadlock: a bug */
	} while (!done && !ret);
out:
	if (box) {
		for (size_t k = 0; k < (size_t)n * (size_t)n; k++)
			while (box[k]) {
				struct lb_msg *m = box[k];

				box[k] = m->next;
				hipFreeAsync(m->data, s);
				free(m);
			}
	}
	if (tmp)
		for (int r = 0; r < n; r++)
			if (tmp[r])
				hipFreeAsync(tmp[r], s);
	if (sym)
		for (int r = 0; r < n; r++)
			if (sym[r])
				hipFreeAsync(sym[r], s);
	if (pl)
		for (int r = 0; r < n; r++)
			plan_free(&pl[r]);
	free(pl);
	free(pc);
	free(arrived);
	free(tmp);
	free(sym);
	free(box);
	return ret;
}
