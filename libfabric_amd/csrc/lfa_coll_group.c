/*
 * lfa_coll_group.c — joining and closing groups (liblfa_coll.so; split out
 * of lfa_coll.c in round 6): coll_join_collective (coll_coll.c:912-995) —
 * the cid-mask BAND allreduce over the parent, the RCCL split or a members'
 * communicator — its completion on the EQ (coll_join_comp, :690-720), and
 * lfa_mc_close.
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

static void free_mask(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc)
{
	if (!mc->mask_host)
		return;
	if (ep->dom->host)
		free(mc->mask_host);
	else
		hipHostFree(mc->mask_host);
	mc->mask_host = NULL;
}

LFA_INTERNAL void join_finish(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc)
{
	/* coll_join_comp (coll_coll.c:690-720): group id = lowest set bit of the
	 * BAND of every member's free-id mask; mark it used locally. */
	int gid = -1;

	for (int b = 0; b < LFA_MAX_GROUP_ID; b++) {
		if (mc->mask_host[b / 8] & (1u << (b % 8))) {
			gid = b;
			break;
		}
	}
	if (gid >= 0) {
		mc->group_id = (uint16_t)gid;
		ep->cid_mask[gid / 8] &= (uint8_t)~(1u << (gid % 8));
	}
	mc->seq = 0;
	free_mask(ep, mc);
	if (ep->eqn < 64) {
		size_t i = (ep->eqh + ep->eqn) % 64;

		ep->eq[i].event = LFA_JOIN_COMPLETE;
		ep->eq[i].entry.fid = mc;
		ep->eq[i].entry.context = mc->join_context;
		ep->eq[i].entry.data = 0;
		ep->eqn++;
	}
}

/* ---------------------------------------------------------------------- */
/* join                                                                    */
/* ---------------------------------------------------------------------- */

/*
 * A device domain's communicator for a group formed by its members alone
 * (lfa_join_members on a strict subset): the first member's RCCL unique id
 * reaches the others point-to-point over the parent's communicator — only
 * the members take part in those transfers — and the members then create
 * their communicator together.  The transfers are enqueued under ep->lock
 * (this rank's position in the parent's operation order); the waits run
 * outside it, so progress keeps reaping completions meanwhile.
 */
static int members_comm(struct lfa_coll_ep *ep, struct lfa_coll_mc *parent,
			const int *ranks, size_t n, int pos, ncclComm_t *out)
{
	ncclUniqueId uid;
	hipEvent_t ev = NULL;
	void *d = NULL;
	int ret = 0;

	memset(&uid, 0, sizeof(uid));
	hipSetDevice(ep->dom->device);
	if (pos == 0 && ncclGetUniqueId(&uid) != ncclSuccess)
		ret = -LFA_EIO;         /* the others still get (and fail on) zeros */
	if (hipMalloc(&d, sizeof(uid)) != hipSuccess ||
	    hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
		if (d)
			hipFree(d);
		return -LFA_ENOMEM;
	}
	pthread_mutex_lock(&ep->lock);
	if ((pos == 0 && hipMemcpyAsync(d, &uid, sizeof(uid), hipMemcpyHostToDevice,
					ep->stream) != hipSuccess) ||
	    ncclGroupStart() != ncclSuccess)
		ret = -LFA_EIO;
	for (size_t k = 1; k < n && pos == 0; k++)
		if (ncclSend(d, sizeof(uid), ncclUint8, ranks[k], parent->comm,
			     ep->stream) != ncclSuccess)
			ret = -LFA_EIO;
	if (pos != 0 && ncclRecv(d, sizeof(uid), ncclUint8, ranks[0], parent->comm,
				 ep->stream) != ncclSuccess)
		ret = -LFA_EIO;
	if (ncclGroupEnd() != ncclSuccess ||
	    hipMemcpyAsync(&uid, d, sizeof(uid), hipMemcpyDeviceToHost,
			   ep->stream) != hipSuccess ||
	    hipEventRecord(ev, ep->stream) != hipSuccess)
		ret = -LFA_EIO;
	pthread_mutex_unlock(&ep->lock);
	if (hipEventSynchronize(ev) != hipSuccess)
		ret = -LFA_EIO;
	hipEventDestroy(ev);
	hipFree(d);
	{
		/* a first member without an id sent zeros: everyone stops here */
		static const ncclUniqueId none;

		if (!memcmp(&uid, &none, sizeof(uid)))
			return ret ? ret : -LFA_EIO;
	}
	pthread_mutex_lock(&ep->comm_lock);
	if (ncclCommInitRank(out, (int)n, uid, pos) != ncclSuccess)
		ret = ret ? ret : -LFA_EIO;
	pthread_mutex_unlock(&ep->comm_lock);
	return ret;
}

/* members_only: lfa_join_members — the agreement runs over the new group
 * itself, so only its members call (see lfa_coll.h). */
static int join_impl(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
		     const int *ranks, size_t nmembers, uint64_t flags,
		     struct lfa_coll_mc **mcp, void *context, int members_only)
{
	struct lfa_coll_mc *parent, *mc;
	int member = 0, pos = -1, ret = 0, host;
	void *dmask;

	if (!ep || !mcp)
		return -LFA_EINVAL;
	if (flags & ~LFA_COLLECTIVE)
		return -LFA_EBADFLAGS;
	host = ep->dom->host;
	parent = mc_of(ep, coll_addr);
	if (!mc_member(parent))
		return -LFA_EINVAL;
	if (members_only && !ranks)
		return -LFA_EINVAL;
	if (ranks) {
		/* ranks[i] is the parent rank of group rank i, in any order: the
		 * group numbers its members by their position in the joined set,
		 * as prov/coll does (coll_find_local_rank, coll_coll.c:669-689:
		 * local_rank = index in the av_set's fi_addr_array) */
		uint8_t *seen;

		if (!nmembers || nmembers > (size_t)parent->size)
			return -LFA_EINVAL;
		seen = calloc((size_t)parent->size / 8 + 1, 1);
		if (!seen)
			return -LFA_ENOMEM;
		for (size_t i = 0; i < nmembers; i++) {
			if (ranks[i] < 0 || ranks[i] >= parent->size ||
			    (seen[ranks[i] / 8] & (1u << (ranks[i] % 8)))) {
				free(seen);
				return -LFA_EINVAL;     /* out of range or listed twice */
			}
			seen[ranks[i] / 8] |= (uint8_t)(1u << (ranks[i] % 8));
			if (ranks[i] == parent->rank) {
				member = 1;
				pos = (int)i;
			}
		}
		free(seen);
	} else {
		member = 1;
		pos = parent->rank;
		nmembers = (size_t)parent->size;
	}
	if (members_only) {
		if (!member)
			return -LFA_EINVAL;     /* only members call this form */
		if (!host && nmembers == (size_t)parent->size)
			members_only = 0;       /* the whole group: every rank calls */
	}
	mc = calloc(1, sizeof(*mc));
	if (!mc)
		return -LFA_ENOMEM;
	mc->ep = ep;
	mc->join_context = context;
	mc->group_id = LFA_MAX_GROUP_ID;        /* none until the join completes */
	if (!ranks) {
		mc->comm = parent->comm;
		mc->rank = parent->rank;
		mc->size = parent->size;
		if (host && parent->members) {
			mc->members = malloc(nmembers * sizeof(*mc->members));
			if (!mc->members)
				ret = -LFA_ENOMEM;
			else
				memcpy(mc->members, parent->members,
				       nmembers * sizeof(*mc->members));
		}
	} else if (host) {
		/* prov/coll's av_set: group rank -> the owner's address (here
		 * the domain rank) */
		mc->rank = pos;
		mc->size = (int)nmembers;
		mc->members = malloc(nmembers * sizeof(*mc->members));
		if (!mc->members)
			ret = -LFA_ENOMEM;
		for (size_t i = 0; !ret && i < nmembers; i++)
			mc->members[i] = world_rank(parent, ranks[i]);
	} else if (members_only) {
		/* a strict subset formed by its members alone: no split (that
		 * needs every parent rank) but a communicator of its own */
		ret = members_comm(ep, parent, ranks, nmembers, pos, &mc->comm);
		mc->owns_comm = !ret;
		mc->rank = pos;
		mc->size = (int)nmembers;
	} else {
		/*
		 * Every parent rank takes part in the split (non-members with
		 * NCCL_SPLIT_NOCOLOR).  The split is a blocking rendezvous of the
		 * parent's members; it is issued under comm_lock, in this rank's
		 * call order, and NOT under ep->lock, so completions keep being
		 * reaped (lfa_cq_read, e.g. from off_lfa's progress thread)
		 * while the members meet (DESIGN.md §6 "ordering").
		 */
		ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;

		pthread_mutex_lock(&ep->comm_lock);
		hipSetDevice(ep->dom->device);
		/* key = the position in the set: RCCL numbers the new
		 * communicator by key, so its rank is the group rank */
		if (ncclCommSplit(parent->comm, member ? 0 : NCCL_SPLIT_NOCOLOR,
				  member ? pos : parent->rank, &mc->comm, &cfg) != ncclSuccess)
			ret = -LFA_EIO;
		pthread_mutex_unlock(&ep->comm_lock);
		mc->owns_comm = !ret;
		mc->rank = pos;
		mc->size = (int)nmembers;
	}
	/*
	 * A non-member (every parent rank calls join, as every rank of the
	 * reference's parent group takes part in the join allreduce) gets a
	 * handle with no communicator: it completes the join like the members
	 * but cannot issue collectives on it (-LFA_EINVAL).
	 */
	if (!member) {
		mc->comm = NULL;
		mc->rank = -1;
		mc->size = (int)nmembers;
	}
	pthread_mutex_lock(&ep->lock);
	/* agree on the group id: BAND of the free-id masks over the PARENT
	 * group (coll_join_collective, coll_coll.c:969-973), UINT8 x 32 — or,
	 * members_only, over the new group itself under the reserved id
	 * LFA_MAX_GROUP_ID (the av_set's own coll_mc as the parent) */
	if (!ret && host) {
		mc->mask_host = malloc(2 * LFA_CID_BYTES);
		if (!mc->mask_host)
			ret = -LFA_ENOMEM;
		if (!ret) {
			memcpy(mc->mask_host + LFA_CID_BYTES, ep->cid_mask, LFA_CID_BYTES);
			ret = host_submit(ep, members_only ? mc : parent, LFA_ALLREDUCE,
					  mc->mask_host + LFA_CID_BYTES, mc->mask_host,
					  LFA_CID_BYTES, -1, LFA_UINT8, LFA_BAND,
					  context, 1, mc, 0, LFA_ALGO_TREE);
		}
	} else if (!ret) {
		struct lfa_coll_mc *over = members_only ? mc : parent;
		const uint64_t t0 = over->p2p_ticket;

		hipSetDevice(ep->dom->device);
		ret = hipHostMalloc((void **)&mc->mask_host, 2 * LFA_CID_BYTES, 0) ==
		      hipSuccess ? 0 : -LFA_ENOMEM;
		if (!ret && grow_staging(ep, 4 * LFA_CID_BYTES))
			ret = -LFA_ENOMEM;
		if (!ret) {
			dmask = ep->hs[0];
			memcpy(mc->mask_host + LFA_CID_BYTES, ep->cid_mask, LFA_CID_BYTES);
			hipMemcpyAsync(dmask, mc->mask_host + LFA_CID_BYTES, LFA_CID_BYTES,
				       hipMemcpyHostToDevice, ep->stream);
			/* the join's own agreement: a fixed schedule, whatever
			 * algorithm each member has selected for its collectives */
			ret = run_device(ep, over, LFA_ALLREDUCE, dmask,
					 (char *)dmask + LFA_CID_BYTES, LFA_CID_BYTES, -1,
					 LFA_UINT8, LFA_BAND, ep->stream, LFA_ALGO_TREE);
			if (!ret)
				hipMemcpyAsync(mc->mask_host, (char *)dmask + LFA_CID_BYTES,
					       LFA_CID_BYTES, hipMemcpyDeviceToHost, ep->stream);
		}
		if (!ret)
			ret = enqueue_completion(ep, ep->stream, context, 1, mc, 0, NULL);
		if (!ret)
			tag_p2p(ep, over, t0);
	}
	if (ret)
		free_mask(ep, mc);
	pthread_mutex_unlock(&ep->lock);
	if (ret) {
		if (mc->owns_comm && mc->comm) {
			pthread_mutex_lock(&ep->comm_lock);
			ncclCommDestroy(mc->comm);
			pthread_mutex_unlock(&ep->comm_lock);
		}
		free(mc->members);
		free(mc);
		return ret;
	}
	*mcp = mc;
	return 0;
}

int lfa_join_collective(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
			const int *ranks, size_t nmembers, uint64_t flags,
			struct lfa_coll_mc **mcp, void *context)
{
	return join_impl(ep, coll_addr, ranks, nmembers, flags, mcp, context, 0);
}

int lfa_join_members(struct lfa_coll_ep *ep, lfa_addr_t coll_addr,
		     const int *ranks, size_t nmembers, uint64_t flags,
		     struct lfa_coll_mc **mcp, void *context)
{
	return join_impl(ep, coll_addr, ranks, nmembers, flags, mcp, context, 1);
}

int lfa_mc_close(struct lfa_coll_mc *mc)
{
	struct lfa_coll_ep *ep;

	if (!mc)
		return -LFA_EINVAL;
	if (mc->is_world)
		return -LFA_EINVAL;
	ep = mc->ep;
	lfa_coll_ep_flush(ep);
	/* a join still queued for this handle completes without it */
	pthread_mutex_lock(&ep->lock);
	for (size_t i = 0; i < ep->qlen; i++) {
		struct pending *p = &ep->q[(ep->qhead + i) % ep->qcap];

		if (p->kind == 1 && p->mc == mc) {
			p->kind = 2;
			p->mc = NULL;
		}
		if (p->pmc == mc) {
			/* the stream has drained (flush above): the word is final */
			p->timed_out = p2p_timed_out(p);
			p->pmc = NULL;
		}
	}
	free_mask(ep, mc);
	/* release the group id only if the join assigned one (a
	 * never-completed join must not free the world's reserved id 0) */
	if (mc->group_id < LFA_MAX_GROUP_ID)
		ep->cid_mask[mc->group_id / 8] |= (uint8_t)(1u << (mc->group_id % 8));
	pthread_mutex_unlock(&ep->lock);
	if (!ep->dom->host) {
		pthread_mutex_lock(&ep->comm_lock);
		p2p_release(mc);
		if (mc->owns_comm && mc->comm)
			ncclCommDestroy(mc->comm);
		pthread_mutex_unlock(&ep->comm_lock);
	} else {
		p2p_release(mc);        /* a peer domain's device workspace */
	}
	sig_word_free(mc);
	free(mc->members);
	free(mc);
	return 0;
}
