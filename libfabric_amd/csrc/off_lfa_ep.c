/*
 * off_lfa_ep.c — the off_lfa provider's endpoint (liboff_lfa-fi.so; split
 * out of off_lfa.c in round 6): progress (the thread and rxm's util_ep
 * slot), the RCCL unique-id bootstrap and the owner's tagged transport,
 * joins (coll_join_collective's role, coll_coll.c:912-995) and the
 * fi_ops_collective slots that forward to liblfa_coll.so.
 */
#define _GNU_SOURCE
#include "off_lfa_int.h"

/* -------------------------------------------------------------- helpers -- */

static int olfa_env_int(const char *name, int dflt)
{
	const char *v = getenv(name);

	return v && *v ? atoi(v) : dflt;
}

static struct olfa_mc *olfa_mc_lookup(struct olfa_ep *ep, fi_addr_t coll_addr)
{
	struct olfa_mc *m;

	for (m = ep->mcs; m; m = m->next)
		if ((fi_addr_t)(uintptr_t)m == coll_addr)
			return m;
	return NULL;
}

/* coll_addr -> liblfa_coll group address, or LFA_ADDR_NOTAVAIL */
static lfa_addr_t olfa_resolve(struct olfa_ep *ep, fi_addr_t coll_addr)
{
	struct olfa_mc *m;
	lfa_addr_t a = LFA_ADDR_NOTAVAIL;

	pthread_mutex_lock(&ep->lock);
	m = olfa_mc_lookup(ep, coll_addr);
	if (m)
		a = m->laddr;
	pthread_mutex_unlock(&ep->lock);
	return a;
}

static void olfa_mc_register(struct olfa_ep *ep, struct olfa_mc *m)
{
	m->ep = ep;
	m->next = ep->mcs;
	ep->mcs = m;
}

OLFA_INTERNAL void olfa_mc_unregister(struct olfa_ep *ep, struct olfa_mc *m)
{
	struct olfa_mc **pp;

	for (pp = &ep->mcs; *pp; pp = &(*pp)->next)
		if (*pp == m) {
			*pp = m->next;
			break;
		}
	m->next = NULL;
}

/* Test knob (LFA_TEST_JOIN_DELAY_US, never a deployer parameter): a pause
 * between a join's lfa_join_* call and its registration, which widens the
 * window olfa_post_join covers (tests/test_off_lfa.py). */
static void olfa_test_join_delay(void)
{
	const char *v = lfa_param("LFA_TEST_JOIN_DELAY_US");
	long us = v ? strtol(v, NULL, 0) : 0;

	if (us > 0) {
		struct timespec t = { us / 1000000, (us % 1000000) * 1000 };

		nanosleep(&t, NULL);
	}
}

/* ------------------------------------------------------------ progress -- */

static void olfa_emit_join(struct olfa_ep *ep, struct olfa_mc *m,
			   const struct lfa_eq_entry *lev)
{
	struct fi_eq_entry e;

	memset(&e, 0, sizeof(e));
	e.fid = m ? &m->mc_fid.fid : NULL;
	e.context = lev->context;
	e.data = lev->data;
	if (ep->eq)
		fi_eq_write(ep->eq->peer_eq, FI_JOIN_COMPLETE, &e, sizeof(e), 0);
	else
		olfa_warn("join completed with no EQ bound", NULL, 0);
}

/* A join event to the owner's EQ with the fid of its registered group;
 * -FI_EAGAIN when the group is not registered yet but a join is between
 * its lfa_join_* call and its registration (the event may be its own: a
 * one-member join completes inside the call).  The count is read before the
 * registry, so a miss with a join counted means that join's registration,
 * which comes before its decrement, had not happened.  An event whose group
 * is gone (closed before its event was read) goes out without a fid, as
 * before. */
static int olfa_post_join(struct olfa_ep *ep, const struct lfa_eq_entry *lev)
{
	const int joining = atomic_load(&ep->joins_in_flight);
	struct olfa_mc *m;

	pthread_mutex_lock(&ep->lock);
	for (m = ep->mcs; m; m = m->next)
		if (m->lmc && (void *)m->lmc == lev->fid)
			break;
	pthread_mutex_unlock(&ep->lock);
	if (!m && joining)
		return -FI_EAGAIN;
	olfa_emit_join(ep, m, lev);
	return 0;
}

/* Moves finished collectives and joins to the owner: CQ entries through
 * the peer CQ's owner_ops (coll_coll.c:725-733), join events through the
 * peer EQ (coll_coll.c:708-717).  Returns how many it moved. */
OLFA_INTERNAL int olfa_progress(struct olfa_ep *ep)
{
	struct lfa_cq_entry ent[16];
	struct lfa_cq_err_entry lerr;
	uint32_t event;
	ssize_t n;
	int moved = 0;

	if (!ep->le)
		return 0;
	/* plock keeps owner writes in completion order when the thread and
	 * the owner progress at once; the registry lock is not held across
	 * owner callbacks. */
	pthread_mutex_lock(&ep->plock);
	for (;;) {
		n = lfa_cq_read(ep->le, ent, 16);
		if (n > 0) {
			for (ssize_t i = 0; i < n; i++) {
				ssize_t w = -FI_EAGAIN;

				if (ep->cq)
					w = ep->cq->peer_cq->owner_ops->write(
						ep->cq->peer_cq, ent[i].op_context,
						FI_COLLECTIVE, 0, NULL, 0, 0,
						FI_ADDR_NOTAVAIL);
				if (w)
					olfa_warn("owner CQ write failed", NULL, (long)w);
			}
			moved += (int)n;
			continue;
		}
		if (n == -LFA_EIO && lfa_cq_readerr(ep->le, &lerr) > 0) {
			struct fi_cq_err_entry e;

			memset(&e, 0, sizeof(e));
			e.op_context = lerr.op_context;
			e.flags = FI_COLLECTIVE;
			e.err = lerr.err;
			e.prov_errno = lerr.prov_errno;
			e.src_addr = FI_ADDR_NOTAVAIL;
			if (ep->cq)
				ep->cq->peer_cq->owner_ops->writeerr(ep->cq->peer_cq, &e);
			moved++;
			continue;
		}
		break;
	}
	/* join events in order; one whose group is still being registered is
	 * held (and the ones behind it wait) until a later pass */
	for (;;) {
		if (!ep->have_held) {
			if (lfa_eq_read(ep->le, &event, &ep->held) <= 0)
				break;
			ep->have_held = 1;
		}
		if (olfa_post_join(ep, &ep->held) < 0)
			break;
		ep->have_held = 0;
		moved++;
	}
	pthread_mutex_unlock(&ep->plock);
	return moved;
}

static void olfa_util_progress(void *util_ep)
{
	olfa_progress((struct olfa_ep *)util_ep);
}

/* FI_PROGRESS_AUTO.  Spins (yielding) while work came through recently and
 * backs off to 20 us naps after a quiet spell, so a latency-bound chain of
 * peer transfers is advanced within microseconds without a busy core when
 * the endpoint idles. */
static void *olfa_progress_thread(void *arg)
{
	struct olfa_ep *ep = arg;
	const struct timespec idle = { 0, 20000 };
	unsigned quiet = 0;

	while (!atomic_load(&ep->stop)) {
		if (olfa_progress(ep)) {
			quiet = 0;
		} else if (++quiet < 4096) {
			sched_yield();
		} else {
			nanosleep(&idle, NULL);
		}
	}
	return NULL;
}

/* ------------------------------------------------------------ bootstrap -- */

static int olfa_uid_rendezvous(int rank, unsigned char *id)
{
	const char *dir = olfa_param("bootstrap_dir");
	const char *key = olfa_param("bootstrap_key");
	int timeout = olfa_param_int("bootstrap_timeout", 120);
	char path[4096], tmp[4200];
	const struct timespec nap = { 0, 10000000 };
	struct timespec t0, t;
	int fd, ret;

	if (!dir || !*dir)
		return -FI_EINVAL;
	snprintf(path, sizeof(path), "%s/off_lfa-%s.uid", dir,
		 key && *key ? key : "world");
	if (rank == 0) {
		ret = lfa_coll_get_unique_id(id, LFA_UNIQUE_ID_BYTES);
		if (ret)
			return ret;
		snprintf(tmp, sizeof(tmp), "%s.tmp.%d", path, (int)getpid());
		fd = open(tmp, O_WRONLY | O_CREAT | O_TRUNC, 0600);
		if (fd < 0)
			return -FI_EIO;
		ret = write(fd, id, LFA_UNIQUE_ID_BYTES) == LFA_UNIQUE_ID_BYTES ? 0 : -FI_EIO;
		close(fd);
		if (!ret && rename(tmp, path))
			ret = -FI_EIO;
		return ret;
	}
	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (;;) {
		fd = open(path, O_RDONLY);
		if (fd >= 0) {
			ret = read(fd, id, LFA_UNIQUE_ID_BYTES) == LFA_UNIQUE_ID_BYTES ? 0 : -FI_EIO;
			close(fd);
			return ret;
		}
		clock_gettime(CLOCK_MONOTONIC, &t);
		if (t.tv_sec - t0.tv_sec > timeout)
			return -FI_ETIMEDOUT;
		nanosleep(&nap, NULL);
	}
}

/*
 * Peer transport (OFF_LFA_TRANSPORT=peer): the collective's transfers ride on
 * the OWNER's tagged messaging, exactly as prov/coll's do on rxm's —
 * fi_tsendmsg / fi_trecvmsg(FI_PEER_TRANSFER) on the owner endpoint with
 * prov/coll's tag (coll_coll.c:770-814); the owner reports each finished
 * transfer through peer_ops->complete (rxm_cq.c:1532-1546, 846-872), which
 * lands in olfa_peer_complete below.  Buffers are host memory; reductions
 * run in liblfa's host combine (lfa_coll_domain_open_host).
 */
struct olfa_xfer {
	atomic_int done;                /* 1 ok, -err failed */
	struct iovec iov;
};

static int olfa_xpost(struct olfa_ep *ep, int send, int peer, void *buf,
		      size_t bytes, uint64_t tag, void **req)
{
	struct olfa_xfer *x = calloc(1, sizeof(*x));
	struct fi_msg_tagged msg;
	ssize_t ret;

	if (!x)
		return -LFA_ENOMEM;
	x->iov.iov_base = buf;
	x->iov.iov_len = bytes;
	memset(&msg, 0, sizeof(msg));
	msg.msg_iov = &x->iov;
	msg.iov_count = 1;
	msg.addr = ep->waddr[peer];
	msg.tag = tag;
	msg.context = x;
	ret = send ? fi_tsendmsg(ep->peer_ep, &msg, FI_PEER_TRANSFER) :
		     fi_trecvmsg(ep->peer_ep, &msg, FI_PEER_TRANSFER);
	if (ret) {
		free(x);
		return ret == -FI_EAGAIN ? -LFA_EAGAIN : (int)ret;
	}
	*req = x;
	return 0;
}

static int olfa_xsend(void *ctx, int peer, const void *buf, size_t bytes,
		      uint64_t tag, void **req)
{
	return olfa_xpost(ctx, 1, peer, (void *)buf, bytes, tag, req);
}

static int olfa_xrecv(void *ctx, int peer, void *buf, size_t bytes, uint64_t tag,
		      void **req)
{
	return olfa_xpost(ctx, 0, peer, buf, bytes, tag, req);
}

static int olfa_xtest(void *ctx, void *req)
{
	struct olfa_xfer *x = req;
	int d = atomic_load(&x->done);

	if (!d)
		return 0;
	free(x);
	return d > 0 ? 1 : d;
}

static const struct lfa_peer_xfer_ops olfa_xops = {
	olfa_xsend, olfa_xrecv, olfa_xtest,
};

/* Creates the liblfa_coll domain + endpoint for the world group — over RCCL
 * (blocking, like ncclCommInitRank) or over the owner's transfers — and
 * starts progress.  `addrs` are the members' owner AV addresses in rank
 * order. */
static int olfa_bootstrap(struct olfa_ep *ep, int rank, int nranks,
			  const fi_addr_t *addrs)
{
	unsigned char id[LFA_UNIQUE_ID_BYTES];
	int ret = 0;

	/* the world's addresses: the peer transport's destinations, and the
	 * rank map of later joins over an av_set's own address */
	ep->waddr = malloc((size_t)nranks * sizeof(*ep->waddr));
	if (!ep->waddr)
		return -FI_ENOMEM;
	memcpy(ep->waddr, addrs, (size_t)nranks * sizeof(*ep->waddr));
	ep->nworld = (size_t)nranks;
	if (ep->peer_xport) {
		/* on the endpoint's GPU, so device buffers run the kernels with
		 * staged transfers (lfa_coll_domain_open_peer); a host without a
		 * usable GPU keeps host buffers only, unless a device was named */
		ret = lfa_coll_domain_open_peer(ep->device, rank, nranks, &olfa_xops, ep,
						&ep->ld);
		if (ret == -LFA_EINVAL && !ep->device_set)
			ret = lfa_coll_domain_open_peer(-1, rank, nranks, &olfa_xops, ep,
							&ep->ld);
		if (ret)
			goto err_addr;
		goto open_ep;
	}
	if (ep->have_uid)
		memcpy(id, ep->uid, sizeof(id));
	else if (nranks == 1)
		ret = lfa_coll_get_unique_id(id, sizeof(id));
	else
		ret = olfa_uid_rendezvous(rank, id);
	if (!ep->have_uid && ret) {
		olfa_warn("no unique id: set OFF_LFA_OPT_UNIQUE_ID or "
			  "OFF_LFA_BOOTSTRAP_DIR", NULL, ret);
		goto err_addr;
	}
	ret = lfa_coll_domain_open(ep->device, rank, nranks, id, sizeof(id), &ep->ld);
	if (ret)
		goto err_addr;
open_ep:
	ret = lfa_coll_ep_open(ep->ld, &ep->le);
	if (ret)
		goto err_dom;
	if (ep->algo >= 0 && (ret = lfa_coll_ep_set_algo(ep->le, ep->algo)))
		goto err_ep;
	if (ep->chunk && (ret = lfa_coll_ep_set_chunk(ep->le, ep->chunk)))
		goto err_ep;
	if (!ep->manual_progress) {
		atomic_store(&ep->stop, 0);
		if (pthread_create(&ep->thread, NULL, olfa_progress_thread, ep)) {
			ret = -FI_ENOMEM;
			goto err_ep;
		}
		ep->thread_running = 1;
	}
	return 0;
err_ep:
	lfa_coll_ep_close(ep->le);
	ep->le = NULL;
err_dom:
	lfa_coll_domain_close(ep->ld);
	ep->ld = NULL;
err_addr:
	free(ep->waddr);
	ep->waddr = NULL;
	ep->nworld = 0;
	return ret;
}

/* ------------------------------------------------------------------ mc -- */

static int olfa_mc_close(struct fid *fid)
{
	struct olfa_mc *m = olfa_container_of(fid, struct olfa_mc, mc_fid.fid);
	struct olfa_ep *ep = m->ep;

	if (ep) {
		/* a held join event of this group goes with it: its lfa handle is
		 * freed below, and a later join's could reuse the address (plock
		 * before the registry lock, as in olfa_progress) */
		pthread_mutex_lock(&ep->plock);
		if (ep->have_held && m->lmc && ep->held.fid == (void *)m->lmc)
			ep->have_held = 0;
		pthread_mutex_unlock(&ep->plock);
		pthread_mutex_lock(&ep->lock);
		olfa_mc_unregister(ep, m);
		if (ep->world == m)
			ep->world = NULL;
		pthread_mutex_unlock(&ep->lock);
	}
	if (m->lmc)
		lfa_mc_close(m->lmc);
	free(m->members);
	free(m);
	return 0;
}

static struct fi_ops olfa_mc_fi_ops = OLFA_FI_OPS(olfa_mc_close, olfa_no_bind,
						  olfa_no_control);

/* position of addr in list, or -1 */
OLFA_INTERNAL long olfa_index(const fi_addr_t *list, size_t n, fi_addr_t addr)
{
	for (size_t i = 0; i < n; i++)
		if (list[i] == addr)
			return (long)i;
	return -1;
}

/* A join whose parent is the set itself: its members, as world ranks, form
 * the group through lfa_join_members; the other world ranks call nothing.
 * Group rank i is the set's i-th address (coll_find_local_rank,
 * coll_coll.c:669-689), whatever order insert / remove left it in. */
static int olfa_join_self(struct olfa_ep *ep, struct olfa_av_set *set,
			  struct olfa_mc *m, uint64_t flags, void *context)
{
	size_t n = set->count;
	int *ranks = malloc(n * sizeof(int)), ret = 0;

	m->members = malloc(n * sizeof(fi_addr_t));
	if (!ranks || !m->members) {
		ret = -FI_ENOMEM;
		goto out;
	}
	pthread_mutex_lock(&ep->lock);
	for (size_t i = 0; i < n && !ret; i++) {
		long r = ep->waddr ? olfa_index(ep->waddr, ep->nworld, set->addr[i]) : -1;

		if (r < 0)
			ret = -FI_EINVAL;       /* not in the bootstrapped world */
		else
			ranks[i] = (int)r;
	}
	pthread_mutex_unlock(&ep->lock);
	if (ret)
		goto out;
	for (size_t i = 0; i < n; i++)
		m->members[i] = set->addr[i];   /* lfa_join_members rejects repeats */
	m->nmembers = n;
	atomic_fetch_add(&ep->joins_in_flight, 1);    /* olfa_post_join */
	ret = lfa_join_members(ep->le, lfa_coll_world_addr(ep->le), ranks, n, flags,
			       &m->lmc, context);
	olfa_test_join_delay();
	if (!ret) {
		pthread_mutex_lock(&ep->lock);
		m->laddr = lfa_mc_addr(m->lmc);
		olfa_mc_register(ep, m);
		pthread_mutex_unlock(&ep->lock);
	}
	atomic_fetch_sub(&ep->joins_in_flight, 1);
out:
	free(ranks);
	if (ret) {
		free(m->members);
		m->members = NULL;
	}
	return ret;
}

/* fi_join_collective (coll_coll.c:912-995).  The parent group is the one
 * coll_addr names; FI_ADDR_NOTAVAIL means the set's world group, which the
 * first such join creates; the set's own address (fi_av_set_addr) means the
 * set's members alone (olfa_join_self). */
static int olfa_join(struct fid_ep *ep_fid, const void *addr, uint64_t flags,
		     struct fid_mc **mc_fid, void *context)
{
	struct olfa_ep *ep = (struct olfa_ep *)ep_fid;
	const struct fi_collective_addr *ca = addr;
	struct olfa_av_set *set;
	struct olfa_mc *parent, *m;
	fi_addr_t my_addr;
	int *ranks = NULL, ret, self;
	size_t n;
	lfa_addr_t paddr;

	if (!(flags & FI_COLLECTIVE))
		return -FI_ENOSYS;                  /* coll_coll.c:926-927 */
	if (!ca || !ca->set || !mc_fid || !ep->av)
		return -FI_EINVAL;
	set = olfa_container_of(ca->set, struct olfa_av_set, set_fid);
	n = set->count;
	if (!n)
		return -FI_EINVAL;
	my_addr = ep->av->peer_av->owner_ops->ep_addr(ep->av->peer_av, ep->peer_ep);

	m = calloc(1, sizeof(*m));
	if (!m)
		return -FI_ENOMEM;
	m->mc_fid.fid.fclass = FI_CLASS_MC;
	m->mc_fid.fid.context = context;
	m->mc_fid.fid.ops = &olfa_mc_fi_ops;
	m->mc_fid.fi_addr = (fi_addr_t)(uintptr_t)m;
	m->laddr = LFA_ADDR_NOTAVAIL;

	/* coll_addr = fi_av_set_addr of this very set: prov/coll then takes the
	 * set's own coll_mc as the parent (coll_av_set.c:166-175,
	 * coll_coll.c:939-941), so the set's members alone take part — fabtests
	 * core_coll.c joins every test group this way (:138-178) */
	self = ca->coll_addr == (fi_addr_t)(uintptr_t)&set->set_mc;
	if ((ca->coll_addr == FI_ADDR_NOTAVAIL || self) && !ep->le) {
		/* world bootstrap: every member of the set takes part */
		long rank = olfa_index(set->addr, n, my_addr);

		if (rank < 0) {
			ret = -FI_EINVAL;       /* a world needs this rank in it */
			goto err;
		}
		ret = olfa_bootstrap(ep, (int)rank, (int)n, set->addr);
		if (ret)
			goto err;
		m->members = malloc(n * sizeof(fi_addr_t));
		if (!m->members) {
			ret = -FI_ENOMEM;
			goto err;
		}
		memcpy(m->members, set->addr, n * sizeof(fi_addr_t));
		m->nmembers = n;
		free(set->set_mc.members);
		set->set_mc.members = malloc(n * sizeof(fi_addr_t));
		if (!set->set_mc.members) {
			ret = -FI_ENOMEM;
			goto err;
		}
		memcpy(set->set_mc.members, set->addr, n * sizeof(fi_addr_t));
		set->set_mc.nmembers = n;
		/* not under the registry lock: the join's communicator work must
		 * not hold up the progress thread's EQ hand-off */
		atomic_fetch_add(&ep->joins_in_flight, 1);    /* olfa_post_join */
		ret = lfa_join_collective(ep->le, LFA_ADDR_NOTAVAIL, NULL, 0, flags,
					  &m->lmc, context);
		olfa_test_join_delay();
		pthread_mutex_lock(&ep->lock);
		if (!ret) {
			m->laddr = lfa_mc_addr(m->lmc);
			olfa_mc_register(ep, m);
			ep->world = m;
			/* fi_av_set_addr of this set names the world group */
			set->set_mc.laddr = lfa_coll_world_addr(ep->le);
			olfa_mc_register(ep, &set->set_mc);
		}
		pthread_mutex_unlock(&ep->lock);
		atomic_fetch_sub(&ep->joins_in_flight, 1);
		if (ret)
			goto err;
		*mc_fid = &m->mc_fid;
		return 0;
	}

	if (self) {
		ret = olfa_join_self(ep, set, m, flags, context);
		if (ret)
			goto err;
		*mc_fid = &m->mc_fid;
		return 0;
	}
	pthread_mutex_lock(&ep->lock);
	parent = ca->coll_addr == FI_ADDR_NOTAVAIL ? ep->world :
		 olfa_mc_lookup(ep, ca->coll_addr);
	if (!parent || parent->laddr == LFA_ADDR_NOTAVAIL || !parent->members) {
		pthread_mutex_unlock(&ep->lock);
		ret = -FI_EINVAL;
		goto err;
	}
	paddr = parent->laddr;
	ranks = malloc(n * sizeof(int));
	m->members = malloc(n * sizeof(fi_addr_t));
	if (!ranks || !m->members) {
		pthread_mutex_unlock(&ep->lock);
		ret = -FI_ENOMEM;
		goto err;
	}
	for (size_t i = 0; i < n; i++) {
		long r = olfa_index(parent->members, parent->nmembers, set->addr[i]);

		if (r < 0) {                    /* not in the parent group */
			pthread_mutex_unlock(&ep->lock);
			ret = -FI_EINVAL;
			goto err;
		}
		ranks[i] = (int)r;
		m->members[i] = set->addr[i];   /* group rank i: the set's order */
	}
	m->nmembers = n;
	pthread_mutex_unlock(&ep->lock);
	atomic_fetch_add(&ep->joins_in_flight, 1);    /* olfa_post_join */
	ret = lfa_join_collective(ep->le, paddr, ranks, n, flags, &m->lmc, context);
	olfa_test_join_delay();
	pthread_mutex_lock(&ep->lock);
	if (!ret) {
		m->laddr = lfa_mc_addr(m->lmc);
		olfa_mc_register(ep, m);
	}
	pthread_mutex_unlock(&ep->lock);
	atomic_fetch_sub(&ep->joins_in_flight, 1);
	free(ranks);
	ranks = NULL;
	if (ret)
		goto err;
	*mc_fid = &m->mc_fid;
	return 0;
err:
	free(ranks);
	free(m->members);
	free(m);
	return ret;
}

/* --------------------------------------------------------- collectives -- */

#define OLFA_EP(fid) ((struct olfa_ep *)(fid))
#define OLFA_GROUP(ep, coll_addr, a)                                 \
	do {                                                          \
		if (!(ep)->le)                                        \
			return -FI_EINVAL;                            \
		(a) = olfa_resolve((ep), (coll_addr));                \
		if ((a) == LFA_ADDR_NOTAVAIL)                         \
			return -FI_EINVAL;                            \
	} while (0)

static ssize_t olfa_barrier2(struct fid_ep *ep_fid, fi_addr_t coll_addr,
			     uint64_t flags, void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_barrier(ep->le, a, context);
}

static ssize_t olfa_barrier(struct fid_ep *ep_fid, fi_addr_t coll_addr,
			    void *context)
{
	return olfa_barrier2(ep_fid, coll_addr, 0, context);
}

static ssize_t olfa_broadcast(struct fid_ep *ep_fid, void *buf, size_t count,
			      void *desc, fi_addr_t coll_addr, fi_addr_t root_addr,
			      enum fi_datatype datatype, uint64_t flags,
			      void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_broadcast(ep->le, buf, count, desc, a, root_addr,
			     (enum lfa_datatype)datatype, flags, context);
}

static ssize_t olfa_alltoall(struct fid_ep *ep_fid, const void *buf,
			     size_t count, void *desc, void *result,
			     void *result_desc, fi_addr_t coll_addr,
			     enum fi_datatype datatype, uint64_t flags,
			     void *context)
{
	return -FI_ENOSYS;          /* coll_ep_alltoall: not offered either */
}

static ssize_t olfa_allreduce(struct fid_ep *ep_fid, const void *buf,
			      size_t count, void *desc, void *result,
			      void *result_desc, fi_addr_t coll_addr,
			      enum fi_datatype datatype, enum fi_op op,
			      uint64_t flags, void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_allreduce(ep->le, buf, count, desc, result, result_desc, a,
			     (enum lfa_datatype)datatype, (enum lfa_op)op, flags,
			     context);
}

static ssize_t olfa_allgather(struct fid_ep *ep_fid, const void *buf,
			      size_t count, void *desc, void *result,
			      void *result_desc, fi_addr_t coll_addr,
			      enum fi_datatype datatype, uint64_t flags,
			      void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_allgather(ep->le, buf, count, desc, result, result_desc, a,
			     (enum lfa_datatype)datatype, flags, context);
}

static ssize_t olfa_reduce_scatter(struct fid_ep *ep_fid, const void *buf,
				   size_t count, void *desc, void *result,
				   void *result_desc, fi_addr_t coll_addr,
				   enum fi_datatype datatype, enum fi_op op,
				   uint64_t flags, void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_reduce_scatter(ep->le, buf, count, desc, result, result_desc,
				  a, (enum lfa_datatype)datatype,
				  (enum lfa_op)op, flags, context);
}

static ssize_t olfa_reduce(struct fid_ep *ep_fid, const void *buf, size_t count,
			   void *desc, void *result, void *result_desc,
			   fi_addr_t coll_addr, fi_addr_t root_addr,
			   enum fi_datatype datatype, enum fi_op op,
			   uint64_t flags, void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_reduce(ep->le, buf, count, desc, result, result_desc, a,
			  root_addr, (enum lfa_datatype)datatype,
			  (enum lfa_op)op, flags, context);
}

static ssize_t olfa_scatter(struct fid_ep *ep_fid, const void *buf, size_t count,
			    void *desc, void *result, void *result_desc,
			    fi_addr_t coll_addr, fi_addr_t root_addr,
			    enum fi_datatype datatype, uint64_t flags,
			    void *context)
{
	struct olfa_ep *ep = OLFA_EP(ep_fid);
	lfa_addr_t a;

	OLFA_GROUP(ep, coll_addr, a);
	return lfa_scatter(ep->le, buf, count, desc, result, result_desc, a,
			   root_addr, (enum lfa_datatype)datatype, flags, context);
}

static ssize_t olfa_gather(struct fid_ep *ep_fid, const void *buf, size_t count,
			   void *desc, void *result, void *result_desc,
			   fi_addr_t coll_addr, fi_addr_t root_addr,
			   enum fi_datatype datatype, uint64_t flags,
			   void *context)
{
	return -FI_ENOSYS;          /* coll_ep_gather: not offered either */
}

static ssize_t olfa_msg(struct fid_ep *ep_fid, const struct fi_msg_collective *msg,
			struct fi_ioc *resultv, void **result_desc,
			size_t result_count, uint64_t flags)
{
	return -FI_ENOSYS;
}

static struct fi_ops_collective olfa_coll_ops = {
	.size = sizeof(struct fi_ops_collective),
	.barrier = olfa_barrier,
	.broadcast = olfa_broadcast,
	.alltoall = olfa_alltoall,
	.allreduce = olfa_allreduce,
	.allgather = olfa_allgather,
	.reduce_scatter = olfa_reduce_scatter,
	.reduce = olfa_reduce,
	.scatter = olfa_scatter,
	.gather = olfa_gather,
	.msg = olfa_msg,
	.barrier2 = olfa_barrier2,
};

/* ------------------------------------------------------------ endpoint -- */

static int olfa_ep_close(struct fid *fid)
{
	struct olfa_ep *ep = olfa_container_of(fid, struct olfa_ep, util.ep_fid.fid);

	if (ep->thread_running) {
		atomic_store(&ep->stop, 1);
		pthread_join(ep->thread, NULL);
		ep->thread_running = 0;
	}
	if (ep->le) {
		lfa_coll_ep_flush(ep->le);
		olfa_progress(ep);          /* hand the last completions over */
	}
	/* multicast handles still open lose their endpoint */
	while (ep->mcs) {
		struct olfa_mc *m = ep->mcs;

		ep->mcs = m->next;
		m->next = NULL;
		m->ep = NULL;
		if (m->lmc) {
			lfa_mc_close(m->lmc);
			m->lmc = NULL;
		}
		m->laddr = LFA_ADDR_NOTAVAIL;
	}
	if (ep->cq && ep->cq->ep == ep)
		ep->cq->ep = NULL;
	if (ep->le)
		lfa_coll_ep_close(ep->le);
	if (ep->ld)
		lfa_coll_domain_close(ep->ld);
	free(ep->waddr);
	pthread_mutex_destroy(&ep->lock);
	pthread_mutex_destroy(&ep->plock);
	free(ep);
	return 0;
}

static int olfa_ep_bind(struct fid *fid, struct fid *bfid, uint64_t flags)
{
	struct olfa_ep *ep = olfa_container_of(fid, struct olfa_ep, util.ep_fid.fid);

	switch (bfid->fclass) {
	case FI_CLASS_AV:
		ep->av = olfa_container_of(bfid, struct olfa_av, av_fid.fid);
		return 0;
	case FI_CLASS_CQ:
		ep->cq = olfa_container_of(bfid, struct olfa_cq, cq_fid.fid);
		ep->cq->ep = ep;
		return 0;
	case FI_CLASS_EQ:
		ep->eq = olfa_container_of(bfid, struct olfa_eq, eq_fid.fid);
		return 0;
	default:
		return -FI_EINVAL;
	}
}

static int olfa_ep_control(struct fid *fid, int command, void *arg)
{
	struct olfa_ep *ep = olfa_container_of(fid, struct olfa_ep, util.ep_fid.fid);

	if (command != FI_ENABLE)
		return -FI_ENOSYS;
	if (!ep->av || !ep->cq)
		return -FI_ENOCQ;
	ep->enabled = 1;
	return 0;
}

static struct fi_ops olfa_ep_fi_ops = OLFA_FI_OPS(olfa_ep_close, olfa_ep_bind,
						  olfa_ep_control);

static ssize_t olfa_ep_cancel(fid_t fid, void *context)
{
	return -FI_ENOSYS;
}

static int olfa_ep_getopt(fid_t fid, int level, int optname, void *optval,
			  size_t *optlen)
{
	struct olfa_ep *ep = olfa_container_of(fid, struct olfa_ep, util.ep_fid.fid);

	if (level != FI_OPT_ENDPOINT || !optval || !optlen)
		return -FI_EINVAL;
	switch (optname) {
	case OFF_LFA_OPT_UNIQUE_ID:
		if (*optlen < LFA_UNIQUE_ID_BYTES)
			return -FI_ETOOSMALL;
		*optlen = LFA_UNIQUE_ID_BYTES;
		return lfa_coll_get_unique_id(optval, LFA_UNIQUE_ID_BYTES);
	case OFF_LFA_OPT_ALGO:
	case OFF_LFA_OPT_DEVICE:
	case OFF_LFA_OPT_TRANSPORT:
		if (*optlen < sizeof(int))
			return -FI_ETOOSMALL;
		*(int *)optval = optname == OFF_LFA_OPT_ALGO ? ep->algo :
				 optname == OFF_LFA_OPT_DEVICE ? ep->device : ep->peer_xport;
		*optlen = sizeof(int);
		return 0;
	case OFF_LFA_OPT_CHUNK:
		if (*optlen < sizeof(size_t))
			return -FI_ETOOSMALL;
		*(size_t *)optval = ep->chunk;
		*optlen = sizeof(size_t);
		return 0;
	default:
		return -FI_ENOPROTOOPT;
	}
}

static int olfa_ep_setopt(fid_t fid, int level, int optname, const void *optval,
			  size_t optlen)
{
	struct olfa_ep *ep = olfa_container_of(fid, struct olfa_ep, util.ep_fid.fid);

	if (level != FI_OPT_ENDPOINT || !optval)
		return -FI_EINVAL;
	switch (optname) {
	case OFF_LFA_OPT_UNIQUE_ID:
		if (optlen != LFA_UNIQUE_ID_BYTES)
			return -FI_EINVAL;
		if (ep->le)
			return -FI_EBUSY;       /* the world group already exists */
		memcpy(ep->uid, optval, LFA_UNIQUE_ID_BYTES);
		ep->have_uid = 1;
		return 0;
	case OFF_LFA_OPT_ALGO:
		if (optlen != sizeof(int))
			return -FI_EINVAL;
		if (ep->le) {
			int ret = lfa_coll_ep_set_algo(ep->le, *(const int *)optval);

			if (ret)
				return ret;
		} else if (*(const int *)optval < LFA_ALGO_TREE ||
			   *(const int *)optval > LFA_ALGO_AUTO) {
			return -FI_EINVAL;
		}
		ep->algo = *(const int *)optval;
		return 0;
	case OFF_LFA_OPT_CHUNK:
		if (optlen != sizeof(size_t))
			return -FI_EINVAL;
		if (ep->le) {
			int ret = lfa_coll_ep_set_chunk(ep->le, *(const size_t *)optval);

			if (ret)
				return ret;
		}
		ep->chunk = *(const size_t *)optval;
		return 0;
	case OFF_LFA_OPT_DEVICE:
		if (optlen != sizeof(int) || *(const int *)optval < 0)
			return -FI_EINVAL;
		if (ep->le)
			return -FI_EBUSY;
		ep->device = *(const int *)optval;
		ep->device_set = 1;
		return 0;
	case OFF_LFA_OPT_TRANSPORT:
		if (optlen != sizeof(int) || (unsigned)*(const int *)optval > 1)
			return -FI_EINVAL;
		if (ep->le)
			return -FI_EBUSY;
		ep->peer_xport = *(const int *)optval;
		return 0;
	default:
		return -FI_ENOPROTOOPT;
	}
}

static int olfa_ep_tx_ctx(struct fid_ep *sep, int index, struct fi_tx_attr *attr,
			  struct fid_ep **tx_ep, void *context)
{
	return -FI_ENOSYS;
}

static int olfa_ep_rx_ctx(struct fid_ep *sep, int index, struct fi_rx_attr *attr,
			  struct fid_ep **rx_ep, void *context)
{
	return -FI_ENOSYS;
}

static ssize_t olfa_ep_size_left(struct fid_ep *ep)
{
	return -FI_ENOSYS;
}

static int olfa_ep_export_xpu(struct fid_ep *ep, uint64_t flags,
			      struct fid_xpu_ep *xpu_ep)
{
	return -FI_ENOSYS;
}

static struct fi_ops_ep olfa_ep_ops = {
	.size = sizeof(struct fi_ops_ep),
	.cancel = olfa_ep_cancel,
	.getopt = olfa_ep_getopt,
	.setopt = olfa_ep_setopt,
	.tx_ctx = olfa_ep_tx_ctx,
	.rx_ctx = olfa_ep_rx_ctx,
	.rx_size_left = olfa_ep_size_left,
	.tx_size_left = olfa_ep_size_left,
	.export_xpu = olfa_ep_export_xpu,
};

/* coll_ep.c:36-41: the name is the owner endpoint's */
static int olfa_getname(fid_t fid, void *addr, size_t *addrlen)
{
	struct olfa_ep *ep = olfa_container_of(fid, struct olfa_ep, util.ep_fid.fid);

	return fi_getname(&ep->peer_ep->fid, addr, addrlen);
}

static int olfa_setname(fid_t fid, void *addr, size_t addrlen)
{
	return -FI_ENOSYS;
}
static int olfa_getpeer(struct fid_ep *ep, void *addr, size_t *addrlen)
{
	return -FI_ENOSYS;
}
static int olfa_connect(struct fid_ep *ep, const void *addr, const void *param,
			size_t paramlen)
{
	return -FI_ENOSYS;
}
static int olfa_listen(struct fid_pep *pep)
{
	return -FI_ENOSYS;
}
static int olfa_accept(struct fid_ep *ep, const void *param, size_t paramlen)
{
	return -FI_ENOSYS;
}
static int olfa_reject(struct fid_pep *pep, fid_t handle, const void *param,
		       size_t paramlen)
{
	return -FI_ENOSYS;
}
static int olfa_shutdown(struct fid_ep *ep, uint64_t flags)
{
	return -FI_ENOSYS;
}

static struct fi_ops_cm olfa_cm_ops = {
	.size = sizeof(struct fi_ops_cm),
	.setname = olfa_setname,
	.getname = olfa_getname,
	.getpeer = olfa_getpeer,
	.connect = olfa_connect,
	.listen = olfa_listen,
	.accept = olfa_accept,
	.reject = olfa_reject,
	.shutdown = olfa_shutdown,
	.join = olfa_join,
};

/* Completions of the transfers this provider asked the owner to make with
 * FI_PEER_TRANSFER (coll_peer_xfer_complete, coll_coll.c:1218-1265): the
 * context is the olfa_xfer the executor's test() polls.  Over RCCL no such
 * transfer is ever issued. */
static ssize_t olfa_peer_complete(struct fid_ep *ep, struct fi_cq_tagged_entry *buf,
				  fi_addr_t src_addr)
{
	struct olfa_ep *e = (struct olfa_ep *)ep;
	struct olfa_xfer *x;

	if (!buf || !buf->op_context || !e->peer_xport) {
		olfa_warn("unexpected peer-transfer completion", NULL, 0);
		return -FI_EINVAL;
	}
	x = buf->op_context;
	atomic_store(&x->done, 1);
	return 0;
}

static ssize_t olfa_peer_comperr(struct fid_ep *ep, struct fi_cq_err_entry *buf)
{
	struct olfa_ep *e = (struct olfa_ep *)ep;
	struct olfa_xfer *x;

	if (!buf || !buf->op_context || !e->peer_xport) {
		olfa_warn("unexpected peer-transfer error", NULL, buf ? buf->err : 0);
		return -FI_EINVAL;
	}
	x = buf->op_context;
	atomic_store(&x->done, -(buf->err ? buf->err : FI_EIO));
	return 0;
}

static struct fi_ops_transfer_peer olfa_peer_xfer_ops = {
	.size = sizeof(struct fi_ops_transfer_peer),
	.complete = olfa_peer_complete,
	.comperr = olfa_peer_comperr,
};

/* coll_endpoint (coll_ep.c:116-170) */
OLFA_INTERNAL int olfa_endpoint(struct fid_domain *domain, struct fi_info *info,
			 struct fid_ep **ep_fid, void *context)
{
	struct fi_peer_transfer_context *pc = context;
	struct olfa_ep *ep;
	const char *algo;

	if (!info || !(info->mode & FI_PEER_TRANSFER))
		return -FI_EINVAL;
	if (!pc || pc->size < sizeof(*pc) || !pc->ep)
		return -FI_EINVAL;
	ep = calloc(1, sizeof(*ep));
	if (!ep)
		return -FI_ENOMEM;
	ep->util.ep_fid.fid.fclass = FI_CLASS_EP;
	ep->util.ep_fid.fid.context = context;
	ep->util.ep_fid.fid.ops = &olfa_ep_fi_ops;
	ep->util.ep_fid.ops = &olfa_ep_ops;
	ep->util.ep_fid.cm = &olfa_cm_ops;
	ep->util.ep_fid.collective = &olfa_coll_ops;
	ep->util.type = FI_EP_RDM;
	ep->util.caps = OLFA_CAPS;
	ep->util.progress = olfa_util_progress;
	ep->domain = olfa_container_of(domain, struct olfa_domain, domain_fid);
	ep->peer_ep = pc->ep;
	pc->peer_ops = &olfa_peer_xfer_ops;
	pthread_mutex_init(&ep->lock, NULL);
	pthread_mutex_init(&ep->plock, NULL);
	ep->device = olfa_param_int("device", olfa_env_int("LOCAL_RANK", 0));
	ep->device_set = olfa_param("device") != NULL;
	algo = olfa_param("algo");
	ep->algo = algo && *algo ? atoi(algo) : -1;
	ep->manual_progress = olfa_param("progress") && !strcmp(olfa_param("progress"), "manual");
	ep->peer_xport = olfa_param("transport") && !strcmp(olfa_param("transport"), "peer");
	*ep_fid = &ep->util.ep_fid;
	return 0;
}
