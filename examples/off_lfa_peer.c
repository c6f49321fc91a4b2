/*
 * off_lfa_peer — N processes drive liboff_lfa-fi.so with the provider's
 * PEER transport: every transfer of a collective goes through the owner
 * endpoint's tagged messaging (fi_tsendmsg / fi_trecvmsg with
 * FI_PEER_TRANSFER), the way prov/coll's do through rxm
 * (prov/coll/src/coll_coll.c:770-814), and the owner reports each finished
 * transfer back through the peer_ops->complete the provider installed
 * (rxm_cq.c:846-872, 1532-1546).
 *
 *   off_lfa_peer <liboff_lfa-fi.so> <nranks> <outdir> [manual] [latency] [core]
 *                [device]
 *
 * The owner here is a minimal stand-in for rxm over a socket provider: one
 * AF_UNIX socket pair per rank pair (made before fork), non-blocking,
 * messages framed as {tag, length, payload}, matched per (source, tag) in
 * arrival order; sends complete once written, receives once matched.  Each
 * rank joins the world group over an av_set of every rank, runs allreduce /
 * reduce_scatter / reduce / allgather / broadcast / barrier and a subset
 * join, and writes every input and output under <outdir> (r<rank>_<case>_in /
 * _out .bin) for tests/test_off_lfa.py to check against the oracle; the
 * known answer of fabtests/multinode/src/core_coll.c:230-277 is checked
 * here.  CPU only: no HIP call is made.  Prints "OK peer" and exits 0 when
 * every rank passed.  With "latency" it instead times BASELINE configs[0]'s
 * shape — a 4 KiB float FI_SUM fi_allreduce — 100 warm-up then 1000 timed
 * operations, and rank 0 prints "LATENCY_US <median> <p10> <p90>".  With
 * "core" it runs the reference's own multinode suite, fabtests core_coll.c's
 * test table, unchanged in flow (core_suite below); rank 0 prints
 * "CORE <test> passed" per test.  With "device" (GPU box) the reducing
 * collectives take hipMalloc'd buffers and add the P2P algorithm: the
 * provider runs the gfx950 kernels and stages the owner's transfers.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <rdma/fabric.h>
#include <rdma/fi_cm.h>
#include <rdma/fi_collective.h>
#include <rdma/fi_domain.h>
#include <rdma/fi_endpoint.h>
#include <rdma/fi_eq.h>
#include <rdma/fi_errno.h>
#include <rdma/fi_tagged.h>
#include <rdma/providers/fi_peer.h>
#include <rdma/providers/fi_prov.h>

#include "off_lfa.h"
#include "fi_param_stub.h"

#define MAXR 16
static int failures, me, nranks;
#define CHECK(cond, ...)                                                        \
	do {                                                                    \
		if (!(cond)) {                                                  \
			fprintf(stderr, "rank %d FAIL %s:%d: ", me, __FILE__, __LINE__); \
			fprintf(stderr, __VA_ARGS__);                           \
			fprintf(stderr, "\n");                                  \
			failures++;                                             \
		}                                                               \
	} while (0)

/* ------------------------------------------ the owner's tagged transport -- */

struct msg {
	struct msg *next;
	uint64_t tag;
	size_t len, off;
	unsigned char *data;         /* owned copy (sends, unexpected receives) */
	void *user;                  /* posted receive buffer */
	void *context;               /* provider's fi_msg_tagged.context */
};

struct link {
	int fd;
	struct msg *sendq, **send_tail;
	struct msg *posted, *unexp;  /* receives: posted / arrived unmatched */
	unsigned char hdr[16];
	size_t hdr_got;
	struct msg *in;              /* message being read */
};

static struct owner {
	struct fid_ep ep;
	struct fi_ops ep_fi_ops;
	struct fi_ops_cm cm;
	struct fi_ops_tagged tagged;
	struct fid_domain domain;
	struct fid_peer_av peer_av;
	struct fi_ops_av_owner av_ops;
	struct fid_peer_cq peer_cq;
	struct fi_ops_cq_owner cq_ops;
	struct fid_eq eq;
	struct fi_ops_eq eq_ops;
	struct fid_ep *offload;              /* the off_lfa endpoint */
	struct fi_ops_transfer_peer *xfer;   /* its peer_ops */
	struct link link[MAXR];
	pthread_mutex_t lock;                /* the provider's progress thread
					      * posts while we progress */
	void *comp[256];
	int ncomp;
	struct fi_eq_entry eve[64];
	uint32_t ev[64];
	int nev;
	uint64_t bytes_sent, bytes_recv;
} own;

/* the harness's own out-of-band messages (pm_barrier) complete here, not
 * into the provider */
static int oob_done[2 * MAXR];

static void complete_xfer(void *context, uint64_t flags, size_t len, uint64_t tag)
{
	struct fi_cq_tagged_entry e;

	if ((int *)context >= oob_done && (int *)context < oob_done + 2 * MAXR) {
		*(int *)context = 1;
		return;
	}
	memset(&e, 0, sizeof(e));
	e.op_context = context;
	e.flags = flags | FI_TAGGED;
	e.len = len;
	e.tag = tag;
	CHECK(own.xfer->complete(own.offload, &e, FI_ADDR_NOTAVAIL) == 0, "peer complete");
}

static ssize_t owner_tsendmsg(struct fid_ep *ep, const struct fi_msg_tagged *m,
			      uint64_t flags)
{
	struct link *l;
	struct msg *x;
	size_t len = 0;

	if (!(flags & FI_PEER_TRANSFER) || m->addr >= (fi_addr_t)nranks ||
	    (int)m->addr == me)
		return -FI_EINVAL;
	for (size_t i = 0; i < m->iov_count; i++)
		len += m->msg_iov[i].iov_len;
	x = calloc(1, sizeof(*x));
	x->data = malloc(16 + len);
	memcpy(x->data, &m->tag, 8);
	memcpy(x->data + 8, &len, 8);
	for (size_t i = 0, o = 16; i < m->iov_count; o += m->msg_iov[i].iov_len, i++)
		memcpy(x->data + o, m->msg_iov[i].iov_base, m->msg_iov[i].iov_len);
	x->len = 16 + len;
	x->tag = m->tag;
	x->context = m->context;
	l = &own.link[m->addr];
	pthread_mutex_lock(&own.lock);
	*l->send_tail = x;
	l->send_tail = &x->next;
	pthread_mutex_unlock(&own.lock);
	return 0;
}

static ssize_t owner_trecvmsg(struct fid_ep *ep, const struct fi_msg_tagged *m,
			      uint64_t flags)
{
	struct link *l;
	struct msg **pp, *x;

	if (!(flags & FI_PEER_TRANSFER) || m->iov_count != 1 ||
	    m->addr >= (fi_addr_t)nranks || (int)m->addr == me)
		return -FI_EINVAL;
	l = &own.link[m->addr];
	pthread_mutex_lock(&own.lock);
	for (pp = &l->unexp; *pp && (*pp)->tag != m->tag; pp = &(*pp)->next)
		;
	if ((x = *pp)) {             /* arrived before it was posted */
		*pp = x->next;
		own.bytes_recv += x->len;       /* under the lock: deliver() counts too */
		pthread_mutex_unlock(&own.lock);
		CHECK(x->len == m->msg_iov[0].iov_len, "length %zu vs %zu", x->len,
		      m->msg_iov[0].iov_len);
		memcpy(m->msg_iov[0].iov_base, x->data, x->len);
		complete_xfer(m->context, FI_RECV, x->len, x->tag);
		free(x->data);
		free(x);
		return 0;
	}
	x = calloc(1, sizeof(*x));
	x->tag = m->tag;
	x->len = m->msg_iov[0].iov_len;
	x->user = m->msg_iov[0].iov_base;
	x->context = m->context;
	for (pp = &l->posted; *pp; pp = &(*pp)->next)
		;
	*pp = x;
	pthread_mutex_unlock(&own.lock);
	return 0;
}

/* A message arrived whole: the first posted receive with its tag takes it,
 * else it waits in the unexpected list (rxm's eager path). */
static void deliver(struct link *l, struct msg *in)
{
	struct msg **pp, *r;

	for (pp = &l->posted; *pp && (*pp)->tag != in->tag; pp = &(*pp)->next)
		;
	if (!(r = *pp)) {
		struct msg **t = &l->unexp;

		while (*t)
			t = &(*t)->next;
		*t = in;
		return;
	}
	*pp = r->next;
	CHECK(r->len == in->len, "length %zu vs %zu", r->len, in->len);
	memcpy(r->user, in->data, in->len);
	own.bytes_recv += in->len;
	complete_xfer(r->context, FI_RECV, in->len, in->tag);
	free(in->data);
	free(in);
	free(r);
}

/* The owner's progress (rxm's, driven by fi_cq_read): move bytes both ways. */
static void owner_progress(void)
{
	pthread_mutex_lock(&own.lock);
	for (int p = 0; p < nranks; p++) {
		struct link *l = &own.link[p];
		ssize_t n;

		if (p == me)
			continue;
		while (l->sendq) {
			struct msg *x = l->sendq;

			n = write(l->fd, x->data + x->off, x->len - x->off);
			if (n <= 0)
				break;
			x->off += (size_t)n;
			if (x->off < x->len)
				break;
			l->sendq = x->next;
			if (!l->sendq)
				l->send_tail = &l->sendq;
			own.bytes_sent += x->len - 16;
			complete_xfer(x->context, FI_SEND, x->len - 16, x->tag);
			free(x->data);
			free(x);
		}
		for (;;) {
			if (!l->in) {
				n = read(l->fd, l->hdr + l->hdr_got, 16 - l->hdr_got);
				if (n <= 0)
					break;
				l->hdr_got += (size_t)n;
				if (l->hdr_got < 16)
					continue;
				l->in = calloc(1, sizeof(*l->in));
				memcpy(&l->in->tag, l->hdr, 8);
				memcpy(&l->in->len, l->hdr + 8, 8);
				l->in->data = malloc(l->in->len ? l->in->len : 1);
				l->hdr_got = 0;
			}
			if (l->in->off < l->in->len) {
				n = read(l->fd, l->in->data + l->in->off, l->in->len - l->in->off);
				if (n <= 0)
					break;
				l->in->off += (size_t)n;
			}
			if (l->in->off == l->in->len) {
				struct msg *in = l->in;

				l->in = NULL;
				deliver(l, in);
			}
		}
	}
	pthread_mutex_unlock(&own.lock);
}

static int owner_av_query(struct fid_peer_av *av, struct fi_av_attr *attr)
{
	memset(attr, 0, sizeof(*attr));
	attr->count = nranks;
	return 0;
}

static fi_addr_t owner_ep_addr(struct fid_peer_av *av, struct fid_ep *ep)
{
	return ep == &own.ep ? (fi_addr_t)me : FI_ADDR_NOTAVAIL;
}

static ssize_t owner_cq_write(struct fid_peer_cq *cq, void *context, uint64_t flags,
			      size_t len, void *buf, uint64_t data, uint64_t tag,
			      fi_addr_t src)
{
	CHECK(flags & FI_COLLECTIVE, "cq flags");
	__atomic_store_n(&own.comp[__atomic_fetch_add(&own.ncomp, 1, __ATOMIC_ACQ_REL) & 255],
			 context, __ATOMIC_RELEASE);
	return 0;
}

static ssize_t owner_cq_writeerr(struct fid_peer_cq *cq, const struct fi_cq_err_entry *e)
{
	CHECK(0, "collective error %d", e->err);
	return 0;
}

static ssize_t owner_eq_write(struct fid_eq *eq, uint32_t event, const void *buf,
			      size_t len, uint64_t flags)
{
	int i = own.nev;

	if (i >= 64 || len != sizeof(struct fi_eq_entry))
		return -FI_EINVAL;
	own.ev[i] = event;
	memcpy(&own.eve[i], buf, len);
	__atomic_store_n(&own.nev, i + 1, __ATOMIC_RELEASE);
	return (ssize_t)len;
}

static int owner_getname(fid_t fid, void *addr, size_t *addrlen)
{
	if (*addrlen < sizeof(uint64_t)) {
		*addrlen = sizeof(uint64_t);
		return -FI_ETOOSMALL;
	}
	*(uint64_t *)addr = 0x4c4641ull + (uint64_t)me;
	*addrlen = sizeof(uint64_t);
	return 0;
}

static void owner_init(void)
{
	own.cm.size = sizeof(own.cm);
	own.cm.getname = owner_getname;
	own.tagged.size = sizeof(own.tagged);
	own.tagged.sendmsg = owner_tsendmsg;
	own.tagged.recvmsg = owner_trecvmsg;
	own.ep_fi_ops.size = sizeof(own.ep_fi_ops);
	own.ep.fid.fclass = FI_CLASS_EP;
	own.ep.fid.ops = &own.ep_fi_ops;
	own.ep.cm = &own.cm;
	own.ep.tagged = &own.tagged;
	own.domain.fid.fclass = FI_CLASS_DOMAIN;
	own.av_ops.size = sizeof(own.av_ops);
	own.av_ops.query = owner_av_query;
	own.av_ops.ep_addr = owner_ep_addr;
	own.peer_av.fid.fclass = FI_CLASS_PEER_AV;
	own.peer_av.owner_ops = &own.av_ops;
	own.cq_ops.size = sizeof(own.cq_ops);
	own.cq_ops.write = owner_cq_write;
	own.cq_ops.writeerr = owner_cq_writeerr;
	own.peer_cq.fid.fclass = FI_CLASS_PEER_CQ;
	own.peer_cq.owner_ops = &own.cq_ops;
	own.eq_ops.size = sizeof(own.eq_ops);
	own.eq_ops.write = owner_eq_write;
	own.eq.fid.fclass = FI_CLASS_EQ;
	own.eq.ops = &own.eq_ops;
	pthread_mutex_init(&own.lock, NULL);
	for (int p = 0; p < nranks; p++)
		own.link[p].send_tail = &own.link[p].sendq;
}

/* --------------------------------------------------------------- driving -- */

struct util_ep_prefix {          /* include/ofi_util.h:280-306 */
	struct fid_ep ep_fid;
	void *domain, *av, *av_entry[2], *eq, *rx_cq;
	uint64_t rx_op_flags;
	void *tx_cq;
	uint64_t tx_op_flags, inject_op_flags, tx_msg_flags, rx_msg_flags;
	void *cntrs[6];
	void (*cntr_inc_funcs[6])(void *);
	enum fi_ep_type type;
	uint64_t caps, flags;
	void (*progress)(void *);
};

static int manual, latency, core;

static void drive(void)
{
	owner_progress();
	if (manual)
		((struct util_ep_prefix *)own.offload)->progress(own.offload);
}

static int wait_comp(void *ctx)
{
	struct timespec t0, t;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (;;) {
		int n = __atomic_load_n(&own.ncomp, __ATOMIC_ACQUIRE);

		for (int i = 0; i < n && i < 256; i++)
			if (__atomic_load_n(&own.comp[i], __ATOMIC_ACQUIRE) == ctx) {
				own.comp[i] = NULL;
				return 0;
			}
		drive();
		clock_gettime(CLOCK_MONOTONIC, &t);
		if (t.tv_sec - t0.tv_sec > 60) {
			CHECK(0, "completion %p timed out", ctx);
			return -1;
		}
	}
}

static int wait_join(struct fid_mc *mc)
{
	struct timespec t0, t;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (;;) {
		int n = __atomic_load_n(&own.nev, __ATOMIC_ACQUIRE);

		for (int i = 0; i < n; i++)
			if (own.eve[i].fid == &mc->fid) {
				CHECK(own.ev[i] == FI_JOIN_COMPLETE, "event %u", own.ev[i]);
				own.eve[i].fid = NULL;
				return 0;
			}
		drive();
		clock_gettime(CLOCK_MONOTONIC, &t);
		if (t.tv_sec - t0.tv_sec > 60) {
			CHECK(0, "join timed out");
			return -1;
		}
	}
}

static const char *outdir;

/* fabtests' pm_barrier (multinode/src/harness.c:164-185) over the owner's
 * links: everyone tells rank 0, rank 0 releases everyone.  Its tags have bit
 * 63 set; the provider's (cid | rank << 32, cid < 2^25) never do. */
static void oob_barrier(void)
{
	static uint64_t seq;
	const uint64_t tag = 1ull << 63 | seq++;
	unsigned char byte = 0, sink[MAXR];
	struct iovec iov;
	struct fi_msg_tagged m;
	int want = 0;

	memset(oob_done, 0, sizeof(oob_done));
	memset(&m, 0, sizeof(m));
	m.msg_iov = &iov;
	m.iov_count = 1;
	m.tag = tag;
	for (int p = 0; p < nranks; p++) {
		if (p == me || (me != 0 && p != 0))
			continue;
		iov.iov_base = &sink[p];
		iov.iov_len = 1;
		m.addr = (fi_addr_t)p;
		m.context = &oob_done[p];
		CHECK(owner_trecvmsg(&own.ep, &m, FI_PEER_TRANSFER) == 0, "oob recv");
		want++;
	}
	if (me != 0) {                       /* arrive */
		iov.iov_base = &byte;
		iov.iov_len = 1;
		m.addr = 0;
		m.context = &oob_done[MAXR];
		CHECK(owner_tsendmsg(&own.ep, &m, FI_PEER_TRANSFER) == 0, "oob send");
		want++;
	}
	for (;;) {                           /* rank 0: all arrived; else released */
		int got = 0;

		for (int i = 0; i < 2 * MAXR; i++)
			got += __atomic_load_n(&oob_done[i], __ATOMIC_ACQUIRE);
		if (got == want)
			break;
		owner_progress();
	}
	if (me == 0) {                       /* release */
		memset(oob_done, 0, sizeof(oob_done));
		for (int p = 1; p < nranks; p++) {
			iov.iov_base = &byte;
			iov.iov_len = 1;
			m.addr = (fi_addr_t)p;
			m.context = &oob_done[MAXR + p];
			CHECK(owner_tsendmsg(&own.ep, &m, FI_PEER_TRANSFER) == 0, "oob release");
		}
		for (int got = 0; got < nranks - 1;) {
			owner_progress();
			got = 0;
			for (int p = 1; p < nranks; p++)
				got += __atomic_load_n(&oob_done[MAXR + p], __ATOMIC_ACQUIRE);
		}
	}
}

static void dump(const char *name, const char *io, const void *p, size_t n)
{
	char path[4096];
	FILE *f;

	snprintf(path, sizeof(path), "%s/r%d_%s_%s.bin", outdir, me, name, io);
	f = fopen(path, "wb");
	if (!f || fwrite(p, 1, n, f) != n)
		CHECK(0, "write %s", path);
	if (f)
		fclose(f);
}

static uint64_t lcg_state;

static uint64_t lcg(void)
{
	lcg_state = lcg_state * 6364136223846793005ull + 1442695040888963407ull;
	return lcg_state >> 11;
}

static double unif(double lo, double hi)
{
	return lo + (hi - lo) * (double)lcg() / (double)(1ull << 53);
}

static void seed(int c)
{
	lcg_state = 0x5EEDull + (uint64_t)me * 1000003ull + (uint64_t)c * 7919ull;
}

typedef struct fi_provider *(*ini_fn)(void);

/* ------------------------------------------- "device": GPU buffers ------- */

/* With "device" the reducing collectives hand the provider hipMalloc'd
 * buffers: it runs the kernels on them and stages every transfer through
 * host memory, so this owner still moves host bytes only.  HIP is loaded on
 * demand (CPU runs never touch it), after fork, in each rank. */
static int devmode;
static struct {
	int (*malloc)(void **, size_t);
	int (*memcpy)(void *, const void *, size_t, int);   /* 1 H2D, 2 D2H */
	int (*free)(void *);
} hip;

static int hip_load(void)
{
	void *h = dlopen("libamdhip64.so.7", RTLD_NOW | RTLD_GLOBAL);

	if (!h)
		h = dlopen("libamdhip64.so", RTLD_NOW | RTLD_GLOBAL);
	if (!h)
		return -1;
	hip.malloc = (int (*)(void **, size_t))dlsym(h, "hipMalloc");
	hip.memcpy = (int (*)(void *, const void *, size_t, int))dlsym(h, "hipMemcpy");
	hip.free = (int (*)(void *))dlsym(h, "hipFree");
	if (!hip.malloc || !hip.memcpy || !hip.free)
		return -1;
	{   /* a usable GPU, or fail now rather than in every collective */
		void *probe = NULL;

		if (hip.malloc(&probe, 1) != 0)
			return -1;
		hip.free(probe);
	}
	return 0;
}

/* the buffer the provider sees: `h` itself, or a device copy of it */
static void *xbuf(void *h, size_t n)
{
	void *d = NULL;

	if (!devmode)
		return h;
	CHECK(hip.malloc(&d, n ? n : 1) == 0, "hipMalloc");
	CHECK(hip.memcpy(d, h, n, 1) == 0, "hipMemcpy H2D");
	return d;
}

/* results back into `h` (device mode), and the device copy freed */
static void xdone(void *h, void *x, size_t n)
{
	if (!devmode)
		return;
	if (h && n)
		CHECK(hip.memcpy(h, x, n, 2) == 0, "hipMemcpy D2H");
	hip.free(x);
}

/* ------------------------------------------------ fabtests core_coll.c -- */

/*
 * The reference's own multinode collective suite, in its order and with its
 * setup / run / pm_barrier / teardown cycle (fabtests/multinode/src/
 * core_coll.c:453-521, 607-648): every test builds an av_set (count 0,
 * start, end = N-1, stride), joins with coll_addr = fi_av_set_addr of that
 * set — the set's own address — only on the ranks in it (:138-168), runs,
 * meets the others in pm_barrier, closes mc and set.  Expected values are
 * the ones core_coll.c checks.
 */
enum core_run { CORE_JOIN, CORE_BARRIER, CORE_SUM, CORE_ALLGATHER, CORE_SCATTER,
		CORE_BROADCAST };

static const struct core_test {
	const char *name;
	uint64_t start, stride;
	enum fi_collective_op coll;
	enum fi_op op;
	enum fi_datatype dt;
	enum core_run run;
} core_tests[] = {
	{ "join_test", 0, 1, FI_BARRIER, FI_NOOP, FI_VOID, CORE_JOIN },
	{ "barrier_test", 0, 1, FI_BARRIER, FI_NOOP, FI_VOID, CORE_BARRIER },
	{ "sum_all_reduce_test", 0, 1, FI_ALLREDUCE, FI_SUM, FI_UINT64, CORE_SUM },
	{ "sum_all_reduce_w_stride_test", 1, 2, FI_ALLREDUCE, FI_SUM, FI_UINT64, CORE_SUM },
	{ "all_gather_test", 0, 1, FI_ALLGATHER, FI_NOOP, FI_UINT64, CORE_ALLGATHER },
	{ "scatter_test", 0, 1, FI_SCATTER, FI_NOOP, FI_UINT64, CORE_SCATTER },
	{ "broadcast_test", 0, 1, FI_BROADCAST, FI_NOOP, FI_UINT64, CORE_BROADCAST },
};

static int core_member(const struct core_test *t)      /* core_coll.c:66-77 */
{
	return (uint64_t)me >= t->start && (uint64_t)me <= (uint64_t)nranks - 1 &&
	       ((uint64_t)me - t->start) % t->stride == 0;
}

static int core_run_one(struct fid_ep *ep, struct fid_mc *mc, const struct core_test *t)
{
	fi_addr_t ca = fi_mc_addr(mc);
	int ctx = 0, before = failures;

	switch (t->run) {
	case CORE_JOIN:
		return 0;
	case CORE_BARRIER:
		CHECK(fi_barrier(ep, ca, &ctx) == 0, "barrier");
		break;
	case CORE_SUM: {                                /* :230-277 */
		uint64_t data = 1234 + (uint64_t)me, result = 0, want = 0;

		for (uint64_t i = t->start; i <= (uint64_t)nranks - 1; i += t->stride)
			want += 1234 + i;
		CHECK(fi_allreduce(ep, &data, 1, NULL, &result, NULL, ca, FI_UINT64, FI_SUM,
				   0, &ctx) == 0, "allreduce");
		wait_comp(&ctx);
		CHECK(result == want, "%s: %lu vs %lu", t->name, (unsigned long)result,
		      (unsigned long)want);
		return failures != before;
	}
	case CORE_ALLGATHER: {                          /* :279-334 */
		uint64_t data = (uint64_t)me, result[MAXR];

		CHECK(fi_allgather(ep, &data, 1, NULL, result, NULL, ca, FI_UINT64, 0,
				   &ctx) == 0, "allgather");
		wait_comp(&ctx);
		for (int i = 0; i < nranks; i++)
			CHECK(result[i] == (uint64_t)i, "allgather [%d] = %lu", i,
			      (unsigned long)result[i]);
		return failures != before;
	}
	case CORE_SCATTER: {                            /* :336-387 */
		uint64_t data[MAXR], result = ~0ull;

		for (int i = 0; i < nranks; i++)
			data[i] = (uint64_t)i;
		CHECK(fi_scatter(ep, me == 0 ? data : NULL, 1, NULL, &result, NULL, ca, 0,
				 FI_UINT64, 0, &ctx) == 0, "scatter");
		wait_comp(&ctx);
		CHECK(result == data[me], "scatter %lu", (unsigned long)result);
		return failures != before;
	}
	case CORE_BROADCAST: {                          /* :389-451 */
		uint64_t data[MAXR], result[MAXR];

		for (int i = 0; i < nranks; i++)
			data[i] = (uint64_t)(nranks - 1 - i);
		CHECK(fi_broadcast(ep, me == 0 ? data : result, (size_t)nranks, NULL, ca, 0,
				   FI_UINT64, 0, &ctx) == 0, "broadcast");
		wait_comp(&ctx);
		for (int i = 0; me != 0 && i < nranks; i++)
			CHECK(result[i] == data[i], "broadcast [%d]", i);
		return failures != before;
	}
	}
	wait_comp(&ctx);
	return failures != before;
}

static int core_suite(struct fid_domain *domain, struct fid_av *av, struct fid_ep *ep)
{
	for (size_t k = 0; k < sizeof(core_tests) / sizeof(core_tests[0]); k++) {
		const struct core_test *t = &core_tests[k];
		struct fi_collective_attr attr = { 0 };
		struct fi_av_set_attr sattr = { 0 };
		struct fid_av_set *set = NULL;
		struct fid_mc *mc = NULL;
		fi_addr_t addr;
		int ret, jctx;

		attr.op = t->op;                       /* test_query, :200-210 */
		attr.datatype = t->dt;
		attr.mode = 0;
		ret = fi_query_collective(domain, t->coll, &attr, 0);
		CHECK(ret == 0, "%s: query %d", t->name, ret);
		if (ret)
			continue;
		if (core_member(t)) {                  /* setup, :138-168 */
			sattr.count = 0;
			sattr.start_addr = t->start;
			sattr.end_addr = (fi_addr_t)nranks - 1;
			sattr.stride = t->stride;
			CHECK(fi_av_set(av, &sattr, &set, NULL) == 0, "%s: av_set", t->name);
			CHECK(fi_av_set_addr(set, &addr) == 0, "%s: av_set_addr", t->name);
			ret = fi_join_collective(ep, addr, set, 0, &mc, &jctx);
			CHECK(ret == 0, "%s: join %d", t->name, ret);
			if (ret)
				return 1;
			wait_join(mc);
			if (core_run_one(ep, mc, t))
				return 1;
		}
		oob_barrier();                         /* :640 */
		if (mc) {                              /* teardown, :180-192 */
			CHECK(fi_close(&mc->fid) == 0, "%s: close mc", t->name);
			CHECK(fi_close(&set->fid) == 0, "%s: close set", t->name);
		}
		if (me == 0)
			printf("CORE %s passed\n", t->name), fflush(stdout);
	}
	return failures ? 1 : 0;
}

/*
 * Groups over sets whose address order is not ascending.
 * prov/coll numbers a group's members by their index in the joined av_set's
 * address array (coll_find_local_rank, coll_coll.c:669-689); insert appends
 * and remove moves the last address into the hole (coll_av_set.c:127-164),
 * so the order is the one these calls leave.  Two sets:
 *   A: stride {0, 2, 4, ...}, insert 1 (and 3), then remove 2 when N >= 4
 *      — e.g. N = 5: {0,2,4} +1 +3 = {0,2,4,1,3}, -2 = {0,3,4,1};
 *      joined over the world group (every rank calls; non-members refused);
 *   B: every rank, diff {0}: {N-1, 1, 2, ..., N-2}; joined over its own
 *      address (members only).
 * Each group runs an allgather of the parent ranks (the block order shows
 * the numbering), a float SUM allreduce (association order), a reduce to
 * group rank 1 and a broadcast from the last group rank, and dumps the set's
 * order and every input and output (tests/test_off_lfa.py checks them).
 */
static void ordered_group(struct fid_ep *ep, struct fid_mc *g, const char *tag,
			  const fi_addr_t *order, size_t n)
{
	fi_addr_t ga = fi_mc_addr(g);
	int pos = -1, req[4];
	char name[64];

	for (size_t i = 0; i < n; i++)
		if ((int)order[i] == me)
			pos = (int)i;
	if (pos < 0) {
		float x = 0;

		CHECK(fi_allreduce(ep, &x, 1, NULL, &x, NULL, ga, FI_FLOAT, FI_SUM, 0,
				   &req[0]) == -FI_EINVAL, "%s: non-member refused", tag);
		return;
	}
	{
		int32_t mine[3] = { me, 10 * me, pos }, all[3 * MAXR];

		CHECK(fi_allgather(ep, mine, 3, NULL, all, NULL, ga, FI_INT32, 0,
				   &req[0]) == 0, "%s allgather", tag);
		wait_comp(&req[0]);
		for (size_t k = 0; k < n; k++)
			CHECK(all[3 * k] == (int32_t)order[k] && all[3 * k + 2] == (int32_t)k,
			      "%s allgather block %zu holds rank %d", tag, k, all[3 * k]);
		snprintf(name, sizeof(name), "%s_allgather", tag);
		dump(name, "out", all, 3 * n * 4);
	}
	{
		float x[4099], y[4099];
		double d[333], e[333], b[9];

		seed(40 + me);
		for (int i = 0; i < 4099; i++)
			x[i] = (float)unif(-1, 1);
		CHECK(fi_allreduce(ep, x, 4099, NULL, y, NULL, ga, FI_FLOAT, FI_SUM, 0,
				   &req[1]) == 0, "%s allreduce", tag);
		wait_comp(&req[1]);
		snprintf(name, sizeof(name), "%s_sum_f32", tag);
		dump(name, "in", x, sizeof(x));
		dump(name, "out", y, sizeof(y));
		seed(60 + me);
		for (int i = 0; i < 333; i++)
			d[i] = unif(-1, 1);
		memset(e, 0, sizeof(e));
		CHECK(fi_reduce(ep, d, 333, NULL, e, NULL, ga, n > 1 ? 1 : 0, FI_DOUBLE,
				FI_SUM, 0, &req[2]) == 0, "%s reduce", tag);
		wait_comp(&req[2]);
		snprintf(name, sizeof(name), "%s_reduce_f64", tag);
		dump(name, "in", d, sizeof(d));
		if (pos == (n > 1 ? 1 : 0))
			dump(name, "out", e, sizeof(e));
		for (int i = 0; i < 9; i++)
			b[i] = pos == (int)n - 1 ? 1000.0 * me + i : -1.0;
		CHECK(fi_broadcast(ep, b, 9, NULL, ga, (fi_addr_t)n - 1, FI_DOUBLE, 0,
				   &req[3]) == 0, "%s broadcast", tag);
		wait_comp(&req[3]);
		for (int i = 0; i < 9; i++)
			CHECK(b[i] == 1000.0 * (double)order[n - 1] + i,
			      "%s broadcast from group rank %zu", tag, n - 1);
	}
}

static void ordered_sets(struct fid_av *av, struct fid_ep *ep, struct fid_mc *world_mc)
{
	struct fi_av_set_attr sattr = { 0 };
	struct fid_av_set *a, *b, *zero;
	struct fid_mc *ga, *gb;
	fi_addr_t order[MAXR], self_addr;
	size_t n = 0;
	int req[2];

	sattr.count = (size_t)nranks;
	sattr.start_addr = 0;
	sattr.end_addr = (fi_addr_t)nranks - 1;
	sattr.stride = 2;
	CHECK(fi_av_set(av, &sattr, &a, NULL) == 0, "set A");
	/* the expected order, by the reference's rules */
	for (int r = 0; r < nranks; r += 2)
		order[n++] = (fi_addr_t)r;
	if (nranks > 1) {
		CHECK(fi_av_set_insert(a, 1) == 0, "insert 1");
		order[n++] = 1;
	}
	if (nranks > 3) {
		CHECK(fi_av_set_insert(a, 3) == 0, "insert 3");
		order[n++] = 3;
		CHECK(fi_av_set_remove(a, 2) == 0, "remove 2");
		order[1] = order[--n];          /* 2 sat at index 1 */
	}
	dump("setA", "order", order, n * sizeof(fi_addr_t));
	CHECK(fi_join_collective(ep, fi_mc_addr(world_mc), a, 0, &ga, &req[0]) == 0,
	      "join A");
	wait_join(ga);
	ordered_group(ep, ga, "setA", order, n);

	/* B = every rank diff {0} */
	sattr.stride = 1;
	CHECK(fi_av_set(av, &sattr, &b, NULL) == 0, "set B");
	sattr.end_addr = 0;
	CHECK(fi_av_set(av, &sattr, &zero, NULL) == 0, "set {0}");
	CHECK(fi_av_set_diff(b, zero) == 0, "diff");
	n = 0;
	for (int r = 0; r < nranks; r++)
		order[n++] = (fi_addr_t)r;
	order[0] = order[--n];
	dump("setB", "order", order, n * sizeof(fi_addr_t));
	if (me != 0 && n) {
		/* coll_addr = the set's own address: its members alone join */
		CHECK(fi_av_set_addr(b, &self_addr) == 0, "set B addr");
		CHECK(fi_join_collective(ep, self_addr, b, 0, &gb, &req[1]) == 0, "join B");
		wait_join(gb);
		ordered_group(ep, gb, "setB", order, n);
		fi_close(&gb->fid);
	}
	fi_close(&ga->fid);
	fi_close(&zero->fid);
	fi_close(&b->fid);
	fi_close(&a->fid);

	/* C = the world in descending order (empty set + inserts) intersected
	 * with [0, 2, 1] (N >= 5), [0, 1] (N = 3, 4) or [0]: coll_av_set.c:71-96
	 * leaves the
	 * common addresses in SRC's order, so group rank k is src[k], not the
	 * k-th address of dst's order */
	{
		struct fid_av_set *c, *csrc;
		struct fid_mc *gc;
		fi_addr_t src[3] = { 0, 2, 1 };
		size_t ns = nranks >= 5 ? 3 : (nranks >= 3 ? 2 : 1);

		if (ns == 2)
			src[1] = 1;
		sattr.start_addr = FI_ADDR_NOTAVAIL;
		sattr.end_addr = FI_ADDR_NOTAVAIL;
		CHECK(fi_av_set(av, &sattr, &c, NULL) == 0, "set C");
		CHECK(fi_av_set(av, &sattr, &csrc, NULL) == 0, "set C src");
		for (int r = nranks - 1; r >= 0; r--)
			CHECK(fi_av_set_insert(c, (fi_addr_t)r) == 0, "C insert %d", r);
		for (size_t k = 0; k < ns; k++)
			CHECK(fi_av_set_insert(csrc, src[k]) == 0, "C src insert");
		CHECK(fi_av_set_intersect(c, csrc) == 0, "intersect");
		for (n = 0; n < ns; n++)
			order[n] = src[n];
		dump("setC", "order", order, n * sizeof(fi_addr_t));
		CHECK(fi_join_collective(ep, fi_mc_addr(world_mc), c, 0, &gc, &req[0]) == 0,
		      "join C");
		wait_join(gc);
		ordered_group(ep, gc, "setC", order, n);
		fi_close(&gc->fid);
		fi_close(&csrc->fid);
		fi_close(&c->fid);
	}
}

static int run_rank(const char *prov_path)
{
	void *dl;
	struct fi_provider *prov;
	struct fi_info *hints, *info = NULL;
	struct fid_fabric *fabric;
	struct fid_domain *domain;
	struct fid_av *av;
	struct fid_cq *cq;
	struct fid_eq *eq;
	struct fid_ep *ep;
	struct fid_av_set *set, *sub_set;
	struct fid_mc *mc, *sub;
	struct fi_peer_domain_context dctx = { sizeof(dctx), NULL };
	struct fi_peer_av_context actx = { sizeof(actx), NULL };
	struct fi_peer_cq_context cctx = { sizeof(cctx), NULL };
	struct fi_peer_eq_context ectx = { sizeof(ectx), NULL };
	struct fi_peer_transfer_context tctx;
	struct fi_av_attr av_attr = { 0 };
	struct fi_cq_attr cq_attr = { 0 };
	struct fi_eq_attr eq_attr = { 0 };
	struct fi_av_set_attr sattr = { 0 };
	fi_addr_t world, subaddr;
	int req[32], one = 1, ival;
	size_t len;

	owner_init();
	if (devmode && hip_load()) {
		fprintf(stderr, "rank %d: no HIP runtime for device mode\n", me);
		return 1;
	}
	dl = dlopen(prov_path, RTLD_NOW);
	if (!dl) {
		fprintf(stderr, "dlopen: %s\n", dlerror());
		return 1;
	}
	prov = ((ini_fn)dlsym(dl, "fi_prov_ini"))();
	hints = calloc(1, sizeof(*hints));
	hints->fabric_attr = calloc(1, sizeof(*hints->fabric_attr));
	hints->mode = FI_PEER_TRANSFER;
	hints->fabric_attr->prov_name = OFF_LFA_PROV_NAME;
	CHECK(prov->getinfo(FI_VERSION(2, 0), NULL, NULL, 0, hints, &info) == 0, "getinfo");
	free(hints->fabric_attr);
	free(hints);
	if (!info)
		return 1;
	CHECK(prov->fabric(info->fabric_attr, &fabric, NULL) == 0, "fabric");
	dctx.domain = &own.domain;
	CHECK(fi_domain2(fabric, info, &domain, FI_PEER, &dctx) == 0, "domain2");
	actx.av = &own.peer_av;
	av_attr.flags = FI_PEER;
	CHECK(fi_av_open(domain, &av_attr, &av, &actx) == 0, "av");
	cctx.cq = &own.peer_cq;
	cq_attr.flags = FI_PEER;
	CHECK(fi_cq_open(domain, &cq_attr, &cq, &cctx) == 0, "cq");
	ectx.eq = &own.eq;
	eq_attr.flags = FI_PEER;
	CHECK(fi_eq_open(fabric, &eq_attr, &eq, &ectx) == 0, "eq");
	memset(&tctx, 0, sizeof(tctx));
	tctx.size = sizeof(tctx);
	tctx.info = info;
	tctx.ep = &own.ep;
	CHECK(fi_endpoint(domain, info, &ep, &tctx) == 0, "endpoint");
	own.offload = ep;
	own.xfer = tctx.peer_ops;
	CHECK(fi_ep_bind(ep, &av->fid, 0) == 0, "bind av");
	CHECK(fi_ep_bind(ep, &cq->fid, FI_TRANSMIT | FI_RECV) == 0, "bind cq");
	CHECK(fi_ep_bind(ep, &eq->fid, 0) == 0, "bind eq");
	CHECK(fi_enable(ep) == 0, "enable");
	/* the peer transport: transfers through this owner's tagged ops */
	CHECK(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_TRANSPORT, &one,
			sizeof(one)) == 0, "transport option");
	ival = -1;
	len = sizeof(ival);
	CHECK(fi_getopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_TRANSPORT, &ival, &len) == 0 &&
	      ival == 1, "transport readback");
	if (core) {
		int bad = core_suite(domain, av, ep);

		fi_close(&ep->fid);
		fi_close(&eq->fid);
		fi_close(&cq->fid);
		fi_close(&av->fid);
		fi_close(&domain->fid);
		fi_close(&fabric->fid);
		return bad || failures ? 1 : 0;
	}

	/* world: an av_set of every rank (fabtests core_coll.c:453-521 order) */
	sattr.count = (size_t)nranks;
	sattr.start_addr = 0;
	sattr.end_addr = (fi_addr_t)nranks - 1;
	sattr.stride = 1;
	CHECK(fi_av_set(av, &sattr, &set, NULL) == 0, "av_set");
	CHECK(fi_join_collective(ep, FI_ADDR_NOTAVAIL, set, 0, &mc, &req[0]) == 0, "join");
	wait_join(mc);
	CHECK(fi_av_set_addr(set, &world) == 0, "av_set_addr");
	if (latency) {
		static double us[1000];
		float x[1024], y[1024];
		struct timespec a, b;

		seed(0);
		for (int i = 0; i < 1024; i++)
			x[i] = (float)unif(-1, 1);
		for (int it = 0; it < 1100; it++) {
			clock_gettime(CLOCK_MONOTONIC, &a);
			CHECK(fi_allreduce(ep, x, 1024, NULL, y, NULL, world, FI_FLOAT, FI_SUM, 0,
					   &req[1]) == 0, "allreduce");
			wait_comp(&req[1]);
			clock_gettime(CLOCK_MONOTONIC, &b);
			if (it >= 100)
				us[it - 100] = (b.tv_sec - a.tv_sec) * 1e6 +
					       (b.tv_nsec - a.tv_nsec) * 1e-3;
		}
		for (int i = 1; i < 1000; i++)          /* insertion sort */
			for (int j = i; j > 0 && us[j - 1] > us[j]; j--) {
				double t = us[j];

				us[j] = us[j - 1];
				us[j - 1] = t;
			}
		if (me == 0)
			printf("LATENCY_US %.2f %.2f %.2f\n", us[500], us[100], us[900]);
		fflush(stdout);
		CHECK(fi_barrier(ep, world, &req[2]) == 0, "barrier");
		wait_comp(&req[2]);
		fi_close(&mc->fid);
		fi_close(&set->fid);
		fi_close(&ep->fid);
		return failures ? 1 : 0;
	}
	CHECK(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_TRANSPORT, &one,
			sizeof(one)) == -FI_EBUSY, "transport fixed after the join");

	{   /* the reference's known answer: uint64 SUM of 1234 + rank */
		uint64_t x = 1234 + (uint64_t)me, y = 0, want = 0;

		for (int r = 0; r < nranks; r++)
			want += 1234 + (uint64_t)r;
		CHECK(fi_allreduce(ep, &x, 1, NULL, &y, NULL, world, FI_UINT64, FI_SUM, 0,
				   &req[1]) == 0, "allreduce ka");
		wait_comp(&req[1]);
		CHECK(y == want, "known answer %lu vs %lu", (unsigned long)y,
		      (unsigned long)want);
	}
	/* TREE, the reference's RD schedule, and (device buffers) P2P */
	for (int k = 0; k < (devmode ? 3 : 2); k++) {
		static const int algos[3] = { 0, 1, 4 };
		static const char *const sfxs[3] = { "", "_rd", "_p2p" };
		int algo = algos[k];
		const char *sfx = sfxs[k];
		char name[64];
		float *fx = malloc(1000 * 4), *fy = calloc(1000, 4);
		double *dx = malloc(4099 * 8), *dy = calloc(4099, 8);
		int64_t lx[33], ly[33] = { 0 };
		void *a[6];

		CHECK(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_ALGO, &algo,
				sizeof(algo)) == 0, "algo");
		seed(1);
		for (int i = 0; i < 1000; i++)
			fx[i] = (float)unif(-1, 1);
		seed(2);
		for (int i = 0; i < 4099; i++)
			dx[i] = unif(0.9, 1.1);
		seed(3);
		for (int i = 0; i < 33; i++)
			lx[i] = (int64_t)(lcg() << 11 ^ lcg());
		a[0] = xbuf(fx, 1000 * 4);
		a[1] = xbuf(fy, 1000 * 4);
		a[2] = xbuf(dx, 4099 * 8);
		a[3] = xbuf(dy, 4099 * 8);
		a[4] = xbuf(lx, sizeof(lx));
		a[5] = xbuf(ly, sizeof(ly));
		CHECK(fi_allreduce(ep, a[0], 1000, NULL, a[1], NULL, world, FI_FLOAT, FI_SUM, 0,
				   &req[2]) == 0, "allreduce f32");
		CHECK(fi_allreduce(ep, a[2], 4099, NULL, a[3], NULL, world, FI_DOUBLE, FI_PROD,
				   0, &req[3]) == 0, "allreduce f64");
		CHECK(fi_allreduce(ep, a[4], 33, NULL, a[5], NULL, world, FI_INT64, FI_BXOR, 0,
				   &req[4]) == 0, "allreduce bxor");
		/* three in flight at once; complete in any order here */
		wait_comp(&req[2]);
		wait_comp(&req[3]);
		wait_comp(&req[4]);
		xdone(NULL, a[0], 0);
		xdone(fy, a[1], 1000 * 4);
		xdone(NULL, a[2], 0);
		xdone(dy, a[3], 4099 * 8);
		xdone(NULL, a[4], 0);
		xdone(ly, a[5], sizeof(ly));
		snprintf(name, sizeof(name), "sum_f32%s", sfx);
		dump(name, "in", fx, 1000 * 4);
		dump(name, "out", fy, 1000 * 4);
		snprintf(name, sizeof(name), "prod_f64%s", sfx);
		dump(name, "in", dx, 4099 * 8);
		dump(name, "out", dy, 4099 * 8);
		snprintf(name, sizeof(name), "bxor_i64%s", sfx);
		dump(name, "in", lx, sizeof(lx));
		dump(name, "out", ly, sizeof(ly));
		free(fx);
		free(fy);
		free(dx);
		free(dy);
	}
	ival = 0;
	fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_ALGO, &ival, sizeof(ival));
	{   /* reduce_scatter: rank r gets block r (ragged at N = 3) */
		size_t count = 1000, base = count / (size_t)nranks, extra = count % (size_t)nranks;
		size_t mlen = base + ((size_t)me < extra);
		float *x = malloc(count * 4), *y = calloc(mlen ? mlen : 1, 4);
		void *ax, *ay;

		seed(4);
		for (size_t i = 0; i < count; i++)
			x[i] = (float)unif(-1, 1);
		ax = xbuf(x, count * 4);
		ay = xbuf(y, (mlen ? mlen : 1) * 4);
		CHECK(fi_reduce_scatter(ep, ax, count, NULL, ay, NULL, world, FI_FLOAT, FI_SUM,
					0, &req[5]) == 0, "reduce_scatter");
		wait_comp(&req[5]);
		xdone(NULL, ax, 0);
		xdone(y, ay, mlen * 4);
		dump("rs_f32", "in", x, count * 4);
		dump("rs_f32", "out", y, mlen * 4);
		free(x);
		free(y);
	}
	{   /* reduce to the last rank */
		double *x = malloc(777 * 8), *y = calloc(777, 8);

		void *ax, *ay;

		seed(5);
		for (int i = 0; i < 777; i++)
			x[i] = unif(-1, 1);
		ax = xbuf(x, 777 * 8);
		ay = xbuf(y, 777 * 8);
		CHECK(fi_reduce(ep, ax, 777, NULL, ay, NULL, world, (fi_addr_t)nranks - 1,
				FI_DOUBLE, FI_SUM, 0, &req[6]) == 0, "reduce");
		wait_comp(&req[6]);
		xdone(NULL, ax, 0);
		xdone(y, ay, 777 * 8);
		dump("reduce_f64", "in", x, 777 * 8);
		if (me == nranks - 1)
			dump("reduce_f64", "out", y, 777 * 8);
		free(x);
		free(y);
	}
	{   /* allgather, broadcast, barrier */
		int32_t g[10], all[10 * MAXR];
		int64_t b[5];

		for (int i = 0; i < 10; i++)
			g[i] = 100 * me + i;
		CHECK(fi_allgather(ep, g, 10, NULL, all, NULL, world, FI_INT32, 0,
				   &req[7]) == 0, "allgather");
		wait_comp(&req[7]);
		for (int r = 0; r < nranks; r++)
			for (int i = 0; i < 10; i++)
				CHECK(all[r * 10 + i] == 100 * r + i, "allgather [%d][%d]", r, i);
		for (int i = 0; i < 5; i++)
			b[i] = me == 0 ? 77 + i : -1;
		CHECK(fi_broadcast(ep, b, 5, NULL, world, 0, FI_INT64, 0, &req[8]) == 0,
		      "broadcast");
		wait_comp(&req[8]);
		for (int i = 0; i < 5; i++)
			CHECK(b[i] == 77 + i, "broadcast [%d]", i);
		CHECK(fi_barrier(ep, world, &req[9]) == 0, "barrier");
		wait_comp(&req[9]);
	}
	/* subset join: the first and the last rank (coll_coll.c:912-995) */
	sattr.count = 2;
	sattr.start_addr = 0;
	sattr.end_addr = (fi_addr_t)nranks - 1;
	sattr.stride = nranks > 1 ? (uint64_t)nranks - 1 : 1;
	CHECK(fi_av_set(av, &sattr, &sub_set, NULL) == 0, "subset av_set");
	CHECK(fi_join_collective(ep, fi_mc_addr(mc), sub_set, 0, &sub, &req[10]) == 0,
	      "subset join");
	wait_join(sub);
	subaddr = fi_mc_addr(sub);
	if (me == 0 || me == nranks - 1) {
		float x[100], y[100];

		seed(6);
		for (int i = 0; i < 100; i++)
			x[i] = (float)unif(-1, 1);
		CHECK(fi_allreduce(ep, x, 100, NULL, y, NULL, subaddr, FI_FLOAT, FI_SUM, 0,
				   &req[11]) == 0, "subset allreduce");
		wait_comp(&req[11]);
		dump("sub_f32", "in", x, sizeof(x));
		dump("sub_f32", "out", y, sizeof(y));
	} else {
		float x = 0;

		CHECK(fi_allreduce(ep, &x, 1, NULL, &x, NULL, subaddr, FI_FLOAT, FI_SUM, 0,
				   &req[11]) == -FI_EINVAL, "non-member refused");
	}
	ordered_sets(av, ep, mc);
	/* let the last transfers drain before anyone closes its sockets */
	CHECK(fi_barrier(ep, world, &req[12]) == 0, "final barrier");
	wait_comp(&req[12]);
	CHECK(own.bytes_sent > 0 || nranks == 1, "the owner carried the transfers");
	fi_close(&sub->fid);
	fi_close(&sub_set->fid);
	fi_close(&mc->fid);
	fi_close(&set->fid);
	fi_close(&ep->fid);
	fi_close(&eq->fid);
	fi_close(&cq->fid);
	fi_close(&av->fid);
	fi_close(&domain->fid);
	fi_close(&fabric->fid);
	return failures ? 1 : 0;
}

int main(int argc, char **argv)
{
	int sp[MAXR][MAXR][2], status, bad = 0;
	pid_t pid[MAXR];

	if (argc < 4) {
		fprintf(stderr, "usage: %s <liboff_lfa-fi.so> <nranks> <outdir> [manual] [latency] [core] [device]\n",
			argv[0]);
		return 2;
	}
	nranks = atoi(argv[2]);
	outdir = argv[3];
	for (int i = 4; i < argc; i++) {
		manual |= !strcmp(argv[i], "manual");
		latency |= !strcmp(argv[i], "latency");
		core |= !strcmp(argv[i], "core");
		devmode |= !strcmp(argv[i], "device");
	}
	if (manual)
		setenv("OFF_LFA_PROGRESS", "manual", 1);
	if (nranks < 1 || nranks > MAXR)
		return 2;
	for (int i = 0; i < nranks; i++)
		for (int j = i + 1; j < nranks; j++)
			if (socketpair(AF_UNIX, SOCK_STREAM, 0, sp[i][j]))
				return 1;
	for (int r = 0; r < nranks; r++) {
		pid[r] = fork();
		if (pid[r] < 0)
			return 1;
		if (pid[r] == 0) {
			me = r;
			for (int i = 0; i < nranks; i++)
				for (int j = i + 1; j < nranks; j++) {
					if (i == r)
						own.link[j].fd = sp[i][j][0];
					else
						close(sp[i][j][0]);
					if (j == r)
						own.link[i].fd = sp[i][j][1];
					else
						close(sp[i][j][1]);
				}
			for (int p = 0; p < nranks; p++)
				if (p != r)
					fcntl(own.link[p].fd, F_SETFL,
					      fcntl(own.link[p].fd, F_GETFL) | O_NONBLOCK);
			_exit(run_rank(argv[1]));
		}
	}
	for (int i = 0; i < nranks; i++)
		for (int j = i + 1; j < nranks; j++) {
			close(sp[i][j][0]);
			close(sp[i][j][1]);
		}
	for (int r = 0; r < nranks; r++) {
		if (waitpid(pid[r], &status, 0) < 0 || !WIFEXITED(status) ||
		    WEXITSTATUS(status)) {
			fprintf(stderr, "rank %d failed (status %#x)\n", r, status);
			bad = 1;
		}
	}
	if (bad)
		return 1;
	printf("OK peer%s\n", manual ? " manual" : "");
	return 0;
}
