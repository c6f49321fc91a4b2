/*
 * off_lfa_host — drives liboff_lfa-fi.so the way rxm drives an offload
 * collective provider, with a minimal owner (peer AV / CQ / EQ / endpoint)
 * standing in for rxm.  Uses libfabric's public headers only; no
 * libfabric.so is needed because every fi_* call used here is a static
 * inline dispatch through the provider's ops tables.
 *
 *   off_lfa_host <provider.so> cpu            discovery, objects, options,
 *                                             query mask, av_set algebra —
 *                                             no GPU calls
 *   off_lfa_host <provider.so> gpu [manual]   + world join, every collective
 *                                             on device and host buffers,
 *                                             completions through the owner,
 *                                             subset join (world size 1)
 *   off_lfa_host <provider.so> avset          av_set union / intersect /
 *                                             diff on sets read from stdin,
 *                                             result order printed (CPU)
 *   off_lfa_host <provider.so> params [LFA_X...]  the parameters the
 *                                             provider defined (fi_info -e
 *                                             style), then the values liblfa
 *                                             sees for the named knobs (CPU)
 *
 * Sequence mirrored from rxm: rxm_fabric.c:85-121 (getinfo with
 * FI_PEER_TRANSFER, fi_fabric), rxm_domain.c:944-953 (fi_domain2 FI_PEER),
 * rxm_domain.c:878-893 (capability mask), rxm_domain.c:274-287 (peer AV),
 * rxm_cq.c:2160-2199 (peer CQ), rxm_ep.c:1709-1720 (peer transfer
 * context), rxm_ep.c:1453-1492 (binds), rxm_cq.c:1928-1951 (owner write),
 * rxm_cq.c:2082-2099 (progress through the util_ep slot).
 * Prints "OK <mode>" and exits 0 when every check passed.
 */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <rdma/fabric.h>
#include <rdma/fi_cm.h>
#include <rdma/fi_collective.h>
#include <rdma/fi_domain.h>
#include <rdma/fi_endpoint.h>
#include <rdma/fi_eq.h>
#include <rdma/fi_errno.h>
#include <rdma/providers/fi_peer.h>
#include <rdma/providers/fi_prov.h>

#include <hip/hip_runtime_api.h>

#include "off_lfa.h"
#include "fi_param_stub.h"

static int failures;
#define CHECK(cond, ...)                                                  \
	do {                                                              \
		if (!(cond)) {                                            \
			fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
			fprintf(stderr, __VA_ARGS__);                     \
			fprintf(stderr, "\n");                            \
			failures++;                                       \
		}                                                         \
	} while (0)
#define CHECK_RC(expr, want)                                              \
	do {                                                              \
		long _rc = (long)(expr);                                  \
		CHECK(_rc == (long)(want), "%s = %ld, want %ld", #expr,   \
		      _rc, (long)(want));                                 \
	} while (0)

/* ------------------------------------------------------ the owner side -- */

#define MAX_COMP 64
struct comp {
	void *context;
	uint64_t flags;
	int err;
};

static struct owner {
	struct fid_ep ep;
	struct fi_ops ep_fi_ops;
	struct fi_ops_cm cm;
	struct fid_domain domain;
	struct fid_peer_av peer_av;
	struct fi_ops_av_owner av_ops;
	struct fid_peer_cq peer_cq;
	struct fi_ops_cq_owner cq_ops;
	struct fid_eq eq;
	struct fi_ops_eq eq_ops;
	int nranks;
	fi_addr_t my_addr;
	struct comp comp[MAX_COMP];
	volatile int ncomp;
	uint32_t ev[8];
	struct fi_eq_entry eve[8];
	volatile int nev;
} own;

static int owner_av_query(struct fid_peer_av *av, struct fi_av_attr *attr)
{
	memset(attr, 0, sizeof(*attr));
	attr->count = own.nranks;
	return 0;
}

static fi_addr_t owner_ep_addr(struct fid_peer_av *av, struct fid_ep *ep)
{
	return ep == &own.ep ? own.my_addr : FI_ADDR_NOTAVAIL;
}

static ssize_t owner_cq_write(struct fid_peer_cq *cq, void *context,
			      uint64_t flags, size_t len, void *buf,
			      uint64_t data, uint64_t tag, fi_addr_t src)
{
	int i = own.ncomp;

	if (i >= MAX_COMP)
		return -FI_EAGAIN;
	own.comp[i].context = context;
	own.comp[i].flags = flags;
	own.comp[i].err = 0;
	__atomic_store_n(&own.ncomp, i + 1, __ATOMIC_RELEASE);
	return 0;
}

static ssize_t owner_cq_writeerr(struct fid_peer_cq *cq,
				 const struct fi_cq_err_entry *e)
{
	int i = own.ncomp;

	if (i >= MAX_COMP)
		return -FI_EAGAIN;
	own.comp[i].context = e->op_context;
	own.comp[i].flags = e->flags;
	own.comp[i].err = e->err;
	__atomic_store_n(&own.ncomp, i + 1, __ATOMIC_RELEASE);
	return 0;
}

static ssize_t owner_eq_write(struct fid_eq *eq, uint32_t event,
			      const void *buf, size_t len, uint64_t flags)
{
	int i = own.nev;

	if (i >= 8 || len != sizeof(struct fi_eq_entry))
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
	*(uint64_t *)addr = 0x4c4641ull + own.my_addr;
	*addrlen = sizeof(uint64_t);
	return 0;
}

static void owner_init(int nranks, fi_addr_t me)
{
	memset(&own, 0, sizeof(own));
	own.nranks = nranks;
	own.my_addr = me;
	own.cm.size = sizeof(own.cm);
	own.cm.getname = owner_getname;
	own.ep_fi_ops.size = sizeof(own.ep_fi_ops);
	own.ep.fid.fclass = FI_CLASS_EP;
	own.ep.fid.ops = &own.ep_fi_ops;
	own.ep.cm = &own.cm;
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
}

/* The util_ep progress slot rxm calls (rxm_cq.c:2095-2098): same prefix
 * layout as include/ofi_util.h:280-306. */
struct util_ep_prefix {
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

static int manual;

static void drive(struct fid_ep *ep)
{
	if (manual)
		((struct util_ep_prefix *)ep)->progress(ep);
}

/* waits for the completion carrying `ctx` (the owner's req pointer) */
static int wait_comp(struct fid_ep *ep, void *ctx, int *err)
{
	struct timespec t0, t;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (;;) {
		int n = __atomic_load_n(&own.ncomp, __ATOMIC_ACQUIRE);

		for (int i = 0; i < n; i++)
			if (own.comp[i].context == ctx) {
				CHECK(own.comp[i].flags & FI_COLLECTIVE,
				      "completion flags %#lx", (unsigned long)own.comp[i].flags);
				if (err)
					*err = own.comp[i].err;
				own.comp[i].context = NULL;
				return 0;
			}
		drive(ep);
		clock_gettime(CLOCK_MONOTONIC, &t);
		if (t.tv_sec - t0.tv_sec > 60)
			return -1;
	}
}

static int wait_join(struct fid_ep *ep, struct fid_mc *mc, void *ctx)
{
	struct timespec t0, t;

	clock_gettime(CLOCK_MONOTONIC, &t0);
	for (;;) {
		int n = __atomic_load_n(&own.nev, __ATOMIC_ACQUIRE);

		for (int i = 0; i < n; i++)
			if (own.eve[i].fid == &mc->fid) {
				CHECK(own.ev[i] == FI_JOIN_COMPLETE, "event %u", own.ev[i]);
				CHECK(own.eve[i].context == ctx, "join context");
				own.eve[i].fid = NULL;
				return 0;
			}
		drive(ep);
		clock_gettime(CLOCK_MONOTONIC, &t);
		if (t.tv_sec - t0.tv_sec > 60)
			return -1;
	}
}

/* ---------------------------------------------------------------- main -- */

typedef struct fi_provider *(*ini_fn)(void);
typedef void (*freeinfo_fn)(struct fi_info *);

/* An av_set holding exactly `a[0..n)` in that order: an empty set (start =
 * end = FI_ADDR_NOTAVAIL, coll_av_set.c:255-262), then inserts. */
static struct fid_av_set *ordered_set(struct fid_av *av, const fi_addr_t *a, int n)
{
	struct fi_av_set_attr sattr = { 0 };
	struct fid_av_set *s = NULL;

	sattr.count = 64;
	sattr.start_addr = FI_ADDR_NOTAVAIL;
	sattr.end_addr = FI_ADDR_NOTAVAIL;
	CHECK_RC(fi_av_set(av, &sattr, &s, NULL), 0);
	for (int i = 0; s && i < n; i++)
		CHECK_RC(fi_av_set_insert(s, a[i]), 0);
	return s;
}

/*
 * avset mode: a batch of set operations read from stdin, one per line,
 *   <op> <nd> d0 .. d(nd-1) <ns> s0 .. s(ns-1)      op: u | i | d
 * builds dst and src in those orders, applies union / intersect / diff
 * (dst op= src) and prints "<rc> <count> <addresses in dst's order>".  The
 * fi_av_set API has no call that lists a set, so the order is read through
 * the provider's exported test accessor off_lfa_test_set_order (the order a
 * join would number the members by).
 */
typedef long (*set_order_fn)(struct fid_av_set *, fi_addr_t *, size_t);

static int avset_batch(void *dl, struct fid_av *av)
{
	set_order_fn order = (set_order_fn)dlsym(dl, "off_lfa_test_set_order");
	char op;
	int nd, ns, lines = 0;

	if (!order) {
		fprintf(stderr, "off_lfa_test_set_order missing\n");
		return 1;
	}
	while (scanf(" %c %d", &op, &nd) == 2) {
		fi_addr_t d[64], s[64], out[64];
		struct fid_av_set *ds, *ss;
		long n;
		int rc = -1;

		if (nd < 0 || nd > 64)
			return 1;
		for (int i = 0; i < nd; i++)
			if (scanf("%lu", (unsigned long *)&d[i]) != 1)
				return 1;
		if (scanf("%d", &ns) != 1 || ns < 0 || ns > 64)
			return 1;
		for (int i = 0; i < ns; i++)
			if (scanf("%lu", (unsigned long *)&s[i]) != 1)
				return 1;
		ds = ordered_set(av, d, nd);
		ss = ordered_set(av, s, ns);
		if (!ds || !ss)
			return 1;
		if (op == 'u')
			rc = fi_av_set_union(ds, ss);
		else if (op == 'i')
			rc = fi_av_set_intersect(ds, ss);
		else if (op == 'd')
			rc = fi_av_set_diff(ds, ss);
		n = order(ds, out, 64);
		printf("%d %ld", rc, n);
		for (long i = 0; i < n; i++)
			printf(" %lu", (unsigned long)out[i]);
		printf("\n");
		fi_close(&ss->fid);
		fi_close(&ds->fid);
		lines++;
	}
	fflush(stdout);
	return failures ? 1 : 0;
}

int main(int argc, char **argv)
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
	struct fid_av_set *set, *set2;
	struct fi_peer_domain_context dctx = { sizeof(dctx), NULL };
	struct fi_peer_av_context actx = { sizeof(actx), NULL };
	struct fi_peer_cq_context cctx = { sizeof(cctx), NULL };
	struct fi_peer_eq_context ectx = { sizeof(ectx), NULL };
	struct fi_peer_transfer_context tctx;
	struct fi_av_attr av_attr = { 0 };
	struct fi_cq_attr cq_attr = { 0 };
	struct fi_eq_attr eq_attr = { 0 };
	struct fi_av_set_attr sattr = { 0 };
	struct fi_collective_attr ca;
	freeinfo_fn freeinfo;
	uint64_t mask = 0;
	int gpu, ival;
	size_t len;

	if (argc < 3) {
		fprintf(stderr, "usage: %s <liboff_lfa-fi.so> cpu|gpu|avset [manual]\n", argv[0]);
		return 2;
	}
	gpu = !strcmp(argv[2], "gpu");
	manual = argc > 3 && !strcmp(argv[3], "manual");
	if (manual)
		setenv("OFF_LFA_PROGRESS", "manual", 1);

	/* discovery, as the core does for a DSO provider (src/fabric.c:683-689) */
	dl = dlopen(argv[1], RTLD_NOW);
	if (!dl) {
		fprintf(stderr, "dlopen: %s\n", dlerror());
		return 1;
	}
	prov = ((ini_fn)dlsym(dl, "fi_prov_ini"))();
	freeinfo = (freeinfo_fn)dlsym(dl, "off_lfa_freeinfo");
	CHECK(prov && !strncmp(prov->name, "off_", 4), "offload prefix");
	CHECK(!strcmp(prov->name, OFF_LFA_PROV_NAME), "name %s", prov->name);
	CHECK(FI_MAJOR(prov->fi_version) == FI_MAJOR_VERSION, "fi_version");
	if (!strcmp(argv[2], "params")) {
		typedef const char *(*param_fn)(const char *);
		param_fn lp = (param_fn)dlsym(dl, "lfa_param");

		stub_print_params(stdout);
		for (int i = 3; i < argc && lp; i++)
			printf("LFA %s=%s\n", argv[i], lp(argv[i]) ? lp(argv[i]) : "(unset)");
		fflush(stdout);
		return failures || !lp ? 1 : 0;
	}

	/* getinfo: FI_PEER_TRANSFER required (coll_init.c:39-43) */
	hints = calloc(1, sizeof(*hints));
	hints->fabric_attr = calloc(1, sizeof(*hints->fabric_attr));
	CHECK_RC(prov->getinfo(FI_VERSION(2, 0), NULL, NULL, 0, hints, &info),
		 -FI_ENODATA);
	hints->mode = FI_PEER_TRANSFER;
	hints->fabric_attr->prov_name = "off_coll";
	CHECK_RC(prov->getinfo(FI_VERSION(2, 0), NULL, NULL, 0, hints, &info),
		 -FI_ENODATA);
	hints->fabric_attr->prov_name = OFF_LFA_PROV_NAME;
	CHECK_RC(prov->getinfo(FI_VERSION(2, 0), NULL, NULL, 0, hints, &info), 0);
	free(hints->fabric_attr);
	free(hints);
	if (!info)
		return 1;
	CHECK(info->mode & FI_PEER_TRANSFER, "mode");
	CHECK(info->caps & FI_COLLECTIVE, "caps");
	CHECK(info->domain_attr->progress == FI_PROGRESS_AUTO, "progress");
	CHECK(info->domain_attr->threading == FI_THREAD_SAFE, "threading");
	CHECK(!strcmp(info->fabric_attr->prov_name, OFF_LFA_PROV_NAME), "prov_name");

	CHECK_RC(prov->fabric(info->fabric_attr, &fabric, NULL), 0);

	/* domain: FI_PEER only (coll_domain.c:88-92) */
	owner_init(1, 0);
	dctx.domain = &own.domain;
	CHECK_RC(fi_domain(fabric, info, &domain, &dctx), -FI_EINVAL);
	CHECK_RC(fi_domain2(fabric, info, &domain, FI_PEER, &dctx), 0);

	/* rxm_get_coll_caps (rxm_domain.c:878-893), verbatim probe */
	ca.datatype = FI_INT8;
	ca.datatype_attr.count = 1;
	ca.datatype_attr.size = sizeof(int8_t);
	ca.mode = 0;
	for (int i = FI_BARRIER; i <= FI_GATHER; i++) {
		ca.op = (i == FI_BARRIER) ? FI_NOOP : FI_MIN;
		if (fi_query_collective(domain, i, &ca, 0) == FI_SUCCESS)
			mask |= 1ull << i;
	}
	CHECK(mask == ((1ull << FI_BARRIER) | (1ull << FI_BROADCAST) |
		       (1ull << FI_ALLREDUCE) | (1ull << FI_ALLGATHER) |
		       (1ull << FI_REDUCE_SCATTER) | (1ull << FI_REDUCE) |
		       (1ull << FI_SCATTER)), "coll mask %#lx", (unsigned long)mask);
	memset(&ca, 0, sizeof(ca));
	ca.op = FI_SUM;
	ca.datatype = FI_FLOAT;
	CHECK_RC(fi_query_collective(domain, FI_ALLREDUCE, &ca, 0), 0);
	CHECK(ca.datatype_attr.size == 4 && ca.max_members == 0x7fffffff,
	      "query attr size %zu members %zu", ca.datatype_attr.size, ca.max_members);
	ca.op = FI_BOR;
	CHECK_RC(fi_query_collective(domain, FI_ALLREDUCE, &ca, 0), -FI_EOPNOTSUPP);
	ca.op = FI_CSWAP;
	CHECK_RC(fi_query_collective(domain, FI_ALLREDUCE, &ca, 0), -FI_ENOSYS);

	/* peer AV / CQ / EQ */
	actx.av = &own.peer_av;
	CHECK_RC(fi_av_open(domain, &av_attr, &av, &actx), -FI_EINVAL);
	av_attr.flags = FI_PEER;
	CHECK_RC(fi_av_open(domain, &av_attr, &av, &actx), 0);
	cctx.cq = &own.peer_cq;
	CHECK_RC(fi_cq_open(domain, &cq_attr, &cq, &cctx), -FI_EINVAL);
	cq_attr.flags = FI_PEER;
	CHECK_RC(fi_cq_open(domain, &cq_attr, &cq, &cctx), 0);
	ectx.eq = &own.eq;
	eq_attr.flags = FI_PEER;
	CHECK_RC(fi_eq_open(fabric, &eq_attr, &eq, &ectx), 0);
	if (!strcmp(argv[2], "avset")) {
		own.nranks = 64;
		return failures ? 1 : avset_batch(dl, av);
	}

	/* endpoint with a peer transfer context (coll_ep.c:116-170) */
	memset(&tctx, 0, sizeof(tctx));
	tctx.size = sizeof(tctx);
	tctx.info = info;
	tctx.ep = &own.ep;
	CHECK_RC(fi_endpoint(domain, info, &ep, &tctx), 0);
	CHECK(tctx.peer_ops && tctx.peer_ops->complete, "peer_ops filled in");
	CHECK(((struct util_ep_prefix *)ep)->progress != NULL, "util_ep progress slot");
	CHECK_RC(fi_enable(ep), -FI_ENOCQ);
	CHECK_RC(fi_ep_bind(ep, &av->fid, 0), 0);
	CHECK_RC(fi_ep_bind(ep, &cq->fid, FI_TRANSMIT | FI_RECV), 0);
	CHECK_RC(fi_ep_bind(ep, &eq->fid, 0), 0);
	CHECK_RC(fi_enable(ep), 0);
	{
		uint64_t name = 0;

		len = sizeof(name);
		CHECK_RC(fi_getname(&ep->fid, &name, &len), 0);
		CHECK(name == 0x4c4641ull, "getname is the owner's");
	}

	/* provider-specific options (fi_ext.h convention) */
	ival = 3;
	CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_ALGO, &ival, sizeof(ival)), 0);
	ival = -1;
	len = sizeof(ival);
	CHECK_RC(fi_getopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_ALGO, &ival, &len), 0);
	CHECK(ival == 3 && len == sizeof(int), "algo roundtrip");
	ival = 9;
	CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_ALGO, &ival, sizeof(ival)),
		 -FI_EINVAL);
	ival = 0;
	CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_ALGO, &ival, sizeof(ival)), 0);
	CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, FI_OPT_MIN_MULTI_RECV, &len, sizeof(len)),
		 -FI_ENOPROTOOPT);
	{
		unsigned char small[16];

		len = sizeof(small);
		CHECK_RC(fi_getopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_UNIQUE_ID, small, &len),
			 -FI_ETOOSMALL);
		CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_UNIQUE_ID, small,
				   sizeof(small)), -FI_EINVAL);
	}

	/* av_set algebra (coll_av_set.c) */
	sattr.count = 8;
	sattr.start_addr = 0;
	sattr.end_addr = 6;
	sattr.stride = 2;
	own.nranks = 8;
	CHECK_RC(fi_av_set(av, &sattr, &set, NULL), 0);          /* {0,2,4,6} */
	CHECK_RC(fi_av_set_insert(set, 2), -FI_EINVAL);
	CHECK_RC(fi_av_set_insert(set, 7), 0);                   /* {0,2,4,6,7} */
	CHECK_RC(fi_av_set_remove(set, 3), -FI_EINVAL);
	CHECK_RC(fi_av_set_remove(set, 4), 0);                   /* {0,2,7,6} */
	sattr.start_addr = 1;
	sattr.end_addr = 2;
	sattr.stride = 1;
	CHECK_RC(fi_av_set(av, &sattr, &set2, NULL), 0);         /* {1,2} */
	CHECK_RC(fi_av_set_intersect(set2, set), 0);             /* {2} */
	CHECK_RC(fi_av_set_union(set2, set), 0);                 /* {2,0,7,6} */
	CHECK_RC(fi_av_set_remove(set2, 2), 0);                  /* {6,0,7} */
	CHECK_RC(fi_av_set_diff(set, set2), 0);                  /* {2} */
	CHECK_RC(fi_close(&set2->fid), 0);
	CHECK_RC(fi_av_set_remove(set, 2), 0);                   /* {} */
	CHECK_RC(fi_av_set_remove(set, 0), -FI_EINVAL);
	sattr.start_addr = 0;
	sattr.end_addr = FI_ADDR_NOTAVAIL;
	CHECK_RC(fi_av_set(av, &sattr, &set2, NULL) == -FI_EINVAL, 1);
	sattr.count = 2;
	sattr.start_addr = 0;
	sattr.end_addr = 4;
	sattr.stride = 1;
	CHECK_RC(fi_av_set(av, &sattr, &set2, NULL) == -FI_EINVAL, 1);  /* too many */
	CHECK_RC(fi_close(&set->fid), 0);
	own.nranks = 1;

	/* before any join every collective is refused */
	{
		fi_addr_t bogus = 0x1234;
		float x = 1, y = 0;

		CHECK_RC(fi_allreduce(ep, &x, 1, NULL, &y, NULL, bogus, FI_FLOAT, FI_SUM,
				      0, NULL), -FI_EINVAL);
		CHECK_RC(fi_barrier(ep, bogus, NULL), -FI_EINVAL);
		CHECK_RC(fi_join_collective(ep, FI_ADDR_NOTAVAIL, NULL, 0, NULL, NULL),
			 -FI_EINVAL);
	}
	drive(ep);                       /* progress with nothing to do */
	{
		struct fi_cq_tagged_entry e;

		CHECK_RC(fi_cq_read(cq, &e, 1), -FI_EAGAIN);
	}

	if (gpu) {
		const size_t n = 1 << 20;
		struct fid_mc *mc, *sub;
		fi_addr_t world, setaddr;
		float *d_x, *d_y, *h_x, *h_y;
		int req[20], err = -1;
		unsigned char uid[128];
		struct fi_cq_err_entry dummy;

		(void)dummy;
		len = sizeof(uid);
		CHECK_RC(fi_getopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_UNIQUE_ID, uid, &len), 0);
		CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_UNIQUE_ID, uid,
				   sizeof(uid)), 0);
		sattr.count = 1;
		sattr.start_addr = 0;
		sattr.end_addr = 0;
		sattr.stride = 1;
		CHECK_RC(fi_av_set(av, &sattr, &set, NULL), 0);
		CHECK_RC(fi_join_collective(ep, FI_ADDR_NOTAVAIL, set, 0, &mc, &req[0]), 0);
		CHECK_RC(wait_join(ep, mc, &req[0]), 0);
		world = fi_mc_addr(mc);
		CHECK_RC(fi_setopt(&ep->fid, FI_OPT_ENDPOINT, OFF_LFA_OPT_UNIQUE_ID, uid,
				   sizeof(uid)), -FI_EBUSY);

		hipMalloc((void **)&d_x, n * 4);
		hipMalloc((void **)&d_y, n * 4);
		h_x = malloc(n * 4);
		h_y = malloc(n * 4);
		for (size_t i = 0; i < n; i++)
			h_x[i] = (float)(i % 1000) * 0.25f - 7.0f;
		hipMemcpy(d_x, h_x, n * 4, hipMemcpyHostToDevice);
		hipMemset(d_y, 0, n * 4);
		hipDeviceSynchronize();   /* the caller orders its own writes */

		/* device buffers: allreduce -> owner CQ carries our context */
		CHECK_RC(fi_allreduce(ep, d_x, n, NULL, d_y, NULL, world, FI_FLOAT, FI_SUM,
				      0, &req[1]), 0);
		CHECK_RC(wait_comp(ep, &req[1], &err), 0);
		CHECK(err == 0, "allreduce err %d", err);
		memset(h_y, 0, n * 4);
		hipMemcpy(h_y, d_y, n * 4, hipMemcpyDeviceToHost);
		CHECK(!memcmp(h_x, h_y, n * 4), "device allreduce result");

		/* host buffers (staged through HBM) */
		memset(h_y, 0, n * 4);
		CHECK_RC(fi_allreduce(ep, h_x, n, NULL, h_y, NULL, world, FI_FLOAT, FI_MAX,
				      0, &req[2]), 0);
		CHECK_RC(wait_comp(ep, &req[2], NULL), 0);
		CHECK(!memcmp(h_x, h_y, n * 4), "host allreduce result");

		/* the rest of fi_ops_collective */
		memset(h_y, 0, n * 4);
		CHECK_RC(fi_reduce_scatter(ep, h_x, n, NULL, h_y, NULL, world, FI_FLOAT,
					   FI_SUM, 0, &req[3]), 0);
		CHECK_RC(wait_comp(ep, &req[3], NULL), 0);
		CHECK(!memcmp(h_x, h_y, n * 4), "reduce_scatter");
		memset(h_y, 0, n * 4);
		CHECK_RC(fi_reduce(ep, h_x, n, NULL, h_y, NULL, world, 0, FI_FLOAT, FI_MIN,
				   0, &req[4]), 0);
		CHECK_RC(wait_comp(ep, &req[4], NULL), 0);
		CHECK(!memcmp(h_x, h_y, n * 4), "reduce");
		memset(h_y, 0, n * 4);
		CHECK_RC(fi_allgather(ep, h_x, n, NULL, h_y, NULL, world, FI_FLOAT, 0,
				      &req[5]), 0);
		CHECK_RC(wait_comp(ep, &req[5], NULL), 0);
		CHECK(!memcmp(h_x, h_y, n * 4), "allgather");
		memset(h_y, 0, n * 4);
		CHECK_RC(fi_scatter(ep, h_x, n, NULL, h_y, NULL, world, 0, FI_FLOAT, 0,
				    &req[6]), 0);
		CHECK_RC(wait_comp(ep, &req[6], NULL), 0);
		CHECK(!memcmp(h_x, h_y, n * 4), "scatter");
		memcpy(h_y, h_x, n * 4);
		CHECK_RC(fi_broadcast(ep, h_y, n, NULL, world, 0, FI_FLOAT, 0, &req[7]), 0);
		CHECK_RC(wait_comp(ep, &req[7], NULL), 0);
		CHECK(!memcmp(h_x, h_y, n * 4), "broadcast");
		CHECK_RC(fi_barrier(ep, world, &req[8]), 0);
		CHECK_RC(wait_comp(ep, &req[8], NULL), 0);
		CHECK_RC(fi_barrier2(ep, world, 0, &req[9]), 0);
		CHECK_RC(wait_comp(ep, &req[9], NULL), 0);

		/* argument errors come back synchronously, as from coll_ep_* */
		CHECK_RC(fi_allreduce(ep, d_x, n, NULL, d_y, NULL, world, FI_FLOAT, FI_BOR,
				      0, &req[10]), -FI_EOPNOTSUPP);
		CHECK_RC(fi_reduce(ep, d_x, n, NULL, d_y, NULL, world, 5, FI_FLOAT, FI_SUM,
				   0, &req[10]), -FI_EINVAL);
		CHECK_RC(fi_alltoall(ep, d_x, n, NULL, d_y, NULL, world, FI_FLOAT, 0,
				     &req[10]), -FI_ENOSYS);

		/* the av_set's own address names the world group */
		CHECK_RC(fi_av_set_addr(set, &setaddr), 0);
		hipMemset(d_y, 0, n * 4);
		hipDeviceSynchronize();   /* the caller orders its own writes */
		CHECK_RC(fi_allreduce(ep, d_x, n, NULL, d_y, NULL, setaddr, FI_FLOAT,
				      FI_SUM, 0, &req[11]), 0);
		CHECK_RC(wait_comp(ep, &req[11], NULL), 0);
		hipMemcpy(h_y, d_y, n * 4, hipMemcpyDeviceToHost);
		CHECK(!memcmp(h_x, h_y, n * 4), "allreduce on av_set addr");

		/* subset join over the world group (ncclCommSplit underneath) */
		CHECK_RC(fi_join_collective(ep, world, set, 0, &sub, &req[12]), 0);
		CHECK_RC(wait_join(ep, sub, &req[12]), 0);
		hipMemset(d_y, 0, n * 4);
		hipDeviceSynchronize();   /* the caller orders its own writes */
		CHECK_RC(fi_allreduce(ep, d_x, n, NULL, d_y, NULL, fi_mc_addr(sub),
				      FI_FLOAT, FI_SUM, 0, &req[13]), 0);
		CHECK_RC(wait_comp(ep, &req[13], NULL), 0);
		hipMemcpy(h_y, d_y, n * 4, hipMemcpyDeviceToHost);
		CHECK(!memcmp(h_x, h_y, n * 4), "allreduce on subset group");
		CHECK_RC(fi_close(&sub->fid), 0);
		CHECK_RC(fi_barrier(ep, fi_mc_addr(sub), NULL), -FI_EINVAL);

		/* a join over a new set's OWN address (fabtests core_coll.c:138-168:
		 * the set's members alone form the group, lfa_join_members), then
		 * core_coll.c's known answer on it */
		{
			struct fid_av_set *own_set;
			struct fid_mc *own_mc;
			fi_addr_t own_addr;
			uint64_t ka = 1234, kr = 0, *d_ka;

			sattr.count = 0;
			sattr.start_addr = 0;
			sattr.end_addr = 0;
			sattr.stride = 1;
			CHECK_RC(fi_av_set(av, &sattr, &own_set, NULL), 0);
			CHECK_RC(fi_av_set_addr(own_set, &own_addr), 0);
			CHECK_RC(fi_join_collective(ep, own_addr, own_set, 0, &own_mc, &req[14]), 0);
			CHECK_RC(wait_join(ep, own_mc, &req[14]), 0);
			hipMalloc((void **)&d_ka, 2 * sizeof(uint64_t));
			hipMemcpy(d_ka, &ka, sizeof(ka), hipMemcpyHostToDevice);
			CHECK_RC(fi_allreduce(ep, d_ka, 1, NULL, d_ka + 1, NULL, fi_mc_addr(own_mc),
					      FI_UINT64, FI_SUM, 0, &req[15]), 0);
			CHECK_RC(wait_comp(ep, &req[15], NULL), 0);
			hipMemcpy(&kr, d_ka + 1, sizeof(kr), hipMemcpyDeviceToHost);
			CHECK(kr == 1234, "self-joined group known answer %lu", (unsigned long)kr);
			hipFree(d_ka);
			CHECK_RC(fi_close(&own_mc->fid), 0);
			CHECK_RC(fi_close(&own_set->fid), 0);
		}

		CHECK_RC(fi_close(&mc->fid), 0);
		CHECK_RC(fi_close(&set->fid), 0);
		hipFree(d_x);
		hipFree(d_y);
		free(h_x);
		free(h_y);
	}

	CHECK_RC(fi_close(&ep->fid), 0);
	CHECK_RC(fi_close(&eq->fid), 0);
	CHECK_RC(fi_close(&cq->fid), 0);
	CHECK_RC(fi_close(&av->fid), 0);
	CHECK_RC(fi_close(&domain->fid), 0);
	CHECK_RC(fi_close(&fabric->fid), 0);
	if (freeinfo)
		freeinfo(info);
	if (failures) {
		fprintf(stderr, "%d check(s) failed\n", failures);
		return 1;
	}
	printf("OK %s%s\n", argv[2], manual ? " manual" : "");
	return 0;
}
