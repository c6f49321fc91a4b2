/*
 * off_lfa — libfabric offload-collective provider over the gfx950 path.
 *
 * A dl-loadable libfabric provider (liboff_lfa-fi.so, entry point
 * fi_prov_ini, include/rdma/providers/fi_prov.h:59-74) that stands where
 * prov/coll's util provider stands behind rxm, and forwards every
 * fi_ops_collective call to liblfa_coll.so (include/lfa_coll.h): schedules
 * as data, RCCL over xGMI for transport, the gfx950 combine kernels for
 * every reduction.  Written against libfabric's PUBLIC headers only
 * (rdma/fabric.h and friends, rdma/providers/fi_prov.h and fi_peer.h).
 *
 * How a host provider drives it (the peer-provider protocol, fi_peer.h):
 *
 *   prov->getinfo   requires FI_PEER_TRANSFER in hints->mode  (coll_init.c:39)
 *   prov->fabric    fi_fabric over the returned fabric_attr   (rxm_fabric.c:85-121)
 *   fi_domain2      FI_PEER + fi_peer_domain_context          (coll_domain.c:80-108,
 *                                                               rxm_domain.c:944-953)
 *   fi_query_collective  per-op capability probe              (rxm_domain.c:878-893)
 *   fi_av_open      FI_PEER + fi_peer_av_context              (coll_av.c:68-106,
 *                                                               rxm_domain.c:274-287)
 *   fi_cq_open      FI_PEER + fi_peer_cq_context              (coll_cq.c:68-100,
 *                                                               rxm_cq.c:2160-2199)
 *   fi_eq_open      FI_PEER + fi_peer_eq_context              (coll_eq.c:66-98)
 *   fi_endpoint     fi_peer_transfer_context; we fill peer_ops (coll_ep.c:116-170,
 *                                                               rxm_ep.c:1709-1720)
 *   fi_join_collective  av_set + parent coll_addr             (coll_coll.c:912-995)
 *   fi_allreduce / fi_reduce_scatter / fi_reduce / fi_allgather / fi_broadcast /
 *   fi_scatter / fi_barrier  -> lfa_*; completion is the owner's
 *       peer_cq->owner_ops->write(cq, context, FI_COLLECTIVE, 0, 0, 0, 0, ...)
 *                                                               (coll_coll.c:725-733)
 *   join completion  fi_eq_write(peer_eq, FI_JOIN_COMPLETE)   (coll_coll.c:691-718)
 *
 * Progress.  The provider advertises FI_PROGRESS_AUTO and backs it with a
 * progress thread per endpoint.  rxm also calls the offload endpoint's
 * util_ep->progress slot (rxm_cq.c:2082-2099), so the endpoint begins with
 * a layout-compatible prefix of struct util_ep (include/ofi_util.h:280-311)
 * whose progress slot points at olfa_util_progress.  fi_cq_read on the
 * off_lfa CQ progresses too (and returns -FI_EAGAIN: completions belong to
 * the owner's CQ).
 *
 * coll_addr.  fi_mc_addr of an off_lfa multicast handle, or fi_av_set_addr
 * of the av_set a world join was made over.  Addresses this provider did not
 * hand out are rejected with -FI_EINVAL (they are looked up, never
 * dereferenced).
 */
#define _GNU_SOURCE
#include <errno.h>
#include <fcntl.h>
#include <pthread.h>
#include <sched.h>
#include <stdatomic.h>
#include <stddef.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
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

#include "lfa_coll.h"
#include "off_lfa.h"

#define OLFA_VERSION FI_VERSION(0, 3)
#define OLFA_CAPS (FI_COLLECTIVE | FI_HMEM)
#define olfa_container_of(ptr, type, field) \
	((type *)((char *)(ptr) - offsetof(type, field)))

/* ---------------------------------------------------------- parameters -- */

/*
 * Provider parameters, registered the libfabric way:
 * fi_param_define at fi_prov_ini makes each one FI_OFF_LFA_<NAME> and lists
 * it with its help in `fi_info -e` (src/var.c:188-231; rxm does the same,
 * prov/rxm/src/rxm_init.c:633-671); fi_param_get reads it.  The provider's
 * own knobs are kept here; the kernel and executor knobs (LFA_*) go to
 * liblfa through lfa_param_set, before any domain opens.  A host without
 * libfabric's core (the test owners, an embedder) may leave fi_param_* out:
 * they are weak here, and then the raw names (OFF_LFA_*, LFA_*) are read
 * from the environment, as before round 6.  "provisional" marks defaults
 * tuned with 2-4 processes time-sharing ONE MI355X, not on
 * the 8-GPU xGMI topology.
 */
#pragma weak fi_param_define
#pragma weak fi_param_get

static const struct olfa_param {
	const char *name;       /* FI_OFF_LFA_<NAME> */
	enum fi_param_type type;
	const char *raw;        /* the environment name it replaces, and for
				 * LFA_* the liblfa knob it sets */
	const char *help;
} olfa_params[] = {
	{ "transport", FI_PARAM_STRING, "OFF_LFA_TRANSPORT",
	  "group transport: rccl (default: RCCL over xGMI) or peer (the owner's tagged messages)" },
	{ "progress", FI_PARAM_STRING, "OFF_LFA_PROGRESS",
	  "auto (a progress thread per endpoint, FI_PROGRESS_AUTO) or manual" },
	{ "algo", FI_PARAM_INT, "OFF_LFA_ALGO",
	  "enum lfa_coll_algo: 0 tree, 1 recursive doubling, 2 rccl, 3 tree over RCCL collectives, 4 p2p, 5 auto (default)" },
	{ "device", FI_PARAM_INT, "OFF_LFA_DEVICE",
	  "HIP device ordinal (default $LOCAL_RANK, else 0; -1 with the peer transport: host buffers only)" },
	{ "bootstrap_dir", FI_PARAM_STRING, "OFF_LFA_BOOTSTRAP_DIR",
	  "directory of the file rendezvous for the RCCL unique id (without fi_setopt)" },
	{ "bootstrap_key", FI_PARAM_STRING, "OFF_LFA_BOOTSTRAP_KEY",
	  "file rendezvous key (default world)" },
	{ "bootstrap_timeout", FI_PARAM_INT, "OFF_LFA_BOOTSTRAP_TIMEOUT",
	  "seconds to wait at the file rendezvous (default 120)" },
	{ "debug", FI_PARAM_BOOL, "OFF_LFA_DEBUG", "warnings on stderr" },
	{ "sig_timeout_ms", FI_PARAM_INT, "LFA_SIG_TIMEOUT_MS",
	  "bound of every GPU-side wait (flag barrier, one-shot, completion word), ms (default 20000)" },
	{ "oneshot_allreduce_bytes", FI_PARAM_SIZE_T, "LFA_OS_AG_BYTES",
	  "allreduce/reduce buckets up to this many bytes summed over the members run as one one-shot kernel (default 2 MiB; provisional)" },
	{ "oneshot_rs_bytes", FI_PARAM_SIZE_T, "LFA_OS_RS_BYTES",
	  "reduce_scatter buckets up to this many bytes per member run as one one-shot kernel (default 4 MiB; provisional)" },
	{ "group_chunk_bytes", FI_PARAM_SIZE_T, "LFA_GROUP_CHUNK_BYTES",
	  "chunk every member of a group splits large operations into (0 off; default: 32 MiB chunks from 64 MiB per member)" },
	{ "stage_pool_bytes", FI_PARAM_SIZE_T, "LFA_STAGE_POOL_BYTES",
	  "idle device staging bytes a peer domain keeps (default 1 GiB)" },
	{ "ws_mem", FI_PARAM_STRING, "LFA_WS_MEM",
	  "P2P workspace memory: uncached (default), fine or coarse" },
	{ "ws_cache_bytes", FI_PARAM_SIZE_T, "LFA_WS_CACHE_BYTES",
	  "released P2P workspaces kept for reuse per process (default 4 GiB)" },
	{ "ws_quarantine_bytes", FI_PARAM_SIZE_T, "LFA_WS_QUARANTINE_BYTES",
	  "released P2P workspaces held, never reused, per process (default 4 GiB)" },
	{ "host_zero_copy", FI_PARAM_BOOL, "LFA_HOST_ZERO_COPY",
	  "combine pinned/registered host buffers on their device mappings (default 1)" },
	{ "host_small_bytes", FI_PARAM_SIZE_T, "LFA_HOST_SMALL_BYTES",
	  "host buckets up to this size combine in the host loop (default 1 MiB)" },
	{ "host_register_bytes", FI_PARAM_SIZE_T, "LFA_HOST_REGISTER_BYTES",
	  "pageable host buckets from this size are registered for the call when no other call is staging (default 64 MiB)" },
	{ "direct", FI_PARAM_BOOL, "LFA_DIRECT",
	  "one-member small collectives through liblfa's own HSA queue (default 1)" },
};
#define OLFA_NPARAMS (sizeof(olfa_params) / sizeof(olfa_params[0]))
/* the provider's own knobs as read at fi_prov_ini (string form) */
static char olfa_param_val[OLFA_NPARAMS][256];
static int olfa_param_isset[OLFA_NPARAMS];

/* Register and read every parameter once (fi_prov_ini). */
static void olfa_params_init(struct fi_provider *prov)
{
	static int done;

	if (done++)
		return;
	for (size_t i = 0; i < OLFA_NPARAMS; i++) {
		const struct olfa_param *p = &olfa_params[i];
		char buf[256];
		int have = 0;

		if (fi_param_define && fi_param_get) {
			union { char *s; int i; size_t z; } v;

			memset(&v, 0, sizeof(v));
			fi_param_define(prov, p->name, p->type, "%s", p->help);
			if (fi_param_get(prov, p->name, &v) == FI_SUCCESS) {
				have = 1;
				if (p->type == FI_PARAM_STRING)
					snprintf(buf, sizeof(buf), "%s", v.s ? v.s : "");
				else if (p->type == FI_PARAM_SIZE_T)
					snprintf(buf, sizeof(buf), "%zu", v.z);
				else
					snprintf(buf, sizeof(buf), "%d", v.i);
			}
		}
		if (!have && getenv(p->raw)) {
			have = 1;
			snprintf(buf, sizeof(buf), "%s", getenv(p->raw));
		}
		if (!have)
			continue;
		olfa_param_isset[i] = 1;
		snprintf(olfa_param_val[i], sizeof(olfa_param_val[i]), "%s", buf);
		if (!strncmp(p->raw, "LFA_", 4))
			lfa_param_set(p->raw, buf);
	}
}

/* The provider's own knob `name` (its string), or NULL when unset. */
static const char *olfa_param(const char *name)
{
	for (size_t i = 0; i < OLFA_NPARAMS; i++)
		if (!strcmp(olfa_params[i].name, name))
			return olfa_param_isset[i] ? olfa_param_val[i] : NULL;
	return NULL;
}

static int olfa_param_int(const char *name, int dflt)
{
	const char *v = olfa_param(name);

	return v && *v ? atoi(v) : dflt;
}

static int olfa_debug = -1;

static void olfa_warn(const char *fmt, const char *arg, long v)
{
	if (olfa_debug < 0)
		olfa_debug = olfa_param("debug") && strcmp(olfa_param("debug"), "0");
	if (olfa_debug)
		fprintf(stderr, "off_lfa: %s %s (%ld)\n", fmt, arg ? arg : "", v);
}

/* ------------------------------------------------------------ objects -- */

struct olfa_fabric {
	struct fid_fabric fabric_fid;
};

struct olfa_domain {
	struct fid_domain domain_fid;
	struct fid_domain *peer_domain;
};

struct olfa_eq {
	struct fid_eq eq_fid;
	struct fid_eq *peer_eq;
};

struct olfa_ep;

struct olfa_cq {
	struct fid_cq cq_fid;
	struct fid_peer_cq *peer_cq;
	struct olfa_ep *ep;            /* the endpoint bound to it, if any */
};

struct olfa_av {
	struct fid_av av_fid;
	struct fid_peer_av *peer_av;
};

struct olfa_mc {
	struct fid_mc mc_fid;
	struct olfa_ep *ep;
	struct lfa_coll_mc *lmc;       /* NULL for an av_set's bound address */
	lfa_addr_t laddr;              /* LFA_ADDR_NOTAVAIL until bound */
	fi_addr_t *members;            /* owner AV addresses, group-rank order */
	size_t nmembers;
	struct olfa_mc *next;          /* ep->mcs registry */
};

struct olfa_av_set {
	struct fid_av_set set_fid;
	struct olfa_av *av;
	fi_addr_t *addr;
	size_t count, cap;
	struct olfa_mc set_mc;         /* what fi_av_set_addr hands out */
};

/* Layout-compatible prefix of struct util_ep (include/ofi_util.h:280-306),
 * for rxm_ep_progress_coll (rxm_cq.c:2095-2098), which reaches the offload
 * endpoint's progress function through container_of(..., struct util_ep,
 * ep_fid).  Only `progress` is ever read through it. */
#define OLFA_UTIL_CNTR_CNT 6           /* enum ofi_cntr_index, ofi_util.h:265-273 */
struct olfa_util_ep_prefix {
	struct fid_ep ep_fid;
	void *domain;
	void *av;
	void *av_entry[2];
	void *eq;
	void *rx_cq;
	uint64_t rx_op_flags;
	void *tx_cq;
	uint64_t tx_op_flags;
	uint64_t inject_op_flags;
	uint64_t tx_msg_flags;
	uint64_t rx_msg_flags;
	void *cntrs[OLFA_UTIL_CNTR_CNT];
	void (*cntr_inc_funcs[OLFA_UTIL_CNTR_CNT])(void *);
	enum fi_ep_type type;
	uint64_t caps;
	uint64_t flags;
	void (*progress)(void *util_ep);
};

struct olfa_ep {
	struct olfa_util_ep_prefix util;   /* must stay first */
	struct olfa_domain *domain;
	struct olfa_av *av;
	struct olfa_cq *cq;
	struct olfa_eq *eq;
	struct fid_ep *peer_ep;            /* the owner endpoint */
	int enabled;

	pthread_mutex_t lock;              /* mc registry */
	pthread_mutex_t plock;             /* one progress pass at a time */
	struct olfa_mc *mcs;
	struct olfa_mc *world;             /* world group, after bootstrap */

	/* bootstrap */
	int device;
	int device_set;                    /* OFF_LFA_DEVICE / the option given */
	int algo;
	size_t chunk;
	int peer_xport;                    /* OFF_LFA_TRANSPORT=peer */
	fi_addr_t *waddr;                  /* world rank -> owner AV address */
	size_t nworld;                     /* entries of waddr */
	int have_uid;
	unsigned char uid[LFA_UNIQUE_ID_BYTES];
	struct lfa_coll_domain *ld;
	struct lfa_coll_ep *le;

	/* progress thread */
	int manual_progress;
	pthread_t thread;
	int thread_running;
	atomic_int stop;
};

/* -------------------------------------------------------- enosys stubs -- */

static int olfa_no_bind(struct fid *fid, struct fid *bfid, uint64_t flags)
{
	return -FI_ENOSYS;
}
static int olfa_no_control(struct fid *fid, int command, void *arg)
{
	return -FI_ENOSYS;
}
static int olfa_no_ops_open(struct fid *fid, const char *name, uint64_t flags,
			    void **ops, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_no_tostr(const struct fid *fid, char *buf, size_t len)
{
	return -FI_ENOSYS;
}
static int olfa_no_ops_set(struct fid *fid, const char *name, uint64_t flags,
			   void *ops, void *context)
{
	return -FI_ENOSYS;
}

#define OLFA_FI_OPS(close_fn, bind_fn, control_fn) {                      \
	.size = sizeof(struct fi_ops), .close = close_fn, .bind = bind_fn, \
	.control = control_fn, .ops_open = olfa_no_ops_open,                \
	.tostr = olfa_no_tostr, .ops_set = olfa_no_ops_set }

/* ----------------------------------------------------------- fi_info -- */

static void olfa_freeinfo(struct fi_info *fi)
{
	while (fi) {
		struct fi_info *next = fi->next;

		free(fi->src_addr);
		free(fi->dest_addr);
		free(fi->tx_attr);
		free(fi->rx_attr);
		free(fi->ep_attr);
		if (fi->domain_attr)
			free(fi->domain_attr->name);
		free(fi->domain_attr);
		if (fi->fabric_attr) {
			free(fi->fabric_attr->name);
			free(fi->fabric_attr->prov_name);
		}
		free(fi->fabric_attr);
		free(fi);
		fi = next;
	}
}

/* One fi_info, allocated the way the core's fi_freeinfo releases it
 * (every attribute and string from malloc). */
static struct fi_info *olfa_info(uint32_t version)
{
	struct fi_info *fi = calloc(1, sizeof(*fi));

	if (!fi)
		return NULL;
	fi->tx_attr = calloc(1, sizeof(*fi->tx_attr));
	fi->rx_attr = calloc(1, sizeof(*fi->rx_attr));
	fi->ep_attr = calloc(1, sizeof(*fi->ep_attr));
	fi->domain_attr = calloc(1, sizeof(*fi->domain_attr));
	fi->fabric_attr = calloc(1, sizeof(*fi->fabric_attr));
	if (!fi->tx_attr || !fi->rx_attr || !fi->ep_attr || !fi->domain_attr ||
	    !fi->fabric_attr)
		goto err;
	fi->caps = OLFA_CAPS;
	fi->mode = FI_PEER_TRANSFER;
	fi->addr_format = FI_FORMAT_UNSPEC;

	fi->tx_attr->caps = OLFA_CAPS;
	fi->tx_attr->mode = FI_PEER_TRANSFER;
	fi->tx_attr->size = 1 << 16;
	fi->tx_attr->iov_limit = 1;
	fi->rx_attr->caps = OLFA_CAPS;
	fi->rx_attr->mode = FI_PEER_TRANSFER;
	fi->rx_attr->size = 1 << 16;
	fi->rx_attr->iov_limit = 1;

	fi->ep_attr->type = FI_EP_RDM;
	fi->ep_attr->protocol = FI_PROTO_UNSPEC;
	fi->ep_attr->max_msg_size = SIZE_MAX;
	fi->ep_attr->tx_ctx_cnt = 1;
	fi->ep_attr->rx_ctx_cnt = 1;

	/* coll_attr.c:69-85, but the progress claim is real here */
	fi->domain_attr->name = strdup(OFF_LFA_PROV_NAME);
	fi->domain_attr->threading = FI_THREAD_SAFE;
	fi->domain_attr->control_progress = FI_PROGRESS_AUTO;
	fi->domain_attr->progress = FI_PROGRESS_AUTO;
	fi->domain_attr->resource_mgmt = FI_RM_ENABLED;
	fi->domain_attr->av_type = FI_AV_UNSPEC;
	fi->domain_attr->caps = FI_COLLECTIVE;
	fi->domain_attr->cq_cnt = 1 << 16;
	fi->domain_attr->ep_cnt = 1 << 15;
	fi->domain_attr->tx_ctx_cnt = 1;
	fi->domain_attr->rx_ctx_cnt = 1;
	fi->domain_attr->max_ep_tx_ctx = 1;
	fi->domain_attr->max_ep_rx_ctx = 1;
	fi->domain_attr->mr_iov_limit = 1;

	fi->fabric_attr->name = strdup(OFF_LFA_PROV_NAME);
	fi->fabric_attr->prov_name = strdup(OFF_LFA_PROV_NAME);
	fi->fabric_attr->prov_version = OLFA_VERSION;
	fi->fabric_attr->api_version = version;
	if (!fi->domain_attr->name || !fi->fabric_attr->name ||
	    !fi->fabric_attr->prov_name)
		goto err;
	return fi;
err:
	olfa_freeinfo(fi);
	return NULL;
}

static int olfa_getinfo(uint32_t version, const char *node, const char *service,
			uint64_t flags, const struct fi_info *hints,
			struct fi_info **info)
{
	if (!info)
		return -FI_EINVAL;
	*info = NULL;
	if (hints) {
		/* coll_init.c:39-43: peer transfers are the only mode */
		if (!(hints->mode & FI_PEER_TRANSFER))
			return -FI_ENODATA;
		if (hints->caps & ~(OLFA_CAPS | FI_MSG | FI_TAGGED | FI_SEND |
				    FI_RECV | FI_LOCAL_COMM | FI_REMOTE_COMM))
			return -FI_ENODATA;
		if (hints->ep_attr && hints->ep_attr->type != FI_EP_UNSPEC &&
		    hints->ep_attr->type != FI_EP_RDM)
			return -FI_ENODATA;
		if (hints->fabric_attr && hints->fabric_attr->prov_name &&
		    strcasecmp(hints->fabric_attr->prov_name, OFF_LFA_PROV_NAME))
			return -FI_ENODATA;
	}
	*info = olfa_info(version);
	return *info ? 0 : -FI_ENOMEM;
}

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

static void olfa_mc_unregister(struct olfa_ep *ep, struct olfa_mc *m)
{
	struct olfa_mc **pp;

	for (pp = &ep->mcs; *pp; pp = &(*pp)->next)
		if (*pp == m) {
			*pp = m->next;
			break;
		}
	m->next = NULL;
}

/* ------------------------------------------------------------ progress -- */

/* Moves finished collectives and joins to the owner: CQ entries through
 * the peer CQ's owner_ops (coll_coll.c:725-733), join events through the
 * peer EQ (coll_coll.c:708-717).  Returns how many it moved. */
static int olfa_progress(struct olfa_ep *ep)
{
	struct lfa_cq_entry ent[16];
	struct lfa_cq_err_entry lerr;
	struct lfa_eq_entry lev;
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
	while (lfa_eq_read(ep->le, &event, &lev) > 0) {
		struct olfa_mc *m;
		struct fi_eq_entry e;

		pthread_mutex_lock(&ep->lock);
		for (m = ep->mcs; m; m = m->next)
			if (m->lmc && (void *)m->lmc == lev.fid)
				break;
		pthread_mutex_unlock(&ep->lock);
		memset(&e, 0, sizeof(e));
		e.fid = m ? &m->mc_fid.fid : NULL;
		e.context = lev.context;
		e.data = lev.data;
		if (ep->eq)
			fi_eq_write(ep->eq->peer_eq, FI_JOIN_COMPLETE, &e, sizeof(e), 0);
		else
			olfa_warn("join completed with no EQ bound", NULL, 0);
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
static long olfa_index(const fi_addr_t *list, size_t n, fi_addr_t addr)
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
	ret = lfa_join_members(ep->le, lfa_coll_world_addr(ep->le), ranks, n, flags,
			       &m->lmc, context);
	if (!ret) {
		pthread_mutex_lock(&ep->lock);
		m->laddr = lfa_mc_addr(m->lmc);
		olfa_mc_register(ep, m);
		pthread_mutex_unlock(&ep->lock);
	}
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
		ret = lfa_join_collective(ep->le, LFA_ADDR_NOTAVAIL, NULL, 0, flags,
					  &m->lmc, context);
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
	ret = lfa_join_collective(ep->le, paddr, ranks, n, flags, &m->lmc, context);
	pthread_mutex_lock(&ep->lock);
	if (!ret) {
		m->laddr = lfa_mc_addr(m->lmc);
		olfa_mc_register(ep, m);
	}
	pthread_mutex_unlock(&ep->lock);
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
static int olfa_endpoint(struct fid_domain *domain, struct fi_info *info,
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

/* ------------------------------------------------------------------ CQ -- */

static int olfa_cq_close(struct fid *fid)
{
	struct olfa_cq *cq = olfa_container_of(fid, struct olfa_cq, cq_fid.fid);

	if (cq->ep && cq->ep->cq == cq)
		cq->ep->cq = NULL;
	free(cq);
	return 0;
}

static struct fi_ops olfa_cq_fi_ops = OLFA_FI_OPS(olfa_cq_close, olfa_no_bind,
						  olfa_no_control);

/* Entries land in the owner's CQ; reading ours only makes progress. */
static ssize_t olfa_cq_read(struct fid_cq *cq_fid, void *buf, size_t count)
{
	struct olfa_cq *cq = olfa_container_of(cq_fid, struct olfa_cq, cq_fid);

	if (cq->ep)
		olfa_progress(cq->ep);
	return -FI_EAGAIN;
}

static ssize_t olfa_cq_readfrom(struct fid_cq *cq, void *buf, size_t count,
				fi_addr_t *src_addr)
{
	return olfa_cq_read(cq, buf, count);
}

static ssize_t olfa_cq_readerr(struct fid_cq *cq, struct fi_cq_err_entry *buf,
			       uint64_t flags)
{
	return -FI_EAGAIN;
}

static ssize_t olfa_cq_sread(struct fid_cq *cq, void *buf, size_t count,
			     const void *cond, int timeout)
{
	return -FI_ENOSYS;
}

static ssize_t olfa_cq_sreadfrom(struct fid_cq *cq, void *buf, size_t count,
				 fi_addr_t *src_addr, const void *cond, int timeout)
{
	return -FI_ENOSYS;
}

static int olfa_cq_signal(struct fid_cq *cq)
{
	return -FI_ENOSYS;
}

static const char *olfa_cq_strerror(struct fid_cq *cq, int prov_errno,
				    const void *err_data, char *buf, size_t len)
{
	if (buf && len)
		snprintf(buf, len, "off_lfa provider error %d", prov_errno);
	return buf;
}

static int olfa_cq_export_xpu(struct fid_cq *cq, uint64_t flags,
			      struct fid_xpu_cq *xpu_cq)
{
	return -FI_ENOSYS;
}

static struct fi_ops_cq olfa_cq_ops = {
	.size = sizeof(struct fi_ops_cq),
	.read = olfa_cq_read,
	.readfrom = olfa_cq_readfrom,
	.readerr = olfa_cq_readerr,
	.sread = olfa_cq_sread,
	.sreadfrom = olfa_cq_sreadfrom,
	.signal = olfa_cq_signal,
	.strerror = olfa_cq_strerror,
	.export_xpu = olfa_cq_export_xpu,
};

/* coll_cq_init (coll_cq.c:68-100): FI_PEER + a peer CQ context */
static int olfa_cq_open(struct fid_domain *domain, struct fi_cq_attr *attr,
			struct fid_cq **cq_fid, void *context)
{
	struct fi_peer_cq_context *pc = context;
	struct olfa_cq *cq;

	if (!attr || !(attr->flags & FI_PEER))
		return -FI_EINVAL;
	if (!pc || pc->size < sizeof(*pc) || !pc->cq)
		return -FI_EINVAL;
	cq = calloc(1, sizeof(*cq));
	if (!cq)
		return -FI_ENOMEM;
	cq->cq_fid.fid.fclass = FI_CLASS_CQ;
	cq->cq_fid.fid.context = context;
	cq->cq_fid.fid.ops = &olfa_cq_fi_ops;
	cq->cq_fid.ops = &olfa_cq_ops;
	cq->peer_cq = pc->cq;
	*cq_fid = &cq->cq_fid;
	return 0;
}

/* ------------------------------------------------------------------ EQ -- */

static int olfa_eq_close(struct fid *fid)
{
	free(olfa_container_of(fid, struct olfa_eq, eq_fid.fid));
	return 0;
}

static struct fi_ops olfa_eq_fi_ops = OLFA_FI_OPS(olfa_eq_close, olfa_no_bind,
						  olfa_no_control);

static ssize_t olfa_eq_read(struct fid_eq *eq, uint32_t *event, void *buf,
			    size_t len, uint64_t flags)
{
	return -FI_EAGAIN;          /* events go to the owner's EQ */
}

static ssize_t olfa_eq_readerr(struct fid_eq *eq, struct fi_eq_err_entry *buf,
			       uint64_t flags)
{
	return -FI_EAGAIN;
}

static ssize_t olfa_eq_write(struct fid_eq *eq, uint32_t event, const void *buf,
			     size_t len, uint64_t flags)
{
	return -FI_ENOSYS;
}

static ssize_t olfa_eq_sread(struct fid_eq *eq, uint32_t *event, void *buf,
			     size_t len, int timeout, uint64_t flags)
{
	return -FI_ENOSYS;
}

static const char *olfa_eq_strerror(struct fid_eq *eq, int prov_errno,
				    const void *err_data, char *buf, size_t len)
{
	if (buf && len)
		snprintf(buf, len, "off_lfa provider error %d", prov_errno);
	return buf;
}

static struct fi_ops_eq olfa_eq_ops = {
	.size = sizeof(struct fi_ops_eq),
	.read = olfa_eq_read,
	.readerr = olfa_eq_readerr,
	.write = olfa_eq_write,
	.sread = olfa_eq_sread,
	.strerror = olfa_eq_strerror,
};

/* ofi_coll_eq_open (coll_eq.c:66-98) */
static int olfa_eq_open(struct fid_fabric *fabric, struct fi_eq_attr *attr,
			struct fid_eq **eq_fid, void *context)
{
	struct fi_peer_eq_context *pc = context;
	struct olfa_eq *eq;

	if (!attr || !(attr->flags & FI_PEER))
		return -FI_EINVAL;
	if (!pc || pc->size < sizeof(*pc) || !pc->eq)
		return -FI_EINVAL;
	eq = calloc(1, sizeof(*eq));
	if (!eq)
		return -FI_ENOMEM;
	eq->eq_fid.fid.fclass = FI_CLASS_EQ;
	eq->eq_fid.fid.context = context;
	eq->eq_fid.fid.ops = &olfa_eq_fi_ops;
	eq->eq_fid.ops = &olfa_eq_ops;
	eq->peer_eq = pc->eq;
	*eq_fid = &eq->eq_fid;
	return 0;
}

/* -------------------------------------------------------------- AV set -- */

static int olfa_set_grow(struct olfa_av_set *s, size_t need)
{
	fi_addr_t *p;
	size_t cap = s->cap ? s->cap : 16;

	if (need <= s->cap)
		return 0;
	while (cap < need)
		cap *= 2;
	p = realloc(s->addr, cap * sizeof(*p));
	if (!p)
		return -FI_ENOMEM;
	s->addr = p;
	s->cap = cap;
	return 0;
}

/* coll_av_set_insert / _remove / _union / _intersect / _diff
 * (coll_av_set.c:35-164).  The ORDER they leave matters: it numbers the
 * members of a group joined over the set (olfa_join).  insert and union
 * append, remove moves the last address into the hole (:149-164).
 *
 * intersect (:71-96) walks SRC and moves each address it finds in dst to a
 * front that advances by one per match, so the common addresses come out in
 * src's order ([3,2,1,0] ∩ [0,1] = [0,1]).  The reference's move overwrites
 * the front entry, which loses a common address not yet reached
 * ([a,b,c,d] ∩ [c,a] = [c]); here the two entries swap, so the result is the
 * reference's wherever the reference keeps every common address, and
 * otherwise every common address, still in src's order (the reference's
 * result is then a subsequence of it).
 *
 * diff (:98-125) removes src's addresses one by one, in src's order, as
 * remove would (the last address moves into the hole).  The reference writes
 * the found address over the last one instead, which keeps the address it
 * was asked to drop and drops the last ([a,b,c,d] \ [b] = [a,b,c]); the
 * result is the reference's wherever the reference drops exactly src's
 * addresses.
 *
 * tests/test_off_lfa.py::test_av_set_algebra_against_reference_loops checks
 * both statements exhaustively on small sets against the reference loops
 * restated in Python (DESIGN.md §6a "Group rank numbering"). */
static int olfa_set_insert(struct fid_av_set *set, fi_addr_t addr)
{
	struct olfa_av_set *s = olfa_container_of(set, struct olfa_av_set, set_fid);

	if (olfa_index(s->addr, s->count, addr) >= 0)
		return -FI_EINVAL;
	if (olfa_set_grow(s, s->count + 1))
		return -FI_ENOMEM;
	s->addr[s->count++] = addr;
	return 0;
}

static int olfa_set_remove(struct fid_av_set *set, fi_addr_t addr)
{
	struct olfa_av_set *s = olfa_container_of(set, struct olfa_av_set, set_fid);
	long i = olfa_index(s->addr, s->count, addr);

	if (i < 0)
		return -FI_EINVAL;
	s->addr[i] = s->addr[--s->count];       /* coll_av_set.c:156-160 */
	return 0;
}

static int olfa_set_union(struct fid_av_set *dst, const struct fid_av_set *src)
{
	struct olfa_av_set *d = olfa_container_of(dst, struct olfa_av_set, set_fid);
	const struct olfa_av_set *s =
		olfa_container_of(src, struct olfa_av_set, set_fid);

	for (size_t i = 0; i < s->count; i++) {
		if (olfa_index(d->addr, d->count, s->addr[i]) >= 0)
			continue;
		if (olfa_set_grow(d, d->count + 1))
			return -FI_ENOMEM;
		d->addr[d->count++] = s->addr[i];
	}
	return 0;
}

static int olfa_set_intersect(struct fid_av_set *dst, const struct fid_av_set *src)
{
	struct olfa_av_set *d = olfa_container_of(dst, struct olfa_av_set, set_fid);
	const struct olfa_av_set *s =
		olfa_container_of(src, struct olfa_av_set, set_fid);
	size_t front = 0;

	for (size_t i = 0; i < s->count; i++) {
		long j = olfa_index(d->addr + front, d->count - front, s->addr[i]);

		if (j >= 0) {
			fi_addr_t t = d->addr[front];

			d->addr[front] = d->addr[front + (size_t)j];
			d->addr[front + (size_t)j] = t;
			front++;
		}
	}
	d->count = front;
	return 0;
}

static int olfa_set_diff(struct fid_av_set *dst, const struct fid_av_set *src)
{
	struct olfa_av_set *d = olfa_container_of(dst, struct olfa_av_set, set_fid);
	const struct olfa_av_set *s =
		olfa_container_of(src, struct olfa_av_set, set_fid);

	for (size_t i = 0; i < s->count; i++) {
		long j = olfa_index(d->addr, d->count, s->addr[i]);

		if (j >= 0)
			d->addr[j] = d->addr[--d->count];
	}
	return 0;
}

/* coll_av_set_addr: the set's own group address (coll_av_set.c); usable
 * once a world join over this set has completed. */
static int olfa_set_addr(struct fid_av_set *set, fi_addr_t *coll_addr)
{
	struct olfa_av_set *s = olfa_container_of(set, struct olfa_av_set, set_fid);

	if (!coll_addr)
		return -FI_EINVAL;
	*coll_addr = (fi_addr_t)(uintptr_t)&s->set_mc;
	return 0;
}

static struct fi_ops_av_set olfa_set_ops = {
	.size = sizeof(struct fi_ops_av_set),
	.set_union = olfa_set_union,
	.intersect = olfa_set_intersect,
	.diff = olfa_set_diff,
	.insert = olfa_set_insert,
	.remove = olfa_set_remove,
	.addr = olfa_set_addr,
};

static int olfa_set_close(struct fid *fid)
{
	struct olfa_av_set *s = olfa_container_of(fid, struct olfa_av_set, set_fid.fid);

	if (s->set_mc.ep) {
		pthread_mutex_lock(&s->set_mc.ep->lock);
		olfa_mc_unregister(s->set_mc.ep, &s->set_mc);
		pthread_mutex_unlock(&s->set_mc.ep->lock);
	}
	free(s->set_mc.members);
	free(s->addr);
	free(s);
	return 0;
}

static struct fi_ops olfa_set_fi_ops = OLFA_FI_OPS(olfa_set_close, olfa_no_bind,
						   olfa_no_control);

/* coll_av_set (coll_av_set.c:208-290) */
static int olfa_av_set(struct fid_av *av_fid, struct fi_av_set_attr *attr,
		       struct fid_av_set **set_fid, void *context)
{
	struct olfa_av *av = olfa_container_of(av_fid, struct olfa_av, av_fid);
	struct fi_av_attr av_attr;
	struct olfa_av_set *s;
	int ret;

	if (!attr || !set_fid)
		return -FI_EINVAL;
	memset(&av_attr, 0, sizeof(av_attr));
	ret = av->peer_av->owner_ops->query(av->peer_av, &av_attr);
	if (ret)
		return ret;
	s = calloc(1, sizeof(*s));
	if (!s)
		return -FI_ENOMEM;
	s->av = av;
	if (olfa_set_grow(s, attr->count ? attr->count : (av_attr.count ? av_attr.count : 1))) {
		free(s);
		return -FI_ENOMEM;
	}
	if (attr->start_addr != FI_ADDR_NOTAVAIL &&
	    attr->end_addr != FI_ADDR_NOTAVAIL) {
		size_t max = attr->count ? attr->count : av_attr.count;

		if (!attr->stride) {
			ret = -FI_EINVAL;
			goto err;
		}
		for (fi_addr_t a = attr->start_addr; a <= attr->end_addr;
		     a += attr->stride) {
			if (s->count >= max) {          /* coll_av_set.c:245-252 */
				ret = -FI_EINVAL;
				goto err;
			}
			s->addr[s->count++] = a;
		}
	} else if (attr->start_addr != attr->end_addr) {
		ret = -FI_EINVAL;                   /* coll_av_set.c:255-262 */
		goto err;
	}
	s->set_fid.fid.fclass = FI_CLASS_AV_SET;
	s->set_fid.fid.context = context;
	s->set_fid.fid.ops = &olfa_set_fi_ops;
	s->set_fid.ops = &olfa_set_ops;
	s->set_mc.mc_fid.fid.fclass = FI_CLASS_MC;
	s->set_mc.mc_fid.fi_addr = (fi_addr_t)(uintptr_t)&s->set_mc;
	s->set_mc.laddr = LFA_ADDR_NOTAVAIL;
	*set_fid = &s->set_fid;
	return 0;
err:
	free(s->addr);
	free(s);
	return ret;
}

/* ------------------------------------------------------------------ AV -- */

static int olfa_av_close(struct fid *fid)
{
	free(olfa_container_of(fid, struct olfa_av, av_fid.fid));
	return 0;
}

static struct fi_ops olfa_av_fi_ops = OLFA_FI_OPS(olfa_av_close, olfa_no_bind,
						  olfa_no_control);

/* Address insertion belongs to the owner's AV (peer AV protocol). */
static int olfa_av_insert(struct fid_av *av, const void *addr, size_t count,
			  fi_addr_t *fi_addr, uint64_t flags, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_av_insertsvc(struct fid_av *av, const char *node,
			     const char *service, fi_addr_t *fi_addr,
			     uint64_t flags, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_av_insertsym(struct fid_av *av, const char *node, size_t nodecnt,
			     const char *service, size_t svccnt, fi_addr_t *fi_addr,
			     uint64_t flags, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_av_remove(struct fid_av *av, fi_addr_t *fi_addr, size_t count,
			  uint64_t flags)
{
	return -FI_ENOSYS;
}
static int olfa_av_lookup(struct fid_av *av, fi_addr_t fi_addr, void *addr,
			  size_t *addrlen)
{
	return -FI_ENOSYS;
}
static const char *olfa_av_straddr(struct fid_av *av, const void *addr,
				   char *buf, size_t *len)
{
	return NULL;
}
static int olfa_av_insert_auth_key(struct fid_av *av, const void *auth_key,
				   size_t auth_key_size, fi_addr_t *fi_addr,
				   uint64_t flags)
{
	return -FI_ENOSYS;
}
static int olfa_av_lookup_auth_key(struct fid_av *av, fi_addr_t fi_addr,
				   void *auth_key, size_t *auth_key_size)
{
	return -FI_ENOSYS;
}
static int olfa_av_set_user_id(struct fid_av *av, fi_addr_t fi_addr,
			       fi_addr_t user_id, uint64_t flags)
{
	return -FI_ENOSYS;
}
static int olfa_av_lookup2(struct fid_av *av, fi_addr_t fi_addr, void *buf,
			   size_t *len, uint64_t flags, struct fid_xpu_ctx *ctx)
{
	return -FI_ENOSYS;
}

static struct fi_ops_av olfa_av_ops = {
	.size = sizeof(struct fi_ops_av),
	.insert = olfa_av_insert,
	.insertsvc = olfa_av_insertsvc,
	.insertsym = olfa_av_insertsym,
	.remove = olfa_av_remove,
	.lookup = olfa_av_lookup,
	.straddr = olfa_av_straddr,
	.av_set = olfa_av_set,
	.insert_auth_key = olfa_av_insert_auth_key,
	.lookup_auth_key = olfa_av_lookup_auth_key,
	.set_user_id = olfa_av_set_user_id,
	.lookup2 = olfa_av_lookup2,
};

/* coll_av_open (coll_av.c:68-106) */
static int olfa_av_open(struct fid_domain *domain, struct fi_av_attr *attr,
			struct fid_av **av_fid, void *context)
{
	struct fi_peer_av_context *pc = context;
	struct olfa_av *av;

	if (!attr || !(attr->flags & FI_PEER))
		return -FI_EINVAL;
	if (!pc || pc->size < sizeof(*pc) || !pc->av)
		return -FI_EINVAL;
	av = calloc(1, sizeof(*av));
	if (!av)
		return -FI_ENOMEM;
	av->av_fid.fid.fclass = FI_CLASS_AV;
	av->av_fid.fid.context = context;
	av->av_fid.fid.ops = &olfa_av_fi_ops;
	av->av_fid.ops = &olfa_av_ops;
	av->peer_av = pc->av;
	*av_fid = &av->av_fid;
	return 0;
}

/* -------------------------------------------------------------- domain -- */

/* coll_query_collective semantics, with REDUCE / REDUCE_SCATTER added
 * (lfa_query_collective; the enums are libfabric's). */
static int olfa_query_collective(struct fid_domain *domain,
				 enum fi_collective_op coll,
				 struct fi_collective_attr *attr, uint64_t flags)
{
	struct lfa_collective_attr la;
	int ret;

	if (!attr)
		return -FI_EINVAL;
	memset(&la, 0, sizeof(la));
	la.op = (enum lfa_op)attr->op;
	la.datatype = (enum lfa_datatype)attr->datatype;
	la.datatype_attr.count = attr->datatype_attr.count;
	la.datatype_attr.size = attr->datatype_attr.size;
	la.max_members = attr->max_members;
	la.mode = attr->mode;
	ret = lfa_query_collective(NULL, (enum lfa_collective_op)coll, &la, flags);
	if (ret)
		return ret;
	attr->datatype_attr.count = la.datatype_attr.count;
	attr->datatype_attr.size = la.datatype_attr.size;
	attr->max_members = la.max_members;
	return 0;
}

static int olfa_domain_close(struct fid *fid)
{
	free(olfa_container_of(fid, struct olfa_domain, domain_fid.fid));
	return 0;
}

static struct fi_ops olfa_domain_fi_ops = OLFA_FI_OPS(olfa_domain_close,
						      olfa_no_bind,
						      olfa_no_control);

static int olfa_scalable_ep(struct fid_domain *domain, struct fi_info *info,
			    struct fid_ep **sep, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_cntr_open(struct fid_domain *domain, struct fi_cntr_attr *attr,
			  struct fid_cntr **cntr, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_poll_open(struct fid_domain *domain, struct fi_poll_attr *attr,
			  struct fid_poll **pollset)
{
	return -FI_ENOSYS;
}
static int olfa_stx_ctx(struct fid_domain *domain, struct fi_tx_attr *attr,
			struct fid_stx **stx, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_srx_ctx(struct fid_domain *domain, struct fi_rx_attr *attr,
			struct fid_ep **rx_ep, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_query_atomic(struct fid_domain *domain, enum fi_datatype datatype,
			     enum fi_op op, struct fi_atomic_attr *attr,
			     uint64_t flags)
{
	return -FI_ENOSYS;
}
static int olfa_endpoint2(struct fid_domain *domain, struct fi_info *info,
			  struct fid_ep **ep, uint64_t flags, void *context)
{
	if (flags)
		return -FI_EBADFLAGS;
	return olfa_endpoint(domain, info, ep, context);
}
static int olfa_xpu_ctx(struct fid_domain *domain, struct fi_xpu_attr *attr,
			struct fid_xpu_ctx **ctx, void *context)
{
	return -FI_ENOSYS;
}

static struct fi_ops_domain olfa_domain_ops = {
	.size = sizeof(struct fi_ops_domain),
	.av_open = olfa_av_open,
	.cq_open = olfa_cq_open,
	.endpoint = olfa_endpoint,
	.scalable_ep = olfa_scalable_ep,
	.cntr_open = olfa_cntr_open,
	.poll_open = olfa_poll_open,
	.stx_ctx = olfa_stx_ctx,
	.srx_ctx = olfa_srx_ctx,
	.query_atomic = olfa_query_atomic,
	.query_collective = olfa_query_collective,
	.endpoint2 = olfa_endpoint2,
	.xpu_ctx = olfa_xpu_ctx,
};

/* coll_domain_open2 (coll_domain.c:80-108): FI_PEER only */
static int olfa_domain2(struct fid_fabric *fabric, struct fi_info *info,
			struct fid_domain **dom, uint64_t flags, void *context)
{
	struct fi_peer_domain_context *pc = context;
	struct olfa_domain *d;

	if (!(flags & FI_PEER))
		return -FI_EINVAL;
	if (!pc || pc->size < sizeof(*pc))
		return -FI_EINVAL;
	d = calloc(1, sizeof(*d));
	if (!d)
		return -FI_ENOMEM;
	d->domain_fid.fid.fclass = FI_CLASS_DOMAIN;
	d->domain_fid.fid.context = context;
	d->domain_fid.fid.ops = &olfa_domain_fi_ops;
	d->domain_fid.ops = &olfa_domain_ops;
	d->peer_domain = pc->domain;
	*dom = &d->domain_fid;
	return 0;
}

static int olfa_domain(struct fid_fabric *fabric, struct fi_info *info,
		       struct fid_domain **dom, void *context)
{
	return olfa_domain2(fabric, info, dom, 0, context);
}

/* -------------------------------------------------------------- fabric -- */

static int olfa_fabric_close(struct fid *fid)
{
	free(olfa_container_of(fid, struct olfa_fabric, fabric_fid.fid));
	return 0;
}

static struct fi_ops olfa_fabric_fi_ops = OLFA_FI_OPS(olfa_fabric_close,
						      olfa_no_bind,
						      olfa_no_control);

static int olfa_passive_ep(struct fid_fabric *fabric, struct fi_info *info,
			   struct fid_pep **pep, void *context)
{
	return -FI_ENOSYS;
}
static int olfa_wait_open(struct fid_fabric *fabric, struct fi_wait_attr *attr,
			  struct fid_wait **waitset)
{
	return -FI_ENOSYS;
}
static int olfa_trywait(struct fid_fabric *fabric, struct fid **fids, int count)
{
	return -FI_ENOSYS;
}

static struct fi_ops_fabric olfa_fabric_ops = {
	.size = sizeof(struct fi_ops_fabric),
	.domain = olfa_domain,
	.passive_ep = olfa_passive_ep,
	.eq_open = olfa_eq_open,
	.wait_open = olfa_wait_open,
	.trywait = olfa_trywait,
	.domain2 = olfa_domain2,
};

static int olfa_fabric(struct fi_fabric_attr *attr, struct fid_fabric **fabric,
		       void *context)
{
	struct olfa_fabric *f;

	if (!attr || !fabric)
		return -FI_EINVAL;
	if (attr->name && strcmp(attr->name, OFF_LFA_PROV_NAME))
		return -FI_ENODATA;
	f = calloc(1, sizeof(*f));
	if (!f)
		return -FI_ENOMEM;
	f->fabric_fid.fid.fclass = FI_CLASS_FABRIC;
	f->fabric_fid.fid.context = context;
	f->fabric_fid.fid.ops = &olfa_fabric_fi_ops;
	f->fabric_fid.ops = &olfa_fabric_ops;
	f->fabric_fid.api_version = attr->api_version;
	*fabric = &f->fabric_fid;
	return 0;
}

static void olfa_cleanup(void)
{
}

static struct fi_provider olfa_prov = {
	.version = OLFA_VERSION,
	.fi_version = FI_VERSION(FI_MAJOR_VERSION, FI_MINOR_VERSION),
	.name = OFF_LFA_PROV_NAME,
	.getinfo = olfa_getinfo,
	.fabric = olfa_fabric,
	.cleanup = olfa_cleanup,
};

FI_EXT_INI
{
	olfa_params_init(&olfa_prov);
	return &olfa_prov;
}

/* For hosts that did not get the fi_info from the core (tests, embedders):
 * releases what getinfo returned, as the core's fi_freeinfo would. */
__attribute__((visibility("default"))) void off_lfa_freeinfo(struct fi_info *info)
{
	olfa_freeinfo(info);
}

/* Test accessor: the addresses of an av_set of this provider in the order a
 * join numbers them (group rank = index).  fi_av_set has no listing call;
 * the av_set algebra tests read the order the set calls left through this.
 * Returns the member count (the first `cap` are copied), or -FI_EINVAL. */
__attribute__((visibility("default"))) long off_lfa_test_set_order(struct fid_av_set *set,
								    fi_addr_t *out,
								    size_t cap)
{
	const struct olfa_av_set *s;

	if (!set || set->fid.fclass != FI_CLASS_AV_SET || (!out && cap))
		return -FI_EINVAL;
	s = olfa_container_of(set, struct olfa_av_set, set_fid);
	for (size_t i = 0; i < s->count && i < cap; i++)
		out[i] = s->addr[i];
	return (long)s->count;
}
