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
#include "off_lfa_int.h"

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
	{ "auto_bulk", FI_PARAM_STRING, "LFA_AUTO_BULK",
	  "algo auto above the one-shot bounds: p2p (default: the two-barrier schedule over the xGMI mesh, the tree's bits) or tree; provisional" },
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
OLFA_INTERNAL const char *olfa_param(const char *name)
{
	for (size_t i = 0; i < OLFA_NPARAMS; i++)
		if (!strcmp(olfa_params[i].name, name))
			return olfa_param_isset[i] ? olfa_param_val[i] : NULL;
	return NULL;
}

OLFA_INTERNAL int olfa_param_int(const char *name, int dflt)
{
	const char *v = olfa_param(name);

	return v && *v ? atoi(v) : dflt;
}

static int olfa_debug = -1;

OLFA_INTERNAL void olfa_warn(const char *fmt, const char *arg, long v)
{
	if (olfa_debug < 0)
		olfa_debug = olfa_param("debug") && strcmp(olfa_param("debug"), "0");
	if (olfa_debug)
		fprintf(stderr, "off_lfa: %s %s (%ld)\n", fmt, arg ? arg : "", v);
}

/* -------------------------------------------------------- enosys stubs -- */

OLFA_INTERNAL int olfa_no_bind(struct fid *fid, struct fid *bfid, uint64_t flags)
{
	return -FI_ENOSYS;
}
OLFA_INTERNAL int olfa_no_control(struct fid *fid, int command, void *arg)
{
	return -FI_ENOSYS;
}
OLFA_INTERNAL int olfa_no_ops_open(struct fid *fid, const char *name, uint64_t flags,
			    void **ops, void *context)
{
	return -FI_ENOSYS;
}
OLFA_INTERNAL int olfa_no_tostr(const struct fid *fid, char *buf, size_t len)
{
	return -FI_ENOSYS;
}
OLFA_INTERNAL int olfa_no_ops_set(struct fid *fid, const char *name, uint64_t flags,
			   void *ops, void *context)
{
	return -FI_ENOSYS;
}


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
OLFA_INTERNAL int olfa_av_set(struct fid_av *av_fid, struct fi_av_set_attr *attr,
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

OLFA_INTERNAL int olfa_domain(struct fid_fabric *fabric, struct fi_info *info,
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
