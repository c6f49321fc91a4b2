/*
 * off_lfa_int.h — internal types of the off_lfa provider (liboff_lfa-fi.so),
 * shared by off_lfa.c (parameters, fi_info, fabric / domain, CQ, EQ, AV,
 * av_set, the provider struct) and off_lfa_ep.c (endpoint, progress,
 * bootstrap, joins, the fi_ops_collective slots).  Split in round 6.  Not
 * installed.
 */
#ifndef OFF_LFA_INT_H
#define OFF_LFA_INT_H

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

#include "lfa_atomic.h"
#include "lfa_coll.h"
#include "off_lfa.h"

#define OLFA_VERSION FI_VERSION(0, 3)
#define OLFA_CAPS (FI_COLLECTIVE | FI_HMEM)
#define olfa_container_of(ptr, type, field) \
	((type *)((char *)(ptr) - offsetof(type, field)))
#define OLFA_INTERNAL __attribute__((visibility("hidden")))

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
	/* joins between their lfa_join_* call and their registration: a join
	 * that completes at once (a one-member group) can post its event
	 * before its group is registered, and progress holds such an event
	 * (under plock) until the group is there instead of posting it
	 * fid-less (olfa_post_join) */
	atomic_int joins_in_flight;
	int have_held;
	struct lfa_eq_entry held;

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

#define OLFA_FI_OPS(close_fn, bind_fn, control_fn) {                      \
	.size = sizeof(struct fi_ops), .close = close_fn, .bind = bind_fn, \
	.control = control_fn, .ops_open = olfa_no_ops_open,                \
	.tostr = olfa_no_tostr, .ops_set = olfa_no_ops_set }

/* Entry points shared by the two translation units. */
OLFA_INTERNAL int olfa_no_ops_open(struct fid *fid, const char *name, uint64_t flags,
			    void **ops, void *context);
OLFA_INTERNAL int olfa_no_tostr(const struct fid *fid, char *buf, size_t len);
OLFA_INTERNAL int olfa_no_ops_set(struct fid *fid, const char *name, uint64_t flags,
			   void *ops, void *context);
OLFA_INTERNAL const char *olfa_param(const char *name);
OLFA_INTERNAL int olfa_param_int(const char *name, int dflt);
OLFA_INTERNAL void olfa_warn(const char *fmt, const char *arg, long v);
OLFA_INTERNAL int olfa_no_bind(struct fid *fid, struct fid *bfid, uint64_t flags);
OLFA_INTERNAL int olfa_no_control(struct fid *fid, int command, void *arg);
OLFA_INTERNAL int olfa_av_set(struct fid_av *av_fid, struct fi_av_set_attr *attr,
		       struct fid_av_set **set_fid, void *context);
OLFA_INTERNAL int olfa_domain(struct fid_fabric *fabric, struct fi_info *info,
		       struct fid_domain **dom, void *context);
OLFA_INTERNAL void olfa_mc_unregister(struct olfa_ep *ep, struct olfa_mc *m);
OLFA_INTERNAL int olfa_progress(struct olfa_ep *ep);
OLFA_INTERNAL long olfa_index(const fi_addr_t *list, size_t n, fi_addr_t addr);
OLFA_INTERNAL int olfa_endpoint(struct fid_domain *domain, struct fi_info *info,
			 struct fid_ep **ep_fid, void *context);

#endif
