/*
 * lfa_coll_ws.c — the LFA_ALGO_P2P symmetric workspaces (liblfa_coll.so;
 * split out of lfa_coll.c in round 6): allocation (LFA_WS_MEM, uncached by
 * default), the process-wide cache and quarantine of exported workspaces,
 * the IPC handshake (export, the members' allgather of handles, mapping,
 * identity check, MIN agreement), and a group's P2P state (tickets, the
 * timed-out status word).  These replace prov/coll's transfers through the
 * owner provider (coll_coll.c:770-814) on device buffers.
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

LFA_INTERNAL void sig_word_free(struct lfa_coll_mc *mc)
{
	if (mc->sig_word)
		hipHostFree(mc->sig_word);
	mc->sig_word = NULL;
}

/*
 * Before a P2P operation of `mc`: its timed-out-wait word exists (allocated
 * at the group's first P2P operation: host-mapped, LFA_SIG_NONE) and no wait
 * of the group has timed out — after one the members' flag epochs disagree
 * and a barrier could pass on stale posts, so the group refuses P2P
 * operations (close and re-join it); other groups are unaffected.
 */
LFA_INTERNAL int sig_ready(struct lfa_coll_mc *mc)
{
	if (mc->sig_failed)
		return -LFA_EIO;
	if (!mc->sig_word) {
		hipSetDevice(mc->ep->dom->device);
		if (hipHostMalloc((void **)&mc->sig_word, sizeof(uint64_t),
				  hipHostMallocCoherent) != hipSuccess) {
			mc->sig_word = NULL;
			return -LFA_ENOMEM;
		}
		*(volatile uint64_t *)mc->sig_word = LFA_SIG_NONE;
	}
	if (*(volatile uint64_t *)mc->sig_word != LFA_SIG_NONE)
		return -LFA_EIO;
	return 0;
}

/* The operation just queued ran P2P kernels on `mc` if its ticket moved. */
LFA_INTERNAL void tag_p2p(struct lfa_coll_ep *ep, struct lfa_coll_mc *mc, uint64_t t0)
{
	struct pending *p;

	if (!ep->qlen || mc->p2p_ticket == t0)
		return;
	p = &ep->q[(ep->qhead + ep->qlen - 1) % ep->qcap];
	p->pmc = mc;
	p->ticket = mc->p2p_ticket;
}

/* Did a P2P wait of this operation, or of an earlier one of its group, time
 * out?  (The group's kernels run in order; the word holds the lowest failing
 * ticket.) */
LFA_INTERNAL int p2p_timed_out(const struct pending *p)
{
	if (p->timed_out)
		return 1;
	return p->pmc && p->ticket && p->pmc->sig_word &&
	       *(volatile uint64_t *)p->pmc->sig_word <= p->ticket;
}

int lfa_mc_seed_ticket(struct lfa_coll_ep *ep, lfa_addr_t coll_addr, uint64_t ticket)
{
	struct lfa_coll_mc *mc;
	int ret = 0;

	if (!ep)
		return -LFA_EINVAL;
	mc = mc_of(ep, coll_addr);
	if (!mc)
		return -LFA_EINVAL;
	pthread_mutex_lock(&ep->lock);
	if (ep->qlen)
		ret = -LFA_EINVAL;
	else
		mc->p2p_ticket = ticket;
	pthread_mutex_unlock(&ep->lock);
	return ret;
}

int lfa_mc_ws_info(struct lfa_coll_ep *ep, lfa_addr_t coll_addr, struct lfa_ws_info *out)
{
	struct lfa_coll_mc *mc;
	int ret = 0;

	if (!ep || !out)
		return -LFA_EINVAL;
	mc = mc_of(ep, coll_addr);
	memset(out, 0, sizeof(*out));
	out->mem = lfa_coll_ws_mem();
	pthread_mutex_lock(&ep->comm_lock);
	out->region = mc->sym_region;
	for (int k = 0; mc->sym && k < mc->size && k < LFA_SIG_MAX && !ret; k++) {
		hipPointerAttribute_t at;

		memset(&at, 0, sizeof(at));
		if (!mc->sym[k])
			continue;
		if (hipPointerGetAttributes(&at, mc->sym[k]) != hipSuccess) {
			(void)hipGetLastError();
			ret = -LFA_EIO;
			break;
		}
		out->alloc_flags[k] = at.allocationFlags;
		out->mapped++;
	}
	pthread_mutex_unlock(&ep->comm_lock);
	return ret;
}



/* Open file descriptors of this process (LFA_DEBUG diagnostics: every
 * exported or imported IPC workspace holds a dma-buf descriptor). */
static int open_fds(void)
{
	DIR *d = opendir("/proc/self/fd");
	int n = 0;

	if (!d)
		return -1;
	while (readdir(d))
		n++;
	closedir(d);
	return n - 3;   /* ".", ".." and the directory's own descriptor */
}

/*
 * LFA_DEBUG: a history of the P2P workspaces' virtual address ranges in this
 * process — 'A'llocated and 'F'reed local workspaces, 'I'mported and 'C'losed
 * peer mappings — so a failed export can be matched against the ranges the
 * same addresses held before (the hipIpcGetMemHandle
 * "invalid argument" seen at a workspace growth).
 */
#define VA_HIST 256
static struct va_ev {
	char kind;
	const void *p;
	size_t bytes;
	unsigned long long seq;
} va_hist[VA_HIST];
static unsigned long long va_n;
static pthread_mutex_t va_lock = PTHREAD_MUTEX_INITIALIZER;

static int va_debug(void)
{
	static int on = -1;

	if (on < 0)
		on = lfa_param("LFA_DEBUG") != NULL;
	return on;
}

static void va_note(char kind, const void *p, size_t bytes)
{
	if (!va_debug() || !p)
		return;
	if (!bytes) {
		void *base = NULL;
		size_t sz = 0;

		if (hipMemGetAddressRange(&base, &sz, (void *)p) == hipSuccess)
			bytes = sz;
		else
			(void)hipGetLastError();
	}
	pthread_mutex_lock(&va_lock);
	va_hist[va_n % VA_HIST] = (struct va_ev){ kind, p, bytes, va_n };
	va_n++;
	pthread_mutex_unlock(&va_lock);
}

/* Everything the history knows about [p, p + bytes), and what HIP says of p. */
static void va_explain(const char *what, const void *p, size_t bytes)
{
	hipPointerAttribute_t at;
	void *base = NULL;
	size_t sz = 0;
	hipError_t e1, e2;

	if (!va_debug())
		return;
	memset(&at, 0, sizeof(at));
	e1 = hipPointerGetAttributes(&at, p);
	e2 = hipMemGetAddressRange(&base, &sz, (void *)p);
	(void)hipGetLastError();
	fprintf(stderr, "lfa: %s: %p + %zu B; attributes rc %d type %d device %d "
		"devptr %p hostptr %p; range rc %d base %p size %zu; %d fds open\n",
		what, p, bytes, (int)e1, (int)at.type, at.device, at.devicePointer,
		at.hostPointer, (int)e2, base, sz, open_fds());
	pthread_mutex_lock(&va_lock);
	for (unsigned long long i = va_n > VA_HIST ? va_n - VA_HIST : 0; i < va_n; i++) {
		const struct va_ev *v = &va_hist[i % VA_HIST];
		const char *a = v->p, *b = p;

		if (a < b + bytes && b < a + v->bytes)
			fprintf(stderr, "lfa:   overlaps event #%llu %c %p + %zu B%s\n", v->seq,
				v->kind, v->p, v->bytes, v->p == p ? " (same base)" : "");
	}
	fprintf(stderr, "lfa:   (%llu workspace events so far)\n", va_n);
	pthread_mutex_unlock(&va_lock);
}

/*
 * Exported workspaces are kept, not freed (LFA_WS_CACHE_BYTES, default
 * 4 GiB per process; 0 frees them as before).  The runtime remembers an
 * exported address after hipFree: a later allocation at that address — the
 * allocator hands freed ranges straight back — is refused an export
 * (hsa_status 4096), or exported with a handle its peers map onto other
 * memory, so the owner waits for posts that land elsewhere (round 4, DESIGN.md
 * §12: tools/probe_ipc_growth.py).  A workspace released by a growth or an
 * endpoint close goes to this cache; the next workspace of the same size on
 * the same device takes it back and exports it again — the same memory
 * under the same address — so no fresh allocation ever lands on an address
 * that was exported while a domain is open.
 *
 * Two kinds of released workspace are never handed out again but held
 * (quarantine, VERDICT r4 #3 / ADVICE r4):
 *   - one whose group had a P2P wait time out: a stalled peer may still run
 *     its old kernel, pushing data and posting its old epoch through its old
 *     mapping; in a reused workspace those posts would satisfy the new
 *     group's waits (its epochs restart at 1) with stale data;
 *   - the least recently used above the cap: returning it to hipFree would
 *     reopen the address hazard above.
 * The quarantine is bounded too (LFA_WS_QUARANTINE_BYTES, default 4 GiB):
 * past it the oldest goes back to hipFree, and a later workspace at that
 * address is caught by the export fallback and the identity check
 * (sym_prepare, sym_open: the growth fails on every member with EIO rather
 * than mapping the wrong memory).  When the last GPU domain of the process
 * closes, every kept workspace is freed (lfa_coll_ws_cached_bytes() and
 * lfa_coll_ws_quarantined_bytes() are then 0).
 */
#define WS_CACHE_SLOTS 64
#define WS_QUAR_SLOTS 256
static struct ws_slot {
	char *p;
	size_t bytes;
	int dev;
	unsigned long long used;
} ws_cache[WS_CACHE_SLOTS], ws_quar[WS_QUAR_SLOTS];
static size_t ws_held, ws_quar_held;
static unsigned long long ws_clock;
static int ws_domains;          /* open domains with a GPU (workspace users) */
static pthread_mutex_t ws_lock = PTHREAD_MUTEX_INITIALIZER;

static size_t env_bytes(const char *name, long long dflt)
{
	const char *e = lfa_param(name);
	long long v = e ? atoll(e) : dflt;

	return v < 0 ? 0 : (size_t)v;
}

static size_t ws_cap(void)
{
	static long long cap = -1;

	if (cap < 0)
		cap = (long long)env_bytes("LFA_WS_CACHE_BYTES", 4ll << 30);
	return (size_t)cap;
}

static size_t ws_quar_cap(void)
{
	static long long cap = -1;

	if (cap < 0)
		cap = (long long)env_bytes("LFA_WS_QUARANTINE_BYTES", 4ll << 30);
	return (size_t)cap;
}

/* A kept workspace of exactly `bytes` on the current device, or NULL. */
static char *ws_take(size_t bytes)
{
	int dev = -1;
	char *p = NULL;

	if (hipGetDevice(&dev) != hipSuccess)
		return NULL;
	pthread_mutex_lock(&ws_lock);
	for (int i = 0; i < WS_CACHE_SLOTS && !p; i++)
		if (ws_cache[i].p && ws_cache[i].bytes == bytes && ws_cache[i].dev == dev) {
			p = ws_cache[i].p;
			ws_cache[i].p = NULL;
			ws_held -= bytes;
		}
	pthread_mutex_unlock(&ws_lock);
	return p;
}

/* Hold `s` in the quarantine (ws_lock held); what leaves it to make room is
 * added to evict[]. */
static void ws_quarantine(struct ws_slot s, char **evict, int *ne)
{
	int slot = -1;

	for (int i = 0; i < WS_QUAR_SLOTS && slot < 0; i++)
		if (!ws_quar[i].p)
			slot = i;
	if (slot < 0) {         /* every slot held: the oldest goes */
		slot = 0;
		for (int i = 1; i < WS_QUAR_SLOTS; i++)
			if (ws_quar[i].used < ws_quar[slot].used)
				slot = i;
		evict[(*ne)++] = ws_quar[slot].p;
		ws_quar_held -= ws_quar[slot].bytes;
	}
	s.used = ++ws_clock;
	ws_quar[slot] = s;
	ws_quar_held += s.bytes;
	while (ws_quar_held > ws_quar_cap()) {
		int old = -1;

		for (int i = 0; i < WS_QUAR_SLOTS; i++)
			if (ws_quar[i].p && (old < 0 || ws_quar[i].used < ws_quar[old].used))
				old = i;
		evict[(*ne)++] = ws_quar[old].p;
		ws_quar_held -= ws_quar[old].bytes;
		ws_quar[old].p = NULL;
	}
}

/* Keep workspace `p` (its whole allocation) for a later ws_take, or — when
 * `tainted` (its group timed out) — in the quarantine, never to be reused. */
static void ws_give(char *p, int tainted)
{
	void *base = NULL;
	size_t bytes = 0;
	int dev = -1, slot = -1;
	char *evict[WS_CACHE_SLOTS + WS_QUAR_SLOTS + 2];
	int ne = 0;

	hipPointerAttribute_t at;

	memset(&at, 0, sizeof(at));
	if ((!ws_cap() && !tainted) || hipMemGetAddressRange(&base, &bytes, p) != hipSuccess ||
	    base != (void *)p || hipPointerGetAttributes(&at, p) != hipSuccess) {
		(void)hipGetLastError();
		hipFree(p);
		return;
	}
	dev = at.device;
	pthread_mutex_lock(&ws_lock);
	if (tainted) {
		ws_quarantine((struct ws_slot){ p, bytes, dev, 0 }, evict, &ne);
		goto out;
	}
	for (int i = 0; i < WS_CACHE_SLOTS && slot < 0; i++)
		if (!ws_cache[i].p)
			slot = i;
	if (slot < 0) {         /* every slot held: the least recently used goes */
		slot = 0;
		for (int i = 1; i < WS_CACHE_SLOTS; i++)
			if (ws_cache[i].used < ws_cache[slot].used)
				slot = i;
		ws_held -= ws_cache[slot].bytes;
		ws_quarantine(ws_cache[slot], evict, &ne);
	}
	ws_cache[slot] = (struct ws_slot){ p, bytes, dev, ++ws_clock };
	ws_held += bytes;
	while (ws_held > ws_cap()) {
		int lru = -1;

		for (int i = 0; i < WS_CACHE_SLOTS; i++)
			if (ws_cache[i].p && i != slot &&
			    (lru < 0 || ws_cache[i].used < ws_cache[lru].used))
				lru = i;
		if (lru < 0)
			lru = slot;
		ws_held -= ws_cache[lru].bytes;
		ws_quarantine(ws_cache[lru], evict, &ne);
		ws_cache[lru].p = NULL;
		if (lru == slot)
			break;
	}
out:
	pthread_mutex_unlock(&ws_lock);
	for (int i = 0; i < ne; i++)
		hipFree(evict[i]);
}

/* A GPU domain opened / closed: the last close frees every kept workspace. */
LFA_INTERNAL void ws_domain_ref(int delta)
{
	char *evict[WS_CACHE_SLOTS + WS_QUAR_SLOTS];
	int ne = 0;

	pthread_mutex_lock(&ws_lock);
	ws_domains += delta;
	if (ws_domains == 0) {
		for (int i = 0; i < WS_CACHE_SLOTS; i++)
			if (ws_cache[i].p) {
				evict[ne++] = ws_cache[i].p;
				ws_cache[i].p = NULL;
			}
		for (int i = 0; i < WS_QUAR_SLOTS; i++)
			if (ws_quar[i].p) {
				evict[ne++] = ws_quar[i].p;
				ws_quar[i].p = NULL;
			}
		ws_held = 0;
		ws_quar_held = 0;
	}
	pthread_mutex_unlock(&ws_lock);
	for (int i = 0; i < ne; i++)
		hipFree(evict[i]);
}

size_t lfa_coll_ws_cached_bytes(void)
{
	size_t n;

	pthread_mutex_lock(&ws_lock);
	n = ws_held;
	pthread_mutex_unlock(&ws_lock);
	return n;
}

size_t lfa_coll_ws_quarantined_bytes(void)
{
	size_t n;

	pthread_mutex_lock(&ws_lock);
	n = ws_quar_held;
	pthread_mutex_unlock(&ws_lock);
	return n;
}

/* A P2P wait of the group timed out (reaped, or recorded by a kernel in the
 * status word): its workspace may still receive a stalled peer's posts. */
static int mc_tainted(const struct lfa_coll_mc *mc)
{
	return mc->sig_failed ||
	       (mc->sig_word && *(volatile uint64_t *)mc->sig_word != LFA_SIG_NONE);
}

/* Unmap the peers' workspaces in `sym` and release this rank's `local`. */
static void sym_free(const struct lfa_coll_mc *mc, char **sym, char *local)
{
	if (sym) {
		for (int k = 0; k < mc->size; k++)
			if (k != mc->rank && sym[k]) {
				va_note('C', sym[k], 0);
				hipIpcCloseMemHandle(sym[k]);
			}
		free(sym);
	}
	if (local) {
		va_note('F', local, 0);
		ws_give(local, mc_tainted(mc));
	}
}

/* A new identity word: this process, a count, the clock. */
static uint64_t ws_identity(void)
{
	static uint64_t n;
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ((uint64_t)getpid() << 40) ^ ((uint64_t)__atomic_add_fetch(&n, 1, __ATOMIC_RELAXED) << 24) ^
	       (uint64_t)ts.tv_nsec ^ ((uint64_t)ts.tv_sec << 30) ^ 1;
}

/*
 * The memory a P2P workspace is allocated from (LFA_WS_MEM, read once per
 * process; every member of a group must use the same kind).  Peers write
 * every byte a member reads from its own workspace — the posted epochs, the
 * one-shot slots, the pushed blocks — over xGMI while the member's kernels
 * run, so the workspace is allocated UNCACHED by default
 * (hipExtMallocWithFlags(hipDeviceMallocUncached), MTYPE UC in the GPU page
 * tables of the owner AND of every peer that maps it): no L2 of any GPU ever
 * holds a line of it, so a post or a push is visible to the owner's next
 * load whatever cache state the owner's earlier accesses left.  HIP's
 * default device memory is coarse-grained: its coherence is only guaranteed
 * at kernel boundaries and synchronisation points, which is exactly what a
 * flag polled inside a running kernel does not have.
 *   uncached (default)  hipDeviceMallocUncached
 *   fine                hipDeviceMallocFinegrained
 *   coarse              hipMalloc's memory (rounds 1-5; A/B only)
 */
int lfa_coll_ws_mem(void)
{
	static int f = -1;

	if (f < 0) {
		const char *e = lfa_param("LFA_WS_MEM");

		f = !e || !*e || !strcmp(e, "uncached") ? hipDeviceMallocUncached :
		    !strcmp(e, "fine") ? hipDeviceMallocFinegrained :
		    !strcmp(e, "coarse") ? hipDeviceMallocDefault : hipDeviceMallocUncached;
	}
	return f;
}

static hipError_t ws_malloc(char **p, size_t bytes)
{
	return hipExtMallocWithFlags((void **)p, bytes, (unsigned)lfa_coll_ws_mem());
}

/* A workspace of 2·region + the flag area: a kept one of that size, else a
 * new allocation of LFA_WS_MEM's kind. */
static hipError_t ws_alloc(char **p, size_t region)
{
	const size_t bytes = 2 * region + LFA_SIG_AREA_BYTES;

	*p = ws_take(bytes);
	if (*p)
		return hipSuccess;
	return ws_malloc(p, bytes);
}

/* The flag area zeroed (epoch 0) and the identity word written, before any
 * peer can learn the handle and post into it (the agreement follows). */
static int ws_reset(struct lfa_coll_mc *mc, char *local, size_t region, uint64_t id,
		    int *why)
{
	char *area = local + 2 * region;

	return lfa_hip_note(why, hipMemsetAsync(area, 0, LFA_SIG_AREA_BYTES, mc->ep->stream),
			    "P2P flag area memset") == hipSuccess &&
	       lfa_hip_note(why, hipMemcpyAsync(area + LFA_SIG_ID_OFF, &id, sizeof(id),
						hipMemcpyHostToDevice, mc->ep->stream),
			    "P2P identity word") == hipSuccess &&
	       lfa_hip_note(why, hipStreamSynchronize(mc->ep->stream),
			    "P2P flag area sync") == hipSuccess;
}

LFA_INTERNAL void p2p_release(struct lfa_coll_mc *mc)
{
	sym_free(mc, mc->sym, mc->sym_local);
	mc->sym = NULL;
	mc->sym_local = NULL;
	mc->sym_region = 0;
}

_Static_assert(sizeof(struct sym_rec) <= LFA_SYM_REC_BYTES, "sym_rec");

/* The workspace size p2p_ensure grows to for a need of `region` bytes. */
LFA_INTERNAL size_t sym_grow(const struct lfa_coll_mc *mc, size_t region)
{
	if (region < 2 * mc->sym_region)
		region = 2 * mc->sym_region;
	if (region < (8u << 20))
		region = 8u << 20;
	return (region + (2u << 20) - 1) & ~(size_t)((2u << 20) - 1);
}

/*
 * p2p_ensure in three local parts around two agreements.  A local failure
 * (no memory for the new workspace or its peer table, no IPC handle) is not
 * returned before the agreements: this rank still takes part with ok = 0, so
 * every member fails together instead of leaving its peers waiting (ADVICE
 * r1).  `ok` comes in false when the old workspace could not be quiesced.
 */
LFA_INTERNAL void sym_prepare(struct lfa_coll_mc *mc, size_t region, int ok,
			struct sym_rec *mine, int *why)
{
	int n = mc->size;
	char **old_sym = mc->sym, *old_local = mc->sym_local;

	/* the new workspace is allocated and exported while the old one is
	 * still held, so its IPC handle can never repeat the old one's (an
	 * exporter resource freed and reused at once); the old mappings and
	 * memory go right after */
	mc->sym = NULL;
	mc->sym_local = NULL;
	mc->sym_region = 0;
	memset(mine, 0, sizeof(*mine));
	mc->sym = calloc((size_t)n, sizeof(*mc->sym));
	ok = ok && mc->sym;
	ok = ok && lfa_hip_note(why, ws_alloc(&mc->sym_local, region),
				"P2P workspace allocation") == hipSuccess;
	if (!ok)
		mc->sym_local = NULL;
	mine->id = ws_identity();
	ok = ok && ws_reset(mc, mc->sym_local, region, mine->id, why);
	/* every member grows at the same operation: the epochs restart with the
	 * zeroed flags, so a count past 2^31 never meets a zero word that reads
	 * as "ahead"  */
	mc->bar_epoch = 0;
	mc->os_epoch = 0;
	if (ok)
		va_note('A', mc->sym_local, 2 * region + LFA_SIG_AREA_BYTES);
	if (ok && n > 1 && hipIpcGetMemHandle(&mine->h, mc->sym_local) != hipSuccess) {
		/*
		 * The runtime refuses to export some fresh allocations: ROCr's IPC
		 * create returns HSA_STATUS_ERROR (AMD_LOG_LEVEL=1: "Failed to
		 * create memory for IPC, failed with hsa_status: 4096"), which
		 * hipIpcGetMemHandle reports as "invalid argument".  Round 4 pinned
		 * it down (tools/probe_ipc_growth.py): 2 to 8 of
		 * 384 to 768 exports; the allocation is ordinary (device memory,
		 * its own base and size), the SAME allocation fails on every retry,
		 * and a replacement allocated after freeing it lands at the same
		 * address and can fail again — the failure follows the address,
		 * which earlier workspaces of this process held and exported.  So
		 * the replacement is allocated while the refused allocation is
		 * still held, which gives it another address, and the refused ones
		 * are freed afterwards; after LFA_EXPORT_TRIES the growth fails on
		 * every member (the agreement below).  With the workspace cache
		 * (ws_give) no fresh allocation lands on a once-exported address,
		 * and this path is the fallback for LFA_WS_CACHE_BYTES=0 and for
		 * workspaces evicted above the cap.
		 */
		hipError_t e = hipGetLastError();
		char *refused[LFA_EXPORT_TRIES];
		int nref = 0;

		if (va_debug()) {
			fprintf(stderr, "lfa: P2P workspace export failed (%s)\n",
				hipGetErrorString(e));
			va_explain("failed export", mc->sym_local,
				   2 * region + LFA_SIG_AREA_BYTES);
		}
		ok = 0;
		while (!ok && mc->sym_local && nref < LFA_EXPORT_TRIES) {
			refused[nref++] = mc->sym_local;
			mc->sym_local = NULL;
			ok = lfa_hip_note(why, ws_malloc(&mc->sym_local,
							 2 * region + LFA_SIG_AREA_BYTES),
					  "P2P workspace allocation (replacement)") == hipSuccess;
			if (!ok) {
				mc->sym_local = NULL;
				break;
			}
			va_note('A', mc->sym_local, 2 * region + LFA_SIG_AREA_BYTES);
			ok = ws_reset(mc, mc->sym_local, region, mine->id, why) &&
			     hipIpcGetMemHandle(&mine->h, mc->sym_local) == hipSuccess;
			if (!ok)
				(void)hipGetLastError();
			if (va_debug())
				va_explain(ok ? "replacement exported" : "replacement refused",
					   mc->sym_local, 2 * region + LFA_SIG_AREA_BYTES);
		}
		if (!ok) {
			lfa_hip_note(why, hipErrorInvalidValue, "P2P workspace hipIpcGetMemHandle");
			if (mc->sym_local) {
				va_note('F', mc->sym_local, 0);
				hipFree(mc->sym_local);
				mc->sym_local = NULL;
			}
		}
		for (int i = 0; i < nref; i++) {
			va_note('F', refused[i], 0);
			hipFree(refused[i]);
		}
	}
	mine->ok = ok;
	sym_free(mc, old_sym, old_local);
}

/* FNV-1a of an IPC handle (LFA_DEBUG lines). */
static uint64_t handle_digest(const hipIpcMemHandle_t *h)
{
	const unsigned char *b = (const unsigned char *)h;
	uint64_t x = 0xcbf29ce484222325ull;

	for (size_t i = 0; i < sizeof(*h); i++)
		x = (x ^ b[i]) * 0x100000001b3ull;
	return x;
}

/* Every member's record in hand: map the peers' workspaces of 2·region + the
 * flag area, and read each one's identity word through the mapping — a
 * mapping onto any other memory fails the handshake on every member (the
 * agreement) instead of leaving its owner waiting for posts that land
 * elsewhere. */
LFA_INTERNAL int sym_open(struct lfa_coll_mc *mc, const struct sym_rec *recs, size_t region,
		    int *why)
{
	int ret = 0;

	for (int k = 0; k < mc->size && !ret; k++)
		if (!recs[k].ok)
			ret = -LFA_ENOMEM;
	for (int k = 0; k < mc->size && !ret; k++) {
		if (k == mc->rank) {
			mc->sym[k] = mc->sym_local;
		} else if (lfa_hip_note(why, hipIpcOpenMemHandle((void **)&mc->sym[k], recs[k].h,
								  hipIpcMemLazyEnablePeerAccess),
					"P2P hipIpcOpenMemHandle") != hipSuccess) {
			mc->sym[k] = NULL;
			ret = -LFA_EIO;
		} else {
			uint64_t id = 0;

			va_note('I', mc->sym[k], 0);
			/* on the endpoint's stream (idle here: the growth synchronised
			 * it), not the null stream, which would wait for the
			 * application's own queued work */
			if (lfa_hip_note(why, hipMemcpyAsync(&id, mc->sym[k] + 2 * region +
								     LFA_SIG_ID_OFF, sizeof(id),
							     hipMemcpyDeviceToHost, mc->ep->stream),
					 "P2P identity read") != hipSuccess ||
			    lfa_hip_note(why, hipStreamSynchronize(mc->ep->stream),
					 "P2P identity read sync") != hipSuccess) {
				ret = -LFA_EIO;
			} else if (id != recs[k].id) {
				lfa_hip_note(why, hipErrorInvalidValue, "P2P workspace identity");
				if (va_debug()) {
					fprintf(stderr, "lfa: peer %d workspace mapped onto other memory: "
						"identity %#llx, read %#llx; handle digest %#llx\n", k,
						(unsigned long long)recs[k].id, (unsigned long long)id,
						(unsigned long long)handle_digest(&recs[k].h));
					va_explain("mismatched mapping", mc->sym[k],
						   2 * region + LFA_SIG_AREA_BYTES);
				}
				ret = -LFA_EIO;
			}
		}
	}
	return ret;
}

/*
 * The P2P symmetric workspace of `mc`, grown to `region` bytes per region.
 * Collective: every member calls it at the same operation (the need depends
 * only on the operation's shape).  The old workspace is released only after
 * this rank's earlier operations have completed — each of which ends with a
 * barrier, so no peer still touches it — and the members learn each other's
 * new handle through one RCCL allgather of {ok, handle} records: a member
 * that failed to allocate makes them all fail together instead of leaving
 * the others waiting in a later barrier.
 */
/* Device domains: the whole handshake, stream-ordered, over RCCL. */
LFA_INTERNAL int p2p_ensure(struct lfa_coll_mc *mc, size_t region)
{
	struct lfa_coll_ep *ep = mc->ep;
	struct sym_rec *recs = ep->ctl_host;    /* nranks records, from ep open */
	void *drec = ep->ctl_dev;
	const size_t rb = sizeof(struct sym_rec);
	int n = mc->size, ret = 0;

	if (region <= mc->sym_region)
		return 0;
	region = sym_grow(mc, region);
	/* the old workspace is released only after this rank's earlier
	 * operations have completed — each of which ends with a barrier, so no
	 * peer still touches it */
	memset(recs, 0, (size_t)n * rb);
	sym_prepare(mc, region, hipStreamSynchronize(ep->stream) == hipSuccess,
		    &recs[mc->rank], NULL);
	if (n > 1 &&
	    (hipMemcpyAsync((char *)drec + (size_t)mc->rank * rb, &recs[mc->rank], rb,
			    hipMemcpyHostToDevice, ep->stream) != hipSuccess ||
	     ncclAllGather((char *)drec + (size_t)mc->rank * rb, drec, rb, ncclUint8,
			   mc->comm, ep->stream) != ncclSuccess ||
	     hipMemcpyAsync(recs, drec, (size_t)n * rb, hipMemcpyDeviceToHost,
			    ep->stream) != hipSuccess ||
	     hipStreamSynchronize(ep->stream) != hipSuccess))
		ret = -LFA_EIO;
	if (!ret)
		ret = sym_open(mc, recs, region, NULL);
	if (n > 1) {
		/* agree that every member mapped every peer (MIN of the flags) */
		int32_t all = ret == 0;

		if (hipMemcpyAsync(drec, &all, sizeof(all), hipMemcpyHostToDevice,
				   ep->stream) != hipSuccess ||
		    ncclAllReduce(drec, drec, 1, ncclInt32, ncclMin, mc->comm,
				  ep->stream) != ncclSuccess ||
		    hipMemcpyAsync(&all, drec, sizeof(all), hipMemcpyDeviceToHost,
				   ep->stream) != hipSuccess ||
		    hipStreamSynchronize(ep->stream) != hipSuccess || !all)
			ret = ret ? ret : -LFA_EIO;
	}
	if (ret) {
		p2p_release(mc);
		return ret;
	}
	mc->sym_region = region;
	return 0;
}
