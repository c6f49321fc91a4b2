/*
 * lfa_coll_plan.h — internal interface between the schedule builder
 * (lfa_coll_plan.c) and the executor (lfa_coll.c, lfa_coll_exec.c,
 * lfa_coll_loopback.c) of liblfa_coll.so.  Not
 * installed; nothing here is exported from the library.
 */
#ifndef LFA_COLL_PLAN_H
#define LFA_COLL_PLAN_H

#include <stddef.h>

#include "lfa_coll.h"

#define LFA_INTERNAL __attribute__((visibility("hidden")))
#define LFA_SMALL_AG_BYTES (256u << 10) /* allgather-then-tree below this */
/* a one-member group's reducing collective of at most this many bytes runs
 * as one copy kernel ending in the completion word (run_solo; LFA_SOLO_BYTES
 * overrides it).  Timed in C through the provider (round 5,
 * tools/probe_world1_sizes.py): 1 MiB 8.3-8.4 us, 4 MiB 10.4-10.7 us against
 * 12.7 us for the TREE plan's copy and event; at 16 MiB the copy's
 * write-through stores lose (19.8 vs 14.5 us), so the TREE plan takes over */
#define LFA_ONESHOT_SOLO_BYTES (4u << 20)
/* ... and through liblfa's own HSA queue up to this many (4 workgroups of
 * 16 KiB): its kernel arguments sit in host memory and every workgroup
 * fetches them over PCIe, so past a few workgroups the HIP launch
 * (device-memory arguments) wins — 64 KiB 6.4 vs 7.6 us, 256 KiB 8.8 vs
 * 8.3 us, 1 MiB 15.4 vs 8.4 us (round 5, tools/probe_solo_multi.py) */
#define LFA_DIRECT_SOLO_BYTES (64u << 10)
/* P2P reduce_scatter: one-shot up to this many input bytes per member (each
 * member pushes block k to member k: the staged schedule's bytes per link,
 * in one kernel instead of four), unless LFA_OS_RS_BYTES in the environment
 * (the same on every member) says otherwise.  Double PROD across 2 / 4
 * processes on one MI355X: 2 MiB 26.9 -> 16.6 / 30.8 -> 24.3 us, 4 MiB
 * 28.2 -> 18.4 / 34.8 -> 28.6 us; from 8 MiB the staged schedule's
 * full-GPU kernels come within 1-3 us (round 5).  1 MiB before
 * round 5. */
#define LFA_OS_RS_BYTES (4u << 20)
LFA_INTERNAL size_t lfa_os_rs_bytes(void);
/* P2P allreduce / reduce: one kernel (the one-shot) while count·esz·n is at
 * most this — LFA_OS_AG_BYTES_DEFAULT unless LFA_OS_AG_BYTES (the same on
 * every member) says otherwise.  The one-shot pushes the whole input to every
 * peer, so each xGMI link carries count·esz (the staged schedule: a quarter
 * of that, in five kernels); at 2 MiB over all members a link carries at
 * most 1 MiB at 2 members and 256 KiB at 8.  On one MI355X shared by 2 / 4
 * processes the one-shot took 16.9 / 29.3 us at 1 MiB per member against
 * 30.4 / 35.2 us staged (round 5); 256 KiB before round 5. */
#define LFA_OS_AG_BYTES_DEFAULT (2u << 20)
LFA_INTERNAL size_t lfa_os_ag_bytes(void);

/* A heap-allocated plan. */
struct plan {
	struct lfa_step *steps;
	struct lfa_ref *refs;
	size_t nsteps, nrefs, tmp;
};

LFA_INTERNAL void plan_free(struct plan *pl);
/* lfa_coll_plan into freshly allocated arrays */
LFA_INTERNAL int plan_make(struct plan *pl, enum lfa_collective_op coll,
			   enum lfa_coll_algo algo, int rank, int n, int root,
			   size_t count, size_t esz);
/* Collective items -> grouped SEND/RECV items; lower_barrier: BARRIER too;
 * lower_oneshot: ONESHOT -> COPY, BARRIER, TREE, BARRIER */
LFA_INTERNAL int lower_plan(const struct plan *in, int r, int n, size_t esz,
			    struct plan *out, int lower_barrier, int lower_oneshot);

#endif
