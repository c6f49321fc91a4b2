/*
 * lfa_bench.c — bench-only helper (liblfa_bench.so; bench.py and tools/,
 * never the product): small-collective latency timed in C.
 *
 * lfa_bench_loop() submits one collective and polls lfa_cq_read until that
 * operation completes, `reps` times, the way a C caller of fi_allreduce /
 * fi_cq_read would (coll_ep_allreduce, coll_coll.c:1040; completion through
 * the owner's CQ, :722-756).  On the host this path costs under 1 us per
 * operation (the provider's submit, schedule and completion); the Python
 * wrapper around each call adds ~10 us, which the bench's Python-timed rows
 * include and this one does not.
 */
#include <errno.h>
#include <stdint.h>
#include <time.h>

#include "lfa_coll.h"

static double now_us(void)
{
	struct timespec ts;

	clock_gettime(CLOCK_MONOTONIC, &ts);
	return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

/* coll: LFA_ALLREDUCE, LFA_REDUCE_SCATTER or LFA_REDUCE (root: group rank).
 * Returns 0 and the mean microseconds per operation in *us_per_op, or the
 * first failing call's negative code (-ETIMEDOUT when an operation does
 * not complete within timeout_ms). */
int lfa_bench_loop(struct lfa_coll_ep *ep, int coll, const void *buf, void *result,
		   size_t count, int root, int dt, int op, lfa_addr_t coll_addr,
		   int reps, int timeout_ms, double *us_per_op)
{
	struct lfa_cq_entry e;
	double t0, deadline;
	ssize_t ret;

	if (!ep || reps <= 0 || !us_per_op)
		return -LFA_EINVAL;
	t0 = now_us();
	for (int i = 0; i < reps; i++) {
		void *ctx = (void *)(uintptr_t)(0x6c666100u + (unsigned)i);

		switch (coll) {
		case LFA_ALLREDUCE:
			ret = lfa_allreduce(ep, buf, count, NULL, result, NULL, coll_addr,
					    (enum lfa_datatype)dt, (enum lfa_op)op, 0, ctx);
			break;
		case LFA_REDUCE_SCATTER:
			ret = lfa_reduce_scatter(ep, buf, count, NULL, result, NULL, coll_addr,
						 (enum lfa_datatype)dt, (enum lfa_op)op, 0, ctx);
			break;
		case LFA_REDUCE:
			ret = lfa_reduce(ep, buf, count, NULL, result, NULL, coll_addr,
					 (lfa_addr_t)root, (enum lfa_datatype)dt,
					 (enum lfa_op)op, 0, ctx);
			break;
		default:
			return -LFA_EINVAL;
		}
		if (ret)
			return (int)ret;
		deadline = now_us() + 1e3 * timeout_ms;
		for (;;) {
			ret = lfa_cq_read(ep, &e, 1);
			if (ret == 1 && e.op_context == ctx)
				break;
			if (ret < 0 && ret != -LFA_EAGAIN)
				return (int)ret;
			if (now_us() > deadline)
				return -ETIMEDOUT;
		}
	}
	*us_per_op = (now_us() - t0) / reps;
	return 0;
}
