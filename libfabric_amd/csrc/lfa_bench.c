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

#include <hip/hip_runtime_api.h>

#include "lfa_atomic.h"
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

/*
 * The same loop keeping every operation's time (latency rows
 * as medians with a spread, not one mean): samples[i] = microseconds from
 * operation i's submit call to its completion read.  0 or as lfa_bench_loop.
 */
int lfa_bench_samples(struct lfa_coll_ep *ep, int coll, const void *buf, void *result,
		      size_t count, int root, int dt, int op, lfa_addr_t coll_addr,
		      int reps, int timeout_ms, double *samples)
{
	struct lfa_cq_entry e;
	double t0, deadline;
	ssize_t ret;

	if (!ep || reps <= 0 || !samples)
		return -LFA_EINVAL;
	for (int i = 0; i < reps; i++) {
		void *ctx = (void *)(uintptr_t)(0x6c666300u + (unsigned)i);

		t0 = now_us();
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
		samples[i] = now_us() - t0;
	}
	return 0;
}

/*
 * The same loop with its time split: out[0] mean us per
 * operation, out[1] of it inside the submit call, out[2] polling lfa_cq_read
 * until the operation completed, out[3] mean lfa_cq_read calls per operation.
 */
int lfa_bench_split(struct lfa_coll_ep *ep, int coll, const void *buf, void *result,
		    size_t count, int root, int dt, int op, lfa_addr_t coll_addr,
		    int reps, int timeout_ms, double out[4])
{
	struct lfa_cq_entry e;
	double t0, t1, t2, sub = 0, poll = 0, calls = 0, deadline;
	ssize_t ret;

	if (!ep || reps <= 0 || !out)
		return -LFA_EINVAL;
	t0 = now_us();
	for (int i = 0; i < reps; i++) {
		void *ctx = (void *)(uintptr_t)(0x6c666200u + (unsigned)i);

		t1 = now_us();
		if (coll == LFA_ALLREDUCE)
			ret = lfa_allreduce(ep, buf, count, NULL, result, NULL, coll_addr,
					    (enum lfa_datatype)dt, (enum lfa_op)op, 0, ctx);
		else if (coll == LFA_REDUCE_SCATTER)
			ret = lfa_reduce_scatter(ep, buf, count, NULL, result, NULL, coll_addr,
						 (enum lfa_datatype)dt, (enum lfa_op)op, 0, ctx);
		else
			return -LFA_EINVAL;
		t2 = now_us();
		sub += t2 - t1;
		if (ret)
			return (int)ret;
		deadline = t2 + 1e3 * timeout_ms;
		for (;;) {
			ret = lfa_cq_read(ep, &e, 1);
			calls++;
			if (ret == 1 && e.op_context == ctx)
				break;
			if (ret < 0 && ret != -LFA_EAGAIN)
				return (int)ret;
			if (now_us() > deadline)
				return -ETIMEDOUT;
		}
		poll += now_us() - t2;
	}
	out[0] = (now_us() - t0) / reps;
	out[1] = sub / reps;
	out[2] = poll / reps;
	out[3] = calls / reps;
	return 0;
}

/*
 * What one small GPU operation costs without the provider, on a stream of
 * its own: the 4 KiB (`bytes`) ATOMIC_WRITE copy kernel (lfa_atomic_write_async)
 *   mode 0: launch + hipEventRecord, then spin on hipEventQuery
 *   mode 1: launch, then hipStreamSynchronize
 *   mode 2: launch alone (host cost; the stream drained every 64)
 *   mode 3: hipEventRecord alone (host cost)
 *   mode 4: hipEventQuery of a completed event (host cost)
 *   mode 5: hipPointerGetAttributes of a device pointer (host cost)
 *   mode 6: lfa_cq_read on an endpoint with nothing queued (ep != NULL)
 * Mean microseconds per iteration in *us.
 */
int lfa_bench_raw(struct lfa_coll_ep *ep, void *dst, const void *src, size_t bytes,
		  int mode, int reps, double *us)
{
	hipStream_t s;
	hipEvent_t ev;
	hipPointerAttribute_t at;
	struct lfa_cq_entry e;
	double t0;
	int rc = 0;

	if (reps <= 0 || !us || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
		return -LFA_EINVAL;
	if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
		hipStreamDestroy(s);
		return -LFA_EIO;
	}
	/* warm: the kernel loaded, the event used once */
	lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8, dst, src, bytes, s);
	hipEventRecord(ev, s);
	hipStreamSynchronize(s);
	t0 = now_us();
	for (int i = 0; i < reps && !rc; i++) {
		switch (mode) {
		case 0:
			rc = lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8, dst, src, bytes, s);
			hipEventRecord(ev, s);
			while (hipEventQuery(ev) == hipErrorNotReady)
				;
			break;
		case 1:
			rc = lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8, dst, src, bytes, s);
			hipStreamSynchronize(s);
			break;
		case 2:
			rc = lfa_atomic_write_async(LFA_ATOMIC_WRITE, LFA_UINT8, dst, src, bytes, s);
			if (i % 64 == 63) {
				double t = now_us();

				hipStreamSynchronize(s);
				t0 += now_us() - t;     /* the drain is not launch cost */
			}
			break;
		case 3:
			hipEventRecord(ev, s);
			break;
		case 4:
			(void)hipEventQuery(ev);
			break;
		case 5:
			(void)hipPointerGetAttributes(&at, dst);
			break;
		case 6:
			if (!ep)
				rc = -LFA_EINVAL;
			else
				(void)lfa_cq_read(ep, &e, 1);
			break;
		default:
			rc = -LFA_EINVAL;
		}
	}
	*us = (now_us() - t0) / reps;
	hipStreamSynchronize(s);
	hipEventDestroy(ev);
	hipStreamDestroy(s);
	return rc;
}
