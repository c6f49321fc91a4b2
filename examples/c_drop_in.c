/*
 * c_drop_in.c — a plain-C libfabric-style caller of the MI355X path.
 *
 * No Python, no torch: links liblfa.so + liblfa_coll.so and /opt/rocm's HIP
 * runtime and RCCL directly, the way a libfabric provider would.
 *   1. the L4 table:   lfa_atomic_write_handlers[FI_SUM][FI_FLOAT](dst, src, n)
 *   2. the async form: lfa_atomic_write_async on a stream
 *   3. the provider:   domain/endpoint (world size 1), fi_allreduce-shaped
 *                      lfa_allreduce on device buffers, completion via
 *                      lfa_cq_read, query_collective.
 * Exit status 0 = every check passed.
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "lfa_atomic.h"
#include "lfa_coll.h"

#define CHECK(c)                                                          \
	do {                                                              \
		if (!(c)) {                                               \
			fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
			return 1;                                         \
		}                                                         \
	} while (0)

int main(void)
{
	enum { N = 1 << 20 };
	float *h_a = malloc(N * sizeof(float)), *h_b = malloc(N * sizeof(float));
	float *h_r = malloc(N * sizeof(float));
	float *d_a, *d_b, *d_r;
	char id[LFA_UNIQUE_ID_BYTES];
	struct lfa_coll_domain *dom;
	struct lfa_coll_ep *ep;
	struct lfa_cq_entry cqe;
	struct lfa_collective_attr attr;
	int ctx_tag = 42, i;
	ssize_t n;

	CHECK(h_a && h_b && h_r);
	for (i = 0; i < N; i++) {
		h_a[i] = (float)(i % 1000) * 0.5f - 3.0f;
		h_b[i] = (float)((i * 7) % 333) * 0.25f;
	}
	CHECK(hipMalloc((void **)&d_a, N * sizeof(float)) == hipSuccess);
	CHECK(hipMalloc((void **)&d_b, N * sizeof(float)) == hipSuccess);
	CHECK(hipMalloc((void **)&d_r, N * sizeof(float)) == hipSuccess);
	CHECK(hipMemcpy(d_a, h_a, N * sizeof(float), hipMemcpyHostToDevice) == hipSuccess);
	CHECK(hipMemcpy(d_b, h_b, N * sizeof(float), hipMemcpyHostToDevice) == hipSuccess);

	/* 1. synchronous table entry, exactly ofi_atomic_write_handler's shape */
	CHECK(lfa_atomic_valid(LFA_FLOAT, LFA_SUM, 0) == 0);
	CHECK(lfa_atomic_valid(LFA_FLOAT, LFA_BOR, 0) == -LFA_EOPNOTSUPP);
	lfa_atomic_write_handlers[LFA_SUM][LFA_FLOAT](d_a, d_b, N);
	CHECK(hipMemcpy(h_r, d_a, N * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess);
	for (i = 0; i < N; i++)
		CHECK(h_r[i] == h_a[i] + h_b[i]);

	/* 2. async form: MIN on the same buffers */
	CHECK(lfa_atomic_write_async(LFA_MIN, LFA_FLOAT, d_a, d_b, N, NULL) == 0);
	CHECK(hipDeviceSynchronize() == hipSuccess);
	CHECK(hipMemcpy(h_r, d_a, N * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess);
	for (i = 0; i < N; i++) {
		float s = h_a[i] + h_b[i];
		CHECK(h_r[i] == (s > h_b[i] ? h_b[i] : s));
	}

	/* 3. provider: world of one rank over RCCL */
	CHECK(lfa_coll_get_unique_id(id, sizeof(id)) == 0);
	CHECK(lfa_coll_domain_open(0, 0, 1, id, sizeof(id), &dom) == 0);
	CHECK(lfa_coll_ep_open(dom, &ep) == 0);
	memset(&attr, 0, sizeof(attr));
	attr.op = LFA_SUM;
	attr.datatype = LFA_FLOAT;
	CHECK(lfa_query_collective(dom, LFA_ALLREDUCE, &attr, 0) == 0);
	CHECK(attr.max_members == 0x7fffffff);
	CHECK(lfa_allreduce(ep, d_b, N, NULL, d_r, NULL, LFA_ADDR_NOTAVAIL,
			    LFA_FLOAT, LFA_SUM, 0, &ctx_tag) == 0);
	do {
		n = lfa_cq_read(ep, &cqe, 1);
	} while (n == -LFA_EAGAIN);
	CHECK(n == 1 && cqe.op_context == &ctx_tag && cqe.flags == LFA_COLLECTIVE);
	CHECK(hipMemcpy(h_r, d_r, N * sizeof(float), hipMemcpyDeviceToHost) == hipSuccess);
	CHECK(memcmp(h_r, h_b, N * sizeof(float)) == 0);
	CHECK(lfa_coll_ep_close(ep) == 0);
	CHECK(lfa_coll_domain_close(dom) == 0);

	hipFree(d_a);
	hipFree(d_b);
	hipFree(d_r);
	free(h_a);
	free(h_b);
	free(h_r);
	printf("c_drop_in: OK (table, async, provider allreduce + CQ)\n");
	return 0;
}
