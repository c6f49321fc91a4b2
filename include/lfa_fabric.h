/*
 * lfa_fabric.h — ABI-compatible enums, flags and error codes for the
 * MI355X-native fi_collective reduction path (libfabric_amd, "lfa").
 *
 * Every enumerator below carries the SAME integer value as the public
 * libfabric ABI, so a libfabric caller can pass its own `enum fi_datatype`,
 * `enum fi_op` and `enum fi_collective_op` values straight through:
 *
 *   lfa_datatype       == enum fi_datatype        include/rdma/fi_domain.h:224-247
 *   lfa_op             == enum fi_op              include/rdma/fi_domain.h:249-273
 *   lfa_collective_op  == enum fi_collective_op   include/rdma/fi_domain.h:279-289
 *   LFA_E*             == FI_E*                   include/rdma/fi_errno.h:57-188
 *   LFA_FETCH_ATOMIC…  == FI_FETCH_ATOMIC…        include/rdma/fi_atomic.h:47-48
 *
 * tests/test_abi.py static-asserts the equality against the reference headers
 * whenever /root/reference is present.
 *
 * Plain C, no HIP or torch types: this header is the drop-in boundary.
 */
#ifndef LFA_FABRIC_H
#define LFA_FABRIC_H

#include <stddef.h>
#include <stdint.h>
#include <errno.h>

#ifdef __cplusplus
extern "C" {
#endif

enum lfa_datatype {
	LFA_INT8 = 0,
	LFA_UINT8,
	LFA_INT16,
	LFA_UINT16,
	LFA_INT32,
	LFA_UINT32,
	LFA_INT64,
	LFA_UINT64,
	LFA_FLOAT,
	LFA_DOUBLE,
	LFA_FLOAT_COMPLEX,
	LFA_DOUBLE_COMPLEX,
	LFA_LONG_DOUBLE,
	LFA_LONG_DOUBLE_COMPLEX,
	LFA_INT128,
	LFA_UINT128,
	LFA_FLOAT16,
	LFA_BFLOAT16,
	LFA_FLOAT8_E4M3,
	LFA_FLOAT8_E5M2,
	LFA_VOID = 256,
};

/* Number of datatypes with a combine-table column (FI_UINT128 + 1),
 * include/ofi_atomic.h:71. */
#define LFA_DATATYPE_CNT (LFA_UINT128 + 1)

enum lfa_op {
	LFA_MIN = 0,
	LFA_MAX,
	LFA_SUM,
	LFA_PROD,
	LFA_LOR,
	LFA_LAND,
	LFA_BOR,
	LFA_BAND,
	LFA_LXOR,
	LFA_BXOR,
	LFA_ATOMIC_READ,
	LFA_ATOMIC_WRITE,
	LFA_CSWAP,
	LFA_CSWAP_NE,
	LFA_CSWAP_LE,
	LFA_CSWAP_LT,
	LFA_CSWAP_GE,
	LFA_CSWAP_GT,
	LFA_MSWAP,
	LFA_DIFF,
	LFA_NOOP = 256,
};

/* Row ranges of the three tables, include/ofi_atomic.h:47-62. */
#define LFA_WRITE_OP_CNT     (LFA_ATOMIC_WRITE + 1)
#define LFA_READWRITE_OP_CNT (LFA_ATOMIC_WRITE + 1)
#define LFA_SWAP_OP_CNT      (LFA_MSWAP - LFA_CSWAP + 1)

enum lfa_collective_op {
	LFA_BARRIER = 0,
	LFA_BROADCAST,
	LFA_ALLTOALL,
	LFA_ALLREDUCE,
	LFA_ALLGATHER,
	LFA_REDUCE_SCATTER,
	LFA_REDUCE,
	LFA_SCATTER,
	LFA_GATHER,
};

/* Flags (same bits as libfabric). */
#define LFA_TAGGED          (1ULL << 3)
#define LFA_COLLECTIVE      (1ULL << 6)
#define LFA_PEER_TRANSFER   (1ULL << 36)
#define LFA_FETCH_ATOMIC    (1ULL << 58)
#define LFA_COMPARE_ATOMIC  (1ULL << 59)

/* Error codes: returned negated, exactly like libfabric (-FI_EINVAL …). */
#define LFA_SUCCESS     0
#define LFA_EAGAIN      EAGAIN
#define LFA_ENOMEM      ENOMEM
#define LFA_EBUSY       EBUSY
#define LFA_EINVAL      EINVAL
#define LFA_ENOSYS      ENOSYS
#define LFA_EOPNOTSUPP  EOPNOTSUPP
#define LFA_EIO         EIO
#define LFA_EOTHER      256
#define LFA_EBADFLAGS   260
#define LFA_ENOEQ       261

typedef uint64_t lfa_addr_t;
#define LFA_ADDR_NOTAVAIL ((uint64_t)-1)

/* Mirrors struct fi_atomic_attr, include/rdma/fi_atomic.h:50-53. */
struct lfa_atomic_attr {
	size_t count;
	size_t size;
};

/* Mirrors struct fi_collective_attr, include/rdma/fi_collective.h:67-73. */
struct lfa_collective_attr {
	enum lfa_op op;
	enum lfa_datatype datatype;
	struct lfa_atomic_attr datatype_attr;
	size_t max_members;
	uint64_t mode;
};

#ifdef __cplusplus
}
#endif

#endif /* LFA_FABRIC_H */
