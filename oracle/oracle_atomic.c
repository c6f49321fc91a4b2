/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.
 *
 * A CPU restatement of libfabric's element-wise combine tables and of
 * prov/coll's recursive-doubling allreduce schedule.  It is the parity
 * checker for the MI355X kernels and the CPU baseline timed by bench.py.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load it; the product path (libfabric_amd, liblfa*.so) never links or calls
 * anything in oracle/.
 *
 * Written from the reference's semantics, not copied:
 *   - combine tables    prov/util/src/util_atomic.c:224-343 (templates),
 *                       :889-922 (shipping HAVE_BUILTIN_MM_ATOMICS table),
 *                       :987-1020 (open-coded table)
 *   - datatype sizes    prov/util/src/util_atomic.c:37-64
 *   - ofi_atomic_valid  prov/util/src/util_atomic.c:1088-1140
 *   - fetch / swap tbl  prov/util/src/util_atomic.c:345-760, :924-980
 *   - allreduce sched   prov/coll/src/coll_coll.c:349-449 (recursive doubling)
 *   - reduce item       prov/coll/src/coll_coll.c:758-768
 *
 * Two variants of every handler:
 *   ORACLE_CAS   — per-element seq_cst compare-exchange / fetch-or, the code
 *                  shape libfabric ships on gcc (configure.ac:389-420);
 *   ORACLE_PLAIN — the open-coded loop (util_atomic.c:119-153).
 * Single-threaded, both produce identical bits; they differ only in speed.
 *
 * Pinning: tests/test_oracle.py checks every (op, datatype) handler here
 * bit-for-bit against oracle/_ref/libft_atomic.so, compiled by oracle/Makefile
 * from the reference's own fabtests/common/ofi_atomic.c (the independent
 * restatement libfabric's fabtests verify provider atomics with,
 * fabtests/common/shared.c:3951-4055), and against tests/golden/ fixtures
 * generated from that library.
 *
 * Build: plain gcc -O2 with -ffp-contract=off and no -march, so float/complex
 * arithmetic rounds exactly as the reference's x86-64 build does.
 */
#define _GNU_SOURCE
#include <complex.h>
#include <errno.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/lfa_fabric.h"

typedef float _Complex cf32_t;
typedef __int128 i128_t;
typedef unsigned __int128 u128_t;

enum { ORACLE_CAS = 0, ORACLE_PLAIN = 1 };

typedef void (*oracle_fn)(void *dst, const void *src, size_t cnt);

/* ------------------------------------------------------------------ */
/* datatype sizes (util_atomic.c:37-64)                                */
/* ------------------------------------------------------------------ */
static const size_t dt_size[LFA_DATATYPE_CNT] = {
	1, 1, 2, 2, 4, 4, 8, 8,             /* int8 .. uint64            */
	4, 8,                               /* float, double             */
	sizeof(float _Complex), sizeof(double _Complex),
	sizeof(long double), sizeof(long double _Complex),
	16, 16,                             /* int128, uint128           */
};

size_t oracle_datatype_size(int dt)
{
	if (dt < 0 || dt >= LFA_DATATYPE_CNT) {
		errno = EINVAL;
		return 0;
	}
	return dt_size[dt];
}

/* ------------------------------------------------------------------ */
/* element semantics                                                   */
/*                                                                     */
/* Integer SUM/PROD wrap modulo 2^bits (the reference computes in C    */
/* with promotion and truncation; x86 wraps).  They are computed here  */
/* in an unsigned type wide enough to avoid C undefined behaviour.     */
/* ------------------------------------------------------------------ */
#define WRAP_ADD(T, W, a, b) ((T)((W)(a) + (W)(b)))
#define WRAP_MUL(T, W, a, b) ((T)((W)(a) * (W)(b)))
#define F_ADD(T, W, a, b)    ((a) + (b))
#define F_MUL(T, W, a, b)    ((a) * (b))
#define LOG_OR(a, b)         ((a) || (b))
#define LOG_AND(a, b)        ((a) && (b))
#define LOG_XOR(a, b)        (((a) && !(b)) || (!(a) && (b)))

/* plain element-wise loop */
#define PLAIN_LOOP(NAME, T, STMT)                                        \
	static void NAME(void *dst, const void *src, size_t cnt)         \
	{                                                                \
		T *d = (T *)dst;                                         \
		const T *s = (const T *)src;                             \
		for (size_t i = 0; i < cnt; i++) {                       \
			T a = d[i], b = s[i];                            \
			(void)a; (void)b;                                \
			STMT;                                            \
		}                                                        \
	}

/* read-modify-CAS loop: the value written is VALUE(a = current dst, b = src) */
#define CAS_LOOP(NAME, T, VALUE)                                         \
	static void NAME(void *dst, const void *src, size_t cnt)         \
	{                                                                \
		T *d = (T *)dst;                                         \
		const T *s = (const T *)src;                             \
		for (size_t i = 0; i < cnt; i++) {                       \
			T a, b = s[i], v;                                \
			do {                                             \
				a = d[i];                                \
				v = (T)(VALUE);                          \
			} while (!__atomic_compare_exchange(&d[i], &a, &v, 0, \
					__ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST)); \
		}                                                        \
	}

/* conditional CAS (MIN/MAX): only swap when COND(a, b) holds */
#define CAS_COND_LOOP(NAME, T, COND)                                     \
	static void NAME(void *dst, const void *src, size_t cnt)         \
	{                                                                \
		T *d = (T *)dst;                                         \
		const T *s = (const T *)src;                             \
		for (size_t i = 0; i < cnt; i++) {                       \
			T a, b = s[i];                                   \
			int done;                                        \
			do {                                             \
				done = 1;                                \
				a = d[i];                                \
				if (COND)                                \
					done = __atomic_compare_exchange(&d[i], &a, &b, 0, \
						__ATOMIC_SEQ_CST, __ATOMIC_SEQ_CST); \
			} while (!done);                                 \
		}                                                        \
	}

#define FETCH_LOOP(NAME, T, BUILTIN)                                     \
	static void NAME(void *dst, const void *src, size_t cnt)         \
	{                                                                \
		T *d = (T *)dst;                                         \
		const T *s = (const T *)src;                             \
		for (size_t i = 0; i < cnt; i++)                         \
			(void)BUILTIN(&d[i], s[i], __ATOMIC_SEQ_CST);    \
	}

/*
 * Per "real" type: MIN MAX SUM PROD LOR LAND LXOR WRITE, both variants.
 * ADD/MUL pick wrapping (integer) or IEEE (float) arithmetic.
 */
#define DEF_REAL(N, T, W, ADD, MUL)                                             \
	PLAIN_LOOP(p_min_##N, T, if (a > b) d[i] = b)                           \
	PLAIN_LOOP(p_max_##N, T, if (a < b) d[i] = b)                           \
	PLAIN_LOOP(p_sum_##N, T, d[i] = ADD(T, W, a, b))                        \
	PLAIN_LOOP(p_prod_##N, T, d[i] = MUL(T, W, a, b))                       \
	PLAIN_LOOP(p_lor_##N, T, d[i] = (T)LOG_OR(a, b))                        \
	PLAIN_LOOP(p_land_##N, T, d[i] = (T)LOG_AND(a, b))                      \
	PLAIN_LOOP(p_lxor_##N, T, d[i] = (T)LOG_XOR(a, b))                      \
	PLAIN_LOOP(p_write_##N, T, d[i] = b)                                    \
	CAS_COND_LOOP(c_min_##N, T, a > b)                                      \
	CAS_COND_LOOP(c_max_##N, T, a < b)                                      \
	CAS_LOOP(c_sum_##N, T, ADD(T, W, a, b))                                 \
	CAS_LOOP(c_prod_##N, T, MUL(T, W, a, b))                                \
	CAS_LOOP(c_lor_##N, T, LOG_OR(a, b))                                    \
	CAS_LOOP(c_land_##N, T, LOG_AND(a, b))                                  \
	CAS_LOOP(c_lxor_##N, T, LOG_XOR(a, b))                                  \
	PLAIN_LOOP(c_write_##N, T, __atomic_store(&d[i], &b, __ATOMIC_SEQ_CST))

/* integer-only bitwise ops */
#define DEF_BITS(N, T)                                                          \
	PLAIN_LOOP(p_bor_##N, T, d[i] = a | b)                                  \
	PLAIN_LOOP(p_band_##N, T, d[i] = a & b)                                 \
	PLAIN_LOOP(p_bxor_##N, T, d[i] = a ^ b)                                 \
	FETCH_LOOP(c_bor_##N, T, __atomic_fetch_or)                             \
	FETCH_LOOP(c_band_##N, T, __atomic_fetch_and)                           \
	FETCH_LOOP(c_bxor_##N, T, __atomic_fetch_xor)

DEF_REAL(i8, int8_t, uint32_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(u8, uint8_t, uint32_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(i16, int16_t, uint32_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(u16, uint16_t, uint32_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(i32, int32_t, uint32_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(u32, uint32_t, uint32_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(i64, int64_t, uint64_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(u64, uint64_t, uint64_t, WRAP_ADD, WRAP_MUL)
DEF_REAL(f32, float, float, F_ADD, F_MUL)
DEF_REAL(f64, double, double, F_ADD, F_MUL)
DEF_BITS(i8, int8_t)
DEF_BITS(u8, uint8_t)
DEF_BITS(i16, int16_t)
DEF_BITS(u16, uint16_t)
DEF_BITS(i32, int32_t)
DEF_BITS(u32, uint32_t)
DEF_BITS(i64, int64_t)
DEF_BITS(u64, uint64_t)

/*
 * 16-byte integers: the shipping table has them when the compiler offers
 * 128-bit __atomic builtins (configure.ac:431-446, HAVE_BUILTIN_MM_INT128_ATOMICS).
 * The values are computed with the plain loop in both variants (16-byte
 * __atomic needs libatomic locks; the result is the same).
 */
PLAIN_LOOP(p_min_i128, i128_t, if (a > b) d[i] = b)
PLAIN_LOOP(p_max_i128, i128_t, if (a < b) d[i] = b)
PLAIN_LOOP(p_sum_i128, i128_t, d[i] = WRAP_ADD(i128_t, u128_t, a, b))
PLAIN_LOOP(p_prod_i128, i128_t, d[i] = WRAP_MUL(i128_t, u128_t, a, b))
PLAIN_LOOP(p_lor_i128, i128_t, d[i] = (i128_t)LOG_OR(a, b))
PLAIN_LOOP(p_land_i128, i128_t, d[i] = (i128_t)LOG_AND(a, b))
PLAIN_LOOP(p_lxor_i128, i128_t, d[i] = (i128_t)LOG_XOR(a, b))
PLAIN_LOOP(p_write_i128, i128_t, d[i] = b)
PLAIN_LOOP(p_bor_i128, i128_t, d[i] = a | b)
PLAIN_LOOP(p_band_i128, i128_t, d[i] = a & b)
PLAIN_LOOP(p_bxor_i128, i128_t, d[i] = a ^ b)
PLAIN_LOOP(p_min_u128, u128_t, if (a > b) d[i] = b)
PLAIN_LOOP(p_max_u128, u128_t, if (a < b) d[i] = b)
PLAIN_LOOP(p_sum_u128, u128_t, d[i] = a + b)
PLAIN_LOOP(p_prod_u128, u128_t, d[i] = a * b)
PLAIN_LOOP(p_lor_u128, u128_t, d[i] = (u128_t)LOG_OR(a, b))
PLAIN_LOOP(p_land_u128, u128_t, d[i] = (u128_t)LOG_AND(a, b))
PLAIN_LOOP(p_lxor_u128, u128_t, d[i] = (u128_t)LOG_XOR(a, b))
PLAIN_LOOP(p_write_u128, u128_t, d[i] = b)
PLAIN_LOOP(p_bor_u128, u128_t, d[i] = a | b)
PLAIN_LOOP(p_band_u128, u128_t, d[i] = a & b)
PLAIN_LOOP(p_bxor_u128, u128_t, d[i] = a ^ b)

/*
 * float complex: SUM PROD LOR LAND LXOR WRITE (include/unix/osd.h:241-271).
 * C99 complex arithmetic exactly as gcc lowers it (inline formula, __mulsc3
 * recovery when both parts come out NaN).  Complex "truth" is re||im != 0.
 */
PLAIN_LOOP(p_sum_c32, cf32_t, d[i] = a + b)
PLAIN_LOOP(p_prod_c32, cf32_t, d[i] = a * b)
PLAIN_LOOP(p_lor_c32, cf32_t, d[i] = (cf32_t)(a || b))
PLAIN_LOOP(p_land_c32, cf32_t, d[i] = (cf32_t)(a && b))
PLAIN_LOOP(p_lxor_c32, cf32_t, d[i] = (cf32_t)LOG_XOR(a, b))
PLAIN_LOOP(p_write_c32, cf32_t, d[i] = b)
CAS_LOOP(c_sum_c32, cf32_t, a + b)
CAS_LOOP(c_prod_c32, cf32_t, a * b)
CAS_LOOP(c_lor_c32, cf32_t, a || b)
CAS_LOOP(c_land_c32, cf32_t, a && b)
CAS_LOOP(c_lxor_c32, cf32_t, LOG_XOR(a, b))
PLAIN_LOOP(c_write_c32, cf32_t, __atomic_store(&d[i], &b, __ATOMIC_SEQ_CST))

/* ------------------------------------------------------------------ */
/* dispatch tables [variant][op][datatype] (util_atomic.c:907-922)     */
/* NULL = the shipping table has no handler.                           */
/* ------------------------------------------------------------------ */
#define ROW_REAL(V, OP)                                                   \
	{ V##_##OP##_i8, V##_##OP##_u8, V##_##OP##_i16, V##_##OP##_u16,  \
	  V##_##OP##_i32, V##_##OP##_u32, V##_##OP##_i64, V##_##OP##_u64, \
	  V##_##OP##_f32, V##_##OP##_f64, NULL, NULL, NULL, NULL,         \
	  p_##OP##_i128, p_##OP##_u128 }
#define ROW_ALL(V, OP)                                                    \
	{ V##_##OP##_i8, V##_##OP##_u8, V##_##OP##_i16, V##_##OP##_u16,  \
	  V##_##OP##_i32, V##_##OP##_u32, V##_##OP##_i64, V##_##OP##_u64, \
	  V##_##OP##_f32, V##_##OP##_f64, V##_##OP##_c32, NULL, NULL, NULL, \
	  p_##OP##_i128, p_##OP##_u128 }
#define ROW_INT(V, OP)                                                    \
	{ V##_##OP##_i8, V##_##OP##_u8, V##_##OP##_i16, V##_##OP##_u16,  \
	  V##_##OP##_i32, V##_##OP##_u32, V##_##OP##_i64, V##_##OP##_u64, \
	  NULL, NULL, NULL, NULL, NULL, NULL,                             \
	  p_##OP##_i128, p_##OP##_u128 }
#define ROW_NONE                                                          \
	{ NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL,                 \
	  NULL, NULL, NULL, NULL, NULL, NULL, NULL, NULL }
#define TABLE(V)                                                          \
	{ ROW_REAL(V, min), ROW_REAL(V, max), ROW_ALL(V, sum),            \
	  ROW_ALL(V, prod), ROW_ALL(V, lor), ROW_ALL(V, land),            \
	  ROW_INT(V, bor), ROW_INT(V, band), ROW_ALL(V, lxor),            \
	  ROW_INT(V, bxor), ROW_NONE, ROW_ALL(V, write) }

static oracle_fn const table[2][LFA_WRITE_OP_CNT][LFA_DATATYPE_CNT] = {
	TABLE(c), TABLE(p),
};

oracle_fn oracle_write_handler(int variant, int op, int dt)
{
	if (variant < 0 || variant > 1 || op < 0 || op >= LFA_WRITE_OP_CNT ||
	    dt < 0 || dt >= LFA_DATATYPE_CNT)
		return NULL;
	return table[variant][op][dt];
}

/* Returns 0, or -LFA_EOPNOTSUPP when the table has no handler. */
int oracle_write(int variant, int op, int dt, void *dst, const void *src,
		 size_t cnt)
{
	oracle_fn fn = oracle_write_handler(variant, op, dt);

	if (!fn)
		return -LFA_EOPNOTSUPP;
	fn(dst, src, cnt);
	return 0;
}

int oracle_has_readwrite(int op, int dt);
int oracle_has_swap(int op, int dt);

/* ofi_atomic_valid (util_atomic.c:1088-1140): write, fetch and compare tables. */
int oracle_atomic_valid(int dt, int op, uint64_t flags)
{
	if (flags & LFA_TAGGED) {
		if (flags & (LFA_FETCH_ATOMIC | LFA_COMPARE_ATOMIC))
			return -LFA_ENOSYS;
	} else if (flags & ~(LFA_FETCH_ATOMIC | LFA_COMPARE_ATOMIC)) {
		return -LFA_EBADFLAGS;
	} else if ((flags & LFA_FETCH_ATOMIC) && (flags & LFA_COMPARE_ATOMIC)) {
		return -LFA_EBADFLAGS;
	}
	if (dt < 0 || dt >= LFA_DATATYPE_CNT)
		return -LFA_EOPNOTSUPP;
	if (flags & LFA_FETCH_ATOMIC) {
		if (op < LFA_MIN || op > LFA_ATOMIC_WRITE)
			return -LFA_EOPNOTSUPP;
		return oracle_has_readwrite(op, dt) ? 0 : -LFA_EOPNOTSUPP;
	}
	if (flags & LFA_COMPARE_ATOMIC) {
		if (op < LFA_CSWAP || op > LFA_MSWAP)
			return -LFA_EOPNOTSUPP;
		return oracle_has_swap(op, dt) ? 0 : -LFA_EOPNOTSUPP;
	}
	if (op < LFA_MIN || op > LFA_ATOMIC_WRITE || op == LFA_ATOMIC_READ)
		return -LFA_EOPNOTSUPP;
	return table[ORACLE_PLAIN][op][dt] ? 0 : -LFA_EOPNOTSUPP;
}

/* ------------------------------------------------------------------ */
/* fetch (readwrite) table (util_atomic.c:345-588, :924-950)           */
/*                                                                     */
/* Every shipping readwrite handler returns the old destination value  */
/* in res[] and then performs the write op (READWRITEEXT CAS loops,    */
/* __atomic_fetch_or/and/xor, __atomic_exchange for ATOMIC_WRITE); the */
/* ATOMIC_READ row only loads.  Single-threaded that is exactly        */
/* "res = dst; dst = dst OP src", in both variants.                    */
/* ------------------------------------------------------------------ */
int oracle_has_readwrite(int op, int dt)
{
	if (op < 0 || op >= LFA_READWRITE_OP_CNT || dt < 0 || dt >= LFA_DATATYPE_CNT)
		return 0;
	if (op == LFA_ATOMIC_READ)  /* ALL handlers (util_atomic.c:936) */
		return table[ORACLE_PLAIN][LFA_ATOMIC_WRITE][dt] != NULL;
	return table[ORACLE_PLAIN][op][dt] != NULL;
}

int oracle_readwrite(int variant, int op, int dt, void *dst, const void *src,
		     void *res, size_t cnt)
{
	if (!oracle_has_readwrite(op, dt))
		return -LFA_EOPNOTSUPP;
	memcpy(res, dst, cnt * dt_size[dt]);
	if (op != LFA_ATOMIC_READ)
		table[variant][op][dt](dst, src, cnt);
	return 0;
}

/* ------------------------------------------------------------------ */
/* compare-swap table (util_atomic.c:590-760, :952-980)                */
/*                                                                     */
/* res = old dst; dst = src when the condition holds:                  */
/*   CSWAP     CAS build: __atomic_compare_exchange — a BYTEWISE       */
/*             compare of dst and cmp (so -0.0 != +0.0 and a NaN       */
/*             equals itself); open-coded build: (cmp) == (dst)       */
/*   CSWAP_NE  (cmp) != (dst)     CSWAP_LE (cmp) <= (dst)               */
/*   CSWAP_LT  (cmp) <  (dst)     CSWAP_GE (cmp) >= (dst)               */
/*   CSWAP_GT  (cmp) >  (dst)                                           */
/*   MSWAP     dst = (src & cmp) | (dst & ~cmp)   (integers)            */
/* ------------------------------------------------------------------ */
#define SWAP_LOOP(T, COND)                                                \
	do {                                                              \
		T *d = (T *)dst;                                          \
		const T *s_ = (const T *)src, *c_ = (const T *)cmp;       \
		T *r = (T *)res;                                          \
		for (size_t i = 0; i < cnt; i++) {                        \
			T a = d[i], b = s_[i], c = c_[i];                 \
			(void)b;                                          \
			r[i] = a;                                         \
			if (COND)                                         \
				d[i] = b;                                 \
		}                                                         \
	} while (0)
#define MSWAP_LOOP(T)                                                     \
	do {                                                              \
		T *d = (T *)dst;                                          \
		const T *s_ = (const T *)src, *c_ = (const T *)cmp;       \
		T *r = (T *)res;                                          \
		for (size_t i = 0; i < cnt; i++) {                        \
			r[i] = d[i];                                      \
			d[i] = (T)((s_[i] & c_[i]) | (d[i] & ~c_[i]));    \
		}                                                         \
	} while (0)

#define SWAP_REAL_CASES(OPV, COND)                                        \
	switch (dt) {                                                     \
	case LFA_INT8: SWAP_LOOP(int8_t, COND); break;                    \
	case LFA_UINT8: SWAP_LOOP(uint8_t, COND); break;                  \
	case LFA_INT16: SWAP_LOOP(int16_t, COND); break;                  \
	case LFA_UINT16: SWAP_LOOP(uint16_t, COND); break;                \
	case LFA_INT32: SWAP_LOOP(int32_t, COND); break;                  \
	case LFA_UINT32: SWAP_LOOP(uint32_t, COND); break;                \
	case LFA_INT64: SWAP_LOOP(int64_t, COND); break;                  \
	case LFA_UINT64: SWAP_LOOP(uint64_t, COND); break;                \
	case LFA_FLOAT: SWAP_LOOP(float, COND); break;                    \
	case LFA_DOUBLE: SWAP_LOOP(double, COND); break;                  \
	case LFA_INT128: SWAP_LOOP(i128_t, COND); break;                  \
	case LFA_UINT128: SWAP_LOOP(u128_t, COND); break;                 \
	default: return -LFA_EOPNOTSUPP;                                  \
	}

int oracle_has_swap(int op, int dt)
{
	int realno = (dt >= LFA_INT8 && dt <= LFA_DOUBLE) || dt == LFA_INT128 ||
		     dt == LFA_UINT128;
	int ints = (dt >= LFA_INT8 && dt <= LFA_UINT64) || dt == LFA_INT128 ||
		   dt == LFA_UINT128;

	switch (op) {
	case LFA_CSWAP:
	case LFA_CSWAP_NE:
		return realno || dt == LFA_FLOAT_COMPLEX;
	case LFA_CSWAP_LE:
	case LFA_CSWAP_LT:
	case LFA_CSWAP_GE:
	case LFA_CSWAP_GT:
		return realno;
	case LFA_MSWAP:
		return ints;
	default:
		return 0;
	}
}

int oracle_swap(int variant, int op, int dt, void *dst, const void *src,
		const void *cmp, void *res, size_t cnt)
{
	size_t esz;

	if (!oracle_has_swap(op, dt))
		return -LFA_EOPNOTSUPP;
	esz = dt_size[dt];
	if (op == LFA_CSWAP && variant == ORACLE_CAS) {
		/* __atomic_compare_exchange(&d, &cmp, &src): bytewise */
		for (size_t i = 0; i < cnt; i++) {
			char *d = (char *)dst + i * esz;

			memcpy((char *)res + i * esz, d, esz);
			if (!memcmp(d, (const char *)cmp + i * esz, esz))
				memcpy(d, (const char *)src + i * esz, esz);
		}
		return 0;
	}
	if (dt == LFA_FLOAT_COMPLEX) {
		if (op == LFA_CSWAP)
			SWAP_LOOP(cf32_t, c == a);
		else
			SWAP_LOOP(cf32_t, c != a);
		return 0;
	}
	switch (op) {
	case LFA_CSWAP: SWAP_REAL_CASES(op, c == a) break;
	case LFA_CSWAP_NE: SWAP_REAL_CASES(op, c != a) break;
	case LFA_CSWAP_LE: SWAP_REAL_CASES(op, c <= a) break;
	case LFA_CSWAP_LT: SWAP_REAL_CASES(op, c < a) break;
	case LFA_CSWAP_GE: SWAP_REAL_CASES(op, c >= a) break;
	case LFA_CSWAP_GT: SWAP_REAL_CASES(op, c > a) break;
	case LFA_MSWAP:
		switch (dt) {
		case LFA_INT8: MSWAP_LOOP(int8_t); break;
		case LFA_UINT8: MSWAP_LOOP(uint8_t); break;
		case LFA_INT16: MSWAP_LOOP(int16_t); break;
		case LFA_UINT16: MSWAP_LOOP(uint16_t); break;
		case LFA_INT32: MSWAP_LOOP(int32_t); break;
		case LFA_UINT32: MSWAP_LOOP(uint32_t); break;
		case LFA_INT64: MSWAP_LOOP(int64_t); break;
		case LFA_UINT64: MSWAP_LOOP(uint64_t); break;
		case LFA_INT128: MSWAP_LOOP(i128_t); break;
		case LFA_UINT128: MSWAP_LOOP(u128_t); break;
		default: return -LFA_EOPNOTSUPP;
		}
		break;
	default:
		return -LFA_EOPNOTSUPP;
	}
	return 0;
}

/* ------------------------------------------------------------------ */
/* recursive-doubling allreduce, simulated for all ranks in-process    */
/* (coll_coll.c:349-449 schedule, :816-890 executor semantics)         */
/* ------------------------------------------------------------------ */
enum { W_SEND, W_RECV, W_REDUCE, W_COPY };

struct witem {
	int type;
	int peer;
	void *a;        /* SEND/RECV buf; REDUCE in; COPY in  */
	void *b;        /* REDUCE inout; COPY out             */
};

struct msg {
	struct msg *next;
	void *data;
};

struct rank_sched {
	struct witem item[2 * 64 + 8];
	int n, pc;
	int pend;       /* index of the posted, unmatched RECV, or -1 */
	void *result, *tmp;
};

static void push(struct rank_sched *r, int type, int peer, void *a, void *b)
{
	r->item[r->n].type = type;
	r->item[r->n].peer = peer;
	r->item[r->n].a = a;
	r->item[r->n].b = b;
	r->n++;
}

static uint64_t pow2_floor(uint64_t v)
{
	uint64_t p = 1;

	while (p * 2 <= v)
		p *= 2;
	return p;
}

/* Build one rank's schedule exactly as coll_do_allreduce orders it. */
static void sched_allreduce(struct rank_sched *r, uint64_t local, uint64_t n)
{
	uint64_t pof2 = pow2_floor(n), rem = n - pof2, newid, mask;

	if (local < 2 * rem) {
		if (local % 2 == 0) {
			push(r, W_SEND, (int)local + 1, r->result, NULL);
			newid = (uint64_t)-1;
		} else {
			push(r, W_RECV, (int)local - 1, r->tmp, NULL);
			push(r, W_REDUCE, -1, r->tmp, r->result);
			newid = local / 2;
		}
	} else {
		newid = local - rem;
	}

	if (newid != (uint64_t)-1) {
		for (mask = 1; mask < pof2; mask <<= 1) {
			uint64_t nr = newid ^ mask;
			uint64_t remote = nr < rem ? nr * 2 + 1 : nr + rem;

			push(r, W_RECV, (int)remote, r->tmp, NULL);
			push(r, W_SEND, (int)remote, r->result, NULL);
			if (remote < local) {
				push(r, W_REDUCE, -1, r->tmp, r->result);
			} else {
				push(r, W_REDUCE, -1, r->result, r->tmp);
				push(r, W_COPY, -1, r->tmp, r->result);
			}
		}
	}

	if (local < 2 * rem) {
		if (local % 2)
			push(r, W_SEND, (int)local - 1, r->result, NULL);
		else
			push(r, W_RECV, (int)local + 1, r->result, NULL);
	}
}

/*
 * Run the N-rank allreduce: send[r] (cnt elements) → result[r].
 * Messages are eager copies taken when the SEND item runs (rxm eager
 * semantics), delivered FIFO per (src, dst) pair.
 * Returns 0, -LFA_EOPNOTSUPP (no handler), -LFA_EINVAL, -LFA_ENOMEM, or
 * -LFA_EIO if the schedule deadlocks (it must not).
 */
int oracle_allreduce(int op, int dt, int nranks, const void *const *send,
		     void *const *result, size_t cnt)
{
	oracle_fn fn;
	size_t bytes;
	struct rank_sched *rs;
	struct msg **box;       /* box[src * n + dst] FIFO head */
	int r, done, progress, ret = 0;

	if (nranks < 1 || nranks > 4096)
		return -LFA_EINVAL;
	if (op < LFA_MIN || op > LFA_BXOR)
		return -LFA_ENOSYS;   /* coll_process_reduce_item :760-761 */
	fn = oracle_write_handler(ORACLE_PLAIN, op, dt);
	if (!fn)
		return -LFA_EOPNOTSUPP;
	bytes = cnt * dt_size[dt];

	rs = calloc((size_t)nranks, sizeof(*rs));
	box = calloc((size_t)nranks * nranks, sizeof(*box));
	if (!rs || !box) {
		free(rs);
		free(box);
		return -LFA_ENOMEM;
	}
	for (r = 0; r < nranks; r++) {
		rs[r].result = result[r];
		rs[r].tmp = calloc(cnt ? cnt : 1, dt_size[dt]);
		if (!rs[r].tmp) {
			ret = -LFA_ENOMEM;
			goto out;
		}
		memcpy(result[r], send[r], bytes);  /* coll_coll.c:364 */
		sched_allreduce(&rs[r], (uint64_t)r, (uint64_t)nranks);
	}

	/*
	 * Executor rule (coll_progress_work, coll_coll.c:153-227): a RECV is
	 * posted and the following SEND may start before it completes (the
	 * loop's RECV has fence 0, :398-401); any REDUCE/COPY/RECV behind it
	 * waits for the posted RECV (the SENDs carry fence 1, :404-407).
	 */
	for (r = 0; r < nranks; r++)
		rs[r].pend = -1;
	do {
		done = 1;
		progress = 0;
		for (r = 0; r < nranks; r++) {
			struct rank_sched *s = &rs[r];

			for (;;) {
				if (s->pend >= 0) {
					struct witem *p = &s->item[s->pend];
					struct msg **head = &box[(size_t)p->peer * nranks + r];
					struct msg *m = *head;

					if (m) {
						*head = m->next;
						memcpy(p->a, m->data, bytes);
						free(m->data);
						free(m);
						s->pend = -1;
						progress = 1;
					}
				}
				if (s->pc >= s->n)
					break;

				struct witem *w = &s->item[s->pc];

				if (w->type == W_SEND) {
					struct msg *m = malloc(sizeof(*m)), **tail;

					if (!m || !(m->data = malloc(bytes ? bytes : 1))) {
						free(m);
						ret = -LFA_ENOMEM;
						goto out;
					}
					memcpy(m->data, w->a, bytes);
					m->next = NULL;
					tail = &box[(size_t)r * nranks + w->peer];
					while (*tail)
						tail = &(*tail)->next;
					*tail = m;
				} else if (s->pend >= 0) {
					break;   /* fenced behind an outstanding RECV */
				} else if (w->type == W_RECV) {
					s->pend = s->pc;
				} else if (w->type == W_REDUCE) {
					fn(w->b, w->a, cnt);  /* (inout, in, count) */
				} else {
					memcpy(w->b, w->a, bytes);
				}
				s->pc++;
				progress = 1;
			}
			if (s->pc < s->n || s->pend >= 0)
				done = 0;
		}
		if (!done && !progress) {
			ret = -LFA_EIO;
			goto out;
		}
	} while (!done);

out:
	for (r = 0; r < nranks; r++)
		free(rs[r].tmp);
	if (box) {
		for (size_t k = 0; k < (size_t)nranks * nranks; k++) {
			while (box[k]) {
				struct msg *m = box[k];

				box[k] = m->next;
				free(m->data);
				free(m);
			}
		}
	}
	free(box);
	free(rs);
	return ret;
}

/* Number of schedule items for a rank (used by tests of the host schedule). */
int oracle_allreduce_sched_len(int rank, int nranks)
{
	struct rank_sched *s = calloc(1, sizeof(*s));
	int n;

	if (!s)
		return -LFA_ENOMEM;
	s->result = s->tmp = NULL;
	sched_allreduce(s, (uint64_t)rank, (uint64_t)nranks);
	n = s->n;
	free(s);
	return n;
}
