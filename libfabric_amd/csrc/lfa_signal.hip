// lfa_signal.hip — device-side barrier of LFA_ALGO_P2P (liblfa.so).
//
// One wave per barrier: lane k (k != rank) posts the epoch into this rank's
// word of peer k's flag row (a system-scope store over xGMI), then polls word
// k of its OWN row until peer k has posted the same epoch.  Polling stays in
// local HBM; the only xGMI traffic is one 4-byte store per peer.  Every
// access is a vector-memory atomic at system scope.  A wait is bounded by the
// GPU's constant-rate wall clock: a member that never arrives (a crashed
// peer, mismatched collectives) turns into an error completion on the host
// (*status, host-mapped) instead of a wave that never retires.
#include <hip/hip_runtime.h>
#include <string.h>

#include "lfa_signal.h"
#include "../../include/lfa_fabric.h"

namespace {

struct BarArgs {
  uint32_t *post[LFA_SIG_MAX];
  const uint32_t *wait;
  uint64_t *status;
  uint64_t timeout;  // wall-clock ticks
  uint64_t ticket;
  uint32_t epoch;
  int n, rank;
};

__global__ __launch_bounds__(64) void flag_barrier(BarArgs a) {
  const int k = threadIdx.x;
  if (k >= a.n || k == a.rank) return;
  // The steps before this one have retired (stream order); this makes their
  // writes visible at system scope before the peer can observe the epoch.
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  __hip_atomic_store(a.post[k], a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  const uint64_t t0 = wall_clock64();
  // epochs wrap: compare by signed distance
  while ((int32_t)(__hip_atomic_load(a.wait + k, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_SYSTEM) - a.epoch) < 0) {
    if (wall_clock64() - t0 > a.timeout) {
      lfa_sig_note_timeout(a.status, a.ticket);
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  // later steps read what the peers wrote before posting
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
}

// One-member copy ending in the completion word (lfa_solo_copy_async).
// Workgroup b copies bytes [b·4 KiB, (b+1)·4 KiB): 16 B per lane when both
// pointers are 16-B aligned, byte-wise otherwise and for the tail.
__global__ __launch_bounds__(256) void solo_copy(char *dst, const char *src, size_t bytes,
                                                 uint32_t *ctr, uint64_t *word,
                                                 uint64_t val) {
  const unsigned t = threadIdx.x;
  const size_t lo = (size_t)blockIdx.x * 4096;
  const size_t hi = lo + 4096 < bytes ? lo + 4096 : bytes;
  const bool vec = (((uintptr_t)dst | (uintptr_t)src) & 15) == 0;
  const size_t vhi = vec ? lo + ((hi - lo) & ~(size_t)15) : lo;
  if (lo + (size_t)t * 16 < vhi) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    // write-through (sc0 sc1): the release below has no dirty lines to write
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(dst + lo, 0, 4096, 0x00020000);
    __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)(src + lo + (size_t)t * 16), r,
                                           t * 16, 0, 17);
  }
  for (size_t o = vhi + t; o < hi; o += 256) dst[o] = src[o];
  // the completion word: this workgroup's stores acknowledged, then the
  // last workgroup publishes `val` (lfa_signal.h); a single workgroup
  // publishes it without the counter.  Write-through stores are in memory
  // once acknowledged (the s_waitcnt), so such a workgroup adds to the
  // counter with no fence of its own; one with byte-wise (plain) stores
  // releases them at system scope first.  The last one acquires the others'
  // adds and releases before the word.  A release per workgroup (an L2
  // write-back each, and one more in an acq_rel add) cost 3.3 us at 1 MiB
  // (256 workgroups: 13.7 -> 10.4 us launch to word, round 5,
  // tools/probe_solo_multi.py).
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (t == 0 && gridDim.x == 1) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  } else if (t == 0) {
    if (vhi != hi) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    const uint32_t seen =
        __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (seen + 1 == gridDim.x) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(word, val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace

extern "C" int lfa_solo_copy_async(void *result, const void *send, size_t bytes,
                                   uint32_t *done_ctr, uint64_t *done_word, uint64_t done_val,
                                   void *stream) {
  if (!bytes) return 0;
  if (!result || !send || !done_ctr || !done_word || bytes > ((size_t)1 << 30))
    return -LFA_EINVAL;
  const unsigned grid = (unsigned)((bytes + 4095) / 4096);
  hipLaunchKernelGGL(solo_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, (char *)result,
                     (const char *)send, bytes, done_ctr, done_word, done_val);
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}

extern "C" size_t lfa__sig_area_bytes(void) { return LFA_SIG_AREA_BYTES; }

extern "C" uint64_t lfa__wallclock_ticks_per_us(void) {
  static uint64_t t = 0;
  if (!t) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess ||
        khz <= 0)
      khz = 100000;  // gfx9's constant 100 MHz
    t = (uint64_t)khz / 1000 ? (uint64_t)khz / 1000 : 1;
  }
  return t;
}

extern "C" int lfa_flag_barrier_async(uint32_t *const *post, const uint32_t *wait, int n,
                                      int rank, uint32_t epoch, uint64_t *status,
                                      uint64_t ticket, uint64_t timeout_us, void *stream) {
  if (n < 1 || n > LFA_SIG_MAX || rank < 0 || rank >= n || !wait || !status || !post)
    return -LFA_EINVAL;
  if (n == 1) return 0;
  BarArgs a;
  memset(&a, 0, sizeof(a));
  for (int k = 0; k < n; k++) {
    if (k != rank && !post[k]) return -LFA_EINVAL;
    a.post[k] = k == rank ? nullptr : post[k];
  }
  a.wait = wait;
  a.status = status;
  a.timeout = timeout_us * lfa__wallclock_ticks_per_us();
  a.epoch = epoch;
  a.ticket = ticket;
  a.n = n;
  a.rank = rank;
  hipLaunchKernelGGL(flag_barrier, dim3(1), dim3(64), 0, (hipStream_t)stream, a);
  return hipGetLastError() == hipSuccess ? 0 : -LFA_EIO;
}
