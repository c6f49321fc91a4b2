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

#include "lfa_solo_body.hpp"
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

// One-member copy ending in the completion word (lfa_solo_copy_async):
// lfa_solo_body.hpp, shared with the direct-dispatch kernel.
__global__ __launch_bounds__(256) void solo_copy(char *dst, const char *src, size_t bytes,
                                                 uint32_t nblocks, uint32_t *ctr,
                                                 uint64_t *word, uint64_t val) {
  lfa_solo_body(dst, src, bytes, nblocks, ctr, word, val);
}

}  // namespace

extern "C" int lfa_solo_copy_async(void *result, const void *send, size_t bytes,
                                   uint32_t *done_ctr, uint64_t *done_word, uint64_t done_val,
                                   void *stream) {
  if (!bytes) return 0;
  if (!result || !send || !done_ctr || !done_word || bytes > ((size_t)1 << 30))
    return -LFA_EINVAL;
  const unsigned grid = lfa_solo_blocks(result, send, bytes);
  hipLaunchKernelGGL(solo_copy, dim3(grid), dim3(256), 0, (hipStream_t)stream, (char *)result,
                     (const char *)send, bytes, grid, done_ctr, done_word, done_val);
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
