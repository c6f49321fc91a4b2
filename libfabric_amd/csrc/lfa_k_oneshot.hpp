// lfa_k_oneshot.hpp — the one-shot kernels of LFA_STEP_ONESHOT (oneshot_reduce, and the LL form oneshot_ll).
// Part of lfa_kernels.hpp (split in round 6); included by it, in order, after
// the shared helpers and the combine kernels.  Not included on its own.
#pragma once

namespace lfa {

// ---------------------------------------------------------------------------
// one-shot reduction (LFA_STEP_ONESHOT, lfa_signal.h): push, post, wait,
// reduce — one launch for a small bucket instead of copy + barrier + tree +
// barrier.  Destination k receives bytes [soff[k], soff[k] + slen[k]) of this
// rank's input (the whole vector for allreduce, block k for reduce_scatter,
// the root alone for reduce).  Workgroup b owns bytes [b·chunk, (b+1)·chunk)
// of every such range and synchronises only with the peers' workgroup b.
// ---------------------------------------------------------------------------
constexpr int kOsMax = LFA_OS_MAX_RANKS;

// One system-scope release / acquire per workgroup (0, the product) or per
// wave (1, round 2's first form).  A workgroup's waves share a CU and so an
// L2, which makes the single pair sufficient on one GPU — every
// cross-process test runs on one MI355X — but its ordering across GPUs over
// xGMI has not run anywhere yet, so the per-wave form stays
// selectable: build with -DLFA_OS_WAVE_FENCES=1.
#ifndef LFA_OS_WAVE_FENCES
#define LFA_OS_WAVE_FENCES 0
#endif

// The one-shot's association tree over at most kOsMax leaves (TreeArgs has
// room for 32): the kernel's argument block is 376 bytes instead of ~670, one
// 64-byte line of it read per 64 bytes on every launch — the n = 1 kernel
// with the larger block took ~1 us longer from launch to completion word
// than a 48-byte one (profiles/r04_solo_2.json).
struct OsTree {
  const void *in[kOsMax];      // own input range (k == rank) or own slot k
  signed char hi[kOsMax];
  signed char lo[kOsMax];
};

struct OsArgs {
  OsTree t;
  char *push[kOsMax];          // peer k's slot of this rank (k != rank)
  uint32_t *post[kOsMax];      // peer k's one-shot rows, column `rank`
  uint32_t soff[kOsMax];       // input range pushed to k (k == rank: reduced)
  uint32_t slen[kOsMax];
  const uint32_t *wait;        // own one-shot rows
  const char *send;
  char *result;
  uint64_t *status;
  uint64_t timeout;            // wall-clock ticks
  size_t chunk;                // a multiple of 16
  uint64_t ticket;
  uint32_t epoch;
  int n, rank;
  int vec;                     // every range start and result 16-B aligned
  int unal;                    // send or result not aligned to the element
  uint32_t *done_ctr;          // completion word (lfa_signal.h), optional
  uint64_t *done_word;
  uint64_t done_val;
};
static_assert(sizeof(OsArgs) == 376, "the one-shot's argument block (see OsTree)");

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void oneshot_reduce(OsArgs a) {
  constexpr size_t E = sizeof(T);
  const unsigned t = threadIdx.x;
  const size_t b = blockIdx.x;
  const size_t lo = b * a.chunk;
  // 1. push this rank's chunk of each destination's range into its slot on
  //    that peer (system-scope write-through stores over xGMI)
  for (int k = 0; k < a.n; k++) {  // wave-uniform
    if (k == a.rank || lo >= a.slen[k]) continue;
    const size_t hi = lo + a.chunk < a.slen[k] ? lo + a.chunk : a.slen[k];
    const size_t vhi = a.vec ? hi & ~(size_t)15 : lo;
    const char *src = a.send + a.soff[k];
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(a.push[k], (unsigned)a.slen[k]);
    for (size_t o = lo + (size_t)t * 16; o < vhi; o += (size_t)kBlock * 16)
      __builtin_amdgcn_raw_buffer_store_b128(*(const u32x4 *)(src + o), r, (unsigned)o, 0,
                                             kSysAux);
    for (size_t o = vhi + t; o < hi; o += kBlock)
      sys_store<uint8_t>((uint8_t *)a.push[k] + o, (uint8_t)src[o]);
  }
  // 2. every wave's pushes acknowledged (write-through, so in the peer's
  //    memory), then ONE system-scope release for the workgroup — its waves
  //    share a CU and so an L2 — and one post per peer
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (a.n > 1 && (LFA_OS_WAVE_FENCES || t < 64))  // wave 0: the posting lanes
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
  if ((int)t < a.n && (int)t != a.rank) {
    __hip_atomic_store(a.post[t] + b * LFA_SIG_MAX, a.epoch, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    // 3. wait for peer t's workgroup b (bounded: *status on timeout)
    const uint32_t *w = a.wait + b * LFA_SIG_MAX + t;
    const uint64_t t0 = wall_clock64();
    while ((int32_t)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) -
                     a.epoch) < 0) {
      if (wall_clock64() - t0 > a.timeout) {
        lfa_sig_note_timeout(a.status, a.ticket);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  // the waiting wave acquires for the workgroup (same CU, same L2), then
  // every wave may read what the peers pushed
  if (a.n > 1 && (LFA_OS_WAVE_FENCES || t < 64)) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  __syncthreads();
  // 4. reduce chunk b of this rank's own range over every rank's input, rank
  //    order (system-scope loads: the slots were written by peers over xGMI)
  const size_t own = a.slen[a.rank];
  bool plain = false;  // this workgroup wrote result bytes with plain stores
  if (lo < own) {
    const size_t hi = lo + a.chunk < own ? lo + a.chunk : own;
    const size_t vhi = a.vec ? hi & ~(size_t)15 : lo;
    plain = a.unal || vhi < hi;
    for (size_t o = lo + (size_t)t * 16; o < vhi; o += (size_t)kBlock * 16) {
      u32x4 v = tree_eval_with<OP, T, u32x4, NLEAF>(a.t, [&](int k) {
        return __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(tile_rsrc(a.t.in[k], (unsigned)own),
                                                         (unsigned)o, 0, kSysLoadAux));
      });
      // write-through: the release before the completion word then has no
      // dirty result lines to write back
      __builtin_amdgcn_raw_buffer_store_b128(v, tile_rsrc(a.result, (unsigned)own), (unsigned)o,
                                             0, kSysAux);
    }
    if (a.unal) {
      // the caller's own input and result, byte-wise (local memory); the
      // peers' slots (256-B aligned) keep their system-scope loads
      for (size_t e = lo / E + t; e < hi / E; e += kBlock)
        st_bytes<T>(a.result, e, tree_eval_with<OP, T, T, NLEAF>(a.t, [&](int k) {
                      return k == a.rank ? ld_bytes<T>(a.t.in[k], e)
                                         : sys_load<T>((const T *)a.t.in[k] + e);
                    }));
    } else {
      for (size_t e = vhi / E + t; e < hi / E; e += kBlock) {
        T v = tree_eval_with<OP, T, T, NLEAF>(
            a.t, [&](int k) { return sys_load<T>((const T *)a.t.in[k] + e); });
        ((T *)a.result)[e] = v;
      }
    }
  }
  // 5. completion word: this workgroup's result stores acknowledged, then it
  //    counts itself; the last workgroup resets the counter for the next
  //    launch on the stream and publishes done_val to the host.  Write-
  //    through stores are in memory once acknowledged, so a workgroup that
  //    made only those adds relaxed with no release of its own (an L2
  //    write-back saved per workgroup, as in lfa_signal.hip solo_copy); one
  //    with plain (byte-wise or tail) stores releases them first at system
  //    scope (its waves share a CU and an L2).  The last one acquires the
  //    others' adds, then releases before the word.
  if (a.done_word) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0 && gridDim.x == 1) {
      // one workgroup: no counter to count in (one device atomic less)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (t == 0) {
      if (plain) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      const uint32_t seen = __hip_atomic_fetch_add(a.done_ctr, 1u, __ATOMIC_RELAXED,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      if (seen + 1 == gridDim.x) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        __hip_atomic_store(a.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// LL one-shot (lfa_signal.h): parts of at most LFA_OS_LL_BYTES.  Lane c owns
// bytes [16c, 16c + 16) of every part: it pushes its 16 bytes of each peer's
// part as two 16-byte stores of {data, flag, data, flag} into that peer's LL
// slot for this rank, then polls its own slots' words until every peer's four
// flags read 2·epoch + 1 — the 8-byte {data, flag} pairs are written and read
// whole, so a matching flag carries its data — and reduces the values in
// prov/coll's association order.  No acknowledgement wait, fence or flag post
// between push and wait, and the poll is the read.  Same completion word and
// timeout as oneshot_reduce.
// ---------------------------------------------------------------------------
struct LlArgs {
  const char *send;
  char *result;
  char *push[kOsMax];          // peer k's LL slot of this rank, this parity
  const char *own;             // this rank's LL slots, this parity
  uint64_t *status;
  uint64_t ticket, timeout;    // timeout: wall-clock ticks
  uint32_t *done_ctr;
  uint64_t *done_word;
  uint64_t done_val;
  uint32_t soff[kOsMax], slen[kOsMax];
  uint32_t flag;
  int n, rank, vec;            // vec: every part start and result 16-B aligned
  signed char hi[kOsMax], lo[kOsMax];  // the association tree's leaves
};

// 16 bytes at base + off, bytes at or past len read as zero (registers only)
__device__ __forceinline__ u32x4 ll_in(const char *base, uint32_t off, uint32_t len, int vec) {
  if (vec && off + 16 <= len) return *(const u32x4 *)(base + off);
  u32x4 v = {0, 0, 0, 0};
#pragma unroll
  for (int w = 0; w < 4; w++) {
    uint32_t x = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t i = off + 4 * w + b;
      if (i < len) x |= (uint32_t)(unsigned char)base[i] << (8 * b);
    }
    v[w] = x;
  }
  return v;
}

__device__ __forceinline__ void ll_out(char *base, uint32_t off, uint32_t len, int vec, u32x4 v) {
  if (vec && off + 16 <= len) {
    *(u32x4 *)(base + off) = v;
    return;
  }
#pragma unroll
  for (int w = 0; w < 4; w++)
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t i = off + 4 * w + b;
      if (i < len) base[i] = (char)(v[w] >> (8 * b));
    }
}

// vals[k] for a wave-uniform k without indexing registers dynamically
__device__ __forceinline__ u32x4 ll_pick(const u32x4 (&v)[kOsMax], int k) {
  u32x4 r = v[0];
#pragma unroll
  for (int i = 1; i < kOsMax; i++)
    if (k == i) r = v[i];
  return r;
}

template <int OP, typename T, int NLEAF>
__global__ __launch_bounds__(kBlock) void oneshot_ll(LlArgs a) {
  const unsigned t = threadIdx.x;
  const uint32_t off = ((uint32_t)blockIdx.x * kBlock + t) * 16u;
  // 1. push this lane's 16 bytes of every peer's part
#pragma unroll
  for (int k = 0; k < kOsMax; k++) {
    if (k >= a.n || k == a.rank || off >= a.slen[k]) continue;
    const u32x4 v = ll_in(a.send + a.soff[k], off, a.slen[k], a.vec);
    const __amdgpu_buffer_rsrc_t r = tile_rsrc(a.push[k], LFA_SIG_LL_SLOT);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[0], a.flag, v[1], a.flag}, r, 2 * off, 0,
                                           kSysAux);
    __builtin_amdgcn_raw_buffer_store_b128(u32x4{v[2], a.flag, v[3], a.flag}, r, 2 * off + 16,
                                           0, kSysAux);
  }
  // 2. this rank's part.  First one lane per wave polls, per peer, the words
  //    of the wave's last chunk (one 16-B load per peer per round instead of
  //    the wave's 128), then every lane reads its own words and polls them
  //    until their flags match — most do on the first read
  const uint32_t own = a.slen[a.rank];
  const uint32_t lane = t & 63u, wave0 = off - lane * 16u;
  if (wave0 < own && lane == 0) {
    const uint32_t last_chunk = (own - 1u) / 16u * 16u;
    const uint32_t last = wave0 + 63u * 16u < last_chunk ? wave0 + 63u * 16u : last_chunk;
    uint32_t pending = 0;
#pragma unroll
    for (int k = 0; k < kOsMax; k++)
      if (k < a.n && k != a.rank) pending |= 1u << k;
    const uint64_t t0 = wall_clock64();
    while (pending) {
#pragma unroll
      for (int k = 0; k < kOsMax; k++) {
        if (!(pending >> k & 1u)) continue;
        const u32x4 w1 = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(
                       tile_rsrc(a.own + (size_t)k * LFA_SIG_LL_SLOT, LFA_SIG_LL_SLOT),
                       2 * last + 16, 0, kSysLoadAux));
        if (w1[1] == a.flag && w1[3] == a.flag) pending &= ~(1u << k);
      }
      if (pending) {
        if (wall_clock64() - t0 > a.timeout) break;   // the lanes below note it
        __builtin_amdgcn_s_sleep(1);
      }
    }
  }
  if (off < own) {
    u32x4 vals[kOsMax];
    uint32_t pending = 0;
    const u32x4 mine = ll_in(a.send + a.soff[a.rank], off, own, a.vec);
#pragma unroll
    for (int k = 0; k < kOsMax; k++) {
      vals[k] = k == a.rank ? mine : u32x4{0, 0, 0, 0};
      if (k < a.n && k != a.rank) pending |= 1u << k;
    }
    const uint64_t t0 = wall_clock64();
    while (pending) {
#pragma unroll
      for (int k = 0; k < kOsMax; k++) {
        if (!(pending >> k & 1u)) continue;
        const __amdgpu_buffer_rsrc_t r =
            tile_rsrc(a.own + (size_t)k * LFA_SIG_LL_SLOT, LFA_SIG_LL_SLOT);
        const u32x4 w0 = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, 2 * off, 0, kSysLoadAux));
        const u32x4 w1 = __builtin_bit_cast(
            u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, 2 * off + 16, 0, kSysLoadAux));
        if (w0[1] == a.flag && w0[3] == a.flag && w1[1] == a.flag && w1[3] == a.flag) {
          vals[k] = u32x4{w0[0], w0[2], w1[0], w1[2]};
          pending &= ~(1u << k);
        }
      }
      if (pending) {
        if (wall_clock64() - t0 > a.timeout) {
          lfa_sig_note_timeout(a.status, a.ticket);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
    }
    ll_out(a.result, off, own, a.vec,
           tree_eval_with<OP, T, u32x4, NLEAF>(a, [&](int k) { return ll_pick(vals, k); }));
  }
  // 3. completion word, as oneshot_reduce's step 5
  if (a.done_word) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (t == 0 && gridDim.x == 1) {
      // one workgroup: no counter to count in (one device atomic less)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    } else if (t == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
      const uint32_t seen = __hip_atomic_fetch_add(a.done_ctr, 1u, __ATOMIC_ACQ_REL,
                                                   __HIP_MEMORY_SCOPE_AGENT);
      if (seen + 1 == gridDim.x) {
        __hip_atomic_store(a.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        __hip_atomic_store(a.done_word, a.done_val, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
  }
}

}  // namespace lfa
