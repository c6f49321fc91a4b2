// Direct dispatch (lfa_signal.h lfa_direct_*): small kernels launched with
// liblfa's own AQL packets on its own HSA queue, bypassing HIP's launch path.
//
// A HIP launch costs ~3.0 us of host time on this part (lfa_bench_raw
// "launch_only"), half of the 6.1 us from a host launch to a host-visible word
// (profiles/r04_solo_2.json).  Writing a 64-byte dispatch packet into a
// user-mode queue and ringing its doorbell is a few stores.  The queue is
// this library's alone, so the kernels on it are not ordered with any HIP
// stream: the provider uses it only for operations that need no ordering with
// stream work — a one-member group's small reducing collective, whose input
// the caller has finished writing before the call and whose output belongs to
// the provider until its completion is read.  Packets on
// the queue carry the barrier bit, so its kernels run and complete in order.
//
// The code object (lfa_direct_k.hip) is a plain gfx950 ELF embedded at build
// time; its kernels take every launch parameter as an explicit argument, so
// a packet's kernarg block is the argument struct below and nothing else.
#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "lfa_fabric.h"
#include "lfa_atomic.h"
#include "lfa_signal.h"

extern "C" const unsigned char lfa_direct_co[], lfa_direct_co_pl[];
extern "C" const size_t lfa_direct_co_size, lfa_direct_co_pl_size;

namespace {

constexpr uint32_t kQueueSize = 256;        // packets; also the kernarg slots

struct SoloArgs {                           // lfa_direct_solo_copy's kernarg block
  void *dst;
  const void *src;
  uint64_t bytes;
  uint32_t nblocks;
  uint32_t pad;
  uint32_t *ctr;
  uint64_t *word;
  uint64_t val;
};
static_assert(sizeof(SoloArgs) == 56, "kernarg layout of lfa_direct_solo_copy");

struct FindGpu {
  uint32_t bdf;
  uint32_t domain;
  hsa_agent_t agent;
  int found;
};

hsa_status_t find_gpu(hsa_agent_t a, void *data) {
  FindGpu *f = (FindGpu *)data;
  hsa_device_type_t type;
  uint32_t bdf = 0, domain = 0;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS ||
      type != HSA_DEVICE_TYPE_GPU)
    return HSA_STATUS_SUCCESS;
  if (hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf) !=
          HSA_STATUS_SUCCESS ||
      hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &domain) !=
          HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (bdf == f->bdf && domain == f->domain) {
    f->agent = a;
    f->found = 1;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg(hsa_region_t r, void *data) {
  uint32_t flags = 0;
  hsa_region_segment_t seg;
  if (hsa_region_get_info(r, HSA_REGION_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_REGION_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  if (hsa_region_get_info(r, HSA_REGION_INFO_GLOBAL_FLAGS, &flags) == HSA_STATUS_SUCCESS &&
      (flags & HSA_REGION_GLOBAL_FLAG_KERNARG)) {
    *(hsa_region_t *)data = r;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

}  // namespace

struct lfa_direct {
  hsa_agent_t gpu;
  hsa_queue_t *q;
  hsa_code_object_reader_t reader, reader_pl;
  hsa_executable_t exe;
  uint64_t solo_kobj;
  uint32_t solo_private, solo_group;
  char *kernarg;                            // kQueueSize slots of 64 B
  uint16_t header;                          // the dispatch packets' header
  pthread_mutex_t lock;
  int hsa_up, have_reader, have_reader_pl, have_exe;
  // 0, or why the queue is no longer used: 1 the runtime reported a queue
  // error (queue_error), 2 the ring stayed full for ring_timeout_ns (its
  // kernels do not finish), 3 marked by a test.  Once set, every submit
  // returns -LFA_EIO and the provider fails the operations whose words the
  // queue still owed (lfa_coll.c word_state).
  int failed;
  uint64_t ring_timeout_ns;
  // Stub queue (CPU tests, lfa__direct_stub_open): no HSA; the packets go to
  // a host ring and the read index is the caller's word.
  int stub;
  uint64_t stub_write;
  const volatile uint64_t *stub_read;
  hsa_kernel_dispatch_packet_t *stub_ring;
};

namespace {

uint64_t now_ns() {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return (uint64_t)t.tv_sec * 1000000000ull + (uint64_t)t.tv_nsec;
}

// The ring's bound: LFA_SIG_TIMEOUT_MS, the provider's bound on every GPU
// wait (default 20 s).
uint64_t ring_timeout_ns() {
  const char *e = lfa_param("LFA_SIG_TIMEOUT_MS");
  const long ms = e ? atol(e) : 0;
  return (uint64_t)(ms > 0 ? ms : 20000) * 1000000ull;
}

void mark_failed(struct lfa_direct *d, int why) {
  int none = 0;
  if (__atomic_compare_exchange_n(&d->failed, &none, why, false, __ATOMIC_ACQ_REL,
                                  __ATOMIC_ACQUIRE))
    fprintf(stderr, "lfa: direct queue %s: its operations fail with EIO, later ones "
            "take the HIP launch\n",
            why == 1 ? "error reported by the runtime"
                     : why == 2 ? "ring full past LFA_SIG_TIMEOUT_MS" : "marked failed");
}

// hsa_queue_create's error callback: the runtime found the queue broken
// (an invalid packet, a kernel that faulted on it).
void queue_error(hsa_status_t status, hsa_queue_t *, void *data) {
  fprintf(stderr, "lfa: direct queue: hsa_status %#x\n", (unsigned)status);
  mark_failed((struct lfa_direct *)data, 1);
}

uint64_t read_index(const struct lfa_direct *d) {
  return d->stub ? __atomic_load_n(d->stub_read, __ATOMIC_ACQUIRE)
                 : hsa_queue_load_read_index_scacquire(d->q);
}

// Room for packet idx: the kernarg slot of packet idx - kQueueSize is free
// once the read index has passed idx - (kQueueSize - 1) (see
// lfa_direct_solo_copy).  Bounded: 0, or -LFA_EIO when the queue has failed
// or the ring has not moved for ring_timeout_ns — the queue is then marked
// failed, since a ring that does not drain holds kernels that do not finish.
int ring_wait(struct lfa_direct *d, uint64_t idx) {
  if (idx - read_index(d) < kQueueSize - 1) return 0;
  const uint64_t t0 = now_ns();
  while (idx - read_index(d) >= kQueueSize - 1) {
    if (__atomic_load_n(&d->failed, __ATOMIC_ACQUIRE)) return -LFA_EIO;
    if (now_ns() - t0 > d->ring_timeout_ns) {
      mark_failed(d, 2);
      return -LFA_EIO;
    }
    __builtin_ia32_pause();
  }
  return 0;
}

}  // namespace

extern "C" int lfa_direct_failed(const struct lfa_direct *d) {
  return d ? __atomic_load_n(&d->failed, __ATOMIC_ACQUIRE) : 0;
}

// Test hook: the queue as if the runtime had reported an error.
extern "C" void lfa__direct_mark_failed(struct lfa_direct *d) {
  if (d) mark_failed(d, 3);
}

// Test hook: a stub queue with no HSA behind it (CPU tests of the bounded
// ring wait).  Its packets land in a host ring; `read_index` plays the
// packet processor's read index; the ring bound is timeout_ms.
extern "C" struct lfa_direct *lfa__direct_stub_open(const volatile uint64_t *read_index,
                                                    uint64_t timeout_ms) {
  if (!read_index) return nullptr;
  struct lfa_direct *d = (struct lfa_direct *)calloc(1, sizeof(*d));
  if (!d) return nullptr;
  d->stub_ring =
      (hsa_kernel_dispatch_packet_t *)calloc(kQueueSize, sizeof(hsa_kernel_dispatch_packet_t));
  d->kernarg = (char *)calloc(kQueueSize, 64);
  if (!d->stub_ring || !d->kernarg) {
    free(d->stub_ring);
    free(d->kernarg);
    free(d);
    return nullptr;
  }
  pthread_mutex_init(&d->lock, nullptr);
  d->stub = 1;
  d->stub_read = read_index;
  d->ring_timeout_ns = timeout_ms * 1000000ull;
  d->header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                         (1u << HSA_PACKET_HEADER_BARRIER));
  return d;
}

// Test hook: packets written to the stub queue so far.
extern "C" uint64_t lfa__direct_stub_written(const struct lfa_direct *d) {
  return d && d->stub ? d->stub_write : 0;
}

extern "C" void lfa_direct_close(struct lfa_direct *d) {
  if (!d) return;
  if (d->stub) {
    free(d->stub_ring);
    free(d->kernarg);
    pthread_mutex_destroy(&d->lock);
    free(d);
    return;
  }
  if (d->q) hsa_queue_destroy(d->q);
  if (d->kernarg) hsa_memory_free(d->kernarg);
  if (d->have_exe) hsa_executable_destroy(d->exe);
  if (d->have_reader) hsa_code_object_reader_destroy(d->reader);
  if (d->have_reader_pl) hsa_code_object_reader_destroy(d->reader_pl);
  if (d->hsa_up) hsa_shut_down();
  pthread_mutex_destroy(&d->lock);
  free(d);
}

extern "C" struct lfa_direct *lfa_direct_open(int device) {
  char bus[32];
  unsigned dom = 0, b = 0, dv = 0, fn = 0;
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess ||
      sscanf(bus, "%x:%x:%x.%x", &dom, &b, &dv, &fn) != 4) {
    (void)hipGetLastError();
    return nullptr;
  }
  struct lfa_direct *d = (struct lfa_direct *)calloc(1, sizeof(*d));
  if (!d) return nullptr;
  pthread_mutex_init(&d->lock, nullptr);
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    lfa_direct_close(d);
    return nullptr;
  }
  d->hsa_up = 1;
  FindGpu f = {(b << 8) | (dv << 3) | fn, dom, {0}, 0};
  hsa_iterate_agents(find_gpu, &f);
  hsa_region_t karg = {0};
  hsa_executable_symbol_t sym;
  uint32_t kernarg_size = 0;
  bool ok = f.found;
  d->gpu = f.agent;
  ok = ok && hsa_agent_iterate_regions(d->gpu, find_kernarg, &karg) == HSA_STATUS_INFO_BREAK;
  // LFA_DIRECT_PRELOAD=1: the build whose arguments the packet processor
  // preloads into SGPRs (lfa_direct_k.hip)
  const char *pe = lfa_param("LFA_DIRECT_PRELOAD");
  const bool pl = pe && pe[0] == '1';
  ok = ok && hsa_code_object_reader_create_from_memory(lfa_direct_co, lfa_direct_co_size,
                                                       &d->reader) == HSA_STATUS_SUCCESS;
  d->have_reader = ok;
  ok = ok && hsa_code_object_reader_create_from_memory(lfa_direct_co_pl, lfa_direct_co_pl_size,
                                                       &d->reader_pl) == HSA_STATUS_SUCCESS;
  d->have_reader_pl = ok;
  ok = ok && hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT,
                                       nullptr, &d->exe) == HSA_STATUS_SUCCESS;
  d->have_exe = ok;
  ok = ok && hsa_executable_load_agent_code_object(d->exe, d->gpu, pl ? d->reader_pl : d->reader,
                                                   nullptr, nullptr) == HSA_STATUS_SUCCESS &&
       hsa_executable_freeze(d->exe, nullptr) == HSA_STATUS_SUCCESS &&
       hsa_executable_get_symbol_by_name(
           d->exe, pl ? "lfa_direct_solo_copy_pl.kd" : "lfa_direct_solo_copy.kd", &d->gpu,
           &sym) == HSA_STATUS_SUCCESS &&
       hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT,
                                      &d->solo_kobj) == HSA_STATUS_SUCCESS &&
       hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE,
                                      &kernarg_size) == HSA_STATUS_SUCCESS &&
       hsa_executable_symbol_get_info(sym,
                                      HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE,
                                      &d->solo_private) == HSA_STATUS_SUCCESS &&
       hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE,
                                      &d->solo_group) == HSA_STATUS_SUCCESS;
  // the kernarg block must be exactly the argument struct (no hidden arguments)
  ok = ok && kernarg_size == sizeof(SoloArgs) && d->solo_kobj;
  ok = ok && hsa_memory_allocate(karg, (size_t)kQueueSize * 64, (void **)&d->kernarg) ==
                 HSA_STATUS_SUCCESS;
  // single producer (every write under d->lock); the runtime reports a broken
  // queue to queue_error instead of leaving its words unwritten silently
  d->ring_timeout_ns = ring_timeout_ns();
  ok = ok && hsa_queue_create(d->gpu, kQueueSize, HSA_QUEUE_TYPE_SINGLE, queue_error, d,
                              UINT32_MAX, UINT32_MAX, &d->q) == HSA_STATUS_SUCCESS &&
       d->q->size >= kQueueSize;    // the ring wait below counts kernarg slots
  if (!ok) {
    lfa_direct_close(d);
    return nullptr;
  }
  // The packet's acquire / release fence scopes.  The kernel itself releases
  // its stores at system scope before it publishes the completion word, so
  // the packet's end-of-kernel release adds nothing the host or a later kernel
  // needs; at system scope it is a cache writeback that the next packet (the
  // barrier bit) waits for.  LFA_DIRECT_FENCE: two letters, acquire then
  // release, s(ystem) / a(gent) / n(one); default "an".
  const char *fe = lfa_param("LFA_DIRECT_FENCE");
  auto scope = [](char c) {
    return c == 's' ? HSA_FENCE_SCOPE_SYSTEM : c == 'a' ? HSA_FENCE_SCOPE_AGENT
                                                        : HSA_FENCE_SCOPE_NONE;
  };
  const char acq = fe && fe[0] ? fe[0] : 'a', rel = fe && fe[0] && fe[1] ? fe[1] : 'n';
  d->header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                         (1u << HSA_PACKET_HEADER_BARRIER) |
                         (scope(acq) << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                         (scope(rel) << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
  return d;
}

// Enqueue lfa_direct_solo_copy.  The kernarg slot of packet i is reused by
// packet i + kQueueSize.  The read index passes i + 1 only once the packet
// processor has consumed packet i + 1, whose barrier bit held it until packet
// i's kernel completed — so the writer waits for that before reusing i's slot
// (one slot of the ring stays unused).  The wait is bounded (ring_wait) and
// happens before the write index moves, so a submit that gives up leaves no
// hole in the ring: 0, -LFA_EINVAL, or -LFA_EIO (the queue failed; the
// caller launches through HIP instead).
extern "C" int lfa_direct_solo_copy(struct lfa_direct *d, void *result, const void *send,
                                    size_t bytes, uint32_t *done_ctr, uint64_t *done_word,
                                    uint64_t done_val) {
  if (!bytes) return 0;
  if (!d || !result || !send || !done_ctr || !done_word || bytes > ((size_t)1 << 30))
    return -LFA_EINVAL;
  if (__atomic_load_n(&d->failed, __ATOMIC_ACQUIRE)) return -LFA_EIO;
  const uint32_t nblocks = lfa_solo_blocks(result, send, bytes);
  pthread_mutex_lock(&d->lock);
  const uint64_t idx = d->stub ? d->stub_write : hsa_queue_load_write_index_relaxed(d->q);
  const int rc = ring_wait(d, idx);
  if (rc) {
    pthread_mutex_unlock(&d->lock);
    return rc;
  }
  if (d->stub)
    d->stub_write = idx + 1;
  else
    hsa_queue_store_write_index_relaxed(d->q, idx + 1);
  SoloArgs *ka = (SoloArgs *)(d->kernarg + (idx % kQueueSize) * 64);
  ka->dst = result;
  ka->src = send;
  ka->bytes = bytes;
  ka->nblocks = nblocks;
  ka->pad = 0;
  ka->ctr = done_ctr;
  ka->word = done_word;
  ka->val = done_val;
  hsa_kernel_dispatch_packet_t *p =
      d->stub ? d->stub_ring + (idx % kQueueSize)
              : (hsa_kernel_dispatch_packet_t *)d->q->base_address + (idx % d->q->size);
  p->workgroup_size_x = 256;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->reserved0 = 0;
  p->grid_size_x = nblocks * 256u;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = d->solo_private;
  p->group_segment_size = d->solo_group;
  p->kernel_object = d->solo_kobj;
  p->kernarg_address = ka;
  p->reserved2 = 0;
  p->completion_signal.handle = 0;
  const uint16_t header = d->header;
  const uint16_t setup = 1u << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  __atomic_store_n((uint32_t *)p, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
  if (!d->stub) hsa_signal_store_screlease(d->q->doorbell_signal, (hsa_signal_value_t)idx);
  pthread_mutex_unlock(&d->lock);
  return 0;
}
