// bg_ring.cc -- the persistent classify kernel's host side (bg_ring_*,
// include/bessgpu.h): SURVEY §7 H1 without a launch per batch.
//
// BESS hands a module <= 32 packets per ProcessBatch (core/pktbatch.h:70);
// a kernel launch per batch is launch-bound (~5 us each). Like the Queue
// module (core/modules/queue.cc:173 enqueues in ProcessBatch, 190 emits
// from RunTask), a submit here only writes one 32-byte descriptor into a
// ring in pinned host memory; em_ring_kernel (bg_kernels.hip), launched
// once, claims tickets in order, classifies each batch and publishes
// done[t % slots] = t + 1 in host memory, which wait/poll read.
//
// One lane of the grid (the dispatcher) polls the host's published count
// over PCIe and mirrors it in device memory, where the other workgroups
// wait: hundreds of waiting workgroups poll L2 instead of all issuing
// PCIe reads. Liveness: when nothing is published for
// the idle time the dispatcher stops the grid, so the kernel always drains
// on its own (also when the owner never destroys the ring); submit and
// wait relaunch it from the oldest unfinished ticket when it has ended.
// Descriptor words carry the ticket's tag (bg_kernels.h RingArgs), so a
// descriptor is read whole without fences.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <mutex>

#include "../../include/bessgpu.h"
#include "bg_internal.h"
#include "bg_kernels.h"

using namespace bg;

struct bg_ring {
  int device = 0;
  uint32_t nslots = 0;
  int blocks = 0;
  int read_end = 0;         // bytes of a slot the kernel reads
  hipStream_t st = nullptr;  // the kernel's own stream
  hipEvent_t ev = nullptr;   // recorded after each launch: has it ended?
  uint64_t *h_desc = nullptr;  // nslots x 4 words, host (coherent, mapped)
  uint32_t *h_done = nullptr;  // nslots, host
  uint32_t *h_stop = nullptr;  // 1 word, host
  uint64_t *h_pub = nullptr;   // tickets published, host
  uint64_t *h_reset = nullptr;  // pinned source of the device words' reset
  unsigned long long *d_dev = nullptr;  // next ticket, published, stop
  uint8_t *d_table = nullptr;  // the ring's own copy of the table image
  RingArgs a{};
  uint64_t next = 0;      // next ticket to publish
  uint64_t done_upto = 0;  // every ticket < done_upto has completed
  bool running = false;
  uint64_t launches = 0;
  std::mutex mu;  // one ring per worker; the lock only guards misuse
};

namespace {

constexpr uint64_t kMaskAddr = (1ull << 48) - 1;

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

bool done_at(const bg_ring *r, uint64_t t) {
  const uint32_t v = __atomic_load_n(r->h_done + (t % r->nslots), __ATOMIC_ACQUIRE);
  return v == (uint32_t)(t + 1);
}

// Advance done_upto over completed tickets (in order).
void retire(bg_ring *r) {
  while (r->done_upto < r->next && done_at(r, r->done_upto)) r->done_upto++;
}

// (Re)launch the kernel from the oldest unfinished ticket if it is not
// running. A grid that stopped itself (idle) has ended once its event has.
int ensure_running(bg_ring *r) {
  if (r->running) {
    const hipError_t q = hipEventQuery(r->ev);
    if (q == hipErrorNotReady) return 0;
    if (q != hipSuccess)
      return fail(EIO, "ring kernel: %s", hipGetErrorString(q));
    r->running = false;
  }
  retire(r);
  if (r->done_upto == r->next) return 0;  // nothing outstanding
  int rc = set_device(r->device);
  if (rc) return rc;
  __atomic_store_n(r->h_stop, 0u, __ATOMIC_RELEASE);
  r->h_reset[0] = r->done_upto;  // claims restart at the oldest unfinished
  r->h_reset[1] = r->done_upto;  // the dispatcher picks up *pub at once
  r->h_reset[2] = 0;
  HIP_TRY(hipMemcpyAsync(r->d_dev, r->h_reset, 24, hipMemcpyHostToDevice, r->st));
  HIP_TRY(launch_em_ring(r->a, r->blocks, r->st));
  HIP_TRY(hipEventRecord(r->ev, r->st));
  r->running = true;
  r->launches++;
  return 0;
}

void ring_release(bg_ring *r) {
  if (r->h_stop) __atomic_store_n(r->h_stop, 1u, __ATOMIC_RELEASE);
  if (r->st) (void)hipStreamSynchronize(r->st);  // every workgroup exits
  if (r->h_desc) (void)hipHostFree(r->h_desc);
  if (r->h_done) (void)hipHostFree(r->h_done);
  if (r->h_stop) (void)hipHostFree(r->h_stop);
  if (r->h_pub) (void)hipHostFree(r->h_pub);
  if (r->h_reset) (void)hipHostFree(r->h_reset);
  if (r->d_dev) (void)hipFree(r->d_dev);
  if (r->d_table) (void)hipFree(r->d_table);
  if (r->ev) (void)hipEventDestroy(r->ev);
  if (r->st) (void)hipStreamDestroy(r->st);
}

template <typename T>
hipError_t host_alloc(T **p, size_t bytes) {
  return hipHostMalloc(reinterpret_cast<void **>(p), bytes,
                       hipHostMallocMapped | hipHostMallocCoherent);
}

template <typename T>
T *dev_alias(T *h) {
  void *d = nullptr;
  return hipHostGetDevicePointer(&d, h, 0) == hipSuccess ? static_cast<T *>(d) : nullptr;
}

}  // namespace

extern "C" {

int bg_em_ring_create(bg_em *em, int device, int slots, int blocks,
                      uint32_t idle_us, bg_ring **out) {
  if (!em || !out) return fail(EINVAL, "bad arguments");
  if (slots < 2 || slots > 32768 || (slots & (slots - 1)))
    return fail(EINVAL, "slots %d: a power of two in [2, 32768]", slots);
  if (idle_us < 100 || idle_us > 60000000)
    return fail(EINVAL, "idle_us %u not in [100, 60000000]", idle_us);
  int rc = set_device(device);
  if (rc) return rc;
  bg_ring *r = new bg_ring();
  r->device = device;
  r->nslots = (uint32_t)slots;
  // workers + the dispatcher
  r->blocks = (blocks > 0 ? blocks : 2 * num_cus(device)) + 1;
  hipError_t e = hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ev, hipEventDisableTiming);
  if (e == hipSuccess) e = host_alloc(&r->h_desc, (size_t)slots * 32);
  if (e == hipSuccess) e = host_alloc(&r->h_done, (size_t)slots * 4);
  if (e == hipSuccess) e = host_alloc(&r->h_stop, 64);
  if (e == hipSuccess) e = host_alloc(&r->h_pub, 64);
  if (e == hipSuccess) e = hipHostMalloc(reinterpret_cast<void **>(&r->h_reset), 64);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&r->d_dev), 64);
  if (e != hipSuccess) {
    ring_release(r);
    delete r;
    return fail(EIO, "ring allocation: %s", hipGetErrorString(e));
  }
  memset(r->h_desc, 0, (size_t)slots * 32);  // tag 0: no ticket's
  memset(r->h_done, 0, (size_t)slots * 4);
  *r->h_stop = 0;
  *r->h_pub = 0;
  RingArgs &a = r->a;
  a.desc = dev_alias(r->h_desc);
  a.done = dev_alias(r->h_done);
  a.stop = dev_alias(r->h_stop);
  a.pub = dev_alias(r->h_pub);
  a.dev = r->d_dev;
  a.nslots = (uint32_t)slots;
  a.idle_ticks = (uint64_t)idle_us * 100;  // s_memrealtime: 100 MHz
  if (!a.desc || !a.done || !a.stop || !a.pub) {
    ring_release(r);
    delete r;
    return fail(EIO, "no device address for the ring's host memory");
  }
  rc = em_device_plan(em, device, r->st, &a.fp, &a.t, &r->read_end);
  if (rc == 0) {
    // The ring classifies with the rule set as of its creation: it keeps
    // its own copy of the table image, so a later rule change (bessd makes
    // them with the workers paused) never frees memory the running kernel
    // reads; a worker re-creates its ring after one.
    const size_t bytes = (size_t)a.t.part_bytes * a.t.nparts;
    e = hipMalloc(reinterpret_cast<void **>(&r->d_table), std::max<size_t>(bytes, 256));
    if (e == hipSuccess)
      e = hipMemcpyAsync(r->d_table, a.t.base, bytes, hipMemcpyDeviceToDevice, r->st);
    if (e == hipSuccess) e = hipStreamSynchronize(r->st);
    if (e != hipSuccess) rc = fail(EIO, "ring table copy: %s", hipGetErrorString(e));
    a.t.base = r->d_table;
  }
  if (rc) {
    ring_release(r);
    delete r;
    return rc;
  }
  *out = r;
  return 0;
}

void bg_ring_destroy(bg_ring *r) {
  if (!r) return;
  ring_release(r);
  delete r;
}

int64_t bg_ring_submit(bg_ring *r, const void *frames, size_t stride, size_t n,
                       uint16_t default_gate, uint16_t *gates) {
  if (n > 0xFFFFFFFFu || stride == 0 || stride > 0xFFFF)
    return fail(EINVAL, "n %zu / stride %zu out of range", n, stride);
  if ((int)stride < r->read_end)
    return fail(EINVAL, "fields read %d bytes, past the %zu-byte slot",
                r->read_end, stride);
  if ((((uintptr_t)frames | (uintptr_t)gates) & ~kMaskAddr) ||
      ((uintptr_t)frames & 15) || (stride & 15))
    return fail(EINVAL, "frames 16-byte aligned with stride %% 16 == 0 below 2^48");
  std::lock_guard<std::mutex> lk(r->mu);
  // ring full: the oldest ticket must finish before its slot is reused
  const double t0 = now_s();
  while (r->next - r->done_upto >= r->nslots) {
    retire(r);
    if (r->next - r->done_upto < r->nslots) break;
    if (int rc = ensure_running(r)) return rc;
    if (now_s() - t0 > 10.0) return fail(ETIMEDOUT, "ring full for 10 s");
    _mm_pause();
  }
  const uint64_t t = r->next;
  const uint64_t tag = ((t + 1) & 0xFFFF) << 48;
  uint64_t *d = r->h_desc + (t % r->nslots) * 4;
  __atomic_store_n(d + 0, ((uint64_t)(uintptr_t)frames & kMaskAddr) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(d + 1, ((uint64_t)(uintptr_t)gates & kMaskAddr) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(d + 2, (uint64_t)n | ((uint64_t)stride << 32) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(d + 3, (uint64_t)default_gate | tag, __ATOMIC_RELAXED);
  __atomic_store_n(r->h_pub, t + 1, __ATOMIC_RELEASE);
  r->next = t + 1;
  if (int rc = ensure_running(r)) return rc;
  return (int64_t)t;
}

int bg_ring_wait(bg_ring *r, int64_t ticket) {
  std::lock_guard<std::mutex> lk(r->mu);
  if (ticket < 0 || (uint64_t)ticket >= r->next)
    return fail(EINVAL, "ticket %lld not submitted", (long long)ticket);
  const double t0 = now_s();
  for (;;) {
    retire(r);
    if ((uint64_t)ticket < r->done_upto) return 0;
    if (int rc = ensure_running(r)) return rc;
    if (now_s() - t0 > 10.0) return fail(ETIMEDOUT, "ticket %lld: 10 s", (long long)ticket);
    _mm_pause();
  }
}

int64_t bg_ring_completed(bg_ring *r) {
  std::lock_guard<std::mutex> lk(r->mu);
  retire(r);
  if (int rc = ensure_running(r)) return rc;
  return (int64_t)r->done_upto;
}

int bg_ring_run(bg_ring *r, const void *frames, size_t stride, size_t n,
                size_t burst, uint16_t default_gate, uint16_t *gates) {
  if (burst < 1) return fail(EINVAL, "burst must be >= 1");
  int64_t last = -1;
  for (size_t i = 0; i < n; i += burst) {
    last = bg_ring_submit(r, static_cast<const uint8_t *>(frames) + i * stride, stride,
                          std::min(burst, n - i), default_gate, gates + i);
    if (last < 0) return (int)last;
  }
  return last < 0 ? 0 : bg_ring_wait(r, last);
}

int bg_ring_info(const bg_ring *r, uint64_t *launches, int *blocks) {
  if (launches) *launches = r->launches;
  if (blocks) *blocks = r->blocks - 1;  // workers
  return 0;
}

}  // extern "C"
