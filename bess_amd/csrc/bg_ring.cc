// bg_ring.cc -- the persistent classify kernel's host side (bg_ring_*,
// include/bessgpu.h): SURVEY §7 H1 without a launch per batch.
//
// BESS hands a module <= 32 packets per ProcessBatch (core/pktbatch.h:70);
// a kernel launch per batch is launch-bound (~5 us each). Like the Queue
// module (core/modules/queue.cc:173 enqueues in ProcessBatch, 190 emits
// from RunTask), a submit here only writes one descriptor (a 64-byte line) into a
// ring in pinned host memory; em_ring_kernel (bg_kernels.hip), launched
// once, claims tickets in order, classifies each batch and publishes
// done[t % slots] = t + 1 in host memory, which wait/poll read.
//
// Where the descriptors live: in device memory when the host can write it
// (the PCIe BAR maps all of it on MI355X; scripts/bar_probe.hip measured a
// 32-byte descriptor write at 1.5 ns, posted), uncached on the device, so
// a worker reads its descriptor from HBM (~1 us) instead of over PCIe (a
// round trip that queued to 8-23 us per ticket under 16 submitters,
// profiles/r03_ring_trace.jsonl). Otherwise (no CPU mapping of device
// memory, or the path flag BG_PATH_RING_HOST_DESC) in pinned host memory,
// read over PCIe.
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
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>
#include <unistd.h>
#include <time.h>
#include <x86intrin.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/bessgpu.h"
#include "bg_internal.h"
#include "bg_kernels.h"
#include "bg_launch.h"

using namespace bg;

// One submission lane: a worker thread's own ring of descriptors. Lanes sit
// on lines of their own (128 B: the adjacent-line prefetcher pairs 64 B
// lines), as each is written by its own submitter.
struct alignas(128) RingLane {
  uint64_t *h_desc = nullptr;  // nslots x kRingDescWords (the host's view)
  uint32_t *h_done = nullptr;  // nslots
  uint64_t *h_pub = nullptr;   // tickets published (its own 64-byte line)
  uint64_t next = 0;           // next ticket to publish
  std::atomic<uint64_t> done_upto{0};  // every ticket below has completed
  // One worker per lane: a second thread inside the lane's calls at the
  // same time gets EBUSY. A flag with plain loads and stores, not a lock:
  // a locked instruction drains the CPU's write-combining buffers, which
  // hold the descriptors bound for device memory (~300 ns per ticket,
  // scripts/bar_probe.hip), so a mutex here cost every submit a flush.
  std::atomic<uint32_t> busy{0};
};

struct bg_ring {
  int device = 0;
  uint32_t nslots = 0, nlanes = 0;
  int blocks = 0;
  int read_end = 0;         // bytes of a slot the kernel reads
  uint64_t version = 0;     // the rule version of its table copy
  uint64_t coherence = kRingSysAcquire | kRingRelease;  // descriptor word 3 flags
  hipStream_t st = nullptr;  // the kernel's own stream
  hipEvent_t ev = nullptr;   // recorded after each launch: has it ended?
  uint64_t *h_desc = nullptr;  // nlanes x nslots x kRingDescWords (pinned host) ...
  uint64_t *d_desc = nullptr;  // ... or in device memory, written by the host
  uint32_t *h_done = nullptr;  // nlanes x nslots
  uint64_t *h_pub = nullptr;   // nlanes x kRingLaneWords
  uint32_t *h_stop = nullptr;  // 1 word, host
  uint32_t *h_ended = nullptr;  // launch id of the grid that ended, host
  uint64_t *h_reset = nullptr;  // pinned source of the device words' reset
  unsigned long long *d_dev = nullptr;  // per lane: next ticket, published; stop
  uint8_t *d_table = nullptr;  // the ring's own copy of the table image
  RingArgs a{};
  bool wm = false;  // a WildcardMatch ring: wa is its table's arguments
  WmArgs wa{};
  std::atomic<uint32_t> launch_id{0};  // of the grid launched last (0: none)
  uint64_t launches = 0;
  std::mutex run_mu;  // (re)launches
  RingLane lanes[kRingMaxLanes];
};

namespace {

constexpr uint64_t kMaskAddr = (1ull << 48) - 1;
constexpr size_t kTicketMaxPkts = (size_t)1 << 27;  // packets per ticket

// A thread waiting for a ticket's completion spins for a while (~0.1-0.2
// ms of pause loops: a slot's usual latency), then sleeps between checks,
// leaving the CPU to the workers (the GPU box's CPUs are a quota shared
// with the HIP runtime's threads). `spin` counts the checks so far. (A
// submitter waiting for lane space keeps spinning: that wait is the
// pipe's backpressure, and its latency is the worker's.)
void wait_pause(uint64_t spin) {
  if (spin < (1u << 15)) {
    _mm_pause();
    return;
  }
  timespec ts{0, 10000L};
  nanosleep(&ts, nullptr);
}

double now_s() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

bool done_at(const bg_ring *r, const RingLane &l, uint64_t t) {
  const uint32_t v = __atomic_load_n(l.h_done + (t % r->nslots), __ATOMIC_ACQUIRE);
  return v == (uint32_t)(t + 1);
}

// Advance the lane's done_upto over completed tickets (in order); the
// lane's owner only.
void retire(bg_ring *r, RingLane &l) {
  uint64_t d = l.done_upto.load(std::memory_order_relaxed);
  while (d < l.next && done_at(r, l, d)) d++;
  l.done_upto.store(d, std::memory_order_release);
}

// Is the last launched grid still serving? Its dispatcher writes its launch
// id to h_ended on the way out, so the submit path reads one host word and
// makes no HIP call.
bool grid_live(const bg_ring *r) {
  const uint32_t id = r->launch_id.load(std::memory_order_acquire);
  return id != 0 && __atomic_load_n(r->h_ended, __ATOMIC_ACQUIRE) != id;
}

// (Re)launch the grid if it has ended and a lane has unfinished tickets;
// every lane's claims restart at its oldest unfinished ticket (later ones
// that already finished are classified again: same gates).
int ensure_running(bg_ring *r) {
  if (grid_live(r)) return 0;
  std::lock_guard<std::mutex> lk(r->run_mu);
  if (grid_live(r)) return 0;
  int rc = set_device(r->device);
  if (rc) return rc;
  if (r->launch_id.load() != 0) HIP_TRY(hipEventSynchronize(r->ev));  // all exited
  bool work = false;
  for (uint32_t i = 0; i < r->nlanes; i++) {
    RingLane &l = r->lanes[i];
    // the lane's published count and its oldest unfinished ticket (read
    // without its owner's lock: done_upto only grows, pub is atomic)
    const uint64_t pub = __atomic_load_n(l.h_pub, __ATOMIC_ACQUIRE);
    uint64_t d = l.done_upto.load(std::memory_order_acquire);
    while (d < pub && done_at(r, l, d)) d++;
    work |= d < pub;
    r->h_reset[i * kRingLaneWords + 0] = d;  // claims restart here
    r->h_reset[i * kRingLaneWords + 1] = d;  // the dispatcher picks up pub
  }
  if (!work) return 0;
  r->h_reset[(size_t)r->nlanes * kRingLaneWords] = 0;  // stop word
  __atomic_store_n(r->h_stop, 0u, __ATOMIC_RELEASE);
  HIP_TRY(hipMemcpyAsync(r->d_dev, r->h_reset,
                         ((size_t)r->nlanes * kRingLaneWords + 1) * 8,
                         hipMemcpyHostToDevice, r->st));
  const uint32_t id = r->launch_id.load() + 1;
  r->a.launch_id = id;
  HIP_TRY(r->wm ? launch_wm_ring(r->a, r->wa, r->blocks, r->st)
                : launch_em_ring(r->a, r->blocks, r->st));
  HIP_TRY(hipEventRecord(r->ev, r->st));
  r->launch_id.store(id, std::memory_order_release);
  r->launches++;
  return 0;
}

void ring_release(bg_ring *r) {
  if (r->h_stop) __atomic_store_n(r->h_stop, 1u, __ATOMIC_RELEASE);
  if (r->st) (void)hipStreamSynchronize(r->st);  // every workgroup exits
  if (r->h_desc) (void)hipHostFree(r->h_desc);
  if (r->d_desc) (void)hipFree(r->d_desc);
  if (r->h_done) (void)hipHostFree(r->h_done);
  if (r->h_pub) (void)hipHostFree(r->h_pub);
  if (r->h_stop) (void)hipHostFree(r->h_stop);
  if (r->h_ended) (void)hipHostFree(r->h_ended);
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

// device memory for the descriptors that this process can also write from
// the host (the allocation's addresses are mapped on the CPU side: mincore
// fails with ENOMEM on an unmapped range); nullptr when it cannot
uint64_t *host_writable_device_alloc(size_t bytes) {
  if (path_flags() & kPathRingHostDesc) return nullptr;
  void *d = nullptr;
  if (hipExtMallocWithFlags(&d, bytes, hipDeviceMallocUncached) != hipSuccess) return nullptr;
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  const uintptr_t lo = (uintptr_t)d & ~(pg - 1);
  const size_t len = (((uintptr_t)d + bytes + pg - 1) & ~(pg - 1)) - lo;
  unsigned char vec[64];
  if (mincore(reinterpret_cast<void *>(lo), pg, vec) != 0 ||
      mincore(reinterpret_cast<void *>(lo + len - pg), pg, vec) != 0) {
    (void)hipFree(d);
    return nullptr;
  }
  return static_cast<uint64_t *>(d);
}

// the lane for this call (see RingLane::busy); ok false: in use elsewhere.
// `claim`: take the flag with an exchange (wait / completed, which are not
// per-ticket paths); submit checks it with plain loads and stores (no
// locked instruction per ticket), so there EBUSY is best-effort detection
// of a second thread on the lane, not a guarantee (include/bessgpu.h)
struct LaneUse {
  RingLane &l;
  const bool ok;
  LaneUse(RingLane &x, bool claim)
      : l(x),
        ok(claim ? x.busy.exchange(1, std::memory_order_acquire) == 0
                 : x.busy.load(std::memory_order_acquire) == 0) {
    if (ok && !claim) l.busy.store(1, std::memory_order_relaxed);
  }
  ~LaneUse() {
    if (ok) l.busy.store(0, std::memory_order_release);
  }
};

// The grid faulted or was aborted (its dispatcher never wrote h_ended):
// -EIO with the HIP error. Called on the slow paths only (lane full,
// waiting), never per ticket.
int grid_failed(bg_ring *r) {
  if (r->launch_id.load(std::memory_order_acquire) == 0) return 0;
  const hipError_t e = hipEventQuery(r->ev);
  if (e == hipSuccess || e == hipErrorNotReady) return 0;
  return fail(EIO, "ring kernel: HIP error %d: %s", (int)e, hipGetErrorString(e));
}

int lane_busy(int lane) {
  return fail(EBUSY, "lane %d in use by another thread (one worker per lane)", lane);
}

int bad_lane(const bg_ring *r, int lane) {
  return fail(EINVAL, "lane %d not in [0,%u)", lane, r->nlanes);
}

}  // namespace

namespace bg {

uint64_t ring_version(const bg_ring *r) { return r->version; }

bool ring_live(const bg_ring *r) { return grid_live(r); }

bool ring_done(const bg_ring *r, int lane, int64_t ticket) {
  const RingLane &l = r->lanes[lane];
  if ((uint64_t)ticket < l.done_upto.load(std::memory_order_acquire)) return true;
  return done_at(r, l, (uint64_t)ticket);
}

}  // namespace bg

extern "C" {

int bg_em_ring_create(bg_em *em, int device, int lanes, int slots, int blocks,
                      uint32_t idle_us, int win_off, bg_ring **out) {
  return bg::em_ring_create(em, device, lanes, slots, blocks, idle_us, win_off,
                            bg::kSlabMeta, out);
}

int bg_wm_ring_create(bg_wm *wm, int device, int lanes, int slots, int blocks,
                      uint32_t idle_us, int win_off, bg_ring **out) {
  return bg::wm_ring_create(wm, device, lanes, slots, blocks, idle_us, win_off,
                            bg::kSlabMeta, out);
}

}  // extern "C"

// The ring's memory and host state (both table kinds)
static int ring_alloc(int device, int lanes, int slots, int blocks, uint32_t idle_us,
                      bg_ring **out) {
  if (lanes < 1 || lanes > kRingMaxLanes)
    return fail(EINVAL, "lanes %d not in [1,%d]", lanes, kRingMaxLanes);
  if (slots < 2 || slots > 32768 || (slots & (slots - 1)))
    return fail(EINVAL, "slots %d: a power of two in [2, 32768]", slots);
  if (idle_us < 100 || idle_us > 60000000)
    return fail(EINVAL, "idle_us %u not in [100, 60000000]", idle_us);
  int rc = set_device(device);
  if (rc) return rc;
  bg_ring *r = new bg_ring();
  r->device = device;
  r->nslots = (uint32_t)slots;
  r->nlanes = (uint32_t)lanes;
  // workers (at least one per lane; four-wave workgroups, 4 per CU beside a
  // 38 KB LDS table) + the dispatcher
  int wk = blocks > 0 ? blocks : 4 * num_cus(device);
  wk = std::max(wk, lanes);
  r->blocks = wk + 1;
  const size_t nl = (size_t)lanes, ns = (size_t)slots;
  hipError_t e = hipStreamCreateWithFlags(&r->st, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&r->ev, hipEventDisableTiming);
  if (e == hipSuccess && !(r->d_desc = host_writable_device_alloc(nl * ns * kRingDescWords * 8)))
    e = host_alloc(&r->h_desc, nl * ns * kRingDescWords * 8);
  if (e == hipSuccess) e = host_alloc(&r->h_done, nl * ns * 4);
  if (e == hipSuccess) e = host_alloc(&r->h_pub, nl * kRingLaneWords * 8);
  if (e == hipSuccess) e = host_alloc(&r->h_stop, 64);
  if (e == hipSuccess) e = host_alloc(&r->h_ended, 64);
  if (e == hipSuccess)
    e = hipHostMalloc(reinterpret_cast<void **>(&r->h_reset), (nl * kRingLaneWords + 8) * 8);
  if (e == hipSuccess)
    e = hipMalloc(reinterpret_cast<void **>(&r->d_dev), (nl * kRingLaneWords + 8) * 8);
  if (e == hipSuccess && r->d_desc) e = hipMemset(r->d_desc, 0, nl * ns * kRingDescWords * 8);  // tag 0
  if (e != hipSuccess) {
    ring_release(r);
    delete r;
    return fail(EIO, "ring allocation: %s", hipGetErrorString(e));
  }
  if (r->h_desc) memset(r->h_desc, 0, nl * ns * kRingDescWords * 8);  // tag 0: no ticket's
  uint64_t *desc = r->d_desc ? r->d_desc : r->h_desc;  // the host's view
  memset(r->h_done, 0, nl * ns * 4);
  memset(r->h_pub, 0, nl * kRingLaneWords * 8);
  *r->h_stop = 0;
  *r->h_ended = 0;
  for (size_t i = 0; i < nl; i++) {
    RingLane &l = r->lanes[i];
    l.h_desc = desc + i * ns * kRingDescWords;
    l.h_done = r->h_done + i * ns;
    l.h_pub = r->h_pub + i * kRingLaneWords;
  }
  RingArgs &a = r->a;
  a.desc = r->d_desc ? r->d_desc : dev_alias(r->h_desc);
  a.done = dev_alias(r->h_done);
  a.stop = dev_alias(r->h_stop);
  a.pub = dev_alias(r->h_pub);
  a.ended = dev_alias(r->h_ended);
  a.dev = r->d_dev;
  a.nslots = (uint32_t)slots;
  a.nlanes = (uint32_t)lanes;
  a.idle_ticks = (uint64_t)idle_us * 100;  // s_memrealtime: 100 MHz
  if (!a.desc || !a.done || !a.stop || !a.pub || !a.ended) {
    ring_release(r);
    delete r;
    return fail(EIO, "no device address for the ring's host memory");
  }
  *out = r;
  return 0;
}

// The ring classifies with the rule set as of its creation: it keeps its own
// copy of the table image, so a later rule change (bessd makes them with the
// workers paused) never frees memory the running kernel reads; a worker
// re-creates its ring after one.
static int ring_copy_table(bg_ring *r, const uint8_t *src, size_t bytes) {
  hipError_t e = hipMalloc(reinterpret_cast<void **>(&r->d_table), std::max<size_t>(bytes, 256));
  if (e == hipSuccess) e = hipMemcpyAsync(r->d_table, src, bytes, hipMemcpyDeviceToDevice, r->st);
  if (e == hipSuccess) e = hipStreamSynchronize(r->st);
  if (e != hipSuccess) return fail(EIO, "ring table copy: %s", hipGetErrorString(e));
  return 0;
}

int bg::em_ring_create(bg_em *em, int device, int lanes, int slots, int blocks,
                       uint32_t idle_us, int win_off, int meta_row, bg_ring **out) {
  if (!em || !out) return fail(EINVAL, "bad arguments");
  bg_ring *r = nullptr;
  if (int rc = ring_alloc(device, lanes, slots, blocks, idle_us, &r)) return rc;
  RingArgs &a = r->a;
  int rc = em_device_plan(em, device, r->st, win_off, meta_row, &a.fp, &a.t, &r->read_end,
                          &r->version);
  if (rc == 0) rc = ring_copy_table(r, a.t.base, (size_t)a.t.part_bytes * a.t.nparts);
  if (rc) {
    ring_release(r);
    delete r;
    return rc;
  }
  a.t.base = r->d_table;
  *out = r;
  return 0;
}

int bg::wm_ring_create(bg_wm *wm, int device, int lanes, int slots, int blocks,
                       uint32_t idle_us, int win_off, int meta_row, bg_ring **out) {
  if (!wm || !out) return fail(EINVAL, "bad arguments");
  bg_ring *r = nullptr;
  if (int rc = ring_alloc(device, lanes, slots, blocks, idle_us, &r)) return rc;
  WmArgs &w = r->wa;
  uint64_t bytes = 0;
  int rc = wm_device_plan(wm, device, r->st, win_off, meta_row, &w, &bytes, &r->read_end,
                          &r->version);
  if (rc == 0) rc = ring_copy_table(r, w.t.base, (size_t)bytes);
  if (rc) {
    ring_release(r);
    delete r;
    return rc;
  }
  r->wm = true;
  w.t.base = r->d_table;
  // the workgroups' LDS holds a table of <= 40 KB whole; anything larger
  // (tag words, a key filter) is probed in L2/MALL, leaving the CUs' LDS to
  // the modules' other kernels
  if (w.t.lds != kLdsTable) w.t.lds = kLdsNone;
  w.default_gate = kRingNoGate;
  w.frames = nullptr;
  w.gates = nullptr;
  w.n = 0;
  r->a.fp = w.fp;  // the serving loop builds the keys
  r->a.t = w.t;
  *out = r;
  return 0;
}

extern "C" {

void bg_ring_destroy(bg_ring *r) {
  if (!r) return;
  ring_release(r);
  delete r;
}

int64_t bg_ring_submit(bg_ring *r, int lane, const void *frames, size_t stride,
                       size_t n, uint16_t default_gate, uint16_t *gates) {
  if (lane < 0 || (uint32_t)lane >= r->nlanes) return bad_lane(r, lane);
  // a run sums up to 16 tickets' counts in 32 bits (ring_serve's prefix
  // sums and `base < total` loop): 16 x 2^27 stays below 2^32
  if (n > kTicketMaxPkts || stride == 0 || stride > 0xFFFF)
    return fail(EINVAL, "n %zu / stride %zu out of range", n, stride);
  if ((int)stride < r->read_end)
    return fail(EINVAL, "fields read %d bytes, past the %zu-byte slot",
                r->read_end, stride);
  if ((((uintptr_t)frames | (uintptr_t)gates) & ~kMaskAddr) ||
      ((uintptr_t)frames & 15) || (stride & 15))
    return fail(EINVAL, "frames 16-byte aligned with stride %% 16 == 0 below 2^48");
  RingLane &l = r->lanes[lane];
  LaneUse use(l, false);
  if (!use.ok) return lane_busy(lane);
  // lane full: its oldest ticket must finish before its slot is reused
  if (l.next - l.done_upto.load(std::memory_order_relaxed) >= r->nslots) {
    if (r->d_desc) _mm_sfence();  // (the last descriptor out before we wait)
    const double t0 = now_s();
    for (uint64_t spin = 0;; spin++) {
      retire(r, l);
      if (l.next - l.done_upto.load(std::memory_order_relaxed) < r->nslots) break;
      if (int rc = ensure_running(r)) return rc;
      if ((spin & 1023) == 1023)
        if (int rc = grid_failed(r)) return rc;
      if (now_s() - t0 > 10.0) {
        if (int rc = grid_failed(r)) return rc;
        return fail(ETIMEDOUT, "ring lane full for 10 s");
      }
      _mm_pause();
    }
  }
  const uint64_t t = l.next;
  const uint64_t tag = ((t + 1) & 0xFFFF) << 48;
  uint64_t *d = l.h_desc + (t % r->nslots) * kRingDescWords;
  __atomic_store_n(d + 0, ((uint64_t)(uintptr_t)frames & kMaskAddr) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(d + 1, ((uint64_t)(uintptr_t)gates & kMaskAddr) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(d + 2, (uint64_t)n | ((uint64_t)stride << 32) | tag, __ATOMIC_RELAXED);
  __atomic_store_n(d + 3, (uint64_t)default_gate | r->coherence | tag, __ATOMIC_RELAXED);
  for (int i = 4; i < kRingDescWords; i++)  // the rest of the line (see kRingDescWords)
    __atomic_store_n(d + i, tag, __ATOMIC_RELAXED);
  // A descriptor in device memory goes through the CPU's write-combining
  // buffers and may reach the device after the count below: the tags make
  // a worker read it again until it has. Its stores fill one 64-byte
  // buffer, which leaves at once. (An sfence per ticket here costs a PCIe
  // flush, ~300 ns: measured in round 4.)
  __atomic_store_n(l.h_pub, t + 1, __ATOMIC_RELEASE);
  l.next = t + 1;
  if (int rc = ensure_running(r)) return rc;
  return (int64_t)t;
}

int bg_ring_wait(bg_ring *r, int lane, int64_t ticket) {
  if (lane < 0 || (uint32_t)lane >= r->nlanes) return bad_lane(r, lane);
  RingLane &l = r->lanes[lane];
  LaneUse use(l, true);
  if (!use.ok) return lane_busy(lane);
  if (ticket < 0 || (uint64_t)ticket >= l.next)
    return fail(EINVAL, "ticket %lld not submitted", (long long)ticket);
  if (r->d_desc) _mm_sfence();  // this submitter's last descriptor out to the device
  const double t0 = now_s();
  for (uint64_t spin = 0;; spin++) {
    retire(r, l);
    if ((uint64_t)ticket < l.done_upto.load(std::memory_order_relaxed)) return 0;
    if (int rc = ensure_running(r)) return rc;
    if ((spin & 1023) == 1023)
      if (int rc = grid_failed(r)) return rc;
    if (now_s() - t0 > 10.0) {
      if (int rc = grid_failed(r)) return rc;
      return fail(ETIMEDOUT, "ticket %lld: 10 s", (long long)ticket);
    }
    wait_pause(spin);
  }
}

int64_t bg_ring_completed(bg_ring *r, int lane) {
  if (lane < 0 || (uint32_t)lane >= r->nlanes) return bad_lane(r, lane);
  RingLane &l = r->lanes[lane];
  LaneUse use(l, true);
  if (!use.ok) return lane_busy(lane);
  retire(r, l);
  if (int rc = ensure_running(r)) return rc;
  return (int64_t)l.done_upto.load(std::memory_order_relaxed);
}

int bg_ring_run(bg_ring *r, int lane, const void *frames, size_t stride, size_t n,
                size_t burst, uint16_t default_gate, uint16_t *gates) {
  if (burst < 1) return fail(EINVAL, "burst must be >= 1");
  int64_t last = -1;
  for (size_t i = 0; i < n; i += burst) {
    last = bg_ring_submit(r, lane, static_cast<const uint8_t *>(frames) + i * stride,
                          stride, std::min(burst, n - i), default_gate, gates + i);
    if (last < 0) return (int)last;
  }
  return last < 0 ? 0 : bg_ring_wait(r, lane, last);
}

double bg_ring_run_lanes(bg_ring *r, int threads, const void *frames, size_t stride,
                         size_t n, size_t burst, uint16_t default_gate, uint16_t *gates,
                         int reps) {
  if (threads < 1 || (uint32_t)threads > r->nlanes || reps < 1)
    return fail(EINVAL, "threads %d / reps %d (lanes %u)", threads, reps, r->nlanes);
  std::vector<std::thread> th;
  std::atomic<int> ready{0}, err{0};
  std::atomic<bool> go{false};
  double t1[kRingMaxLanes] = {};
  for (int i = 0; i < threads; i++) {
    th.emplace_back([&, i] {
      const size_t lo = n * i / threads, hi = n * (i + 1) / threads;
      ready++;
      while (!go.load(std::memory_order_acquire)) _mm_pause();
      for (int k = 0; k < reps && !err.load(); k++) {
        const int rc = bg_ring_run(r, i, static_cast<const uint8_t *>(frames) + lo * stride,
                                   stride, hi - lo, burst, default_gate, gates + lo);
        if (rc < 0) err.store(rc);
      }
      t1[i] = now_s();
    });
  }
  while (ready.load() < threads) _mm_pause();
  const double t0 = now_s();
  go.store(true, std::memory_order_release);
  for (auto &t : th) t.join();
  if (err.load()) return (double)err.load();
  double end = t0;
  for (int i = 0; i < threads; i++) end = std::max(end, t1[i]);
  return (end - t0) / reps;
}


int bg_ring_desc_in_device(const bg_ring *r) { return r && r->d_desc ? 1 : 0; }

int bg_ring_set_coherence(bg_ring *r, int frames, int done) {
  if (!r || frames < 0 || frames > 1 || done < 0 || done > 1)
    return fail(EINVAL, "bad arguments");
  uint64_t c = (frames ? kRingSysAcquire : 0) | (done ? kRingRelease : 0);
  r->coherence = c;
  return 0;
}

int bg_ring_info(const bg_ring *r, uint64_t *launches, int *blocks) {
  if (launches) *launches = r->launches;
  if (blocks) *blocks = r->blocks - 1;  // workers
  return 0;
}

}  // extern "C"
