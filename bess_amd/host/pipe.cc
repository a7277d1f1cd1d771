// pipe.cc -- asynchronous host ingress/egress for a GPU module (bg_pipe_*,
// include/bessgpu.h): the aggregation queue of SURVEY §7 H1 / §8f rank 1.
//
// BESS hands a module <= 32 packets per ProcessBatch (core/pktbatch.h:70);
// one device launch (plus H2D/D2H) per 32 packets is launch-latency bound.
// A drop-in module therefore splits its work like the Queue module does --
// ProcessBatch enqueues (core/modules/queue.cc:173), a task emits later
// (queue.cc:190) -- and this file is that queue:
//
//   submit : the bytes of each packet the device reads (Module::DeviceWindow:
//            the field window for ExactMatch/WildcardMatch, the frame for the
//            checksum modules) are gathered into a pinned staging slot;
//   launch : when a slot holds `batch` packets (or on flush), on the slot's
//            own HIP stream: H2D of the slot -> ProcessDeviceWindow -> D2H of
//            the gates (checksum modules: also the first 128 B of each frame,
//            the bytes whose checksum words the kernel rewrites) -> event;
//   poll   : completed slots, oldest first; checksum header lines are
//            written back into the packet buffers, then (cookie, gate) pairs
//            are returned in submission order -- the EmitPacket calls of the
//            reference's ProcessBatch, per-gate order preserved
//            (core/module.h:268-272).
//
// `depth` slots form a ring, each with its own stream, so the gather of slot
// i+1, the H2D of slot i, the kernel of slot i-1 and the D2H of slot i-2
// overlap. Packets stay owned by the caller until poll returns them (the
// device only ever sees copies of their bytes, core/module.h:224-226).
//
// Ring mode (a module with a persistent kernel, Module::PipeRingFor:
// ExactMatch): a slot's staging and gates live in pinned host memory the
// device maps; launch writes one descriptor on the pipe's lane of the
// module's bg_ring and poll reads the lane's done word -- no HIP call per
// slot, so slots can be small (little in flight per worker, as bessd's
// packet pool is shared by all workers) at no launch cost.
#include <hip/hip_runtime.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

#include <algorithm>
#include <deque>
#include <mutex>
#include <vector>

#include "../../include/bessgpu.h"
#include "../csrc/bg_internal.h"
#include "module.h"

using bg::fail;

namespace {

constexpr size_t kWriteback = 128;  // header line returned to the host

struct Slot {
  uint8_t *h_in = nullptr, *d_in = nullptr;   // staged windows
  uint8_t *h_wb = nullptr;                    // header lines back (writeback)
  uint16_t *h_g = nullptr, *d_g = nullptr;    // gates
  hipStream_t st = nullptr;
  uint64_t *h_done = nullptr;  // pinned, mapped: = seq once the slot's D2H is done
  uint64_t *d_done = nullptr;  // its device address (hipStreamWriteValue64)
  uint64_t seq = 0;            // this launch's number
  std::vector<uint8_t *> heads;  // writeback targets; the lagging gather's sources
  std::vector<uint8_t *> metas;  // metadata areas (modules with attr fields)
  size_t gathered = 0;           // packets [0, gathered) are in h_in
  std::vector<uint16_t> wblen;   // bytes of the header line to write back
  std::vector<void *> cookies;
  size_t n = 0;
  bool inflight = false;
  bool draining = false;  // completed; poll hands out [cursor, n)
  size_t cursor = 0;
  bg_ctx ctx{};  // the context of the slot's packets (Module::CtxUse fields)
  // ring mode: the device addresses of h_in / h_g, and the ticket in flight
  uint8_t *dv_in = nullptr;
  uint16_t *dv_g = nullptr;
  // zero-copy slot (a writeback module's packets in host-registered memory,
  // bg_host_register): the packets' head pointers, device addresses, in
  // pinned host memory the kernel reads; the frames are processed in place
  bool zc = false;
  uint64_t *h_ptr = nullptr, *dv_ptr = nullptr;
  std::shared_ptr<PipeRing> ring;  // the ring (rules) it was submitted to
  int lane = 0;
  int64_t ticket = -1;
  uint64_t t_launch = 0;  // TSC at launch (bg_pipe_stats: launch -> done)
};

}  // namespace

struct bg_pipe {
  bg_module *mod = nullptr;
  int device = 0;
  size_t batch = 0;
  int lo = 0, hi = 0;    // staged frame bytes [lo, hi)
  size_t w = 0;          // staged stride (16-byte multiple)
  // attr fields (Module::MetaWindow): metadata bytes [mlo, mhi) of each
  // packet staged at row offset mat (module.h StagedMetaAt)
  bool meta = false;
  int mlo = 0, mhi = 0;
  size_t mat = 0;
  bool writeback = false;
  bool zc = false;       // the module processes frames in place by pointer
  unsigned ctx_use = 0;  // Module::CtxUse(): the context fields a slot fixes
  bool ring_mode = false;          // slots go to the module's ring
  std::shared_ptr<PipeRing> ring;  // the ring this pipe has a lane on
  int lane = 0;
  std::vector<Slot> slots;
  size_t fill = 0;       // slot being filled
  size_t oldest = 0;     // oldest in-flight slot
  size_t inflight = 0;   // slots in flight
  // completed packets of a slot that had to be reused before poll took
  // them (they leave first); normally poll reads the slots themselves
  std::deque<std::pair<void *, uint16_t>> ready;
  size_t pending = 0;    // submitted, not yet returned by poll
  int err = 0;           // sticky launch error
  uint64_t launched = 0;  // slot launches so far (Slot::seq)
  // bg_pipe_stats: submits, packets, ns in launches (HIP calls), ns a
  // submit waited for a free slot, ns a poll waited
  uint64_t st_submits = 0, st_pkts = 0, st_launch_ns = 0, st_full_ns = 0,
           st_wait_ns = 0;
  uint64_t st_submit_tsc = 0, st_poll_tsc = 0;  // cycles inside submit / poll
  uint64_t st_lat_tsc = 0, st_lat_max = 0;      // slot launch -> seen done
  // ns of a launch by HIP call: H2D copy, module kernel, gate D2H, header
  // lines D2H, completion write (launch mode)
  uint64_t st_call_ns[5] = {0, 0, 0, 0, 0};
  // One worker owns a pipe; the lock is for the module's control path
  // (PipeFlushLocked) and a RunTask on another worker (never contended on
  // the datapath).
  std::mutex mu;
};

static void pipe_release(bg_pipe *p) {
  for (Slot &s : p->slots) {
    if (s.ring) {  // the kernel may still read the staging: let it finish
      if (s.inflight) {
        std::lock_guard<std::mutex> lk(s.ring->lane_mu[s.lane]);
        (void)bg_ring_wait(s.ring->r, s.lane, s.ticket);
      }
      s.ring.reset();
    }
    if (s.st) {
      (void)hipStreamSynchronize(s.st);
      bg::stream_gone(s.st);  // no table image fences on it any more
    }
    if (s.h_in) (void)hipHostFree(s.h_in);
    if (s.h_wb) (void)hipHostFree(s.h_wb);
    if (s.h_g) (void)hipHostFree(s.h_g);
    if (s.h_done) (void)hipHostFree(s.h_done);
    if (s.h_ptr) (void)hipHostFree(s.h_ptr);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_g) (void)hipFree(s.d_g);
    if (s.st) (void)hipStreamDestroy(s.st);
  }
  p->slots.clear();
}

// dst <- src, w bytes (a multiple of 16): fixed-size 16-byte moves, no
// libc call per packet
static inline uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

static inline void copy16(uint8_t *dst, const uint8_t *src, size_t w) {
  switch (w) {
    case 16:
      __builtin_memcpy(dst, src, 16);
      return;
    case 32:
      __builtin_memcpy(dst, src, 32);
      return;
    case 48:
      __builtin_memcpy(dst, src, 48);
      return;
    case 64:
      __builtin_memcpy(dst, src, 64);
      return;
    default:
      memcpy(dst, src, w);
  }
}

// Launch the fill slot (n > 0): H2D, module kernel, D2H, event. (No
// module lock: like bessd's datapath, a pipe relies on THREAD_UNSAFE
// commands running only while its worker is paused, core/module.cc:97-101;
// such a command flushes the pipe first, PipeFlushLocked.)
// The lagging gather (field windows, no writeback): a submit records its
// packets' heads and copies the windows of the packets the PREVIOUS call
// recorded, whose data lines the caller's prefetch has brought in since
// (copying them at once stalled on the line misses the prefetch had just
// started: about a miss latency per 32-packet batch). A slot is gathered
// whole before it launches.
static void gather(bg_pipe *p, Slot &s) {
  uint8_t *dst = s.h_in + s.gathered * p->w;
  if (p->meta) {
    const size_t ml = (size_t)(p->mhi - p->mlo);
    for (size_t j = s.gathered; j < s.n; j++, dst += p->w) {
      copy16(dst, s.heads[j] + p->lo, p->mat);
      memcpy(dst + p->mat, s.metas[j] + p->mlo, ml);
    }
  } else {
    for (size_t j = s.gathered; j < s.n; j++, dst += p->w) copy16(dst, s.heads[j] + p->lo, p->w);
  }
  s.gathered = s.n;
}

static int launch_slot(bg_pipe *p) {
  Slot &s = p->slots[p->fill];
  if (!p->writeback) gather(p, s);
  const size_t n = s.n;
  const uint64_t t0 = mono_ns();
  s.t_launch = __rdtsc();
  if (p->ring_mode) {
    // one descriptor on the pipe's lane of the module's current ring (a new
    // ring after a rule change: a lane there)
    std::shared_ptr<PipeRing> ring;
    uint16_t dflt = 0;
    if (p->ring && p->mod->m->PipeRingCurrent(*p->ring, &dflt)) {
      ring = p->ring;  // (no module lock per slot: workers share the module)
    } else {
      int rc = p->mod->m->PipeRingFor(p->device, &ring, &dflt);
      if (rc < 0) return rc;
    }
    if (!ring) return fail(ENOTSUP, "the module no longer serves pipes through a ring");
    if (ring != p->ring) {
      p->ring = ring;
      p->lane = ring->next_lane.fetch_add(1) % ring->lanes;
    }
    // the gathered windows reach memory before the descriptor that points
    // at them (the descriptor goes out through write-combining buffers,
    // which x86 does not order after earlier write-back stores): one
    // fence per slot
    _mm_sfence();
    int64_t t;
    {
      std::lock_guard<std::mutex> lk(ring->lane_mu[p->lane]);
      t = bg_ring_submit(ring->r, p->lane, s.dv_in, p->w, n, dflt, s.dv_g);
    }
    if (t < 0) return (int)t;
    s.ring = std::move(ring);
    s.lane = p->lane;
    s.ticket = t;
    s.seq = ++p->launched;
    p->st_launch_ns += mono_ns() - t0;
    s.inflight = true;
    p->inflight++;
    p->fill = (p->fill + 1) % p->slots.size();
    return 0;
  }
  int rc = bg::set_device(p->device);
  if (rc) return rc;
  uint64_t t1 = mono_ns(), t2;
  auto lap = [&](int k) {
    t2 = mono_ns();
    p->st_call_ns[k] += t2 - t1;
    t1 = t2;
  };
  bg_ctx c = s.ctx;
  c.device = (int16_t)p->device;
  if (s.zc) {  // the frames in place: no copy either way but the gates
    lap(0);
    int r = p->mod->m->ProcessDevicePtrs(c, s.dv_ptr, (size_t)(p->hi - p->lo), n, s.d_g,
                                         s.st);
    if (r < 0) return r;
  } else {
    HIP_TRY(hipMemcpyAsync(s.d_in, s.h_in, n * p->w, hipMemcpyHostToDevice, s.st));
    lap(0);
    int r = p->mod->m->ProcessDeviceWindow(c, s.d_in, p->w, n, p->lo, s.d_g, s.st);
    if (r < 0) return r;
  }
  lap(1);
  HIP_TRY(hipMemcpyAsync(s.h_g, s.d_g, n * 2, hipMemcpyDeviceToHost, s.st));
  lap(2);
  if (p->writeback && !s.zc) {
    const size_t line = std::min(p->w, kWriteback);
    HIP_TRY(hipMemcpy2DAsync(s.h_wb, line, s.d_in, p->w, line, n,
                             hipMemcpyDeviceToHost, s.st));
  }
  lap(3);
  // completion lands in host memory after the D2H copies: poll reads one
  // word and makes no HIP call
  s.seq = ++p->launched;
  HIP_TRY(hipStreamWriteValue64(s.st, s.d_done, s.seq, 0));
  lap(4);
  p->st_launch_ns += mono_ns() - t0;
  s.inflight = true;
  p->inflight++;
  p->fill = (p->fill + 1) % p->slots.size();
  return 0;
}

// Retire the oldest slot if it is in flight and done (blocking when
// `wait`): header lines written back, the slot's packets ready for poll.
// Returns 1 if it was retired, 0 if not (not in flight / not done), -errno.
static int retire_oldest(bg_pipe *p, bool wait) {
  Slot &s = p->slots[p->oldest];
  if (!s.inflight) return 0;
  if (s.ring) {
    if (!bg::ring_done(s.ring->r, s.lane, s.ticket)) {
      // not yet, and the grid that will finish it is running: no lane lock
      // per poll (the lane is shared with the pipe's own submits)
      if (!wait && bg::ring_live(s.ring->r)) return 0;
      // (through the ring's own check, which relaunches a grid that ended)
      std::lock_guard<std::mutex> lk(s.ring->lane_mu[s.lane]);
      const int64_t c = bg_ring_completed(s.ring->r, s.lane);
      if (c < 0) return (int)c;
      if (c <= s.ticket) {
        if (!wait) return 0;
        const uint64_t t0 = mono_ns();
        if (int rc = bg_ring_wait(s.ring->r, s.lane, s.ticket)) return rc;
        p->st_wait_ns += mono_ns() - t0;
      }
    }
    s.ring.reset();  // the last slot on a replaced ring retires it
    const uint64_t lat = __rdtsc() - s.t_launch;
    p->st_lat_tsc += lat;
    p->st_lat_max = std::max(p->st_lat_max, lat);
  } else if (__atomic_load_n(s.h_done, __ATOMIC_ACQUIRE) != s.seq) {
    if (!wait) return 0;
    const uint64_t t0 = mono_ns();
    int rc = bg::set_device(p->device);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s.st));
    p->st_wait_ns += mono_ns() - t0;
    if (__atomic_load_n(s.h_done, __ATOMIC_ACQUIRE) != s.seq)
      return fail(EIO, "pipe slot %llu: completion word not written",
                  (unsigned long long)s.seq);
  }
  if (!s.ring) {
    const uint64_t lat = __rdtsc() - s.t_launch;
    p->st_lat_tsc += lat;
    p->st_lat_max = std::max(p->st_lat_max, lat);
  }
  if (p->writeback && !s.zc) {
    const size_t line = std::min(p->w, kWriteback);
    for (size_t i = 0; i < s.n; i++)
      memcpy(s.heads[i], s.h_wb + i * line, s.wblen[i]);
  }
  s.inflight = false;
  s.draining = true;
  s.cursor = 0;
  p->inflight--;
  return 1;
}

// The oldest slot, drained: the next one becomes the oldest.
static void release_oldest(bg_pipe *p) {
  Slot &s = p->slots[p->oldest];
  s.draining = false;
  s.n = 0;
  s.gathered = 0;
  p->oldest = (p->oldest + 1) % p->slots.size();
}

// Completed packets in submission order into cookies / gates (cap): the
// spilled ones first, then the oldest slots in place.
static long take_done(bg_pipe *p, bool wait, void **cookies, uint16_t *gates,
                      size_t cap) {
  size_t k = 0;
  while (k < cap && !p->ready.empty()) {
    const auto &e = p->ready.front();
    if (cookies) cookies[k] = e.first;
    if (gates) gates[k] = e.second;
    p->ready.pop_front();
    k++;
  }
  while (k < cap) {
    Slot &s = p->slots[p->oldest];
    if (s.draining) {
      const size_t m = std::min(cap - k, s.n - s.cursor);
      if (cookies) memcpy(cookies + k, s.cookies.data() + s.cursor, m * sizeof(void *));
      if (gates) memcpy(gates + k, s.h_g + s.cursor, m * 2);
      s.cursor += m;
      k += m;
      if (s.cursor == s.n) release_oldest(p);
      continue;
    }
    const int r = retire_oldest(p, wait && k == 0);
    if (r < 0) return r;
    if (r == 0) break;
  }
  p->pending -= k;
  return (long)k;
}

// mapped pinned memory the device reads uncached (see bg_pipe_create)
constexpr size_t kPipeRingMaxBatch = 8192;  // ring-mode slots (bg_pipe_create)

static hipError_t host_alloc_uc(void **p, size_t bytes) {
  return hipHostMalloc(p, bytes, hipHostMallocMapped | hipHostMallocUncached);
}

extern "C" {

int bg_pipe_create(bg_module *m, int device, size_t batch, int depth,
                   size_t span, bg_pipe **out) {
  if (!m || !out) return fail(EINVAL, "bad arguments");
  if (batch < 1 || batch > (1u << 24)) return fail(EINVAL, "batch %zu", batch);
  if (depth < 1 || depth > 16) return fail(EINVAL, "depth %d not in [1,16]", depth);
  int r = bg::set_device(device);
  if (r) return r;
  bg_pipe *p = new bg_pipe();
  p->mod = m;
  p->device = device;
  p->batch = batch;
  m->m->DeviceWindow(&p->lo, &p->hi, &p->writeback);
  r = m->m->MetaWindow(&p->mlo, &p->mhi);
  if (r < 0) {
    delete p;
    return r;
  }
  p->meta = p->mhi > p->mlo;
  if (span && !p->meta && p->lo == 0 && (int)span < p->hi) p->hi = (int)span;
  if (p->hi <= p->lo) p->hi = p->lo + 1;
  p->w = ((size_t)(p->hi - p->lo) + 15) / 16 * 16;
  if (p->meta) {
    p->mat = (size_t)StagedMetaAt(p->lo, p->hi);
    p->w = StagedStride(p->lo, p->hi, p->mlo, p->mhi);
  }
  p->ctx_use = m->m->CtxUse();
  // a writeback module with a by-pointer datapath takes packets that lie in
  // host-registered memory in place (Module::ProcessDevicePtrs asked with n
  // 0); its kernel reads each frame from the pointer on, so only a window
  // that starts at the head (lo 0: the checksum modules) goes in place
  p->zc = p->writeback && !p->meta && p->lo == 0 &&
          m->m->ProcessDevicePtrs(ResolveCtx(nullptr, device), nullptr,
                                  (size_t)(p->hi - p->lo), 0, nullptr, nullptr) == 0;
  // a ring ticket is served by one workgroup: past a few thousand packets
  // a launch per slot spreads them over the whole device instead
  if (!p->writeback && batch <= kPipeRingMaxBatch) {
    uint16_t dflt = 0;
    r = m->m->PipeRingFor(device, &p->ring, &dflt);
    if (r < 0) {
      delete p;
      return r;
    }
    p->ring_mode = p->ring != nullptr;
    if (p->ring_mode) p->lane = p->ring->next_lane.fetch_add(1) % p->ring->lanes;
  }
  p->slots.resize((size_t)depth);
  for (Slot &s : p->slots) {
    if (p->ring_mode) {
      // the kernel reads the windows and writes the gates in place. Mapped
      // uncached (MTYPE UC): a refilled slot's windows are never served
      // from a line an earlier batch left in the device's L2 (coherent host
      // memory alone is cached there as non-coherent lines, and the ring's
      // grid outlives many batches), so the ring's tickets acquire at agent
      // scope only (their CU's L1; bg_ring_set_coherence in the EM module).
      hipError_t e = host_alloc_uc(reinterpret_cast<void **>(&s.h_in), batch * p->w + 64);
      if (e == hipSuccess) e = host_alloc_uc(reinterpret_cast<void **>(&s.h_g), batch * 2 + 64);
      if (e == hipSuccess)
        e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.dv_in), s.h_in, 0);
      if (e == hipSuccess)
        e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.dv_g), s.h_g, 0);
      if (e != hipSuccess) {
        pipe_release(p);
        delete p;
        return fail(EIO, "HIP error %d: %s", (int)e, hipGetErrorString(e));
      }
      s.cookies.resize(batch);
      s.heads.resize(batch);
      if (p->meta) s.metas.resize(batch);
      continue;
    }
    // +64 B: window loads of the last packet may run past its slot
    hipError_t e = hipHostMalloc(reinterpret_cast<void **>(&s.h_in), batch * p->w + 64,
                                 hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_in), batch * p->w + 64);
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void **>(&s.h_g), batch * 2, hipHostMallocDefault);
    if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void **>(&s.d_g), batch * 2);
    if (e == hipSuccess && p->writeback)
      e = hipHostMalloc(reinterpret_cast<void **>(&s.h_wb),
                        batch * std::min(p->w, kWriteback), hipHostMallocDefault);
    if (e == hipSuccess && p->zc)
      e = hipHostMalloc(reinterpret_cast<void **>(&s.h_ptr), batch * 8, hipHostMallocMapped);
    if (e == hipSuccess && p->zc)
      e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.dv_ptr), s.h_ptr, 0);
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking);
    if (e == hipSuccess) bg::own_stream(s.st);
    if (e == hipSuccess)
      e = hipHostMalloc(reinterpret_cast<void **>(&s.h_done), 64,
                        hipHostMallocMapped | hipHostMallocCoherent);
    if (e == hipSuccess) {
      *s.h_done = 0;
      e = hipHostGetDevicePointer(reinterpret_cast<void **>(&s.d_done), s.h_done, 0);
    }
    if (e != hipSuccess) {
      pipe_release(p);
      delete p;
      return fail(EIO, "HIP error %d: %s", (int)e, hipGetErrorString(e));
    }
    s.cookies.resize(batch);
    s.heads.resize(batch);
    if (p->meta) s.metas.resize(batch);
    if (p->writeback) s.wblen.resize(batch);
  }
  {
    std::lock_guard<std::mutex> lk(m->pipes_mu);
    m->pipes.insert(p);
  }
  m->refs.fetch_add(1, std::memory_order_relaxed);  // released by bg_pipe_destroy
  *out = p;
  return 0;
}

void bg_pipe_destroy(bg_pipe *p) {
  if (!p) return;
  {
    std::lock_guard<std::mutex> lk(p->mod->pipes_mu);
    p->mod->pipes.erase(p);
  }
  {
    std::lock_guard<std::mutex> lk(p->mu);
    pipe_release(p);
    p->ring.reset();
  }
  bg_module *m = p->mod;
  delete p;
  ModuleUnref(m);  // the module's last reference may be this pipe's
}

int bg_pipe_window(const bg_pipe *p, int *lo, int *hi, size_t *stride) {
  if (lo) *lo = p->lo;
  if (hi) *hi = p->hi;
  if (stride) *stride = p->w;
  return 0;
}

// Whether two contexts agree on every field the module's device path reads.
static bool same_ctx(unsigned use, const bg_ctx &a, const bg_ctx &b) {
  if ((use & Module::kCtxIgate) && a.igate != b.igate) return false;
  if ((use & Module::kCtxNow) && a.now_ns != b.now_ns) return false;
  return true;
}

static int submit(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                  uint8_t *const *metas, const uint16_t *lens, void *const *cookies,
                  size_t cnt);

int bg_pipe_submit(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                   const uint16_t *lens, void *const *cookies, size_t cnt) {
  return bg_pipe_submit_meta(p, ctx, heads, nullptr, lens, cookies, cnt);
}

int bg_pipe_submit_meta(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                        uint8_t *const *metas, const uint16_t *lens,
                        void *const *cookies, size_t cnt) {
  std::lock_guard<std::mutex> lk(p->mu);
  const uint64_t t0 = __rdtsc();
  const int r = submit(p, ctx, heads, metas, lens, cookies, cnt);
  p->st_submit_tsc += __rdtsc() - t0;
  return r;
}

static int submit(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                  uint8_t *const *metas, const uint16_t *lens, void *const *cookies,
                  size_t cnt) {
  if (p->err) return p->err;
  if (p->meta && !metas && cnt)  // (not sticky: nothing was taken)
    return fail(EINVAL, "the module reads metadata attributes: submit each "
                "packet's metadata area (bg_pipe_submit_meta)");
  int r;
  if (!p->writeback) gather(p, p->slots[p->fill]);  // the previous call's packets
  const bg_ctx c = ResolveCtx(ctx, p->device);
  p->st_submits++;
  p->st_pkts += cnt;
  const size_t span = (size_t)(p->hi - p->lo);
  const Module *mod = p->mod->m.get();
  size_t i = 0;
  while (i < cnt) {
    Slot &s = p->slots[p->fill];
    if (s.inflight) {  // ring full: backpressure until the oldest retires
      const uint64_t t0 = mono_ns(), w0 = p->st_wait_ns;
      r = retire_oldest(p, true);
      if (r < 0) return p->err = r;
      p->st_full_ns += mono_ns() - t0;
      p->st_wait_ns = w0;  // counted as a full ring, not as a poll wait
      continue;
    }
    if (s.draining) {  // completed but not polled: its rest waits aside
      for (size_t j = s.cursor; j < s.n; j++) p->ready.emplace_back(s.cookies[j], s.h_g[j]);
      release_oldest(p);
      continue;
    }
    if (s.n == 0) {
      s.ctx = c;
    } else if (!same_ctx(p->ctx_use, s.ctx, c)) {
      // the slot's packets run with their own context: launch them first
      r = launch_slot(p);
      if (r < 0) return p->err = r;
      continue;
    }
    const size_t take = std::min(cnt - i, p->batch - s.n);
    uint8_t *dst = s.h_in + s.n * p->w;
    size_t j = 0;
    for (; j < take; j++, dst += p->w) {
      const size_t k = i + j;
      const uint8_t *src = heads[k] + p->lo;
      if (!p->writeback) {
        // the window (rounded up to 16 bytes: the bytes past it are not
        // read by the kernel; the packet buffer holds them, SNBUF_DATA) is
        // copied by the next call's gather
        __builtin_prefetch(src);
        s.heads[s.n + j] = heads[k];
        if (p->meta) {
          __builtin_prefetch(metas[k] + p->mlo);
          s.metas[s.n + j] = metas[k];
        }
      } else {
        // a packet in host-registered memory goes in place (its head's
        // device address) when its head is 16-byte aligned, as the kernel's
        // 16-byte frame loads are (a head moved by prepend / adj goes
        // staged); a slot holds packets of one kind
        uint64_t dev = 0;
        const bool zc = p->zc && ((uintptr_t)heads[k] & 15) == 0 &&
                        bg::host_dev_addr(heads[k], span, &dev);
        if (s.n + j == 0)
          s.zc = zc;
        else if (zc != s.zc)
          break;
        if (zc) {
          s.h_ptr[s.n + j] = dev;
        } else {
          if (k + 8 < cnt) __builtin_prefetch(heads[k + 8] + p->lo);
          // the bytes the module reads (data_len when given, or what its
          // headers reach past it, Module::StageReach; at least the header
          // line), zero-padded to the slot
          size_t len =
              lens ? std::min<size_t>(mod->StageReach(heads[k], lens[k]), span) : span;
          const size_t line = std::min(span, kWriteback);
          len = std::max(len, line);
          memcpy(dst, src, len);
          if (len < p->w) memset(dst + len, 0, p->w - len);
          s.wblen[s.n + j] = (uint16_t)line;
        }
        s.heads[s.n + j] = heads[k];
      }
      s.cookies[s.n + j] = cookies ? cookies[k] : heads[k];
    }
    s.n += j;
    i += j;
    p->pending += j;
    if (s.n == p->batch || j < take) {  // full, or the next packet is of the other kind
      r = launch_slot(p);
      if (r < 0) return p->err = r;
    }
  }
  return 0;
}

static int flush(bg_pipe *p) {
  if (p->err) return p->err;
  Slot &s = p->slots[p->fill];
  if (s.inflight || s.draining || s.n == 0) return 0;
  int r = launch_slot(p);
  if (r < 0) return p->err = r;
  return 0;
}

int bg_pipe_flush(bg_pipe *p) {
  std::lock_guard<std::mutex> lk(p->mu);
  return flush(p);
}

long bg_pipe_poll(bg_pipe *p, int wait, void **cookies, uint16_t *gates,
                  size_t cap) {
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->err) return p->err;
  const uint64_t t0 = __rdtsc();
  const long k = take_done(p, wait != 0, cookies, gates, cap);
  p->st_poll_tsc += __rdtsc() - t0;
  if (k < 0) return p->err = (int)k;
  return k;
}

size_t bg_pipe_pending(const bg_pipe *p) { return p->pending; }

int bg_pipe_stats(const bg_pipe *p, uint64_t *out, int n) {
  const uint64_t v[16] = {p->st_submits, p->st_pkts, p->launched, p->st_launch_ns,
                          p->st_full_ns, p->st_wait_ns, (uint64_t)p->batch,
                          p->st_submit_tsc, p->st_poll_tsc, p->st_lat_tsc,
                          p->st_lat_max, p->st_call_ns[0], p->st_call_ns[1],
                          p->st_call_ns[2], p->st_call_ns[3], p->st_call_ns[4]};
  for (int i = 0; i < n && i < 16; i++) out[i] = v[i];
  return 0;
}

}  // extern "C"

// A THREAD_UNSAFE command is about to change the module's rules (its lock
// held exclusively, workers paused): the packets this pipe holds in its
// filling slot were submitted under the old rules, so they launch now.
int PipeFlushLocked(bg_pipe *p) {
  int cur = -1;
  (void)hipGetDevice(&cur);
  int r;
  {
    std::lock_guard<std::mutex> lk(p->mu);
    r = flush(p);
  }
  if (cur >= 0) (void)hipSetDevice(cur);
  return r;
}

extern "C" {

// A BESS worker's loop over this module (Source -> module -> Sink, SURVEY
// §3A): ProcessBatch-sized submits of `burst` packets, completions polled
// after every submit and emitted into ogates[packet index].
int bg_pipe_run(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                const uint16_t *lens, size_t n, size_t burst, uint16_t *ogates) {
  if (burst < 1) return fail(EINVAL, "burst must be >= 1");
  std::vector<void *> ck(burst), done(std::max<size_t>(p->batch, 4096));
  std::vector<uint16_t> g(done.size());
  auto emit = [&](int wait) -> int {
    long k = bg_pipe_poll(p, wait, done.data(), g.data(), done.size());
    if (k < 0) return (int)k;
    for (long j = 0; j < k; j++) ogates[(uintptr_t)done[j]] = g[j];
    return 0;
  };
  for (size_t i = 0; i < n; i += burst) {
    const size_t c = std::min(burst, n - i);
    for (size_t j = 0; j < c; j++) ck[j] = reinterpret_cast<void *>(i + j);
    // the next ProcessBatch's packets: their header lines are in flight
    // while this batch is gathered
    for (size_t j = i + c; j < std::min(n, i + c + burst); j++)
      __builtin_prefetch(heads[j] + p->lo);
    int r = bg_pipe_submit(p, ctx, heads + i, lens ? lens + i : nullptr, ck.data(), c);
    if (r < 0) return r;
    if (p->inflight && (r = emit(0)) < 0) return r;
  }
  int r = bg_pipe_flush(p);
  if (r < 0) return r;
  while (p->pending)
    if ((r = emit(1)) < 0) return r;
  return 0;
}

}  // extern "C"
