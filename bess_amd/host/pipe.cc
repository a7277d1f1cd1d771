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
#include <hip/hip_runtime.h>
#include <string.h>

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
  std::vector<uint8_t *> heads;  // writeback targets
  std::vector<uint16_t> wblen;   // bytes of the header line to write back
  std::vector<void *> cookies;
  size_t n = 0;
  bool inflight = false;
  bg_ctx ctx{};  // the context of the slot's packets (Module::CtxUse fields)
};

}  // namespace

struct bg_pipe {
  bg_module *mod = nullptr;
  int device = 0;
  size_t batch = 0;
  int lo = 0, hi = 0;    // staged frame bytes [lo, hi)
  size_t w = 0;          // staged stride (16-byte multiple)
  bool writeback = false;
  unsigned ctx_use = 0;  // Module::CtxUse(): the context fields a slot fixes
  std::vector<Slot> slots;
  size_t fill = 0;       // slot being filled
  size_t oldest = 0;     // oldest in-flight slot
  size_t inflight = 0;   // slots in flight
  std::deque<std::pair<void *, uint16_t>> ready;  // completed, not returned
  size_t pending = 0;    // submitted, not yet returned by poll
  int err = 0;           // sticky launch error
  uint64_t launched = 0;  // slot launches so far (Slot::seq)
  // One worker owns a pipe; the lock is for the module's control path
  // (PipeFlushLocked) and a RunTask on another worker (never contended on
  // the datapath).
  std::mutex mu;
};

static void pipe_release(bg_pipe *p) {
  for (Slot &s : p->slots) {
    if (s.st) {
      (void)hipStreamSynchronize(s.st);
      bg::stream_gone(s.st);  // no table image fences on it any more
    }
    if (s.h_in) (void)hipHostFree(s.h_in);
    if (s.h_wb) (void)hipHostFree(s.h_wb);
    if (s.h_g) (void)hipHostFree(s.h_g);
    if (s.h_done) (void)hipHostFree(s.h_done);
    if (s.d_in) (void)hipFree(s.d_in);
    if (s.d_g) (void)hipFree(s.d_g);
    if (s.st) (void)hipStreamDestroy(s.st);
  }
  p->slots.clear();
}

// Launch the fill slot (n > 0): H2D, module kernel, D2H, event. (No
// module lock: like bessd's datapath, a pipe relies on THREAD_UNSAFE
// commands running only while its worker is paused, core/module.cc:97-101;
// such a command flushes the pipe first, PipeFlushLocked.)
static int launch_slot(bg_pipe *p) {
  Slot &s = p->slots[p->fill];
  const size_t n = s.n;
  int rc = bg::set_device(p->device);
  if (rc) return rc;
  HIP_TRY(hipMemcpyAsync(s.d_in, s.h_in, n * p->w, hipMemcpyHostToDevice, s.st));
  bg_ctx c = s.ctx;
  c.device = (int16_t)p->device;
  int r = p->mod->m->ProcessDeviceWindow(c, s.d_in, p->w, n, p->lo, s.d_g, s.st);
  if (r < 0) return r;
  HIP_TRY(hipMemcpyAsync(s.h_g, s.d_g, n * 2, hipMemcpyDeviceToHost, s.st));
  if (p->writeback) {
    const size_t line = std::min(p->w, kWriteback);
    HIP_TRY(hipMemcpy2DAsync(s.h_wb, line, s.d_in, p->w, line, n,
                             hipMemcpyDeviceToHost, s.st));
  }
  // completion lands in host memory after the D2H copies: poll reads one
  // word and makes no HIP call
  s.seq = ++p->launched;
  HIP_TRY(hipStreamWriteValue64(s.st, s.d_done, s.seq, 0));
  s.inflight = true;
  p->inflight++;
  p->fill = (p->fill + 1) % p->slots.size();
  return 0;
}

// Retire the oldest in-flight slot (blocking when `wait`). Returns 1 if a
// slot was retired, 0 if not (nothing in flight / not done), or -errno.
static int retire_oldest(bg_pipe *p, bool wait) {
  if (p->inflight == 0) return 0;
  Slot &s = p->slots[p->oldest];
  if (__atomic_load_n(s.h_done, __ATOMIC_ACQUIRE) != s.seq) {
    if (!wait) return 0;
    int rc = bg::set_device(p->device);
    if (rc) return rc;
    HIP_TRY(hipStreamSynchronize(s.st));
    if (__atomic_load_n(s.h_done, __ATOMIC_ACQUIRE) != s.seq)
      return fail(EIO, "pipe slot %llu: completion word not written",
                  (unsigned long long)s.seq);
  }
  if (p->writeback) {
    const size_t line = std::min(p->w, kWriteback);
    for (size_t i = 0; i < s.n; i++)
      memcpy(s.heads[i], s.h_wb + i * line, s.wblen[i]);
  }
  for (size_t i = 0; i < s.n; i++) p->ready.emplace_back(s.cookies[i], s.h_g[i]);
  s.n = 0;
  s.inflight = false;
  p->inflight--;
  p->oldest = (p->oldest + 1) % p->slots.size();
  return 1;
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
  if (span && p->lo == 0 && (int)span < p->hi) p->hi = (int)span;
  if (p->hi <= p->lo) p->hi = p->lo + 1;
  p->w = ((size_t)(p->hi - p->lo) + 15) / 16 * 16;
  p->ctx_use = m->m->CtxUse();
  p->slots.resize((size_t)depth);
  for (Slot &s : p->slots) {
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
    if (e == hipSuccess) e = hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking);
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
    if (p->writeback) {
      s.heads.resize(batch);
      s.wblen.resize(batch);
    }
  }
  {
    std::lock_guard<std::mutex> lk(m->pipes_mu);
    m->pipes.insert(p);
  }
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
  }
  delete p;
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

int bg_pipe_submit(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                   const uint16_t *lens, void *const *cookies, size_t cnt) {
  std::lock_guard<std::mutex> lk(p->mu);
  if (p->err) return p->err;
  int r;
  const bg_ctx c = ResolveCtx(ctx, p->device);
  const size_t span = (size_t)(p->hi - p->lo);
  size_t i = 0;
  while (i < cnt) {
    Slot &s = p->slots[p->fill];
    if (s.inflight) {  // ring full: backpressure until the oldest retires
      r = retire_oldest(p, true);
      if (r < 0) return p->err = r;
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
    for (size_t j = 0; j < take; j++, dst += p->w) {
      const size_t k = i + j;
      if (k + 8 < cnt) __builtin_prefetch(heads[k + 8] + p->lo);
      const uint8_t *src = heads[k] + p->lo;
      if (!p->writeback) {
        memcpy(dst, src, span);
      } else {
        // the frame (data_len bytes when given, at least its header line),
        // zero-padded to the slot
        size_t len = lens ? std::min<size_t>(lens[k], span) : span;
        const size_t line = std::min(span, kWriteback);
        len = std::max(len, line);
        memcpy(dst, src, len);
        if (len < p->w) memset(dst + len, 0, p->w - len);
        s.heads[s.n + j] = heads[k];
        s.wblen[s.n + j] = (uint16_t)line;
      }
      s.cookies[s.n + j] = cookies ? cookies[k] : heads[k];
    }
    s.n += take;
    i += take;
    p->pending += take;
    if (s.n == p->batch) {
      r = launch_slot(p);
      if (r < 0) return p->err = r;
    }
  }
  return 0;
}

static int flush(bg_pipe *p) {
  if (p->err) return p->err;
  Slot &s = p->slots[p->fill];
  if (s.inflight || s.n == 0) return 0;
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
  for (;;) {
    int r = retire_oldest(p, wait && p->ready.empty());
    if (r < 0) return p->err = r;
    if (r == 0) break;
  }
  size_t k = 0;
  while (k < cap && !p->ready.empty()) {
    const auto &e = p->ready.front();
    if (cookies) cookies[k] = e.first;
    if (gates) gates[k] = e.second;
    p->ready.pop_front();
    k++;
  }
  p->pending -= k;
  return (long)k;
}

size_t bg_pipe_pending(const bg_pipe *p) { return p->pending; }

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
