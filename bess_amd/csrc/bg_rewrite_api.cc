// bg_rewrite_api.cc -- C ABI of the Rewrite datapath (include/bessgpu.h
// bg_rewrite_*): the template set (CommandAdd / CommandClear,
// core/modules/rewrite.cc:25-70, with the reference's checks and messages)
// and the round-robin turn live on the host; the templates' device copy is
// refreshed when they change; ProcessBatch runs on a device slab of packet
// slots, or on host packets staged through the calling thread's buffers.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>

#include "bg_internal.h"

using namespace bg;

// One device copy of the templates. A kernel launched against it may still
// be queued on its stream when the templates change, so the copy is never
// overwritten: a change uploads a new generation, and the old one is freed
// once the events recorded behind its launches (one per stream it was
// launched on) have completed -- this handle's own launches only, never the
// device's other work (round 5 synchronized the whole device here, which on
// the datapath waited for other pipes' persistent ring kernels).
struct RwGen {
  int device = -1;
  uint8_t *d_tmpl = nullptr;    // kRwMaxTemplates x kRwMaxSize
  uint16_t *d_size = nullptr;
  std::vector<std::pair<hipStream_t, hipEvent_t>> launched;  // stream -> last launch
  bool done() const {  // every launch against it has finished
    for (auto &e : launched)
      if (hipEventQuery(e.second) == hipErrorNotReady) return false;
    return true;
  }
  void release() {
    for (auto &e : launched) {
      (void)hipEventSynchronize(e.second);
      (void)hipEventDestroy(e.second);
    }
    launched.clear();
    if (d_tmpl) (void)hipFree(d_tmpl);
    if (d_size) (void)hipFree(d_size);
    d_tmpl = nullptr;
    d_size = nullptr;
  }
};

struct bg_rewrite {
  std::vector<uint8_t> tmpl;    // n x kRwMaxSize, zero past each size
  std::vector<uint16_t> size;
  uint64_t next = 0;            // next_turn_
  bool dirty = true;
  RwGen cur;                    // the templates launches read now
  std::vector<RwGen> retired;   // older copies, launches maybe still queued
  std::mutex mu;
  ~bg_rewrite() {
    cur.release();
    for (auto &g : retired) g.release();
  }
};

namespace {

// the current templates on `device`, uploaded on `s` (which later launches
// on `s` follow; other streams: the upload is synchronized)
int sync_templates(bg_rewrite *h, int device, hipStream_t s) {
  if (!h->dirty && h->cur.device == device && h->cur.d_tmpl) return 0;
  if (h->size.empty()) {
    h->dirty = false;
    return 0;
  }
  // free the retired copies whose launches have all finished
  for (size_t i = 0; i < h->retired.size();) {
    if (h->retired[i].done()) {
      h->retired[i].release();
      h->retired.erase(h->retired.begin() + i);
    } else {
      i++;
    }
  }
  if (h->cur.d_tmpl) {
    if (h->cur.launched.empty()) {
      h->cur.release();  // never launched against: reuse nothing, free now
    } else {
      h->retired.push_back(std::move(h->cur));
      h->cur = RwGen();
    }
  }
  RwGen g;
  g.device = device;
  if (hipMalloc(reinterpret_cast<void **>(&g.d_tmpl), (size_t)kRwMaxTemplates * kRwMaxSize) !=
          hipSuccess ||
      hipMalloc(reinterpret_cast<void **>(&g.d_size), kRwMaxTemplates * 2) != hipSuccess) {
    g.release();
    return fail(ENOMEM, "no device memory for the templates");
  }
  if (hipMemcpyAsync(g.d_tmpl, h->tmpl.data(), h->tmpl.size(), hipMemcpyHostToDevice, s) !=
          hipSuccess ||
      hipMemcpyAsync(g.d_size, h->size.data(), h->size.size() * 2, hipMemcpyHostToDevice, s) !=
          hipSuccess ||
      hipStreamSynchronize(s) != hipSuccess) {
    g.release();
    return fail(EIO, "template upload failed");
  }
  h->cur = std::move(g);
  h->dirty = false;
  return 0;
}

// an event behind this launch on `s` (re-recorded per launch: the stream's
// last launch against the current templates)
int note_launch(bg_rewrite *h, hipStream_t s) {
  for (auto &e : h->cur.launched)
    if (e.first == s) {
      HIP_TRY(hipEventRecord(e.second, s));
      return 0;
    }
  hipEvent_t ev;
  HIP_TRY(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  if (hipEventRecord(ev, s) != hipSuccess) {
    (void)hipEventDestroy(ev);
    return fail(EIO, "hipEventRecord failed");
  }
  h->cur.launched.emplace_back(s, ev);
  return 0;
}

// the bytes a packet's rewrite writes past its head: the largest template
// rounded to the reference's 32-byte copy blocks
uint32_t span_of(const bg_rewrite *h) {
  uint32_t m = 0;
  for (uint16_t z : h->size) m = std::max<uint32_t>(m, (z + 31u) & ~31u);
  return m;
}

}  // namespace

extern "C" {

int bg_rewrite_create(bg_rewrite **out) {
  if (!out) return fail(EINVAL, "bad arguments");
  *out = new bg_rewrite();
  return 0;
}

void bg_rewrite_destroy(bg_rewrite *h) { delete h; }

// CommandAdd (rewrite.cc:25-61): all or nothing
int bg_rewrite_add(bg_rewrite *h, const uint8_t *const *templates,
                   const uint32_t *lens, int k) {
  if (k < 0 || (k > 0 && (!templates || !lens))) return fail(EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(h->mu);
  const size_t curr = h->size.size();
  if (curr + (size_t)k > kRwMaxTemplates)
    return fail(EINVAL, "max %zu packet templates can be used %zu %d",
                (size_t)kRwMaxTemplates, curr, k);
  for (int i = 0; i < k; i++)
    if (lens[i] > kRwMaxSize) return fail(EINVAL, "template is too big");
  for (int i = 0; i < k; i++) {
    h->tmpl.resize((curr + i + 1) * kRwMaxSize, 0);
    memcpy(h->tmpl.data() + (curr + i) * kRwMaxSize, templates[i], lens[i]);
    h->size.push_back((uint16_t)lens[i]);
  }
  h->dirty = true;
  return 0;
}

// CommandClear (rewrite.cc:63-67)
void bg_rewrite_clear(bg_rewrite *h) {
  std::lock_guard<std::mutex> lk(h->mu);
  h->next = 0;
  h->size.clear();
  h->tmpl.clear();
  h->dirty = true;
}

size_t bg_rewrite_count(const bg_rewrite *h) { return h->size.size(); }

// add() from a serialized bess.pb.RewriteArg (module_msg.proto: `repeated
// bytes templates = 1`), as bessd hands a plugin its Init / add argument:
// proto3 wire format, unknown fields skipped
int bg_rewrite_add_pb(bg_rewrite *h, const void *arg, size_t len) {
  const uint8_t *p = static_cast<const uint8_t *>(arg), *end = p + len;
  auto varint = [&](uint64_t *v) {
    *v = 0;
    for (int sh = 0; sh < 64 && p < end; sh += 7) {
      const uint8_t b = *p++;
      *v |= (uint64_t)(b & 0x7F) << sh;
      if (!(b & 0x80)) return true;
    }
    return false;
  };
  std::vector<const uint8_t *> ts;
  std::vector<uint32_t> ls;
  while (p < end) {
    uint64_t key, v;
    if (!varint(&key)) return fail(EINVAL, "malformed RewriteArg");
    const uint32_t wt = key & 7;
    if (wt == 0) {
      if (!varint(&v)) return fail(EINVAL, "malformed RewriteArg");
    } else if (wt == 2) {
      if (!varint(&v) || v > (uint64_t)(end - p)) return fail(EINVAL, "malformed RewriteArg");
      if ((key >> 3) == 1) {
        ts.push_back(p);
        ls.push_back((uint32_t)std::min<uint64_t>(v, 0xFFFFFFFFu));
      }
      p += v;
    } else if (wt == 1 || wt == 5) {
      const size_t k = wt == 1 ? 8 : 4;
      if ((size_t)(end - p) < k) return fail(EINVAL, "malformed RewriteArg");
      p += k;
    } else {
      return fail(EINVAL, "malformed RewriteArg");
    }
  }
  return bg_rewrite_add(h, ts.data(), ls.data(), (int)ts.size());
}

int bg_rewrite_process(bg_rewrite *h, int device, void *d_slots, size_t stride,
                       size_t n, uint32_t headroom, uint16_t *d_head, uint32_t *d_len,
                       bg_stream_t stream) {
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(h->mu);
  const uint32_t nt = (uint32_t)h->size.size();
  if (nt == 0) return 0;  // ProcessBatch with no template: packets untouched
  const uint32_t span = span_of(h);
  if (headroom > 0xFFFFu || (size_t)headroom + span > stride)
    return fail(EINVAL, "headroom %u + %u template bytes past the %zu-byte slot",
                headroom, span, stride);
  if (stride % 16 || headroom % 16 || ((uintptr_t)d_slots & 15))
    return fail(EINVAL, "slots and headroom must be 16-byte aligned");
  int r = set_device(device);
  if (r) return r;
  // the caller's stream as given (NULL: the legacy default stream), so the
  // kernel is ordered after the caller's earlier work on the slots and the
  // head / len arrays (a private non-blocking stream would not be)
  hipStream_t s = (hipStream_t)stream;
  r = sync_templates(h, device, s);
  if (r) return r;
  RewriteArgs a;
  memset(&a, 0, sizeof(a));
  a.slots = static_cast<uint8_t *>(d_slots);
  a.stride = stride;
  a.n = n;
  a.tmpl = h->cur.d_tmpl;
  a.tsize = h->cur.d_size;
  a.ntempl = nt;
  a.start = nt == 1 ? 0u : (uint32_t)h->next;  // DoRewriteSingle keeps turn 0
  a.headroom = headroom;
  a.units = span / 16;
  uint32_t lg = 0;
  while ((1u << lg) < a.units && lg < 6) lg++;
  a.lpp_log2 = lg;
  a.head = d_head;
  a.len = d_len;
  HIP_TRY(launch_rewrite(a, num_cus(device), s));
  if ((r = note_launch(h, s))) return r;
  if (nt > 1) h->next = (h->next + n) % nt;  // consecutive batches' turns
  return 0;
}

// Host packets (bessd's snbufs): slots[i] is packet i's buffer; the device
// writes the packets' new data into the calling thread's staging, which is
// copied into each buffer at headroom with head / len set. Synchronous.
int bg_rewrite_process_host(bg_rewrite *h, int device, uint8_t *const *slots,
                            size_t slot_bytes, size_t n, uint32_t headroom,
                            uint16_t *head, uint32_t *len, bg_stream_t stream) {
  if (n == 0) return 0;
  if (!slots || !head || !len) return fail(EINVAL, "bad arguments");
  uint32_t span;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->size.empty()) return 0;
    span = span_of(h);
  }
  if ((size_t)headroom + span > slot_bytes)
    return fail(EINVAL, "headroom %u + %u template bytes past the %zu-byte slot",
                headroom, span, slot_bytes);
  Staging &st = thread_staging();
  int r = set_device(device);
  if (r) return r;
  hipStream_t s = thread_stream(device, (hipStream_t)stream);
  // device slots of `span` bytes (headroom 0), then head (u16) and len (u32)
  const size_t arr = n * 8;
  r = st.ensure(device, n * span + arr, 16);
  if (r) return r;
  uint16_t *dh = reinterpret_cast<uint16_t *>(st.d_in + n * span);
  uint32_t *dl = reinterpret_cast<uint32_t *>(st.d_in + n * span + n * 2 + (n & 1) * 2);
  r = bg_rewrite_process(h, device, st.d_in, span, n, 0, dh, dl, s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.h_in, st.d_in, n * span + arr, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const uint16_t *hh = reinterpret_cast<const uint16_t *>(st.h_in + n * span);
  const uint32_t *hl = reinterpret_cast<const uint32_t *>(st.h_in + n * span + n * 2 + (n & 1) * 2);
  for (size_t i = 0; i < n; i++) {
    memcpy(slots[i] + headroom, st.h_in + i * span + hh[i], (hl[i] + 31u) & ~31u);
    head[i] = (uint16_t)headroom;
    len[i] = hl[i];
  }
  return 0;
}

}  // extern "C"
