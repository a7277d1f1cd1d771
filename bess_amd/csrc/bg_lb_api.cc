// bg_lb_api.cc -- C ABI of the HashLB datapath (include/bessgpu.h bg_hlb_*):
// the per-position CRC32C tables and the gate table the kernel stages in
// LDS (bg_lb.hip), uploaded when the mode or the gates change.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <vector>

#include "bg_internal.h"

using namespace bg;

namespace {

constexpr uint32_t kCrc32cPoly = 0x82F63B78u;  // reflected Castagnoli

// one CRC32C step over a byte (the SSE4.2 crc32 instruction without the
// initial / final inversion: _mm_crc32_u8(crc, b))
uint32_t crc32c_byte(uint32_t crc, uint8_t b) {
  crc ^= b;
  for (int k = 0; k < 8; k++) crc = (crc >> 1) ^ (kCrc32cPoly & (0u - (crc & 1u)));
  return crc;
}

// T[i][v] = CRC32C(init 0) of the L-byte message that is v at position i
// and zero elsewhere: the CRC of v then L-1-i zero bytes.
std::vector<uint32_t> position_tables(uint32_t L) {
  std::vector<uint32_t> T((size_t)L * 256);
  for (uint32_t v = 0; v < 256; v++) {
    uint32_t c = crc32c_byte(0, (uint8_t)v);
    for (int i = (int)L - 1; i >= 0; i--) {
      T[(size_t)i * 256 + v] = c;
      c = crc32c_byte(c, 0);
    }
  }
  return T;
}

}  // namespace

struct bg_hlb {
  int mode = kHlbL4;
  std::vector<bg_field> fields;
  uint32_t L = 4;  // hash input bytes
  std::vector<uint16_t> gates{0};  // gates_[0 .. max(n, 1))
  uint32_t num_gates = 0;
  bool dirty = true;
  int device = -1;
  uint8_t *d_buf = nullptr;  // [crc tables][gate table]
  size_t d_cap = 0;
  std::mutex mu;
  ~bg_hlb() {
    if (d_buf) (void)hipFree(d_buf);
  }
};

static int hlb_sync_locked(bg_hlb *h, int dev, hipStream_t s) {
  if (!h->dirty && h->device == dev && h->d_buf) return 0;
  int r = set_device(dev);
  if (r) return r;
  std::vector<uint32_t> T = position_tables(h->L);
  const size_t tb = T.size() * 4, gb = h->gates.size() * 2;
  if (!h->d_buf || h->d_cap < tb + gb || h->device != dev) {
    if (h->d_buf) (void)hipFree(h->d_buf);
    h->d_buf = nullptr;
    h->d_cap = std::max<size_t>(tb + gb, 64 * 1024 + 32 * 1024 + 64);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&h->d_buf), h->d_cap));
  }
  HIP_TRY(hipMemcpyAsync(h->d_buf, T.data(), tb, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->d_buf + tb, h->gates.data(), gb,
                         hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  h->device = dev;
  h->dirty = false;
  return 0;
}

extern "C" {

int bg_hlb_create(int mode, const bg_field *fields, int nfields, bg_hlb **out) {
  if (mode < BG_HLB_L2 || mode > BG_HLB_FIELDS)
    return fail(EINVAL, "mode %d", mode);
  bg_hlb *h = new bg_hlb();
  int r = bg_hlb_set_mode(h, mode, fields, nfields, -1);
  if (r) {
    delete h;
    return r;
  }
  *out = h;
  return 0;
}

void bg_hlb_destroy(bg_hlb *h) { delete h; }

int bg_hlb_set_mode(bg_hlb *h, int mode, const bg_field *fields, int nfields,
                    int hash_len) {
  if (mode < BG_HLB_L2 || mode > BG_HLB_FIELDS)
    return fail(EINVAL, "mode %d", mode);
  std::lock_guard<std::mutex> lk(h->mu);
  if (mode == BG_HLB_FIELDS) {
    if (nfields < 0 || nfields > BG_MAX_FIELDS || (nfields && !fields))
      return fail(EINVAL, "fields mode takes 0..%d fields", BG_MAX_FIELDS);
    if (hash_len > BG_KEY_BYTES || (hash_len > 0 && hash_len % 8))
      return fail(EINVAL, "hash_len %d", hash_len);
    int acc = 0;
    for (int i = 0; i < nfields; i++) {
      const bg_field &f = fields[i];
      if (f.size < 1 || f.size > 8 || f.offset < 0 || f.offset > 1024 ||
          f.pos != acc || f.attr_id >= 0)
        return fail(EINVAL, "idx %d: bad field", i);
      acc += f.size;
    }
    h->fields.assign(fields, fields + nfields);
    // ExactMatchKeyHash(total_key_size_) unless given
    h->L = hash_len >= 0 ? (uint32_t)hash_len : (uint32_t)(acc + 7) / 8 * 8;
  } else {
    h->fields.clear();
    h->L = mode == BG_HLB_L2 ? 2 : 4;
  }
  h->mode = mode;
  h->dirty = true;
  return 0;
}

int bg_hlb_set_gates(bg_hlb *h, const uint16_t *gates, size_t n,
                     size_t num_gates) {
  if (n > BG_HLB_MAX_GATES || n < 1 || num_gates > n)
    return fail(EINVAL, "gate table of %zu entries (num_gates %zu)", n, num_gates);
  std::lock_guard<std::mutex> lk(h->mu);
  h->gates.assign(gates, gates + n);
  h->num_gates = (uint32_t)num_gates;
  h->dirty = true;
  return 0;
}

void bg_hlb_window(const bg_hlb *h, int *lo, int *hi) {
  if (h->mode == BG_HLB_FIELDS) {
    int l = 1 << 30, u = 0;
    for (auto &f : h->fields) {
      l = std::min(l, f.offset);
      u = std::max(u, f.offset + f.size);
    }
    if (h->fields.empty()) l = u = 0;
    *lo = l;
    *hi = u;
  } else {
    *lo = 0;
    *hi = h->mode == BG_HLB_L2 ? 16 : h->mode == BG_HLB_L3 ? 48 : 80;
  }
}

int bg_hlb_classify(bg_hlb *h, const void *d_frames, size_t stride, size_t n,
                    int win_off, uint16_t *d_gates, bg_stream_t stream) {
  if (stride % 16 || ((uintptr_t)d_frames & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned with stride %% 16 == 0");
  if (win_off != 0 && h->mode != BG_HLB_FIELDS)
    return fail(EINVAL, "l2/l3/l4 modes read the frame from offset 0");
  if (win_off < 0 || win_off > 1024) return fail(EINVAL, "win_off %d", win_off);
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  HlbArgs a;
  memset(&a, 0, sizeof(a));
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->device >= 0) dev = h->device;
    int r = hlb_sync_locked(h, dev, s);
    if (r) return r;
    a.crc_tab = reinterpret_cast<const uint32_t *>(h->d_buf);
    a.gtab = reinterpret_cast<const uint16_t *>(h->d_buf + (size_t)h->L * 1024);
    a.mode = (uint32_t)h->mode;
    a.L = h->L;
    a.num_gates = h->num_gates;
    a.ngtab = (uint32_t)h->gates.size();
    if (h->mode == BG_HLB_FIELDS) {
      std::vector<bg_field> f = h->fields;
      for (auto &x : f) x.mask = 0;  // AddField(offset, size, 0, i): all bits
      a.fp = make_plan(f, false, -win_off);
    }
  }
  if (h->mode != BG_HLB_FIELDS && stride < (size_t)(h->mode == BG_HLB_L2 ? 16 : 64))
    return fail(EINVAL, "stride %zu too small for the mode", stride);
  int r = set_device(dev);
  if (r) return r;
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_gates;
  HIP_TRY(launch_hlb(a, num_cus(dev), s));
  return 0;
}

}  // extern "C"
