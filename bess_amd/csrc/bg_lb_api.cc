// bg_lb_api.cc -- C ABI of the HashLB datapath (include/bessgpu.h bg_hlb_*):
// the per-position CRC32C tables and the gate table the kernel stages in
// LDS (bg_lb.hip), uploaded when the mode or the gates change.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <memory>
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

// one device's image of one mode + gate-table version: [crc tables][gates]
struct HlbImage : DevImage {
  HlbArgs a{};                  // tables into d, mode, geometry
  std::vector<bg_field> fields;  // fields mode: the key's fields
};

struct bg_hlb {
  int mode = kHlbL4;
  std::vector<bg_field> fields;
  uint32_t L = 4;  // hash input bytes
  std::vector<uint16_t> gates{0};  // gates_[0 .. max(n, 1))
  uint32_t num_gates = 0;
  // set_mode / set_gates bump the version; each device's image is rebuilt
  // fresh at its next classify (bg_image.h)
  std::atomic<uint64_t> version{1};
  Published<HlbImage> dev;
  std::mutex mu;
};

static void hlb_changed(bg_hlb *h) { h->version.fetch_add(1, std::memory_order_acq_rel); }

static int hlb_image(bg_hlb *h, int dev, hipStream_t s, HlbImage **out) {
  HlbImage *v = h->dev.get(dev);
  const uint64_t ver = h->version.load(std::memory_order_acquire);
  if (v && v->version == ver) {
    *out = v;
    return 0;
  }
  std::lock_guard<std::mutex> lk(h->mu);
  v = h->dev.get(dev);
  if (!v || v->version != ver) {
    std::vector<uint32_t> T = position_tables(h->L);
    const size_t tb = T.size() * 4, gb = h->gates.size() * 2;
    std::vector<uint8_t> img(tb + gb);
    memcpy(img.data(), T.data(), tb);
    memcpy(img.data() + tb, h->gates.data(), gb);
    std::unique_ptr<HlbImage> p(new HlbImage());
    int r = upload_image(p.get(), dev, img.data(), img.size(), s);
    if (r) return r;
    p->version = ver;
    p->a.crc_tab = reinterpret_cast<const uint32_t *>(p->d);
    p->a.gtab = reinterpret_cast<const uint16_t *>(p->d + tb);
    p->a.mode = (uint32_t)h->mode;
    p->a.L = h->L;
    p->a.num_gates = h->num_gates;
    p->a.ngtab = (uint32_t)h->gates.size();
    p->fields = h->fields;
    for (auto &x : p->fields) x.mask = 0;  // AddField(offset, size, 0, i): all bits
    v = p.get();
    h->dev.publish(dev, p.release());
  }
  *out = v;
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
  hlb_changed(h);
  return 0;
}

int bg_hlb_set_gates(bg_hlb *h, const uint16_t *gates, size_t n,
                     size_t num_gates) {
  if (n > BG_HLB_MAX_GATES || n < 1 || num_gates > n)
    return fail(EINVAL, "gate table of %zu entries (num_gates %zu)", n, num_gates);
  std::lock_guard<std::mutex> lk(h->mu);
  h->gates.assign(gates, gates + n);
  h->num_gates = (uint32_t)num_gates;
  hlb_changed(h);
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
  HlbImage *img;
  if (int r = hlb_image(h, dev, s, &img)) return r;
  HlbArgs a = img->a;
  if (a.mode == (uint32_t)BG_HLB_FIELDS) a.fp = make_plan(img->fields, false, -win_off);
  if (a.mode != (uint32_t)BG_HLB_FIELDS && stride < (size_t)(a.mode == BG_HLB_L2 ? 16 : 64))
    return fail(EINVAL, "stride %zu too small for the mode", stride);
  img->used_on(s);
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_gates;
  HIP_TRY(launch_hlb(a, num_cus(dev), s));
  img->launched_on(s);
  return 0;
}

}  // extern "C"
