// bg_acl_api.cc -- C ABI of the ACL datapath (include/bessgpu.h bg_acl_*):
// the ordered rule list, compiled to the frame's byte order and uploaded
// when it changes (bg_acl.hip reads it with wave-uniform loads).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "bg_internal.h"

using namespace bg;

struct bg_acl {
  std::vector<bg_acl_rule> rules;
  bool dirty = true;
  int device = -1;
  uint32_t *d_rules = nullptr;
  size_t d_cap = 0;  // rules
  std::mutex mu;
  ~bg_acl() {
    if (d_rules) (void)hipFree(d_rules);
  }
};

static uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

static int acl_sync_locked(bg_acl *h, int dev, hipStream_t s) {
  if (!h->dirty && h->device == dev && (h->d_rules || h->rules.empty())) return 0;
  int r = set_device(dev);
  if (r) return r;
  const size_t n = h->rules.size();
  const size_t np = (n + 3) / 4 * 4;  // groups of 4; padding never valid
  std::vector<uint32_t> img(std::max<size_t>(np, 4) * 8, 0);
  for (size_t i = 0; i < n; i++) {
    const bg_acl_rule &x = h->rules[i];
    uint32_t *o = &img[i * 8];
    // Ipv4Prefix::Match: (addr & mask) == (ip & mask), in frame byte order
    o[0] = __builtin_bswap32(x.src_addr & x.src_mask);
    o[1] = __builtin_bswap32(x.src_mask);
    o[2] = __builtin_bswap32(x.dst_addr & x.dst_mask);
    o[3] = __builtin_bswap32(x.dst_mask);
    // ports (be16_t values) as the LE dword at the L4 header; 0 = wildcard
    o[4] = (uint32_t)bswap16(x.src_port) | ((uint32_t)bswap16(x.dst_port) << 16);
    o[5] = (x.src_port ? 0xFFFFu : 0u) | (x.dst_port ? 0xFFFF0000u : 0u);
    o[6] = x.drop ? 1u : 0u;
    o[7] = 1;  // valid
  }
  if (!h->d_rules || h->d_cap < img.size() / 8 || h->device != dev) {
    if (h->d_rules) (void)hipFree(h->d_rules);
    h->d_rules = nullptr;
    h->d_cap = std::max<size_t>(img.size() / 8, 64);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&h->d_rules), h->d_cap * 32));
  }
  HIP_TRY(hipMemcpyAsync(h->d_rules, img.data(), img.size() * 4,
                         hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  h->device = dev;
  h->dirty = false;
  return 0;
}

extern "C" {

int bg_acl_create(bg_acl **out) {
  if (!out) return fail(EINVAL, "bad arguments");
  *out = new bg_acl();
  return 0;
}

void bg_acl_destroy(bg_acl *h) { delete h; }

int bg_acl_add(bg_acl *h, const bg_acl_rule *rules, size_t n) {
  if (n && !rules) return fail(EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(h->mu);
  h->rules.insert(h->rules.end(), rules, rules + n);
  h->dirty = true;
  return 0;
}

void bg_acl_clear(bg_acl *h) {
  std::lock_guard<std::mutex> lk(h->mu);
  h->rules.clear();
  h->dirty = true;
}

size_t bg_acl_count(const bg_acl *h) { return h->rules.size(); }

int bg_acl_classify(bg_acl *h, const void *d_frames, size_t stride, size_t n,
                    uint16_t igate, uint16_t *d_out, bg_stream_t stream) {
  if (stride % 16 || stride < 64 || ((uintptr_t)d_frames & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned, stride a 16-byte "
                "multiple >= 64");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  AclArgs a;
  memset(&a, 0, sizeof(a));
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->device >= 0) dev = h->device;
    int r = acl_sync_locked(h, dev, s);
    if (r) return r;
    a.rules = h->d_rules;
    a.nrules = (uint32_t)((h->rules.size() + 3) / 4 * 4);
  }
  int r = set_device(dev);
  if (r) return r;
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_out;
  a.igate = igate;
  HIP_TRY(launch_acl(a, num_cus(dev), s));
  return 0;
}

}  // extern "C"
