// bg_acl_api.cc -- C ABI of the ACL datapath (include/bessgpu.h bg_acl_*):
// the ordered rule list, compiled to the frame's byte order and uploaded
// when it changes (bg_acl.hip reads it with wave-uniform loads).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
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
  uint32_t *d_bv = nullptr;  // the bit-vector form (bv_args), or none
  size_t bv_cap = 0;         // words
  AclArgs bv_args{};         // its geometry and offsets (bv = d_bv)
  std::mutex mu;
  ~bg_acl() {
    if (d_rules) (void)hipFree(d_rules);
    if (d_bv) (void)hipFree(d_bv);
  }
};

static uint16_t bswap16(uint16_t v) { return (uint16_t)((v >> 8) | (v << 8)); }

// LDS for the two address dimensions' interval starts
static const size_t kAclBvLdsBytes = 64 << 10;

static uint32_t ceil_log2(uint32_t k) {
  uint32_t l = 0;
  while ((1ull << l) < k) l++;
  return l;
}

// The bit-vector image of an ordered rule list (AclArgs in bg_kernels.h).
// Per dimension, elementary intervals and, for each, the bit vector of the
// rules that match there. Returns false when the address interval starts
// would not fit in LDS (the launch then uses the rule scan).
static bool build_bv(const std::vector<bg_acl_rule> &R, std::vector<uint32_t> *img,
                     AclArgs *a) {
  const uint32_t nr = (uint32_t)R.size();
  const uint32_t nw = (nr + 31) / 32;
  const uint32_t grp = std::max<uint32_t>(1, (nw + 31) / 32);
  std::vector<uint32_t> B[2], V[4], S[4];
  uint32_t k[4];
  for (int d = 0; d < 2; d++) {  // addresses: prefix ranges [lo, hi]
    std::vector<uint32_t> &b = B[d];
    b.push_back(0);
    for (const bg_acl_rule &x : R) {
      const uint32_t m = d ? x.dst_mask : x.src_mask;
      const uint32_t lo = (d ? x.dst_addr : x.src_addr) & m, hi = lo | ~m;
      b.push_back(lo);
      if (hi != 0xFFFFFFFFu) b.push_back(hi + 1);
    }
    std::sort(b.begin(), b.end());
    b.erase(std::unique(b.begin(), b.end()), b.end());
    k[d] = (uint32_t)b.size();
    V[d].assign((size_t)k[d] * nw, 0);
    for (uint32_t r = 0; r < nr; r++) {
      const bg_acl_rule &x = R[r];
      const uint32_t m = d ? x.dst_mask : x.src_mask;
      const uint32_t lo = (d ? x.dst_addr : x.src_addr) & m, hi = lo | ~m;
      const size_t ia = std::lower_bound(b.begin(), b.end(), lo) - b.begin();
      const size_t ib = hi == 0xFFFFFFFFu
                            ? b.size() - 1
                            : (size_t)(std::lower_bound(b.begin(), b.end(), hi + 1) -
                                       b.begin()) - 1;
      for (size_t i = ia; i <= ib; i++) V[d][i * nw + r / 32] |= 1u << (r % 32);
    }
  }
  if ((size_t)(k[0] + k[1]) * 4 > kAclBvLdsBytes) return false;
  std::vector<uint16_t> P[2];
  for (int d = 0; d < 2; d++) {  // ports: exact values; 0 = any
    std::vector<uint16_t> vals;
    for (const bg_acl_rule &x : R) {
      const uint16_t p = d ? x.dst_port : x.src_port;
      if (p) vals.push_back(p);
    }
    std::sort(vals.begin(), vals.end());
    vals.erase(std::unique(vals.begin(), vals.end()), vals.end());
    k[2 + d] = (uint32_t)vals.size() + 1;  // class 0: no rule names the port
    P[d].assign(65536, 0);
    for (size_t j = 0; j < vals.size(); j++)  // indexed by the frame's raw bytes
      P[d][bswap16(vals[j])] = (uint16_t)(j + 1);
    std::vector<uint32_t> &v = V[2 + d];
    v.assign((size_t)k[2 + d] * nw, 0);
    for (uint32_t r = 0; r < nr; r++) {
      const uint16_t p = d ? R[r].dst_port : R[r].src_port;
      if (p == 0) {
        for (uint32_t i = 0; i < k[2 + d]; i++) v[(size_t)i * nw + r / 32] |= 1u << (r % 32);
      } else {
        const size_t j = std::lower_bound(vals.begin(), vals.end(), p) - vals.begin() + 1;
        v[j * nw + r / 32] |= 1u << (r % 32);
      }
    }
  }
  for (int d = 0; d < 4; d++) {
    S[d].assign(k[d], 0);
    for (uint32_t i = 0; i < k[d]; i++)
      for (uint32_t w = 0; w < nw; w++)
        if (V[d][(size_t)i * nw + w]) S[d][i] |= 1u << (w / grp);
  }
  std::vector<uint32_t> D(std::max<uint32_t>(nw, 1), 0);
  for (uint32_t r = 0; r < nr; r++)
    if (R[r].drop) D[r / 32] |= 1u << (r % 32);
  // [B0][B1][S0..S3][V0..V3][P2][P3][D]
  img->clear();
  auto put = [&](const uint32_t *p, size_t n) {
    const size_t o = img->size();
    img->insert(img->end(), p, p + n);
    return (uint32_t)o;
  };
  a->b_off[0] = put(B[0].data(), B[0].size());
  a->b_off[1] = put(B[1].data(), B[1].size());
  for (int d = 0; d < 4; d++) a->s_off[d] = put(S[d].data(), S[d].size());
  for (int d = 0; d < 4; d++) a->v_off[d] = put(V[d].data(), V[d].size());
  for (int d = 0; d < 2; d++)
    a->p_off[d] = put(reinterpret_cast<const uint32_t *>(P[d].data()), 65536 / 2);
  a->d_off = put(D.data(), D.size());
  a->k0 = k[0];
  a->k1 = k[1];
  a->lg0 = ceil_log2(k[0]);
  a->lg1 = ceil_log2(k[1]);
  a->nw = nw;
  a->grp = grp;
  return true;
}

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
  // the padding repeats the last rule (it can never be a first match):
  // the LDS scan then needs no validity test per rule
  for (size_t i = n; n && i < np; i++)
    memcpy(&img[i * 8], &img[(n - 1) * 8], 32);
  if (!h->d_rules || h->d_cap < img.size() / 8 || h->device != dev) {
    if (h->d_rules) (void)hipFree(h->d_rules);
    h->d_rules = nullptr;
    h->d_cap = std::max<size_t>(img.size() / 8, 64);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&h->d_rules), h->d_cap * 32));
  }
  HIP_TRY(hipMemcpyAsync(h->d_rules, img.data(), img.size() * 4,
                         hipMemcpyHostToDevice, s));
  std::vector<uint32_t> bv;
  h->bv_args = AclArgs{};
  if (build_bv(h->rules, &bv, &h->bv_args)) {
    if (!h->d_bv || h->bv_cap < bv.size() || h->device != dev) {
      if (h->d_bv) (void)hipFree(h->d_bv);
      h->d_bv = nullptr;
      h->bv_cap = bv.size();
      HIP_TRY(hipMalloc(reinterpret_cast<void **>(&h->d_bv), h->bv_cap * 4));
    }
    HIP_TRY(hipMemcpyAsync(h->d_bv, bv.data(), bv.size() * 4, hipMemcpyHostToDevice, s));
    h->bv_args.bv = h->d_bv;
  }
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
    a = h->bv_args;  // the bit-vector form, when it was built
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
