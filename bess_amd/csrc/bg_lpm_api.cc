// bg_lpm_api.cc -- C ABI of the IPLookup datapath (include/bessgpu.h
// bg_lpm_*): the route table with rte_lpm's add / delete / capacity
// semantics (DPDK 19.11 rte_lpm.c, as IPLookup uses it), laid out as
// DIR-24-8 and uploaded to the device when it changes (bg_lpm.hip).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <map>
#include <memory>
#include <mutex>
#include <vector>

#include "bg_internal.h"

using namespace bg;

namespace {
constexpr uint32_t kTbl24 = 1u << 24;
constexpr uint32_t kMaxGroups = 0x7FFF;  // u16 entries: 15-bit group index
constexpr uint32_t kMaxNextHop = 0x7FFE;  // u16 entries: next hop + 1

uint32_t depth_mask(int depth) {
  return depth == 0 ? 0u : depth >= 32 ? 0xFFFFFFFFu : ~((1u << (32 - depth)) - 1u);
}
}  // namespace

// one device's tables of one route-set version: [tbl24][tbl8][tbl16][tbl2]
struct LpmImage : DevImage {
  LpmArgs a{};  // the table pointers into d
};

struct bg_lpm {
  uint32_t max_rules = 1024, max_tbl8s = 128;
  // (depth, masked ip) -> next hop: map order = ascending depth, the order
  // DIR-24-8 is filled in (longer prefixes overwrite shorter ones)
  std::map<std::pair<int, uint32_t>, uint32_t> rules;
  std::map<uint32_t, int> ext;  // /24 block -> rules deeper than /24 in it
  // route changes bump the version; each device's tables are rebuilt into a
  // fresh image at its next lookup (bg_image.h)
  std::atomic<uint64_t> version{1};
  std::vector<uint8_t> host_img;  // the tables of host_version
  uint64_t off8 = 0, off16 = 0, off2 = 0;  // their offsets (off16 0: none)
  uint64_t host_version = 0;
  Published<LpmImage> dev;
  std::mutex mu;
};

static void lpm_changed(bg_lpm *h) { h->version.fetch_add(1, std::memory_order_acq_rel); }

static int lpm_build_host(bg_lpm *h) {
  std::vector<uint16_t> t24(kTbl24, 0);
  std::vector<uint16_t> t8;
  std::map<uint32_t, std::vector<std::pair<int, uint32_t>>> deep;  // block -> rules
  for (const auto &kv : h->rules) {
    const int depth = kv.first.first;
    const uint32_t ip = kv.first.second, nh = kv.second;
    if (depth <= 24) {
      const uint32_t start = ip >> 8, cnt = 1u << (24 - depth);
      std::fill(t24.begin() + start, t24.begin() + start + cnt, (uint16_t)(nh + 1));
    } else {
      deep[ip >> 8].push_back(kv.first);
    }
  }
  uint32_t g = 0;
  for (const auto &b : deep) {
    t8.resize((size_t)(g + 1) * 256, t24[b.first]);  // the covering <= /24 route
    uint16_t *grp = t8.data() + (size_t)g * 256;
    for (const auto &k : b.second) {  // ascending depth (map order)
      const uint32_t start = k.second & 0xFF, cnt = 1u << (32 - k.first);
      std::fill(grp + start, grp + start + cnt, (uint16_t)(h->rules[k] + 1));
    }
    t24[b.first] = (uint16_t)(0x8000u | g);
    g++;
  }
  // DIR-16-8-8: a /16 block whose 256 tbl24 entries are one plain value
  // keeps it in tbl16; any other block gets a tbl2 group (its entries)
  std::vector<uint16_t> t16(1u << 16), t2;
  bool has16 = true;
  for (uint32_t b = 0; b < (1u << 16) && has16; b++) {
    const uint16_t *seg = t24.data() + (size_t)b * 256;
    const bool flat = !(seg[0] & 0x8000u) && std::all_of(seg, seg + 256, [&](uint16_t v) {
      return v == seg[0];
    });
    if (flat) {
      t16[b] = seg[0];
    } else if (t2.size() / 256 >= kMaxGroups) {
      has16 = false;  // past 15-bit group indices: DIR-24-8 only
    } else {
      t16[b] = (uint16_t)(0x8000u | (t2.size() / 256));
      t2.insert(t2.end(), seg, seg + 256);
    }
  }
  // one image: tbl24, tbl8 (>= 1 group), then tbl16 and tbl2 if built
  h->off8 = align256((uint64_t)kTbl24 * 2);
  const uint64_t end8 = h->off8 + std::max<size_t>(g, 1) * 512;
  h->off16 = has16 ? align256(end8) : 0;
  h->off2 = has16 ? align256(h->off16 + t16.size() * 2) : 0;
  const uint64_t total = has16 ? h->off2 + std::max<size_t>(t2.size(), 256) * 2 : end8;
  std::vector<uint8_t> &img = h->host_img;
  img.assign(total, 0);
  memcpy(img.data(), t24.data(), (size_t)kTbl24 * 2);
  if (g) memcpy(img.data() + h->off8, t8.data(), t8.size() * 2);
  if (has16) {
    memcpy(img.data() + h->off16, t16.data(), t16.size() * 2);
    if (!t2.empty()) memcpy(img.data() + h->off2, t2.data(), t2.size() * 2);
  }
  return 0;
}

// the device's tables of the current routes, rebuilt into a fresh image
// when they changed (the replaced image is retired behind fences)
static int lpm_image(bg_lpm *h, int dev, hipStream_t s, LpmImage **out) {
  LpmImage *v = h->dev.get(dev);
  const uint64_t ver = h->version.load(std::memory_order_acquire);
  if (v && v->version == ver) {
    *out = v;
    return 0;
  }
  std::lock_guard<std::mutex> lk(h->mu);
  v = h->dev.get(dev);
  if (!v || v->version != ver) {
    if (h->host_version != ver) {
      if (int r = lpm_build_host(h)) return r;
      h->host_version = ver;
    }
    std::unique_ptr<LpmImage> img(new LpmImage());
    int r = upload_image(img.get(), dev, h->host_img.data(), h->host_img.size(), s);
    if (r) return r;
    img->version = ver;
    uint16_t *b = reinterpret_cast<uint16_t *>(img->d);
    img->a.tbl24 = b;
    img->a.tbl8 = b + h->off8 / 2;
    img->a.tbl16 = h->off16 ? b + h->off16 / 2 : nullptr;
    img->a.tbl2 = h->off16 ? b + h->off2 / 2 : b + h->off8 / 2;
    v = img.get();
    h->dev.publish(dev, img.release());
  }
  *out = v;
  return 0;
}

extern "C" {

int bg_lpm_create(uint32_t max_rules, uint32_t max_tbl8s, bg_lpm **out) {
  if (!out) return fail(EINVAL, "bad arguments");
  bg_lpm *h = new bg_lpm();
  h->max_rules = max_rules ? max_rules : 1024;
  h->max_tbl8s = max_tbl8s ? max_tbl8s : 128;
  *out = h;
  return 0;
}

void bg_lpm_destroy(bg_lpm *h) { delete h; }

// rte_lpm_add: an existing (prefix, depth) gets the new next hop; a new rule
// needs room in the rule table (max_rules) and, deeper than /24 in a /24
// block that has no such rule yet, a free tbl8 group (max_tbl8s).
int bg_lpm_add(bg_lpm *h, uint32_t ip, int depth, uint32_t next_hop) {
  if (depth < 1 || depth > 32) return fail(EINVAL, "depth %d", depth);
  if (next_hop > kMaxNextHop) return fail(EINVAL, "next hop %u", next_hop);
  std::lock_guard<std::mutex> lk(h->mu);
  const uint32_t ipm = ip & depth_mask(depth);
  auto key = std::make_pair(depth, ipm);
  auto it = h->rules.find(key);
  if (it != h->rules.end()) {
    it->second = next_hop;
    lpm_changed(h);
    return 0;
  }
  if (h->rules.size() >= h->max_rules) return fail(ENOSPC, "rule table full");
  if (depth > 24) {
    auto e = h->ext.find(ipm >> 8);
    if (e == h->ext.end()) {
      if (h->ext.size() >= std::min(h->max_tbl8s, kMaxGroups))
        return fail(ENOSPC, "no free tbl8 group");
      h->ext[ipm >> 8] = 1;
    } else {
      e->second++;
    }
  }
  h->rules[key] = next_hop;
  lpm_changed(h);
  return 0;
}

int bg_lpm_delete(bg_lpm *h, uint32_t ip, int depth) {
  if (depth < 1 || depth > 32) return fail(EINVAL, "depth %d", depth);
  std::lock_guard<std::mutex> lk(h->mu);
  const uint32_t ipm = ip & depth_mask(depth);
  auto it = h->rules.find(std::make_pair(depth, ipm));
  if (it == h->rules.end()) return fail(EINVAL, "no such rule");
  h->rules.erase(it);
  if (depth > 24) {
    auto e = h->ext.find(ipm >> 8);
    if (--e->second == 0) h->ext.erase(e);  // tbl8 group recycled
  }
  lpm_changed(h);
  return 0;
}

void bg_lpm_clear(bg_lpm *h) {
  std::lock_guard<std::mutex> lk(h->mu);
  h->rules.clear();
  h->ext.clear();
  lpm_changed(h);
}

size_t bg_lpm_count(const bg_lpm *h) { return h->rules.size(); }

int bg_lpm_classify(bg_lpm *h, const void *d_frames, size_t stride, size_t n,
                    uint16_t default_gate, uint16_t *d_out, bg_stream_t stream) {
  if (stride % 16 || stride < 64 || ((uintptr_t)d_frames & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned, stride a 16-byte "
                "multiple >= 64");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  LpmImage *img;
  if (int r = lpm_image(h, dev, s, &img)) return r;
  LpmArgs a = img->a;
  img->used_on(s);
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_out;
  a.default_gate = default_gate;
  HIP_TRY(launch_lpm(a, num_cus(dev), s));
  img->launched_on(s);
  return 0;
}

}  // extern "C"
