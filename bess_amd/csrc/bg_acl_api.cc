// bg_acl_api.cc -- C ABI of the ACL datapath (include/bessgpu.h bg_acl_*):
// the ordered rule list, compiled when it changes into the forms bg_acl.hip
// classifies with (the list in the frame's byte order for the scans, the
// per-dimension bit vectors, the decision tree) and uploaded.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <algorithm>
#include <array>
#include <mutex>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <memory>
#include <vector>

#include "bg_internal.h"

using namespace bg;

// one device's image of one rule-list version: [rules][bit vectors][trees]
struct AclImage : DevImage {
  AclArgs a{};  // rules / bv / tree pointers into d and their geometry
};

struct bg_acl {
  std::vector<bg_acl_rule> rules;
  // list changes bump the version; each device's image is rebuilt fresh at
  // its next classify (bg_image.h)
  std::atomic<uint64_t> version{1};
  std::vector<uint32_t> host_img;  // the image of host_version
  AclArgs host_a{};                // its launch arguments, offsets in words
  uint64_t bv_off = 0, tree_off = 0;  // words (0: none)
  uint64_t host_version = 0;
  Published<AclImage> dev;
  std::mutex mu;
};

static void acl_changed(bg_acl *h) { h->version.fetch_add(1, std::memory_order_acq_rel); }

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

// ---- decision trees (AclArgs tree fields, bg_acl.hip AclTreeOp) ---------
//
// Every ACL field is a prefix: the addresses by their prefix length
// (Ipv4Prefix), a port exact (length 16) or 0 = any (length 0). A node is
// the box of packets that agree on the first c[d] bits of each dimension d;
// it cuts k more bits of one dimension into 2^k children. A rule goes to the
// children its prefix allows (all of them when its length is <= c[d]).
// A node's list keeps the list order and ends at the first rule that covers
// its box (length <= c[d] in every dimension): later rules can never be the
// first match there. Lists of <= kLeafMax rules become leaves. Children
// with equal lists share one subtree (equal lists imply equal subtrees: a
// rule in two siblings has no bits left to test in the cut dimension).
//
// One tree over all rules replicates the rules that are wild in the cut
// dimension into every child: 1000 random rules (bench lists) needed up to
// 600 KB. So the rules are split by which address is specific (prefix
// length >= kSpecific; EffiCuts' separation), one tree per class, and the
// packet takes the lowest rule index any tree matches (records carry it).
// A rule that matches every packet ends every class's list.

namespace {

constexpr int kTreeW[4] = {32, 32, 16, 16};
constexpr size_t kAclTreeLdsBytes = 112 << 10;  // + 32 KB stage <= 160 KB
constexpr uint32_t kLeafMax = 8;
constexpr int kCutMax = 8;              // up to 256 children per node
constexpr size_t kTreeMaxRules = 8192;  // larger lists: the scans
constexpr int kSpecific = 8;

struct TreeRule {
  uint32_t v[4];   // host-order value, masked to its prefix
  uint8_t len[4];  // prefix length
  bool drop;
};

bool prefix_len(uint32_t mask, uint8_t *len) {
  const uint32_t inv = ~mask;
  if (inv & (inv + 1)) return false;  // not a prefix mask
  *len = (uint8_t)__builtin_popcount(mask);
  return true;
}

typedef std::array<uint8_t, 4> Box;  // bits fixed per dimension

struct TreeBuilder {
  std::vector<TreeRule> R;
  std::vector<uint32_t> recs;   // leaf records, 4 words each
  std::vector<uint32_t> nodes;  // child arrays; internal refs node-relative
  std::unordered_map<std::string, uint32_t> memo;
  size_t budget_words = kAclTreeLdsBytes / 4;
  bool overflow = false;

  uint32_t bits_of(const TreeRule &r, int d, int c, int k) const {
    return (r.v[d] >> (kTreeW[d] - c - k)) & ((1u << k) - 1);
  }
  bool covers(const TreeRule &r, const Box &c) const {
    for (int d = 0; d < 4; d++)
      if (r.len[d] > c[d]) return false;
    return true;
  }
  // the 2^k children of (lst, c) cut on k bits of d, truncated
  void cut(const std::vector<uint32_t> &lst, const Box &c, int d, int k,
           std::vector<std::vector<uint32_t>> *ch, Box *c2) const {
    const uint32_t nc = 1u << k;
    *c2 = c;
    (*c2)[d] = (uint8_t)(c[d] + k);
    ch->assign(nc, {});
    std::vector<uint8_t> closed(nc, 0);
    auto put = [&](uint32_t j, uint32_t r) {
      if (closed[j]) return;
      (*ch)[j].push_back(r);
      if (covers(R[r], *c2)) closed[j] = 1;
    };
    for (uint32_t r : lst) {
      const TreeRule &x = R[r];
      if (x.len[d] <= c[d]) {
        for (uint32_t j = 0; j < nc; j++) put(j, r);
      } else if (x.len[d] >= c[d] + k) {
        put(bits_of(x, d, c[d], k), r);
      } else {
        const int span = c[d] + k - x.len[d];
        const uint32_t base = bits_of(x, d, c[d], k) & ~((1u << span) - 1);
        for (uint32_t j = 0; j < (1u << span); j++) put(base + j, r);
      }
    }
  }
  static std::string key_of(const std::vector<uint32_t> &lst, const Box &c) {
    std::string s(reinterpret_cast<const char *>(c.data()), 4);
    s.append(reinterpret_cast<const char *>(lst.data()), lst.size() * 4);
    return s;
  }
  uint32_t leaf(const std::vector<uint32_t> &lst) {
    const uint32_t off = (uint32_t)(recs.size() / 4);
    for (uint32_t r : lst) {
      const TreeRule &x = R[r];
      recs.push_back(x.v[0]);
      recs.push_back(x.v[1]);
      recs.push_back(x.v[2] | (x.v[3] << 16));
      recs.push_back((uint32_t)x.len[0] | ((uint32_t)x.len[1] << 6) |
                     ((uint32_t)(x.len[2] != 0) << 12) | ((uint32_t)(x.len[3] != 0) << 13) |
                     ((uint32_t)x.drop << 14) | (r << 16));
    }
    return 0x80000000u | ((uint32_t)lst.size() << 16) | off;
  }
  uint32_t build(const std::vector<uint32_t> &lst, const Box &c) {
    if (overflow) return 0;
    const std::string key = key_of(lst, c);
    auto it = memo.find(key);
    if (it != memo.end()) return it->second;
    uint32_t ref;
    int best_d = -1, best_k = 0;
    size_t best_mx = 0, best_mem = 0;
    if (lst.size() > kLeafMax) {
      std::vector<std::vector<uint32_t>> ch;
      Box c2;
      for (int d = 0; d < 4; d++) {
        bool useful = false;
        for (uint32_t r : lst) useful |= R[r].len[d] > c[d];
        if (!useful) continue;
        for (int k = 1; k <= std::min(kCutMax, kTreeW[d] - (int)c[d]); k++) {
          cut(lst, c, d, k, &ch, &c2);
          std::unordered_set<std::string> uniq;
          size_t mx = 0, mem = (size_t)1 << k;
          for (auto &x : ch) {
            mx = std::max(mx, x.size());
            if (uniq.insert(key_of(x, c2)).second) mem += x.size() * 4;
          }
          // wider cuts only while they stay within a space factor
          if (k > 1 && mem > 16 * lst.size() + 64) break;
          if (best_d < 0 || mx < best_mx || (mx == best_mx && mem < best_mem)) {
            best_d = d;
            best_k = k;
            best_mx = mx;
            best_mem = mem;
          }
        }
      }
    }
    // no useful cut: every rule is covered, so the list is one rule long
    if (best_d < 0) {
      ref = leaf(lst);
    } else {
      std::vector<std::vector<uint32_t>> ch;
      Box c2;
      cut(lst, c, best_d, best_k, &ch, &c2);
      const uint32_t nc = 1u << best_k;
      const uint32_t at = (uint32_t)nodes.size();
      nodes.resize(nodes.size() + nc);
      const int shift = kTreeW[best_d] - c2[best_d] + (best_d == 3 ? 16 : 0);
      ref = ((uint32_t)std::min(best_d, 2) << 25) | ((uint32_t)best_k << 21) |
            ((uint32_t)shift << 16) | at;
      for (uint32_t j = 0; j < nc && !overflow; j++) {
        const uint32_t child = build(ch[j], c2);  // may grow nodes
        nodes[at + j] = child;
      }
    }
    if (recs.size() + nodes.size() > budget_words) overflow = true;
    memo.emplace(key, ref);
    return ref;
  }
};

}  // namespace

// The trees' image [leaf records][child arrays] and their roots, or false
// (no trees: masks that are not prefixes, too many rules, or an image past
// the LDS budget).
static bool build_tree(const std::vector<bg_acl_rule> &rules, std::vector<uint32_t> *img,
                       uint32_t *roots, uint32_t *ntrees) {
  if (rules.empty() || rules.size() > kTreeMaxRules) return false;
  TreeBuilder b;
  for (const bg_acl_rule &x : rules) {
    TreeRule t;
    if (!prefix_len(x.src_mask, &t.len[0]) || !prefix_len(x.dst_mask, &t.len[1]))
      return false;
    t.v[0] = x.src_addr & x.src_mask;
    t.v[1] = x.dst_addr & x.dst_mask;
    t.v[2] = x.src_port;
    t.v[3] = x.dst_port;
    t.len[2] = x.src_port ? 16 : 0;
    t.len[3] = x.dst_port ? 16 : 0;
    t.drop = x.drop != 0;
    b.R.push_back(t);
  }
  // classes: src address specific x dst address specific
  std::vector<uint32_t> cls[4];
  for (uint32_t i = 0; i < rules.size(); i++) {
    const TreeRule &t = b.R[i];
    cls[(t.len[0] >= kSpecific ? 0 : 2) + (t.len[1] >= kSpecific ? 0 : 1)].push_back(i);
    if (b.covers(t, {0, 0, 0, 0})) break;  // matches every packet
  }
  std::vector<uint32_t> r;
  for (auto &l : cls)
    if (!l.empty()) r.push_back(b.build(l, {0, 0, 0, 0}));
  if (b.overflow) return false;
  const uint32_t base = (uint32_t)b.recs.size();  // a multiple of 4
  auto fix = [&](uint32_t ref) { return (ref >> 31) ? ref : ref + base; };
  img->assign(b.recs.begin(), b.recs.end());
  for (uint32_t w : b.nodes) img->push_back(fix(w));
  while (img->size() % 4) img->push_back(0);
  if (img->size() * 4 > kAclTreeLdsBytes || img->size() > 0xFFFF) return false;
  *ntrees = (uint32_t)r.size();
  for (size_t i = 0; i < r.size(); i++) roots[i] = fix(r[i]);
  return true;
}

// the host image of the current list: rules, then the bit-vector form and
// the decision trees when they are built, each 64-byte aligned
static void acl_build_host(bg_acl *h) {
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
  AclArgs &a = h->host_a;
  a = AclArgs{};
  std::vector<uint32_t> bv;
  h->bv_off = h->tree_off = 0;
  if (build_bv(h->rules, &bv, &a)) {  // geometry into a, words appended
    h->bv_off = (img.size() + 15) / 16 * 16;
    img.resize(h->bv_off, 0);
    img.insert(img.end(), bv.begin(), bv.end());
  }
  std::vector<uint32_t> tree;
  uint32_t roots[4] = {}, ntrees = 0;
  if (build_tree(h->rules, &tree, roots, &ntrees)) {
    h->tree_off = (img.size() + 15) / 16 * 16;
    img.resize(h->tree_off, 0);
    img.insert(img.end(), tree.begin(), tree.end());
    a.tree_words = (uint32_t)tree.size();
    a.ntrees = ntrees;
    memcpy(a.roots, roots, sizeof(a.roots));
  }
  a.nrules = (uint32_t)np;
  h->host_img.swap(img);
}

// the device's image of the current list (rebuilt fresh when it changed;
// the replaced image is retired behind fences)
static int acl_image(bg_acl *h, int dev, hipStream_t s, AclImage **out) {
  AclImage *v = h->dev.get(dev);
  const uint64_t ver = h->version.load(std::memory_order_acquire);
  if (v && v->version == ver) {
    *out = v;
    return 0;
  }
  std::lock_guard<std::mutex> lk(h->mu);
  v = h->dev.get(dev);
  if (!v || v->version != ver) {
    if (h->host_version != ver) {
      acl_build_host(h);
      h->host_version = ver;
    }
    std::unique_ptr<AclImage> img(new AclImage());
    int r = upload_image(img.get(), dev, h->host_img.data(), h->host_img.size() * 4, s);
    if (r) return r;
    img->version = ver;
    const uint32_t *b = reinterpret_cast<const uint32_t *>(img->d);
    img->a = h->host_a;
    img->a.rules = b;
    img->a.bv = h->bv_off ? b + h->bv_off : nullptr;
    img->a.tree = h->tree_off ? b + h->tree_off : nullptr;
    v = img.get();
    h->dev.publish(dev, img.release());
  }
  *out = v;
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
  acl_changed(h);
  return 0;
}

void bg_acl_clear(bg_acl *h) {
  std::lock_guard<std::mutex> lk(h->mu);
  h->rules.clear();
  acl_changed(h);
}

size_t bg_acl_count(const bg_acl *h) { return h->rules.size(); }

int bg_acl_tree(bg_acl *h, uint32_t *img, size_t cap, size_t *words, uint32_t *roots,
                int *ntrees) {
  if (!words || !roots || !ntrees) return fail(EINVAL, "bad arguments");
  std::vector<uint32_t> t;
  uint32_t nt = 0;
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (!build_tree(h->rules, &t, roots, &nt))
      return fail(ENOENT, "no decision tree for this rule list");
  }
  *ntrees = (int)nt;
  *words = t.size();
  if (img && cap >= t.size()) memcpy(img, t.data(), t.size() * 4);
  else if (img) return fail(ENOBUFS, "tree needs %zu words", t.size());
  return 0;
}

int bg_acl_classify(bg_acl *h, const void *d_frames, size_t stride, size_t n,
                    uint16_t igate, uint16_t *d_out, bg_stream_t stream) {
  if (stride % 16 || stride < 64 || ((uintptr_t)d_frames & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned, stride a 16-byte "
                "multiple >= 64");
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  AclImage *img;
  if (int r = acl_image(h, dev, s, &img)) return r;
  AclArgs a = img->a;
  img->used_on(s);
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_out;
  a.igate = igate;
  HIP_TRY(launch_acl(a, num_cus(dev), s));
  img->launched_on(s);
  return 0;
}

}  // extern "C"
