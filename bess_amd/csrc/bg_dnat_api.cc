// bg_dnat_api.cc -- C ABI of the NAT datapath (include/bessgpu.h bg_dnat_*).
//
// The NAT map (core/modules/nat.h:129-175: endpoint -> NatEntry, forward and
// reverse entries) lives on the host, where new mappings are made; the
// device keeps a lookup copy (bg_table.h image, entry index values), the
// entries' translated endpoints and their forward timestamps.
// CreateNewEntry (nat.cc:180-258) draws ports from the module's Random and
// may evict an expired mapping that a later packet of the same batch would
// have hit. A hit on a mapping that has NOT expired at `now` is final for the
// whole batch (only expired mappings can be evicted, and a hit refreshes its
// mapping), so every batch is
//   1. dnat_fused_kernel (dnat_fused_slab_kernel for 64-byte slots): lookup
//      and Stamp of every final hit in one pass over the header line,
//      forward timestamps refreshed; forward misses AND forward hits on
//      expired mappings are listed instead;
//   2. only if the list is not empty: the listed packets walked in packet
//      order on the host (find, or CreateNewEntry with its eviction), the
//      device copy updated, and dnat_apply_kernel stamps the listed packets.
// Reverse traffic never creates a mapping, so a reverse batch is step 1.
// The host's forward timestamps are lower bounds of the device's (only the
// device refreshes between walks): a mapping the host sees as unexpired is
// unexpired; one it sees as expired is re-read from the device before the
// port search may evict it.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "bg_internal.h"
#include "bg_launch.h"

using namespace bg;

namespace {

constexpr uint64_t kTimeOutNs = 300ull * 1000 * 1000 * 1000;  // nat.h:167
constexpr int kMaxTrials = 128;                                 // nat.h:170

struct Range {
  uint16_t begin, end;
  bool suspended;
};

uint64_t ep_key(uint32_t addr_raw, uint16_t port_raw, uint16_t proto) {
  return (uint64_t)addr_raw | (uint64_t)port_raw << 32 | (uint64_t)proto << 48;
}

// crc32c_sse42_u32(v, 0) as rte_hash_crc(&addr, 4, 0) computes it: the
// reflected CRC-32C register update over v's bytes in memory order, no
// final inversion (the SSE4.2 crc32 instruction)
uint32_t crc32c_u32(uint32_t v) {
  uint32_t c = 0;
  for (int b = 0; b < 4; b++) {
    c ^= (v >> (8 * b)) & 0xFFu;
    for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
  }
  return c;
}

bool parse_ipv4(const char *s, uint32_t *host) {  // ParseIpv4Address
  unsigned a, b, c, d;
  if (!s || sscanf(s, "%u.%u.%u.%u", &a, &b, &c, &d) != 4 || a >= 256 ||
      b >= 256 || c >= 256 || d >= 256)
    return false;
  *host = a << 24 | b << 16 | c << 8 | d;
  return true;
}

// Host mirror of the device lookup image, kept in step with the map so that
// a batch that adds or evicts mappings sends the device only the 8-byte
// words it changed (dnat_image_kernel) instead of a rebuilt image. Slot key
// words as in bg_dnat.hip lookup_hit: the endpoint with the entry index's
// top byte in bits 56-63, its translation with the index's low half in bits
// 48-63. New keys go in by cuckoo insertion (the builder's placement rule:
// a free slot of b1, then b2, then a random-walk eviction path); past the
// load limit or an insertion failure the next sync rebuilds the image.
struct ImageMirror {
  std::vector<uint8_t> img;
  TableLayout L{};
  std::vector<uint64_t> occ;                   // per slot: endpoint or kFree
  std::unordered_map<uint64_t, uint32_t> at;   // endpoint -> slot
  std::vector<uint32_t> dirty;                 // changed 8-byte words
  uint64_t rng = 0x9E3779B97F4A7C15ull;
  bool valid = false;
  static constexpr uint64_t kFree = ~0ull;
  static constexpr double kMaxLoad = 0.9;

  Probe probe(uint64_t key) const {
    return split_hash(hash_words(&key, 1, L.seed), 1, L.nbp);
  }
  uint32_t *tags() { return reinterpret_cast<uint32_t *>(img.data()); }
  uint64_t *kwords() { return reinterpret_cast<uint64_t *>(img.data() + L.keys_off); }
  uint32_t *vals() { return reinterpret_cast<uint32_t *>(img.data() + L.vals_off); }
  void mark(const void *p) {
    dirty.push_back((uint32_t)((reinterpret_cast<const uint8_t *>(p) - img.data()) / 8));
  }
  // write (or clear, e = ~0u) one slot
  void write_slot(uint32_t slot, uint64_t key, uint32_t e, uint64_t ep) {
    const uint32_t b = slot / kSlots, sh = 8 * (slot % kSlots);
    uint32_t &tw = tags()[b];
    tw &= ~(0xFFu << sh);
    uint64_t *kw = kwords() + (uint64_t)slot * 2;
    if (e == ~0u) {
      kw[0] = kw[1] = 0;
      vals()[slot] = 0;
      occ[slot] = kFree;
    } else {
      tw |= probe(key).tag << sh;
      kw[0] = key | (uint64_t)(e >> 16) << 56;
      kw[1] = (ep & 0xFFFFFFFFFFFFull) | (uint64_t)(e & 0xFFFF) << 48;
      vals()[slot] = e;
      occ[slot] = key;
      at[key] = slot;
    }
    mark(&tw);
    mark(kw);
    mark(kw + 1);
    mark(&vals()[slot]);
  }
  // after a full build: which slot holds which endpoint
  void index(const std::vector<uint8_t> &image, const TableLayout &lay) {
    img = image;
    L = lay;
    occ.assign((size_t)L.nbp * kSlots, kFree);
    at.clear();
    dirty.clear();
    const uint64_t *kw = kwords();
    for (uint32_t sl = 0; sl < occ.size(); sl++) {
      if (!((tags()[sl / kSlots] >> (8 * (sl % kSlots))) & 0xFFu)) continue;
      const uint64_t key = kw[(uint64_t)sl * 2] & 0x00FFFFFFFFFFFFFFull;
      occ[sl] = key;
      at[key] = sl;
    }
    valid = true;
  }
  // insert or update; false: the image must be rebuilt
  bool put(uint64_t key, uint32_t e, uint64_t ep, const std::vector<uint64_t> &ent_ep) {
    if (!valid) return false;
    auto it = at.find(key);
    if (it != at.end()) {
      write_slot(it->second, key, e, ep);
      return true;
    }
    if ((double)(at.size() + 1) > kMaxLoad * (double)occ.size()) return false;
    uint64_t cur = key;
    uint32_t ce = e;
    uint64_t cep = ep;
    Probe p = probe(cur);
    for (uint32_t b : {p.b1, p.b2})
      for (int s = 0; s < kSlots; s++)
        if (occ[b * kSlots + s] == kFree) {
          write_slot(b * kSlots + s, cur, ce, cep);
          return true;
        }
    uint32_t bucket = (rng_next() & 1) ? p.b2 : p.b1;
    for (int step = 0; step < 500; step++) {
      for (int s = 0; s < kSlots; s++)
        if (occ[bucket * kSlots + s] == kFree) {
          write_slot(bucket * kSlots + s, cur, ce, cep);
          return true;
        }
      const uint32_t slot = bucket * kSlots + (uint32_t)(rng_next() % kSlots);
      const uint64_t vkey = occ[slot];
      const uint32_t ve = vals()[slot];
      at.erase(vkey);
      write_slot(slot, cur, ce, cep);
      cur = vkey;
      ce = ve;
      cep = ent_ep[ve];
      const Probe q = probe(cur);
      bucket = q.b1 == bucket ? q.b2 : q.b1;
    }
    valid = false;  // the displaced key has no slot: rebuild
    return false;
  }
  void erase(uint64_t key) {
    if (!valid) return;
    auto it = at.find(key);
    if (it == at.end()) return;
    const uint32_t slot = it->second;
    at.erase(it);
    write_slot(slot, 0, ~0u, 0);
  }
  uint64_t rng_next() {
    rng ^= rng << 13;
    rng ^= rng >> 7;
    rng ^= rng << 17;
    return rng;
  }
};

}  // namespace

struct bg_dnat {
  std::vector<uint32_t> ext;               // ext_addrs_ (raw be32), sorted
  std::vector<std::vector<Range>> ranges;  // port_ranges_ (argument order)
  uint64_t seed;                           // Random::seed_
  // the map: key -> entry index; entries: translated endpoint, timestamp
  std::unordered_map<uint64_t, uint32_t> map;
  // per entry: translated endpoint, forward timestamp (a lower bound of the
  // device's unless `exact`), whether the current walk set it
  std::vector<uint64_t> ent_ep, ent_ts;
  std::vector<uint32_t> exact_walk;  // walk that made ent_ts exact
  uint32_t walk = 1;
  std::vector<uint32_t> free_idx;
  std::vector<uint32_t> changed;  // entries to push to the device
  bool map_dirty = true;          // the lookup images must be rebuilt
  // Two lookup images -- forward entries (internal endpoint -> external)
  // and reverse entries -- since a batch has one direction: its lookups
  // touch half the keys (half the L2 footprint of one combined table)
  std::vector<uint8_t> ent_rev;   // per entry: 1 = reverse entry
  DevTable tab[2];
  ImageMirror mirror[2];          // the images, for word-level updates
  int device = -1;
  hipStream_t walk_stream = nullptr;
  uint64_t *d_ent = nullptr, *d_ts = nullptr;
  size_t d_cap = 0;  // entries the device arrays hold
  uint64_t *d_keys = nullptr;
  uint32_t *d_res = nullptr, *d_nmiss = nullptr, *d_mres = nullptr;
  uint64_t *d_meps = nullptr;
  size_t d_n = 0;
  uint64_t *d_up = nullptr;  // update lists (ensure_up)
  size_t d_upcap = 0;
  // Forward-miss counters: two device words used in turn, each launch
  // zeroing the other (no memset node between calls), and the count read
  // back into pinned host memory. `miss_stale`: a call ended between its
  // launch and its read-back, so the turn's word may not be zero.
  uint32_t *h_nmiss = nullptr;
  uint32_t miss_turn = 0;
  bool miss_stale = false;
  std::mutex mu;
  ~bg_dnat() {
    for (void *p : {(void *)d_ent, (void *)d_ts, (void *)d_keys, (void *)d_res,
                    (void *)d_nmiss, (void *)d_mres, (void *)d_up, (void *)d_meps})
      if (p) (void)hipFree(p);
    if (h_nmiss) (void)hipHostFree(h_nmiss);
  }

  // HashTable::Insert; rev: a reverse entry (external endpoint -> internal)
  uint32_t insert(uint64_t key, uint64_t ep, bool rev) {
    auto it = map.find(key);
    if (it != map.end()) {
      ent_ep[it->second] = ep;
      changed.push_back(it->second);
      // the image carries the translation
      if (ent_rev[it->second] != rev) {  // the key changes direction
        mirror[ent_rev[it->second]].erase(key);
        ent_rev[it->second] = rev;
      }
      if (!mirror[rev].put(key, it->second, ep, ent_ep)) map_dirty = true;
      return it->second;
    }
    uint32_t idx;
    if (!free_idx.empty()) {
      idx = free_idx.back();
      free_idx.pop_back();
      ent_ep[idx] = ep;
      ent_ts[idx] = 0;
      exact_walk[idx] = walk;
      ent_rev[idx] = rev;
    } else {
      idx = (uint32_t)ent_ep.size();
      ent_ep.push_back(ep);
      ent_ts.push_back(0);
      exact_walk.push_back(walk);
      ent_rev.push_back(rev);
    }
    map.emplace(key, idx);
    changed.push_back(idx);
    if (idx >= (1u << 24) || !mirror[rev].put(key, idx, ep, ent_ep)) map_dirty = true;
    return idx;
  }
  void remove(uint64_t key) {
    auto it = map.find(key);
    if (it == map.end()) return;
    free_idx.push_back(it->second);
    mirror[ent_rev[it->second]].erase(key);
    map.erase(it);
  }
  // now - last_refresh > kTimeOutNs (nat.cc:217, u64 arithmetic) with the
  // entry's current timestamp: a host value that says "expired" may be
  // stale, so it is re-read from the device first
  // (a timestamp that cannot be read counts as live: a mapping is never
  // evicted on a guess)
  bool expired(uint32_t e, uint64_t now) {
    if (now - ent_ts[e] <= kTimeOutNs) return false;
    if (exact_walk[e] != walk && d_ts && e < d_cap) {
      uint64_t t = 0;
      if (hipMemcpyAsync(&t, d_ts + e, 8, hipMemcpyDeviceToHost, walk_stream) !=
              hipSuccess ||
          hipStreamSynchronize(walk_stream) != hipSuccess)
        return false;
      ent_ts[e] = std::max(ent_ts[e], t);
      exact_walk[e] = walk;
    }
    return now - ent_ts[e] > kTimeOutNs;
  }
  int64_t find(uint64_t key) const {
    auto it = map.find(key);
    return it == map.end() ? -1 : (int64_t)it->second;
  }
  uint32_t get_range(uint32_t range) {  // Random::GetRange (random.h:58-75)
    seed = seed * 1103515245 + 12345;
    union {
      uint64_t i;
      double d;
    } t;
    t.i = (seed >> 12) | 0x3ff0000000000000ull;
    return (uint32_t)((t.d - 1.0) * range);
  }

  // CreateNewEntry (nat.cc:180-258) -> forward entry index or -1
  int64_t create(uint64_t in, uint64_t now) {
    const uint32_t in_addr = (uint32_t)in;
    const uint16_t in_port = (uint16_t)(in >> 32), proto = (uint16_t)(in >> 48);
    const size_t ai = crc32c_u32(in_addr) % ext.size();  // rte_hash_crc
    const uint16_t port_host = __builtin_bswap16(in_port);
    for (const Range &r : ranges[ai]) {
      if (r.suspended) continue;
      uint16_t min, range;
      if (proto == 1) {  // ICMP
        min = r.begin;
        range = (uint16_t)(r.end - r.begin);
      } else if (port_host == 0) {
        return -1;
      } else if (port_host & ~1023u) {
        if (r.end <= 1024u) continue;
        min = std::max<uint16_t>(1024, r.begin);
        range = (uint16_t)(r.end - min + 1);
      } else {
        if (r.begin >= 1023u) continue;
        min = r.begin;
        range = (uint16_t)(std::min<uint16_t>(1023, r.end) - min);
      }
      const uint16_t start = (uint16_t)(min + get_range(range));
      uint16_t port = start;
      int trials = 0;
      do {
        const uint64_t ext_ep = ep_key(ext[ai], __builtin_bswap16(port), proto);
        const int64_t rev = find(ext_ep);
        bool take = rev < 0;
        if (!take) {
          const int64_t fwd = find(ent_ep[rev]);  // the internal endpoint
          if (fwd >= 0 && expired((uint32_t)fwd, now)) {
            remove(ent_ep[rev]);
            remove(ext_ep);
            take = true;
          }
        }
        if (take) {
          insert(ext_ep, in, true);
          return insert(in, ext_ep, false);
        }
        port++;
        trials++;
        if (port == 0 || port >= min + range) port = min;
      } while (port != start && trials < kMaxTrials);
    }
    return -1;
  }

  // the device buffer of a sync's update lists (grown, never shrunk: a
  // hipMalloc + hipFree per batch cost more than the whole walk)
  int ensure_up(size_t words) {
    if (words <= d_upcap) return 0;
    if (d_up) (void)hipFree(d_up);
    d_up = nullptr;
    d_upcap = std::max<size_t>(words * 2, 4096);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_up), d_upcap * 8));
    return 0;
  }

  int ensure_batch(size_t n) {
    if (n <= d_n) return 0;
    for (void *p : {(void *)d_keys, (void *)d_res, (void *)d_mres, (void *)d_meps})
      if (p) (void)hipFree(p);
    d_n = std::max<size_t>(n, 4096);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_keys), d_n * 8));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_res), d_n * 4));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_mres), d_n * 4));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_meps), d_n * 8));
    if (!d_nmiss) {
      HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_nmiss), 8));
      HIP_TRY(hipMemset(d_nmiss, 0, 8));
    }
    if (!h_nmiss) HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h_nmiss), 4));
    return 0;
  }

  // Device copy: the lookup image (rebuilt when the map changed) and the
  // per-entry arrays, grown by doubling with their device contents kept
  // (the device's timestamps are newer than the host's), then the entries
  // the walk changed scattered in (dnat_scatter_kernel).
  int sync(int dev_id, hipStream_t s) {
    int r = set_device(dev_id);
    if (r) return r;
    if (device != dev_id && device >= 0)
      return fail(EINVAL, "NAT map bound to device %d", device);
    if (map_dirty || !tab[0].valid || !tab[1].valid) {
      if (ent_ep.size() > (1u << 24))
        return fail(ENOSPC, "NAT map past 2^24 entries");
      for (int rev = 0; rev < 2; rev++) {  // forward, reverse
        std::vector<uint64_t> keys, hashes;
        std::vector<uint8_t> vals, img;
        for (auto &kv : map) {  // key words: the endpoint, its translation,
          // the entry index in their spare top bits (bg_dnat.hip lookup_hit)
          const uint64_t e = kv.second;
          if (ent_rev[e] != rev) continue;
          keys.push_back(kv.first | (e >> 16) << 56);
          keys.push_back((ent_ep[e] & 0xFFFFFFFFFFFFull) | (e & 0xFFFF) << 48);
          hashes.push_back(hash_words(&kv.first, 1, kDefaultSeed));
          for (int b = 0; b < 4; b++) vals.push_back((uint8_t)(e >> (8 * b)));
        }
        TableLayout L;
        r = build_image(2, 4, 1, keys, vals, hashes, &img, &L);
        if (r) return r;
        r = tab[rev].upload(dev_id, img, L, s);
        if (r) return r;
        mirror[rev].index(img, L);
      }
      map_dirty = false;
    }
    for (int rev = 0; rev < 2; rev++) {
      if (mirror[rev].dirty.empty()) continue;  // the changed words only
      std::vector<uint32_t> &w = mirror[rev].dirty;
      std::sort(w.begin(), w.end());
      w.erase(std::unique(w.begin(), w.end()), w.end());
      const size_t k = w.size();
      std::vector<uint64_t> up(2 * k);  // word index | value
      const uint64_t *src = reinterpret_cast<const uint64_t *>(mirror[rev].img.data());
      for (size_t i = 0; i < k; i++) {
        up[i] = w[i];
        up[k + i] = src[w[i]];
      }
      if (int e = ensure_up(up.size())) return e;
      HIP_TRY(hipMemcpyAsync(d_up, up.data(), up.size() * 8, hipMemcpyHostToDevice, s));
      HIP_TRY(launch_dnat_image(d_up, k, reinterpret_cast<uint64_t *>(tab[rev].d_image), s));
      HIP_TRY(hipStreamSynchronize(s));  // `up` is host memory
      w.clear();
    }
    const size_t ne = std::max<size_t>(ent_ep.size(), 1);
    if (ne > d_cap) {
      const size_t cap = std::max<size_t>(ne * 2, 1024);
      uint64_t *ne_ep = nullptr, *ne_ts = nullptr;
      HIP_TRY(hipMalloc(reinterpret_cast<void **>(&ne_ep), cap * 8));
      HIP_TRY(hipMalloc(reinterpret_cast<void **>(&ne_ts), cap * 8));
      if (d_cap) {
        HIP_TRY(hipMemcpyAsync(ne_ep, d_ent, d_cap * 8, hipMemcpyDeviceToDevice, s));
        HIP_TRY(hipMemcpyAsync(ne_ts, d_ts, d_cap * 8, hipMemcpyDeviceToDevice, s));
        HIP_TRY(hipStreamSynchronize(s));
        (void)hipFree(d_ent);
        (void)hipFree(d_ts);
      }
      d_ent = ne_ep;
      d_ts = ne_ts;
      d_cap = cap;
    }
    if (!changed.empty()) {
      std::sort(changed.begin(), changed.end());
      changed.erase(std::unique(changed.begin(), changed.end()), changed.end());
      const size_t k = changed.size();
      std::vector<uint64_t> up(3 * k);  // idx | ep | ts
      for (size_t i = 0; i < k; i++) {
        up[i] = changed[i];
        up[k + i] = ent_ep[changed[i]];
        up[2 * k + i] = ent_ts[changed[i]];
      }
      if (int e = ensure_up(up.size())) return e;
      HIP_TRY(hipMemcpyAsync(d_up, up.data(), up.size() * 8, hipMemcpyHostToDevice, s));
      HIP_TRY(launch_dnat_scatter(d_up, k, d_ent, d_ts, s));
      HIP_TRY(hipStreamSynchronize(s));  // `up` is host memory
      changed.clear();
    }
    device = dev_id;
    return 0;
  }
};

extern "C" {

int bg_dnat_create(const char *const *addrs, int naddr, const int32_t *nranges,
                   const int64_t *begin, const int64_t *end,
                   const uint8_t *suspended, uint64_t seed, bg_dnat **out) {
  if (!out || naddr < 0 || (naddr > 0 && (!addrs || !nranges)))
    return fail(EINVAL, "bad arguments");
  // Init (nat.cc:46-96): ranges checked first, then the addresses
  for (int i = 0, k = 0; i < naddr; i++)
    for (int r = 0; r < nranges[i]; r++, k++)
      if (begin[k] >= end[k] || begin[k] > 65535 || end[k] > 65535)
        return fail(EINVAL, "Port range for address %s is malformed", addrs[i]);
  bg_dnat *h = new bg_dnat();
  std::vector<uint32_t> host;
  for (int i = 0, k = 0; i < naddr; i++) {
    uint32_t a;
    if (!parse_ipv4(addrs[i], &a)) {
      delete h;
      return fail(EINVAL, "invalid IP address %s", addrs[i]);
    }
    host.push_back(a);
    std::vector<Range> rl;
    if (nranges[i] == 0) rl.push_back(Range{0, 65535, false});
    for (int r = 0; r < nranges[i]; r++, k++)
      rl.push_back(Range{(uint16_t)begin[k], (uint16_t)end[k], suspended[k] != 0});
    h->ranges.push_back(rl);
  }
  if (host.empty()) {
    delete h;
    return fail(EINVAL, "at least one external IP address must be specified");
  }
  std::sort(host.begin(), host.end());  // be32_t compares values
  for (uint32_t a : host) h->ext.push_back(__builtin_bswap32(a));
  h->seed = seed;
  *out = h;
  return 0;
}

void bg_dnat_destroy(bg_dnat *h) { delete h; }

// GetDesc (nat.cc:377-380): map entries / 2
size_t bg_dnat_count(const bg_dnat *h) { return h->map.size() / 2; }

int bg_dnat_process(bg_dnat *h, void *d_frames, size_t stride, size_t n,
                    int dir, uint64_t now, uint16_t *d_out, bg_stream_t stream) {
  if (dir != 0 && dir != 1) return fail(EINVAL, "dir %d", dir);
  if (n == 0) return 0;
  std::lock_guard<std::mutex> lk(h->mu);
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (h->device >= 0) dev = h->device;
  // the caller's stream as given (NULL: the legacy default stream): the
  // kernels read and rewrite the caller's slab and gates, so they must run
  // after the caller's earlier work on them
  hipStream_t s = (hipStream_t)stream;
  int r = h->sync(dev, s);
  if (r) return r;
  r = h->ensure_batch(n);
  if (r) return r;
  DnatArgs a;
  memset(&a, 0, sizeof(a));
  a.frames = static_cast<uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.dir = (uint32_t)dir;
  a.now = now;
  a.timeout = kTimeOutNs;
  a.t = h->tab[dir].ref();
  if (dir == 1) a.t2 = h->tab[0].ref();  // reverse misses: the forward entries
  a.next = (uint32_t)std::min<size_t>(h->ext.size(), kDnatMaxExt);
  a.list_fwd = h->ext.size() > (size_t)kDnatMaxExt ? 1u : 0u;
  for (uint32_t j = 0; j < a.next; j++) a.ext[j] = h->ext[j];
  a.keys = h->d_keys;
  a.res = h->d_res;
  a.nmiss = h->d_nmiss + h->miss_turn;
  a.nmiss_next = h->d_nmiss + (h->miss_turn ^ 1);
  a.ent = h->d_ent;
  a.ts = h->d_ts;
  a.nent = h->ent_ep.size();
  a.out = d_out;
  if (h->miss_stale) HIP_TRY(hipMemsetAsync(a.nmiss, 0, 4, s));
  h->miss_stale = true;
  const int ncu = num_cus(dev);
  // final hits stamped on the device; forward misses and forward hits on
  // expired mappings listed (reverse traffic never creates a mapping)
  HIP_TRY(launch_dnat_fused(a, ncu, s));
  if (dir == 0)
    HIP_TRY(hipMemcpyAsync(h->h_nmiss, a.nmiss, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  const uint32_t nlist = dir == 0 ? *h->h_nmiss : 0;
  h->miss_turn ^= 1;  // the launch zeroed the other word
  h->miss_stale = false;
  if (nlist == 0) return 0;
  // the listed packets in packet order on the host (DoProcessBatch 321-363)
  std::vector<uint32_t> idx(nlist), ent(nlist);
  std::vector<uint64_t> eps(nlist);
  std::vector<uint64_t> key(nlist);
  HIP_TRY(hipMemcpyAsync(idx.data(), h->d_res, nlist * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(key.data(), h->d_keys, nlist * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  std::vector<uint32_t> ord(nlist);
  for (uint32_t k = 0; k < nlist; k++) ord[k] = k;
  std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return idx[x] < idx[y]; });
  std::vector<uint32_t> sidx(nlist);
  std::vector<uint64_t> skey(nlist);
  h->walk++;  // no host timestamp is known exact yet
  h->walk_stream = s;
  for (uint32_t k = 0; k < nlist; k++) {
    sidx[k] = idx[ord[k]];
    skey[k] = key[ord[k]];
    int64_t e = h->find(skey[k]);
    if (e < 0) e = h->create(skey[k], now);
    if (e >= 0) {  // forward refresh (rfc4787 REQ-6)
      h->ent_ts[e] = now;
      h->exact_walk[e] = h->walk;
      h->changed.push_back((uint32_t)e);
    }
    ent[k] = e < 0 ? kDnatMiss : (uint32_t)e;
    eps[k] = e < 0 ? 0 : h->ent_ep[e];  // Stamp's `after` at this packet's turn
  }
  r = h->sync(dev, s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(h->d_res, sidx.data(), nlist * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->d_keys, skey.data(), nlist * 8, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->d_mres, ent.data(), nlist * 4, hipMemcpyHostToDevice, s));
  HIP_TRY(hipMemcpyAsync(h->d_meps, eps.data(), nlist * 8, hipMemcpyHostToDevice, s));
  a.t = h->tab[dir].ref();
  a.ent = h->d_ent;
  a.ts = h->d_ts;
  a.nent = h->ent_ep.size();
  a.list = 1;
  a.nlist = nlist;
  a.mres = h->d_mres;
  a.meps = h->d_meps;
  HIP_TRY(launch_dnat_apply(a, ncu, s));
  HIP_TRY(hipStreamSynchronize(s));  // the host vectors outlive the copies
  return 0;
}

}  // extern "C"
