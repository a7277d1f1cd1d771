// bg_dnat_api.cc -- C ABI of the NAT datapath (include/bessgpu.h bg_dnat_*).
//
// The NAT map (core/modules/nat.h:129-175: endpoint -> NatEntry, forward and
// reverse entries) lives on the host, where new mappings are made; the
// device keeps a lookup copy (bg_table.h image, entry index values), the
// entries' translated endpoints and their forward timestamps.
// CreateNewEntry (nat.cc:180-258) draws ports from the module's Random and
// may evict an expired mapping that a later packet of the same batch would
// have hit. The host tracks bounds on the forward timestamps, so it knows
// when no mapping can expire at `now` (and reverse traffic never creates
// one). Then a batch is
//   1. dnat_fused_kernel (dnat_fused_slab_kernel for 64-byte slots): lookup
//      and Stamp of every hit in one pass over the header line, forward
//      timestamps refreshed, forward misses listed;
//   2. only if the list is not empty: the misses walked in packet order on
//      the host (find or CreateNewEntry), the device copy rebuilt, and
//      dnat_apply_kernel stamps the listed packets.
// When a mapping may expire, the whole batch is classified first
// (dnat_find_kernel); with no forward miss dnat_apply_kernel rewrites it,
// otherwise every packet is decided on the host in packet order, with the
// device's timestamps read back first, and dnat_apply_kernel rewrites the
// batch from the host's decisions.
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

}  // namespace

struct bg_dnat {
  std::vector<uint32_t> ext;               // ext_addrs_ (raw be32), sorted
  std::vector<std::vector<Range>> ranges;  // port_ranges_ (argument order)
  uint64_t seed;                           // Random::seed_
  // the map: key -> entry index; entries: translated endpoint, timestamp
  std::unordered_map<uint64_t, uint32_t> map;
  std::vector<uint64_t> ent_ep, ent_ts;
  std::vector<uint32_t> free_idx;
  std::vector<uint8_t> ent_fwd;  // live forward entry (its ts can expire)
  // bounds on the forward entries' timestamps: lb exact after every host
  // walk (device refreshes only raise them), ub = the latest `now` seen
  uint64_t ts_lb = ~0ull, ts_ub = 0;
  bool dirty = true;
  int device = -1;
  DevTable dev;
  uint64_t *d_ent = nullptr, *d_ts = nullptr;
  size_t d_cap = 0;  // entries the device arrays hold
  uint64_t *d_keys = nullptr;
  uint32_t *d_res = nullptr, *d_nmiss = nullptr, *d_mres = nullptr;
  size_t d_n = 0;
  std::mutex mu;
  ~bg_dnat() {
    for (void *p : {(void *)d_ent, (void *)d_ts, (void *)d_keys, (void *)d_res,
                    (void *)d_nmiss, (void *)d_mres})
      if (p) (void)hipFree(p);
  }

  uint32_t insert(uint64_t key, uint64_t ep) {  // HashTable::Insert
    auto it = map.find(key);
    if (it != map.end()) {
      ent_ep[it->second] = ep;
      return it->second;
    }
    uint32_t idx;
    if (!free_idx.empty()) {
      idx = free_idx.back();
      free_idx.pop_back();
      ent_ep[idx] = ep;
      ent_ts[idx] = 0;
      ent_fwd[idx] = 0;
    } else {
      idx = (uint32_t)ent_ep.size();
      ent_ep.push_back(ep);
      ent_ts.push_back(0);
      ent_fwd.push_back(0);
    }
    map.emplace(key, idx);
    dirty = true;
    return idx;
  }
  void remove(uint64_t key) {
    auto it = map.find(key);
    if (it == map.end()) return;
    free_idx.push_back(it->second);
    ent_fwd[it->second] = 0;
    map.erase(it);
    dirty = true;
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
          if (fwd >= 0 && now - ent_ts[fwd] > kTimeOutNs) {
            remove(ent_ep[rev]);
            remove(ext_ep);
            take = true;
          }
        }
        if (take) {
          insert(ext_ep, in);
          const uint32_t e = insert(in, ext_ep);
          ent_fwd[e] = 1;
          return e;
        }
        port++;
        trials++;
        if (port == 0 || port >= min + range) port = min;
      } while (port != start && trials < kMaxTrials);
    }
    return -1;
  }

  int ensure_batch(size_t n) {
    if (n <= d_n) return 0;
    for (void *p : {(void *)d_keys, (void *)d_res, (void *)d_mres})
      if (p) (void)hipFree(p);
    d_n = std::max<size_t>(n, 4096);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_keys), d_n * 8));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_res), d_n * 4));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_mres), d_n * 4));
    if (!d_nmiss) HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_nmiss), 4));
    return 0;
  }

  // Can CreateNewEntry evict a mapping at `now`? Only a forward entry with
  // now - ts > kTimeOutNs (u64 arithmetic, nat.cc:217) can go; with every
  // forward ts in [lb, ub], none can when ub <= now and now - lb <= timeout.
  bool may_evict(uint64_t now) const {
    if (ts_lb == ~0ull) return false;  // no forward entry
    return now < ts_ub || now - ts_lb > kTimeOutNs;
  }
  void exact_bounds() {  // host timestamps are exact here
    ts_lb = ~0ull;
    for (size_t e = 0; e < ent_fwd.size(); e++)
      if (ent_fwd[e]) {
        ts_lb = std::min(ts_lb, ent_ts[e]);
        ts_ub = std::max(ts_ub, ent_ts[e]);
      }
  }

  // device copy of the map, entries and timestamps
  int sync(int dev_id, hipStream_t s) {
    if (!dirty && device == dev_id && dev.valid) return 0;
    int r = set_device(dev_id);
    if (r) return r;
    std::vector<uint64_t> keys, hashes;
    std::vector<uint8_t> vals, img;
    for (auto &kv : map) {  // key words: the endpoint, its translation
      keys.push_back(kv.first);
      keys.push_back(ent_ep[kv.second]);
      hashes.push_back(hash_words(&kv.first, 1, kDefaultSeed));
      for (int b = 0; b < 4; b++) vals.push_back((uint8_t)(kv.second >> (8 * b)));
    }
    TableLayout L;
    r = build_image(2, 4, 1, keys, vals, hashes, &img, &L);
    if (r) return r;
    r = dev.upload(dev_id, img, L, s);
    if (r) return r;
    const size_t ne = std::max<size_t>(ent_ep.size(), 1);
    if (ne > d_cap || device != dev_id) {
      if (d_ent) (void)hipFree(d_ent);
      if (d_ts) (void)hipFree(d_ts);
      d_cap = std::max<size_t>(ne * 2, 1024);
      HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_ent), d_cap * 8));
      HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_ts), d_cap * 8));
    }
    if (!ent_ep.empty()) {
      HIP_TRY(hipMemcpyAsync(d_ent, ent_ep.data(), ent_ep.size() * 8,
                             hipMemcpyHostToDevice, s));
      HIP_TRY(hipMemcpyAsync(d_ts, ent_ts.data(), ent_ts.size() * 8,
                             hipMemcpyHostToDevice, s));
    }
    HIP_TRY(hipStreamSynchronize(s));
    device = dev_id;
    dirty = false;
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
  hipStream_t s = (hipStream_t)stream;
  std::lock_guard<std::mutex> lk(h->mu);
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (h->device >= 0) dev = h->device;
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
  a.t = h->dev.ref();
  a.keys = h->d_keys;
  a.res = h->d_res;
  a.nmiss = h->d_nmiss;
  a.ent = h->d_ent;
  a.ts = h->d_ts;
  a.nent = h->ent_ep.size();
  a.out = d_out;
  HIP_TRY(hipMemsetAsync(h->d_nmiss, 0, 4, s));
  const int ncu = num_cus(dev);
  if (dir == 1 || !h->may_evict(now)) {
    // Nothing this batch creates can change another packet's mapping, so
    // hits are final: one pass stamps them and lists the forward misses.
    // Reverse traffic never creates a mapping (a miss drops).
    HIP_TRY(launch_dnat_fused(a, ncu, s));
    if (dir == 1) return 0;
    h->ts_ub = std::max(h->ts_ub, now);
    uint32_t nmiss = 0;
    HIP_TRY(hipMemcpyAsync(&nmiss, h->d_nmiss, 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    if (nmiss == 0) return 0;
    // new flows: CreateNewEntry in packet order on the host
    std::vector<uint32_t> idx(nmiss), ent(nmiss);
    std::vector<uint64_t> key(nmiss);
    HIP_TRY(hipMemcpyAsync(idx.data(), h->d_res, nmiss * 4, hipMemcpyDeviceToHost, s));
    HIP_TRY(hipMemcpyAsync(key.data(), h->d_keys, nmiss * 8, hipMemcpyDeviceToHost, s));
    if (!h->ent_ts.empty())  // forward refreshes made on the device
      HIP_TRY(hipMemcpyAsync(h->ent_ts.data(), h->d_ts, h->ent_ts.size() * 8,
                             hipMemcpyDeviceToHost, s));
    HIP_TRY(hipStreamSynchronize(s));
    std::vector<uint32_t> ord(nmiss);
    for (uint32_t k = 0; k < nmiss; k++) ord[k] = k;
    std::sort(ord.begin(), ord.end(), [&](uint32_t x, uint32_t y) { return idx[x] < idx[y]; });
    std::vector<uint32_t> sidx(nmiss);
    std::vector<uint64_t> skey(nmiss);
    for (uint32_t k = 0; k < nmiss; k++) {
      sidx[k] = idx[ord[k]];
      skey[k] = key[ord[k]];
      int64_t e = h->find(skey[k]);
      if (e < 0) e = h->create(skey[k], now);
      if (e >= 0) h->ent_ts[e] = now;
      ent[k] = e < 0 ? kDnatMiss : (uint32_t)e;
    }
    h->exact_bounds();
    h->dirty = true;
    r = h->sync(dev, s);
    if (r) return r;
    HIP_TRY(hipMemcpyAsync(h->d_res, sidx.data(), nmiss * 4, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(h->d_keys, skey.data(), nmiss * 8, hipMemcpyHostToDevice, s));
    HIP_TRY(hipMemcpyAsync(h->d_mres, ent.data(), nmiss * 4, hipMemcpyHostToDevice, s));
    a.t = h->dev.ref();
    a.ent = h->d_ent;
    a.ts = h->d_ts;
    a.nent = h->ent_ep.size();
    a.refresh = 0;
    a.list = 1;
    a.nlist = nmiss;
    a.mres = h->d_mres;
    HIP_TRY(launch_dnat_apply(a, ncu, s));
    HIP_TRY(hipStreamSynchronize(s));  // the host vectors outlive the copies
    return 0;
  }
  // An expired mapping may be evicted by a new flow, which changes what a
  // later packet of the batch maps to: classify first, and if any forward
  // packet misses, decide the whole batch in packet order on the host.
  HIP_TRY(launch_dnat_find(a, ncu, s));
  uint32_t nmiss = 0;
  HIP_TRY(hipMemcpyAsync(&nmiss, h->d_nmiss, 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  h->ts_ub = std::max(h->ts_ub, now);
  if (nmiss == 0) {  // every valid packet has a mapping
    a.refresh = dir == 0;
    HIP_TRY(launch_dnat_apply(a, ncu, s));
    return 0;
  }
  // in packet order on the host (DoProcessBatch 321-363)
  std::vector<uint64_t> keys(n);
  std::vector<uint32_t> res(n);
  HIP_TRY(hipMemcpyAsync(keys.data(), h->d_keys, n * 8, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(res.data(), h->d_res, n * 4, hipMemcpyDeviceToHost, s));
  if (!h->ent_ts.empty())  // forward refreshes made on the device
    HIP_TRY(hipMemcpyAsync(h->ent_ts.data(), h->d_ts, h->ent_ts.size() * 8,
                           hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (size_t i = 0; i < n; i++) {
    if (res[i] == kDnatInvalid) continue;  // DropPacket
    int64_t e = h->find(keys[i]);
    if (e < 0) e = h->create(keys[i], now);
    if (e < 0) {
      res[i] = kDnatMiss;  // DropPacket
      continue;
    }
    if (dir == 0) h->ent_ts[e] = now;
    res[i] = (uint32_t)e;
  }
  h->exact_bounds();
  h->dirty = true;  // timestamps (and maybe entries) changed
  r = h->sync(dev, s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(h->d_res, res.data(), n * 4, hipMemcpyHostToDevice, s));
  a.t = h->dev.ref();
  a.ent = h->d_ent;
  a.ts = h->d_ts;
  a.nent = h->ent_ep.size();
  a.refresh = 0;
  HIP_TRY(launch_dnat_apply(a, ncu, s));
  HIP_TRY(hipStreamSynchronize(s));  // res (host memory) outlives the copy
  return 0;
}

}  // extern "C"
