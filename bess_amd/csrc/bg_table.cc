// bg_table.cc -- host builder for the device flow-table image (bg_table.h).
//
// Control path only (rule-set changes; THREAD_UNSAFE in the reference,
// exact_match.cc:50-57). Bucketized cuckoo insertion with a random-walk
// eviction path, deterministic for a given (rule set, seed).
#include "bg_table.h"

#include <string.h>

#include <vector>

namespace bg {

TableLayout plan_layout(size_t max_part_entries, uint32_t kw,
                        uint32_t val_bytes, uint32_t nparts, uint64_t seed,
                        double max_load, bool vik) {
  TableLayout L;
  L.vik = vik && val_bytes == 2 ? 1u : 0u;
  L.probe = 0;
  L.rec = 0;
  L.kw = kw;
  L.val_bytes = val_bytes;
  L.nparts = nparts;
  L.seed = seed;
  uint64_t need = (uint64_t)((double)max_part_entries / (kSlots * max_load)) + 1;
  uint32_t nbp = 2;  // >= 2 so that b1 != b2 is always possible
  while (nbp < need && nbp < kMaxBucketsPerPart) nbp <<= 1;
  L.nbp = nbp;
  L.keys_off = align256((uint64_t)nbp * 4);
  L.vals_off = align256(L.keys_off + (uint64_t)nbp * kSlots * kw * 8);
  L.part_bytes = align256(L.vals_off + (L.vik ? 0 : (uint64_t)nbp * kSlots * val_bytes));
  return L;
}

namespace {
struct Xorshift {
  uint64_t s;
  uint64_t next() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
  }
};
}  // namespace

bool build_partition(const TableLayout &L, uint32_t part, size_t n,
                     const uint64_t *keys, const uint8_t *vals,
                     const uint64_t *hashes, uint8_t *dst) {
  const uint32_t nslots = L.nbp * kSlots;
  if (n > nslots) return false;
  std::vector<int32_t> occ(nslots, -1);
  std::vector<Probe> pr(n);
  for (size_t i = 0; i < n; i++) {
    pr[i] = L.probe ? wm_probe((uint32_t)hashes[i], L.nbp)
                    : split_hash(hashes[i], L.nparts, L.nbp);
    if (pr[i].part != part) return false;  // caller filtered wrongly
  }
  Xorshift rng{(L.seed ^ (0x9E3779B97F4A7C15ULL * (part + 1))) | 1};
  for (size_t i = 0; i < n; i++) {
    int32_t cur = (int32_t)i;
    uint32_t bucket = pr[i].b1;
    bool placed = false;
    // first choice: any free slot in b1 then b2
    for (int pass = 0; pass < 2 && !placed; pass++) {
      uint32_t b = pass ? pr[i].b2 : pr[i].b1;
      for (int s = 0; s < kSlots; s++)
        if (occ[b * kSlots + s] < 0) {
          occ[b * kSlots + s] = cur;
          placed = true;
          break;
        }
    }
    if (placed) continue;
    bucket = (rng.next() & 1) ? pr[i].b2 : pr[i].b1;
    for (int step = 0; step < 2000 && !placed; step++) {
      for (int s = 0; s < kSlots; s++)
        if (occ[bucket * kSlots + s] < 0) {
          occ[bucket * kSlots + s] = cur;
          placed = true;
          break;
        }
      if (placed) break;
      int s = (int)(rng.next() % kSlots);
      int32_t victim = occ[bucket * kSlots + s];
      occ[bucket * kSlots + s] = cur;
      cur = victim;
      bucket = (pr[cur].b1 == bucket) ? pr[cur].b2 : pr[cur].b1;
    }
    if (!placed) return false;
  }
  memset(dst, 0, L.part_bytes);
  uint32_t *tags = reinterpret_cast<uint32_t *>(dst);
  uint64_t *kslots = reinterpret_cast<uint64_t *>(dst + L.keys_off);
  uint8_t *vslots = dst + L.vals_off;
  for (uint32_t sl = 0; sl < nslots; sl++) {
    int32_t e = occ[sl];
    if (e < 0) continue;
    uint32_t b = sl / kSlots, s = sl % kSlots;
    tags[b] |= pr[e].tag << (8 * s);
    if (L.rec) {  // key words, then the value, in the slot's record
      memcpy(kslots + (uint64_t)sl * L.rec, keys + (uint64_t)e * L.kw, L.kw * 8);
      memcpy(kslots + (uint64_t)sl * L.rec + L.kw, vals + (uint64_t)e * L.val_bytes,
             L.val_bytes);
      continue;
    }
    memcpy(kslots + (uint64_t)sl * L.kw, keys + (uint64_t)e * L.kw, L.kw * 8);
    if (L.vik) {  // value in the key's last two bytes
      uint16_t v;
      memcpy(&v, vals + (uint64_t)e * 2, 2);
      uint64_t &last = kslots[(uint64_t)sl * L.kw + L.kw - 1];
      last = (last & 0x0000FFFFFFFFFFFFULL) | ((uint64_t)v << 48);
    } else {
      memcpy(vslots + (uint64_t)sl * L.val_bytes, vals + (uint64_t)e * L.val_bytes,
             L.val_bytes);
    }
  }
  return true;
}

}  // namespace bg
