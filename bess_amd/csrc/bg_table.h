// bg_table.h -- device flow-table layout shared by the host builder
// (bg_table.cc) and the HIP classify kernels (bg_kernels.hip).
//
// Replaces the reference's CuckooMap<ExactMatchKey, V> (core/utils/
// cuckoo_map.h) for LOOKUPS on the GPU. Lookup results do not depend on the
// hash or the layout (exact semantics: a key is either present with one
// value or absent), so the layout is chosen for gfx950:
//
//   * bucketized cuckoo hashing, 2 candidate buckets x 4 slots;
//   * one 32-bit "tag word" per bucket holding four 8-bit key fingerprints
//     (0 = empty slot), so a miss costs two 4-byte reads and a hit one
//     16-byte key read (5-tuple) plus the value;
//   * the table is split into `nparts` independent partitions (partition =
//     hash bits 48..50). Both candidate buckets of a key lie in its own
//     partition, so partitions are built independently (one per rank) and
//     concatenated by an all-gather of raw bytes (RCCL over xGMI).
//
// Partition image (all offsets 256-byte aligned, `part_bytes` per part):
//   [tags: nbp x u32][keys: nbp x 4 x kw x u64][vals: nbp x 4 x val_bytes]
#ifndef BESS_AMD_BG_TABLE_H_
#define BESS_AMD_BG_TABLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __HIPCC__
#define BG_HD __host__ __device__ __forceinline__
#else
#define BG_HD inline
#endif

namespace bg {

constexpr int kSlots = 4;       // slots per bucket
constexpr int kMaxKeyWords = 8; // ExactMatchKey: MAX_FIELDS * MAX_FIELD_SIZE / 8
constexpr uint32_t kMaxBucketsPerPart = 1u << 24;

struct TableLayout {
  uint32_t kw;         // key words (total_key_size / 8), 1..8
  uint32_t val_bytes;  // 2 (EM gate) or 8 (WM {prio, gate, tuple})
  uint32_t nparts;     // power of 2, <= 8
  uint32_t nbp;        // buckets per partition, power of 2
  uint64_t part_bytes; // bytes per partition image
  uint64_t keys_off;   // byte offset of keys within a partition
  uint64_t vals_off;   // byte offset of values within a partition
  uint64_t seed;       // hash seed
};

BG_HD uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// Full 64-bit hash of a key: one multiply-xorshift round per word plus a
// splitmix64 finalizer (cheap on gfx950: 32-bit MULs, no CRC instruction).
BG_HD uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ULL;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebULL;
  x ^= x >> 31;
  return x;
}

BG_HD uint64_t hash_words(const uint64_t *k, int n, uint64_t seed) {
  uint64_t h = seed ^ (0x9E3779B97F4A7C15ULL * (uint64_t)(n + 1));
  for (int i = 0; i < n; i++) {
    h = (h ^ k[i]) * 0x9E3779B97F4A7C15ULL;
    h ^= h >> 29;
  }
  return mix64(h);
}

// per-tuple seed for the combined WildcardMatch table
BG_HD uint64_t tuple_seed(uint64_t seed, uint32_t tuple) {
  return seed ^ ((uint64_t)(tuple + 1) * 0xD6E8FEB86659FD93ULL);
}

struct Probe {
  uint32_t part, b1, b2, tag;
};

BG_HD Probe split_hash(uint64_t h, uint32_t nparts, uint32_t nbp) {
  Probe p;
  uint32_t m = nbp - 1;
  p.part = (uint32_t)(h >> 48) & (nparts - 1);
  p.b1 = (uint32_t)h & m;
  p.b2 = (uint32_t)(h >> 24) & m;
  if (p.b2 == p.b1) p.b2 = (p.b1 ^ 1u) & m;
  uint32_t t = (uint32_t)(h >> 56);
  p.tag = t ? t : 1u;
  return p;
}

// Blocked Bloom filter over a table's keys (one 32-bit word per probe, two
// bits set in it). Kept in LDS in front of an L2-resident WildcardMatch
// table so that most (packet, tuple) pairs that cannot match skip both
// scattered tag reads. `nwords` is a power of two <= 2^16.
struct FilterProbe {
  uint32_t word, bits;
};

BG_HD FilterProbe filter_probe(uint64_t h, uint32_t nwords) {
  FilterProbe f;
  f.word = (uint32_t)(h >> 40) & (nwords - 1);
  f.bits = (1u << ((uint32_t)(h >> 8) & 31)) | (1u << ((uint32_t)(h >> 14) & 31));
  return f;
}

TableLayout plan_layout(size_t max_part_entries, uint32_t kw,
                        uint32_t val_bytes, uint32_t nparts, uint64_t seed,
                        double max_load = 0.75);

// Lay out the partition image of `part` at `dst` (layout.part_bytes bytes)
// from the given entries (keys[i*kw .. ], vals[i*val_bytes ..]) that hash
// into this partition (callers filter). `seeds[i]` is the hash seed of entry
// i (tuple seeds for WildcardMatch). Returns false if cuckoo insertion failed
// (caller retries with a bigger nbp).
bool build_partition(const TableLayout &L, uint32_t part, size_t n,
                     const uint64_t *keys, const uint8_t *vals,
                     const uint64_t *seeds, uint8_t *dst);

}  // namespace bg

#endif  // BESS_AMD_BG_TABLE_H_
