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
// or, for WildcardMatch (`rec` words per record), one record per slot:
//   [tags: nbp x u32][records: nbp x 4 x (kw key words, the u64 value, pad)]
// so that a check's key and value lie in one 64 B line (one L2 request).
#ifndef BESS_AMD_BG_TABLE_H_
#define BESS_AMD_BG_TABLE_H_

#ifndef __HIPCC_RTC__
#include <stddef.h>
#include <stdint.h>
#else  // hiprtc (bg_wm_jit.cc): its runtime header declares these in a namespace
using __hip_internal::int32_t;
using __hip_internal::int64_t;
using __hip_internal::uint16_t;
using __hip_internal::uint32_t;
using __hip_internal::uint64_t;
using __hip_internal::uint8_t;
#ifndef offsetof
#define offsetof(t, m) __builtin_offsetof(t, m)
#endif
#endif

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
  uint32_t nbp;        // buckets per partition, power of 2 (probe 0)
  uint64_t part_bytes; // bytes per partition image
  uint64_t keys_off;   // byte offset of keys within a partition
  uint64_t vals_off;   // byte offset of values within a partition
  uint64_t seed;       // hash seed
  // 1: the u16 value sits in the top two bytes of the key's last word (the
  // key has >= 2 bytes past its raw size, which are 0 in every packet key,
  // P4), so one key read also yields the value; no value array
  uint32_t vik;
  // 0: split_hash of a 64-bit hash_words value (ExactMatch, NAT);
  // 1: wm_probe of a 32-bit wm_hash value (WildcardMatch, one partition;
  // nbp any number >= 2)
  uint32_t probe;
  // 0: separate key and value arrays; else the words per slot record (key
  // words, then the 8-byte value at word kw; wm_rec_words), vals_off =
  // keys_off + 8 kw
  uint32_t rec;
};

// WildcardMatch slot records: the key words and the value, padded to a
// power of two (kw 2: 32 B, so a record never straddles a 64 B line)
BG_HD uint32_t wm_rec_words(uint32_t kw) {
  uint32_t r = 1;
  while (r < kw + 1) r <<= 1;
  return r;
}

BG_HD uint64_t align256(uint64_t x) { return (x + 255) & ~uint64_t(255); }

// Key hash, all 32-bit arithmetic (gfx950 has no 64-bit multiply: a
// 64 x 64 product is four 32-bit multiplies plus adds, and a multiply is a
// quarter-rate VALU op). h1 walks the key's u32 halves with one
// multiply-xorshift step each -- a bijection of the state for a fixed
// input word and of the input word for a fixed state, so two keys collide
// only by a 2^-32 chance -- then the murmur3 finalizer. h1 alone gives the
// first bucket, the fingerprint and the WildcardMatch filter probe; h2
// (second bucket, partition) is one more finalizer over h1, so a lookup
// that the filter rejects never computes it.
BG_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

BG_HD uint32_t hash_words_h1(const uint64_t *k, int n, uint64_t seed) {
  uint32_t h = (uint32_t)seed ^ (uint32_t)(seed >> 32) ^ ((uint32_t)n * 0x9E3779B9u);
  for (int i = 0; i < n; i++) {
    h = (h ^ (uint32_t)k[i]) * 0x9E3779B1u;
    h ^= h >> 15;
    h = (h ^ (uint32_t)(k[i] >> 32)) * 0x85EBCA77u;
    h ^= h >> 13;
  }
  return fmix32(h);
}

BG_HD uint32_t hash_h2(uint32_t h1) { return fmix32(h1 ^ 0x5BD1E995u); }

// the full hash: h2 << 32 | h1
BG_HD uint64_t hash_join(uint32_t h1) { return (uint64_t)hash_h2(h1) << 32 | h1; }

BG_HD uint64_t hash_words(const uint64_t *k, int n, uint64_t seed) {
  return hash_join(hash_words_h1(k, n, seed));
}

// per-tuple seed for the combined WildcardMatch table
BG_HD uint64_t tuple_seed(uint64_t seed, uint32_t tuple) {
  return seed ^ ((uint64_t)(tuple + 1) * 0xD6E8FEB86659FD93ULL);
}

struct Probe {
  uint32_t part, b1, b2, tag;
};

// WildcardMatch tuple hash: one multiply-xorshift step per key dword the
// tuple's mask covers (`cover` bit d: mask dword d is not zero -- a masked
// key is 0 everywhere else, so those dwords carry nothing), then a
// one-multiply finalizer. A packet is probed in all (<= 8) tuples, so the
// multiplies (quarter-rate on gfx950) are what bounds the kernel: this
// spends 1 per covered dword + 1, where hash_words + hash_join spend 1 per
// dword + 4.
BG_HD uint32_t wm_seed32(uint64_t tuple_seed) {
  return (uint32_t)tuple_seed ^ (uint32_t)(tuple_seed >> 32);
}
BG_HD uint32_t wm_hash(const uint32_t *kd, uint32_t cover, int ndw, uint32_t seed) {
  uint32_t h = seed;
  for (int d = 0; d < ndw; d++) {
    if (!((cover >> d) & 1u)) continue;
    h = (h ^ kd[d]) * 0x9E3779B1u;
    h ^= h >> 15;
  }
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h;
}

// WildcardMatch tables take any bucket count nbp >= 2 (not only powers of
// two: a table whose tag words live in LDS is sized to its entries, C4's
// 75 K hashed entries take 79 KB of tag words at load 0.95 where the next
// power of two took 128 KB). x in [0, 2^32) scaled to [0, n): the high half
// of a 32 x 32 product (one v_mul_hi_u32).
BG_HD uint32_t wm_range(uint32_t x, uint32_t n) { return (uint32_t)(((uint64_t)x * n) >> 32); }

// The second bucket from the first and the fingerprint alone (partial-key
// cuckoo hashing), so a (first bucket, fingerprint) pair names both buckets
// -- the tag-word kernel queues one entry per (packet, tuple) and its check
// derives the other bucket: b1 plus an offset in [1, nbp) drawn from the
// fingerprint, modulo nbp (never b1).
BG_HD uint32_t wm_b2(uint32_t b1, uint32_t tag, uint32_t nbp) {
  const uint32_t b = b1 + 1u + wm_range(tag * 0x5BD1E995u, nbp - 1u);
  return b >= nbp ? b - nbp : b;
}
// fingerprint from the top byte, first bucket from the low 24 bits scaled
// to [0, nbp), second bucket wm_b2 (nbp >= 2)
BG_HD Probe wm_probe(uint32_t h, uint32_t nbp) {
  Probe p;
  p.part = 0;
  p.b1 = wm_range(h << 8, nbp);
  const uint32_t t = h >> 24;
  p.tag = t ? t : 1u;
  p.b2 = wm_b2(p.b1, p.tag, nbp);
  return p;
}

BG_HD uint32_t log2_pow2(uint32_t x) {
  uint32_t l = 0;
  while ((1u << l) < x) l++;
  return l;
}

// h1: first bucket (low bits) and fingerprint (top byte); h2: second
// bucket (low bits) and partition (top 3 bits). Buckets per partition are
// <= 2^24, so no two fields share a bit.
BG_HD Probe split_hash(uint64_t h, uint32_t nparts, uint32_t nbp) {
  Probe p;
  const uint32_t m = nbp - 1, h1 = (uint32_t)h, h2 = (uint32_t)(h >> 32);
  p.part = (h2 >> 29) & (nparts - 1);
  p.b1 = h1 & m;
  p.b2 = h2 & m;
  if (p.b2 == p.b1) p.b2 = (p.b1 ^ 1u) & m;
  const uint32_t t = h1 >> 24;
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

// from h1 only (the low 32 bits of the hash)
BG_HD FilterProbe filter_probe(uint64_t h, uint32_t nwords) {
  FilterProbe f;
  const uint32_t h1 = (uint32_t)h;
  f.word = (h1 >> 4) & (nwords - 1);
  f.bits = (1u << ((h1 >> 20) & 31)) | (1u << ((h1 >> 25) & 31));
  return f;
}

TableLayout plan_layout(size_t max_part_entries, uint32_t kw,
                        uint32_t val_bytes, uint32_t nparts, uint64_t seed,
                        double max_load = 0.75, bool vik = false);

// Lay out the partition image of `part` at `dst` (layout.part_bytes bytes)
// from the given entries (keys[i*kw .. ], vals[i*val_bytes ..]) that hash
// into this partition (callers filter). `hashes[i]` is entry i's full hash
// (hash_words with its seed -- tuple seeds for WildcardMatch). Returns
// false if cuckoo
// insertion failed (caller retries with a bigger nbp).
bool build_partition(const TableLayout &L, uint32_t part, size_t n,
                     const uint64_t *keys, const uint8_t *vals,
                     const uint64_t *hashes, uint8_t *dst);

}  // namespace bg

#endif  // BESS_AMD_BG_TABLE_H_
