// bg_wm_body.h -- the WildcardMatch tag-word kernel body (WildcardMatch::
// ProcessBatch, core/modules/wildcard_match.cc:159-203, LookupEntry
// 136-157) for tables whose tag words fit in LDS, written over a `Spec`
// that supplies the table's tuple data:
//
//   * WmRuntimeSpec (below): read per tile from the kernel arguments --
//     the kernel bg_wm.hip compiles ahead of time for any table;
//   * a generated spec (bg_wm_jit.cc): the same data as compile-time
//     constants -- hashed-tuple set, per-tuple covered dwords, mask dwords
//     and seeds, the direct tuples' byte specs and the key's byte-permute
//     plan -- compiled at run time (hiprtc) for one rule-set shape, so the
//     per-tuple branches, scalar loads and window-index moves fold away.
//
// Spec interface (static __device__ members):
//   uint32_t hashed(a)               bit tu: tuple tu is probed by hash
//   uint32_t hash<KW>(k, tu, a)      tuple tu's wm_hash of key k (bg_table.h)
//   uint32_t ndirect(a)              direct tuples (<= kMaxDirect)
//   uint32_t dtu(a, d), dspec(a, d)  direct tuple d's tuple index, byte spec
//   void key<KW, NCH>(w, a, k)       the packet key from its header window
//
// This header is compiled by hipcc (bg_wm.hip) and by hiprtc (the text is
// embedded in libbessgpu.so, bg_wm_jit.cc), so it includes nothing beyond
// the kernel headers. Lane = packet, 64 packets per wave tile:
//
//   1. header window -> raw key (WildcardMatch's unmasked 8-byte loads,
//      P4), the next tile's window in flight;
//   2. per tuple (wave-uniform): key & mask, hash, both tag words from
//      LDS (all tuples' reads issued before any is used);
//   3. every (packet, tuple) whose buckets hold the packet's fingerprint
//      goes into a per-wave LDS queue as (first bucket, lane, tuple,
//      fingerprint) -- the second bucket follows from the first and the
//      fingerprint (wm_b2) -- at a scalar base + mbcnt of the tuple's
//      match mask, so the key checks run on dense lanes instead of on
//      whichever lanes matched;
//   4. the queue (<= 256 entries; more go in further rounds) is checked
//      with up to four entries per lane, all their loads in flight at
//      once: a lane loads each entry's slot key and value from L2 and the
//      owning lane's key comes over with ds_bpermute; a hit is folded into
//      the packet's best with a 64-bit LDS atomic max over (priority,
//      tuple, gate) -- the highest priority wins and an equal priority
//      goes to the later tuple, LookupEntry's '>=' (P5);
//   5. gate = the best's gate, or the default gate when nothing matched.
//
// One 1024-thread workgroup per CU (tags <= 128 KB + 1.5 KB per wave).
#ifndef BESS_AMD_BG_WM_BODY_H_
#define BESS_AMD_BG_WM_BODY_H_

#include "bg_kernels.h"
#include "bg_keys_dev.h"

namespace bg {
namespace {

constexpr int kWaves = kWmWaves;
constexpr uint32_t kQueue = kWmQueue;   // entries per wave per round
constexpr int kPerLane = kQueue / 64;   // entries a lane checks per round
constexpr uint32_t kWaveLds = kWmWaveLds;

// The table data from the kernel arguments, read per tile through the
// laundered kernarg pointer (hoisted, the per-tuple data of 8 tuples would
// take more scalar registers than the kernel has)
struct WmRuntimeSpec {
  __device__ static uint32_t hashed(const WmArgs &a) {
    return tuple_words(a, offsetof(WmArgs, hmask))[0];
  }
  template <int KW>
  __device__ static uint32_t hash(const uint64_t (&k)[KW], int tu, const WmArgs &a) {
    return wm_tuple_hash<KW>(k, tuple_masks(a), tu, a);
  }
  __device__ static uint32_t ndirect(const WmArgs &a) {
    return tuple_words(a, offsetof(WmArgs, ndirect))[0];
  }
  __device__ static uint32_t dtu(const WmArgs &a, int d) {
    return tuple_words(a, offsetof(WmArgs, dtu))[d];
  }
  __device__ static uint32_t dspec(const WmArgs &a, int d) {
    return tuple_words(a, offsetof(WmArgs, dspec))[d];
  }
  template <int KW, int NCH>
  __device__ static void key(const uint32_t (&w)[NCH * 4 + 2], const WmArgs &a,
                             uint64_t (&k)[KW]) {
    extract_key<KW, NCH>(w, a.fp, k);
  }
};

// one step of wm_hash (bg_table.h) over masked key dword x
__device__ __forceinline__ uint32_t wm_step(uint32_t h, uint32_t x) {
  h = (h ^ x) * 0x9E3779B1u;
  return h ^ (h >> 15);
}
__device__ __forceinline__ uint32_t wm_final(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  return h ^ (h >> 13);
}

__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// Queue entry: bucket (bits 0-14; tags <= 128 KB, so < 2^15 buckets) |
// lane << 15 | tuple << 21 | fingerprint << 24.
__device__ __forceinline__ uint32_t entry_lane(uint32_t e) { return (e >> 15) & 63u; }
__device__ __forceinline__ uint32_t entry_tuple(uint32_t e) { return (e >> 21) & 7u; }

// The owning lane's key for queue entry e (every lane takes part in the
// permutes)
template <int KW>
__device__ __forceinline__ void owner_key(uint32_t e, const uint64_t (&k)[KW],
                                          uint64_t (&kk)[KW]) {
  const int pl = (int)entry_lane(e);
#pragma unroll
  for (int j = 0; j < KW; j++) {
    const uint32_t lo = shfl32((uint32_t)k[j], pl);
    const uint32_t hi = shfl32((uint32_t)(k[j] >> 32), pl);
    kk[j] = (uint64_t)hi << 32 | lo;
  }
}

// fold a hit of entry e (slot value v) into its packet's best
__device__ __forceinline__ void wm_fold(uint64_t *best, uint32_t e, uint64_t v) {
  // (priority as unsigned order, valid bit, tuple, gate)
  const uint64_t comb = ((uint64_t)((uint32_t)v ^ 0x80000000u) << 32) |
                        (1u << 19) | (entry_tuple(e) << 16) |
                        ((uint32_t)(v >> 32) & 0xFFFFu);
  atomicMax(reinterpret_cast<unsigned long long *>(best + entry_lane(e)),
            (unsigned long long)comb);
}

template <int KW>
__device__ __forceinline__ bool wm_hit(const uint64_t *mlds, uint32_t e,
                                       uint64_t v, const uint64_t (&sk)[KW],
                                       const uint64_t (&kk)[KW]) {
  const uint32_t tu = entry_tuple(e);
  bool hit = (uint32_t)(v >> 48) == tu;
#pragma unroll
  for (int j = 0; j < KW; j++) hit &= sk[j] == (kk[j] & mlds[tu * KW + j]);
  return hit;
}

// fingerprint matches of entry e's tag in bucket b: bit 7 of each byte
__device__ __forceinline__ uint32_t bucket_matches(const uint32_t *tags, uint32_t b,
                                                   uint32_t e) {
  return zero_bytes(tags[b] ^ __builtin_amdgcn_perm(0u, e >> 24, 0u));
}

// Entry e = (packet, tuple, first bucket b1, fingerprint); its second bucket
// is wm_b2(b1, fingerprint). Candidate slots: the matches of b1 (z1), then
// those of b2 (z2); the next candidate's slot index.
__device__ __forceinline__ uint32_t next_slot(uint32_t e, uint32_t nbp, uint32_t z1,
                                              uint32_t z2) {
  const uint32_t b1 = e & 0x7FFFu;
  const uint32_t b = z1 ? b1 : wm_b2(b1, e >> 24, nbp);
  return b * kSlots + (__builtin_ctz(z1 ? z1 : z2) >> 3);
}

// Check queue entries [0, m), m <= kQueue: lane l takes entries l, l + 64,
// ... Each entry is a (packet, tuple) whose tag words hold the packet's
// fingerprint in one of its two buckets: the lane re-reads both tag words,
// and the first candidate slot's key and value loads of every entry are
// issued before any is compared (one L2 round trip). An entry whose first
// candidate is not the key (a fingerprint collision) tries the rest (rare).
// R entries per lane (m <= 64 R); the usual tile has fewer than 64
// entries and takes R = 1
template <int KW, int R>
__device__ __forceinline__ void wm_check_r(const WmArgs &a, const uint32_t *tags,
                                           const uint64_t *mlds, uint64_t *best,
                                           const uint32_t *q, uint32_t m, int lane,
                                           uint32_t nbp, const uint64_t (&k)[KW]) {
  const uint64_t *vals = reinterpret_cast<const uint64_t *>(a.t.base + a.t.vals_off);
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(a.t.base + a.t.keys_off);
  uint32_t e[R], z1[R], z2[R];
  uint64_t v[R], sk[R][KW], kk[R][KW];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t i = (uint32_t)lane + 64u * r;
    e[r] = z1[r] = z2[r] = 0;
    v[r] = 0;
#pragma unroll
    for (int j = 0; j < KW; j++) sk[r][j] = kk[r][j] = 0;
    if (64u * r < m) {  // wave-uniform: the permutes need every lane
      e[r] = q[i];
      owner_key<KW>(e[r], k, kk[r]);
      if (i < m) {
        const uint32_t b1 = e[r] & 0x7FFFu;
        z1[r] = bucket_matches(tags, b1, e[r]);
        z2[r] = bucket_matches(tags, wm_b2(b1, e[r] >> 24, nbp), e[r]);
        const uint32_t slot = next_slot(e[r], nbp, z1[r], z2[r]);
#ifdef BG_AB  // phase timing: checks without their L2 loads
        if (a.ab_phase == 3) continue;
#endif
        v[r] = vals[(uint64_t)slot * wm_rec_words(KW)];
#pragma unroll
        for (int j = 0; j < KW; j++) sk[r][j] = keys[(uint64_t)slot * wm_rec_words(KW) + j];
      }
    }
  }
  bool more = false;
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t i = (uint32_t)lane + 64u * r;
    if (i < m) {
      if (wm_hit<KW>(mlds, e[r], v[r], sk[r], kk[r])) {
        wm_fold(best, e[r], v[r]);
        z1[r] = z2[r] = 0;
      } else if (z1[r]) {  // the candidates not tried yet
        z1[r] &= z1[r] - 1;
      } else {
        z2[r] &= z2[r] - 1;
      }
    } else {
      z1[r] = z2[r] = 0;
    }
    more |= (z1[r] | z2[r]) != 0;
  }
  if (__builtin_amdgcn_ballot_w64(more)) {  // wave-uniform, rare
#pragma unroll
    for (int r = 0; r < R; r++) {
      while (z1[r] | z2[r]) {
        const uint32_t slot = next_slot(e[r], nbp, z1[r], z2[r]);
        if (z1[r])
          z1[r] &= z1[r] - 1;
        else
          z2[r] &= z2[r] - 1;
        const uint64_t vv = vals[(uint64_t)slot * wm_rec_words(KW)];
        uint64_t s2[KW];
#pragma unroll
        for (int j = 0; j < KW; j++) s2[j] = keys[(uint64_t)slot * wm_rec_words(KW) + j];
        if (wm_hit<KW>(mlds, e[r], vv, s2, kk[r])) {
          wm_fold(best, e[r], vv);
          z1[r] = z2[r] = 0;
        }
      }
    }
  }
}

template <int KW, uint32_t QUEUE = kQueue>
__device__ __forceinline__ void wm_check(const WmArgs &a, const uint32_t *tags,
                                         const uint64_t *mlds, uint64_t *best,
                                         const uint32_t *q, uint32_t m, int lane,
                                         uint32_t nbp, const uint64_t (&k)[KW]) {
  if (QUEUE <= 64 || m <= 64)  // wave-uniform (a 64-entry queue: always)
    wm_check_r<KW, 1>(a, tags, mlds, best, q, m, lane, nbp, k);
  else
    wm_check_r<KW, kPerLane>(a, tags, mlds, best, q, m, lane, nbp, k);
}

// bit 7 of each byte of x that is zero, OR-ed over two words (the SWAR
// test of zero_bytes; only the any-match result is exact)
__device__ __forceinline__ uint32_t zero_bytes2(uint32_t x, uint32_t y) {
  return (((x - 0x01010101u) & ~x) | ((y - 0x01010101u) & ~y)) & 0x80808080u;
}

// direct tuple d's value for key k: a one-byte tuple's from its LDS copy
// (after the tuple masks, wm_stage_tags), a two-byte tuple's from its
// 65536-entry table in the image
template <class Spec, int KW>
__device__ __forceinline__ uint64_t wm_direct_value(const WmArgs &a, const uint64_t *mlds,
                                                    const uint64_t (&k)[KW], int d) {
  const uint32_t spec = Spec::dspec(a, d);
  const uint32_t ix = direct_index_k<KW>(k, spec);
  if ((spec >> 24) == 0) return mlds[kMaxTuples * KW + d * 256 + ix];
  const uint64_t off = reinterpret_cast<const __attribute__((address_space(4))) uint64_t *>(
      tuple_words(a, offsetof(WmArgs, doff)))[d];
  return reinterpret_cast<const uint64_t *>(a.t.base + off)[ix];
}

// One tile's lookups (lane = packet idx, its header window w): steps 1-5 of
// the file comment. `prefetch` runs right after the direct tuples' reads are
// issued (wm_tags_body issues the next tile's window there: vector loads
// retire in order, so the direct values, consumed in this tile, must not be
// younger than a prefetch the next tile consumes).
template <class Spec, int KW, int NCH, uint32_t QUEUE = kQueue, class Prefetch>
__device__ __forceinline__ void wm_tile(const WmArgs &a, const uint32_t *tags,
                                        const uint64_t *mlds, uint64_t *best, uint32_t *q,
                                        uint32_t nbp, int lane, uint64_t idx, bool live,
                                        const uint32_t (&w)[NCH * 4 + 2], Prefetch prefetch) {
  uint64_t k[KW];
  Spec::template key<KW, NCH>(w, a, k);
  // direct tuples: one value read each, issued now, folded at the end
  const uint32_t ndir = Spec::ndirect(a);
  uint64_t dv[kMaxDirect];
#pragma unroll
  for (int d = 0; d < kMaxDirect; d++) {
    dv[d] = ~0ull;
    if ((uint32_t)d < ndir && live) dv[d] = wm_direct_value<Spec, KW>(a, mlds, k, d);
  }
  prefetch();
#ifdef BG_AB  // phase timing (scripts/variants.py wmphase): header read only
  if (a.ab_phase == 1) {
    if (live) a.gates[idx] = (uint16_t)(k[0] ^ (k[KW - 1] >> 32));
    return;
  }
#endif
  const uint32_t hmask = Spec::hashed(a);

  // A. every hashed tuple's probe: both tag words from LDS (all reads in
  // flight before any is used); ent[tu] is the packet's queue entry when
  // a bucket holds its fingerprint, else 0 (an entry is never 0: its
  // fingerprint is not)
  uint32_t ent[kMaxTuples];
#pragma unroll
  for (int tu = 0; tu < kMaxTuples; tu++) {
    ent[tu] = 0;
    if ((hmask >> tu) & 1u) {  // wave-uniform (a scalar test, or a constant)
      const Probe p = wm_probe(Spec::template hash<KW>(k, tu, a), nbp);
      const uint32_t tb = __builtin_amdgcn_perm(0u, p.tag, 0u);  // tag in every byte
      const uint32_t zz = zero_bytes2(tags[p.b1] ^ tb, tags[p.b2] ^ tb);
      ent[tu] = zz ? p.b1 | ((uint32_t)lane << 15) | ((uint32_t)tu << 21) | (p.tag << 24)
                   : 0u;
    }
  }
  // B/C. one queue entry per (packet, tuple) with a fingerprint match,
  // tuple-major: the wave's mask of matching lanes gives each lane its
  // position (a scalar base + mbcnt) and the base advances by the mask's
  // popcount. Usually the tile's entries fit one queue; more go in
  // further rounds of kQueue.
  const uint64_t livemask = __builtin_amdgcn_ballot_w64(live);
  uint64_t mk[kMaxTuples];
  uint32_t total = 0;
#pragma unroll
  for (int tu = 0; tu < kMaxTuples; tu++) {
    mk[tu] = __builtin_amdgcn_ballot_w64(ent[tu] != 0) & livemask;
    total += (uint32_t)__popcll(mk[tu]);
  }
  for (uint32_t r0 = 0; r0 < total; r0 += QUEUE) {
    uint32_t base = 0;
#pragma unroll
    for (int tu = 0; tu < kMaxTuples; tu++) {
      const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
          (uint32_t)(mk[tu] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk[tu], base));
      const bool mine = live && ent[tu] != 0;
      if (total <= QUEUE) {  // wave-uniform: one round, no window test
        if (mine) q[pos] = ent[tu];
      } else if (mine && pos - r0 < QUEUE) {
        q[pos - r0] = ent[tu];
      }
      base += (uint32_t)__popcll(mk[tu]);
    }
#ifdef BG_AB  // phase timing: + hashes, tag reads and the queue writes
    if (a.ab_phase == 2) break;
#endif
    lds_fence();
    const uint32_t m = total - r0 < QUEUE ? total - r0 : QUEUE;
    wm_check<KW, QUEUE>(a, tags, mlds, best, q, m, lane, nbp, k);
    lds_fence();  // the queue is rewritten by the next round
  }
  lds_fence();
  uint64_t bb = best[lane];
  best[lane] = 0;
#pragma unroll
  for (int d = 0; d < kMaxDirect; d++) {
    // (an unused direct slot names no tuple: its value is the all-ones
    // "empty", whose tuple field 0xFFFF must not match it)
    const uint32_t tu = (uint32_t)d < ndir ? Spec::dtu(a, d) : 0xFFFFFFFFu;
    if ((uint32_t)(dv[d] >> 48) == tu) {  // same order as wm_fold
      const uint64_t comb = ((uint64_t)((uint32_t)dv[d] ^ 0x80000000u) << 32) |
                            (1u << 19) | (tu << 16) | ((uint32_t)(dv[d] >> 32) & 0xFFFFu);
      bb = comb > bb ? comb : bb;
    }
  }
  if (live)  // (a streaming store)
    __builtin_nontemporal_store(bb ? (uint16_t)bb : (uint16_t)a.default_gate, a.gates + idx);
}

// stage the tag words and the tuple masks (every thread of the workgroup);
// returns the masks' LDS address
template <int KW>
__device__ __forceinline__ uint64_t *wm_stage_tags(const WmArgs &a, uint8_t *lds,
                                                   uint32_t tag_bytes) {
  const uint4 *src = reinterpret_cast<const uint4 *>(a.t.base);
  uint4 *dst = reinterpret_cast<uint4 *>(lds);
  for (uint32_t i = threadIdx.x; i < tag_bytes / 16; i += kWmBlock) dst[i] = src[i];
  uint64_t *mlds = reinterpret_cast<uint64_t *>(lds + tag_bytes);
  const kconst_u64 tm = tuple_masks(a);
  if (threadIdx.x < kMaxTuples * KW)
    mlds[threadIdx.x] = tm[(threadIdx.x / KW) * kMaxKeyWords + threadIdx.x % KW];
  // the one-byte direct tuples' tables (256 values each) after the masks
  // (wm_direct_value reads them there)
  static_assert(kWmDirLds == kMaxDirect * 2048, "one 2 KB table per direct slot");
  const uint32_t nd = tuple_words(a, offsetof(WmArgs, ndirect))[0];
  const uint32_t d = threadIdx.x >> 7;  // 128 threads x 16 B per table
  if (d < nd && d < (uint32_t)kMaxDirect &&
      (tuple_words(a, offsetof(WmArgs, dspec))[d] >> 24) == 0) {
    const uint64_t off = reinterpret_cast<const __attribute__((address_space(4))) uint64_t *>(
        tuple_words(a, offsetof(WmArgs, doff)))[d];
    reinterpret_cast<uint4 *>(mlds + kMaxTuples * KW)[threadIdx.x] =
        reinterpret_cast<const uint4 *>(a.t.base + off)[threadIdx.x & 127];
  }
  return mlds;
}


// PAIR 2 (the line form; dense 64 B slots, the window inside the slot): a
// wave reads its tile's 64 slots (4 KB) with lane-contiguous 16-byte loads
// -- one L2 request per 128 B line, two slots, where the pair loads make
// one per slot (a scattered lookup is bound by the requests a CU keeps in
// flight) -- keeps the two window chunks of each slot in a 2 KB
// per-wave LDS stage, and each lane reads its slot's window there. The
// next tile's loads are in flight meanwhile (16 VGPRs: the queue rounds
// are of 64 entries, whose checks take one entry per lane).
template <class Spec, int KW, int NCH, int PAIR>
__device__ __forceinline__ void wm_tags_body(const WmArgs &a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tag_bytes = (a.t.nbp * 4 + 15) & ~15u;
  const uint64_t *mlds = wm_stage_tags<KW>(a, lds, tag_bytes);
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(lds);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t *wl = lds + tag_bytes + kMaxTuples * KW * 8 + kWmDirLds +
                wid * (PAIR == 2 ? kWmWaveLdsLine : kWaveLds);
  uint64_t *best = reinterpret_cast<uint64_t *>(wl);
  uint32_t *q = reinterpret_cast<uint32_t *>(wl + 64 * 8);
  best[lane] = 0;
  __syncthreads();

  const uint32_t nbp = a.t.nbp;
  const uint64_t ntiles = (a.n + 63) / 64;
  const uint64_t nw = (uint64_t)gridDim.x * kWaves;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  if constexpr (PAIR == 2) {
    static_assert(NCH == 2, "the line form stages two window chunks per slot");
    uint4 *stage = reinterpret_cast<uint4 *>(wl + 64 * 8 + 64 * 4);  // 64 x 2 chunks
    const uint4 *src = reinterpret_cast<const uint4 *>(a.frames);
    const uint32_t q0 = a.fp.win_lo >> 4;
    uint4 v[4];
    auto load_tile = [&](uint64_t tile) {
      const uint64_t p0 = tile * 64;
      const uint64_t units = (a.n - p0 < 64 ? a.n - p0 : 64) * 4;
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t u = c * 64 + lane;
        v[c] = u < units ? ld_stream(src + p0 * 4 + u) : make_uint4(0, 0, 0, 0);
      }
    };
    if (t < ntiles) load_tile(t);
    for (; t < ntiles; t += nw) {
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t u = c * 64 + lane, d = (u & 3) - q0;
        if (d < 2u) stage[(u >> 2) * 2 + d] = v[c];
      }
      lds_fence();
      const uint4 x = stage[lane * 2], y = stage[lane * 2 + 1];
      uint32_t w[10] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, 0u, 0u};
      const uint64_t idx = t * 64 + lane;
      wm_tile<Spec, KW, 2, 64>(
          a, tags, mlds, best, q, nbp, lane, idx, idx < a.n, w, [&]() {
            if (t + nw < ntiles) load_tile(t + nw);
          });
      lds_fence();  // this tile's stage reads retire before the next writes
    }
    return;
  }
  uint32_t wn[PAIR ? 8 : NCH * 4 + 2];
  if constexpr (PAIR) {
    if (t < ntiles) load_pair(a.frames, a.n, t * 64, lane, a.fp.win_lo, (uint32_t)a.stride, wn);
  } else {
    if (t < ntiles && t * 64 + lane < a.n)
      load_window<NCH>(a.frames + (t * 64 + lane) * a.stride, a.fp, wn);
  }
  for (; t < ntiles; t += nw) {
    const uint64_t idx = t * 64 + (PAIR ? pair_slot(lane) : (uint64_t)lane);
    const bool live = idx < a.n;
    uint32_t w[NCH * 4 + 2];
    if constexpr (PAIR) {
      pair_window<NCH>(wn, lane, w);
    } else {
#pragma unroll
      for (int i = 0; i < NCH * 4 + 2; i++) w[i] = wn[i];
    }
    // the next tile's header window
    wm_tile<Spec, KW, NCH>(a, tags, mlds, best, q, nbp, lane, idx, live, w, [&]() {
      if constexpr (PAIR) {
        if (t + nw < ntiles)
          load_pair(a.frames, a.n, (t + nw) * 64, lane, a.fp.win_lo, (uint32_t)a.stride, wn);
      } else {
        const uint64_t nidx = (t + nw) * 64 + lane;
        if (t + nw < ntiles && nidx < a.n)
          load_window<NCH>(a.frames + nidx * a.stride, a.fp, wn);
      }
    });
  }
}

// The probe of one tile (step 2): ent[tu] = the packet's queue entry for
// hashed tuple tu when one of its buckets holds the packet's fingerprint,
// else 0; all tag reads in flight before any is used.
template <class Spec, int KW>
__device__ __forceinline__ void wm_probe_tuples(const WmArgs &a, const uint32_t *tags,
                                                uint32_t nbp, int lane,
                                                const uint64_t (&k)[KW],
                                                uint32_t (&ent)[kMaxTuples]) {
  const uint32_t hmask = Spec::hashed(a);
#pragma unroll
  for (int tu = 0; tu < kMaxTuples; tu++) {
    ent[tu] = 0;
    if ((hmask >> tu) & 1u) {
      const Probe p = wm_probe(Spec::template hash<KW>(k, tu, a), nbp);
      const uint32_t tb = __builtin_amdgcn_perm(0u, p.tag, 0u);
      const uint32_t zz = zero_bytes2(tags[p.b1] ^ tb, tags[p.b2] ^ tb);
      ent[tu] = zz ? p.b1 | ((uint32_t)lane << 15) | ((uint32_t)tu << 21) | (p.tag << 24)
                   : 0u;
    }
  }
}

// A tile whose checks' loads are in flight (the pipelined consumer): lane
// = packet idx; its direct tuples' values; its queue entry (lanes < m: the
// tile's m <= 64 entries, one per lane), the entry's candidate slots left,
// the first candidate's value and key, the owner's key
template <int KW>
struct WmPend {
  uint64_t idx;
  uint32_t live, m;
  uint64_t dv[kMaxDirect];
  uint32_t e, z1, z2;
  uint64_t v, sk[KW], kk[KW];
};

// the pending tile's end (steps 4-5): compare its loaded candidates, fold
// the hits, try further candidates of fingerprint collisions, store gates
template <class Spec, int KW>
__device__ __forceinline__ void wm_finish(const WmArgs &a, const uint32_t *tags,
                                          const uint64_t *mlds, uint64_t *best, int lane,
                                          uint32_t nbp, WmPend<KW> &p) {
  const uint64_t *vals = reinterpret_cast<const uint64_t *>(a.t.base + a.t.vals_off);
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(a.t.base + a.t.keys_off);
  bool more = false;
  if ((uint32_t)lane < p.m) {
    if (wm_hit<KW>(mlds, p.e, p.v, p.sk, p.kk)) {
      wm_fold(best, p.e, p.v);
      p.z1 = p.z2 = 0;
    } else if (p.z1) {
      p.z1 &= p.z1 - 1;
    } else {
      p.z2 &= p.z2 - 1;
    }
    more = (p.z1 | p.z2) != 0;
  }
  if (__builtin_amdgcn_ballot_w64(more)) {  // wave-uniform, rare
    while (p.z1 | p.z2) {
      const uint32_t slot = next_slot(p.e, nbp, p.z1, p.z2);
      if (p.z1)
        p.z1 &= p.z1 - 1;
      else
        p.z2 &= p.z2 - 1;
      const uint64_t vv = vals[(uint64_t)slot * wm_rec_words(KW)];
      uint64_t s2[KW];
#pragma unroll
      for (int j = 0; j < KW; j++) s2[j] = keys[(uint64_t)slot * wm_rec_words(KW) + j];
      if (wm_hit<KW>(mlds, p.e, vv, s2, p.kk)) {
        wm_fold(best, p.e, vv);
        p.z1 = p.z2 = 0;
      }
    }
  }
  lds_fence();
  uint64_t bb = best[lane];
  best[lane] = 0;
  const uint32_t ndir = Spec::ndirect(a);
#pragma unroll
  for (int d = 0; d < kMaxDirect; d++) {
    const uint32_t tu = (uint32_t)d < ndir ? Spec::dtu(a, d) : 0xFFFFFFFFu;
    if ((uint32_t)(p.dv[d] >> 48) == tu) {
      const uint64_t comb = ((uint64_t)((uint32_t)p.dv[d] ^ 0x80000000u) << 32) |
                            (1u << 19) | (tu << 16) | ((uint32_t)(p.dv[d] >> 32) & 0xFFFFu);
      bb = comb > bb ? comb : bb;
    }
  }
  if (p.live)
    __builtin_nontemporal_store(bb ? (uint16_t)bb : (uint16_t)a.default_gate, a.gates + p.idx);
}

// ---------------------------------------------------------------------------
// Streamed form (pair-shaped windows: two 16-byte chunks inside the slot's
// first 64 bytes). The header stream is decoupled from the lookups: in the
// form above every wave prefetches one tile, and its key / value loads from
// L2 retire behind that prefetch (vector loads retire in order), so a wave
// has one tile of windows in flight for part of its time. Here
// kStreamProducers waves per workgroup only load windows -- straight into
// an LDS ring of `a.ring_slots` tiles (global_load_lds), kStreamDepth tiles
// in flight each, waited for with an explicit vmcnt -- and the other waves
// (consumers) take tiles from the ring in order and do the lookups, their
// own loads being only the L2 checks.
//
// Ring protocol: the workgroup's tiles j = 0, 1, ... (global tile blockIdx.x
// + j * gridDim.x) go through ring slot j % R. ready[s] = j + 1 once tile j's
// windows are in slot s; done[s] = j + 1 once its consumer has read them.
// Producer p loads tiles p, p + P, ...; it loads tile j only when the slot's
// previous tile j - R is done, and publishes a tile once kStreamDepth - 1
// younger ones are issued (or at its end). Consumer c takes tiles c, c + C,
// ... Every wait is for a smaller tile index, and R > P * kStreamDepth: the
// smallest unfinished tile can always advance (its producer's pending waits
// are for tiles below it, all done), so the workgroup drains and every wave
// leaves after its last tile.
// ---------------------------------------------------------------------------
// ring flags: a volatile LDS word (an LDS-typed pointer: a generic volatile
// access would be a flat instruction, which counts in vmcnt and would make
// the producer wait for its loads); the data written before a publish has
// landed first (lgkmcnt), and a wave's LDS operations execute in order
typedef volatile __attribute__((address_space(3))) uint32_t lds_flag_t;
__device__ __forceinline__ void lds_wait_eq(const uint32_t *p, uint32_t v) {
  lds_flag_t *f = (lds_flag_t *)(p);
  while (*f != v) __builtin_amdgcn_s_sleep(1);
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void lds_publish(uint32_t *p, uint32_t v) {
  lds_fence();
  *(lds_flag_t *)(p) = v;
}

// the pair-shaped windows of tile p0 (slots p0 .. p0 + 63; indices past
// the slab clamped to n - 1) straight into LDS at `dst` (global_load_lds:
// lane l's 16 bytes land at dst + 16 l, so slot m's window is at dst + 32 m):
// no registers, and the producer alone decides when to wait for them
__device__ __forceinline__ void dma_pair(const uint8_t *__restrict__ frames, uint64_t n,
                                         uint64_t p0, int lane, uint32_t win_lo,
                                         uint64_t stride, uint8_t *dst) {
  uint64_t s0 = p0 + (uint32_t)(lane >> 1), s1 = s0 + 32;
  s0 = s0 < n ? s0 : n - 1;
  s1 = s1 < n ? s1 : n - 1;
  const uint32_t c = (uint32_t)(lane & 1) * 16 + win_lo;
  typedef const __attribute__((address_space(1))) void *gptr;
  typedef __attribute__((address_space(3))) void *lptr;
  __builtin_amdgcn_global_load_lds((gptr)(frames + s0 * stride + c), (lptr)dst, 16, 0, 0);
  __builtin_amdgcn_global_load_lds((gptr)(frames + s1 * stride + c), (lptr)(dst + 1024), 16,
                                   0, 0);
}

template <class Spec, int KW, int D>
__device__ __forceinline__ void wm_stream_impl(const WmArgs &a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  constexpr int P = kStreamProducers, C = kWaves - kStreamProducers;
  constexpr uint32_t kWaveLds = kStreamWaveLds, kQueue = 64;
  const uint32_t tag_bytes = (a.t.nbp * 4 + 15) & ~15u;
  const uint64_t *mlds = wm_stage_tags<KW>(a, lds, tag_bytes);
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(lds);
  // (the wave index in a scalar register: the role and tile branches below
  // are uniform)
  const int lane = threadIdx.x & 63,
            wid = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  uint8_t *waves = lds + tag_bytes + kMaxTuples * KW * 8 + kWmDirLds;
  const uint32_t R = a.ring_slots;
  uint8_t *ring = waves + C * kWaveLds;
  uint32_t *ready = reinterpret_cast<uint32_t *>(ring + (uint64_t)R * kStreamTileBytes);
  uint32_t *done = ready + R;
  for (uint32_t i = threadIdx.x; i < 2 * R; i += kWmBlock) ready[i] = 0;
  if (wid >= P) reinterpret_cast<uint64_t *>(waves + (wid - P) * kWaveLds)[lane] = 0;
  __syncthreads();

  const uint64_t ntiles = (a.n + 63) / 64, G = gridDim.x;
  // the workgroup's tiles (< 2^32: n < 2^38 packets)
  const uint64_t K = ntiles > blockIdx.x ? (ntiles - blockIdx.x + G - 1) / G : 0;
  const uint32_t win_lo = a.fp.win_lo;
  if (wid < P) {  // producer: windows of tiles wid, wid + P, ... into the ring
    const uint32_t I = K > (uint64_t)wid ? (uint32_t)((K - wid + P - 1) / P) : 0u;
    // tile i of this producer: j = wid + P i, slot j % R (kept incrementally)
    uint32_t slot = (uint32_t)wid % R, pslot = slot;  // issue / publish cursors
    uint32_t pj = (uint32_t)wid;
    auto publish = [&]() {  // the oldest issued tile: its windows have landed
      if (lane == 0) *(lds_flag_t *)&ready[pslot] = pj + 1;
      pj += P;
      pslot += P;
      if (pslot >= R) pslot -= R;
    };
    for (uint32_t i = 0; i < I; i++) {
      const uint32_t j = (uint32_t)wid + P * i;
      if (j >= R) lds_wait_eq(&done[slot], j - R + 1);  // the slot's last tile read
      dma_pair(a.frames, a.n, (blockIdx.x + (uint64_t)j * G) * 64, lane, win_lo, a.stride,
               ring + (uint64_t)slot * kStreamTileBytes);
      slot += P;
      if (slot >= R) slot -= R;
      if (i + 1 >= (uint32_t)D) {  // D tiles in flight: the oldest has landed
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * (D - 1)) : "memory");
        publish();
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    while (pj < (uint32_t)wid + P * I) publish();
    return;
  }
  // consumer, software-pipelined one tile deep: the L2 loads of tile j's
  // checks are in flight while tile j + C is taken from the ring, keyed,
  // hashed and probed; then tile j ends and tile j + C's loads are issued.
  // A wave's only vector loads are its own checks' and direct tuples', so
  // ending tile j waits for exactly those (vmcnt in order), never for the
  // header stream.
  const int c = wid - P;
  uint8_t *wl = waves + c * kWaveLds;
  uint64_t *best = reinterpret_cast<uint64_t *>(wl);
  uint32_t *q = reinterpret_cast<uint32_t *>(wl + 64 * 8);
  const uint32_t nbp = a.t.nbp;
  const uint64_t *vals = reinterpret_cast<const uint64_t *>(a.t.base + a.t.vals_off);
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(a.t.base + a.t.keys_off);
  WmPend<KW> pd;
  bool pending = false;
  uint32_t s = (uint32_t)c % R;
  for (uint32_t j = (uint32_t)c; j < K; j += C) {
    // A1: the tile's windows, key, probes and queue
    lds_wait_eq(&ready[s], j + 1);
    const uint4 *src = reinterpret_cast<const uint4 *>(ring + (uint64_t)s * kStreamTileBytes) +
                       2 * lane;
    const uint4 x = src[0], y = src[1];
    uint32_t w[10] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w, 0u, 0u};
    if (lane == 0) lds_publish(&done[s], j + 1);  // (the reads have returned)
    s += C;
    while (s >= R) s -= R;
    const uint64_t idx = (blockIdx.x + (uint64_t)j * G) * 64 + lane;
    const bool live = idx < a.n;
    uint64_t k[KW];
    Spec::template key<KW, 2>(w, a, k);
    uint32_t total;
    {
      uint32_t ent[kMaxTuples];
      wm_probe_tuples<Spec, KW>(a, tags, nbp, lane, k, ent);
      const uint64_t livemask = __builtin_amdgcn_ballot_w64(live);
      uint64_t mk[kMaxTuples];
      total = 0;
#pragma unroll
      for (int tu = 0; tu < kMaxTuples; tu++) {
        mk[tu] = __builtin_amdgcn_ballot_w64(ent[tu] != 0) & livemask;
        total += (uint32_t)__popcll(mk[tu]);
      }
      if (total <= 64) {  // (uniform) the usual tile: one entry per lane at most
        uint32_t base = 0;
#pragma unroll
        for (int tu = 0; tu < kMaxTuples; tu++) {
          const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(mk[tu] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk[tu], base));
          if (live && ent[tu] != 0) q[pos] = ent[tu];
          base += (uint32_t)__popcll(mk[tu]);
        }
      }
    }
    // B: the previous tile ends (its loads have had this tile's front)
    if (pending) wm_finish<Spec, KW>(a, tags, mlds, best, lane, nbp, pd);
    // A2: this tile's loads: direct tuples, then the checks' first candidates
    pd.idx = idx;
    pd.live = live ? 1u : 0u;
    const uint32_t ndir = Spec::ndirect(a);
#pragma unroll
    for (int d = 0; d < kMaxDirect; d++) {
      pd.dv[d] = ~0ull;
      if ((uint32_t)d < ndir && live) pd.dv[d] = wm_direct_value<Spec, KW>(a, mlds, k, d);
    }
    pd.e = pd.z1 = pd.z2 = 0;
    pd.v = 0;
#pragma unroll
    for (int q2 = 0; q2 < KW; q2++) pd.sk[q2] = pd.kk[q2] = 0;
    if (total <= 64) {
      pd.m = total;
      if (total) {  // (uniform)
        lds_fence();  // the queue written above
        if ((uint32_t)lane < total) pd.e = q[lane];
        owner_key<KW>(pd.e, k, pd.kk);
        if ((uint32_t)lane < total) {
          const uint32_t b1 = pd.e & 0x7FFFu;
          pd.z1 = bucket_matches(tags, b1, pd.e);
          pd.z2 = bucket_matches(tags, wm_b2(b1, pd.e >> 24, nbp), pd.e);
          const uint32_t slot = next_slot(pd.e, nbp, pd.z1, pd.z2);
          pd.v = vals[(uint64_t)slot * wm_rec_words(KW)];
#pragma unroll
          for (int q2 = 0; q2 < KW; q2++) pd.sk[q2] = keys[(uint64_t)slot * wm_rec_words(KW) + q2];
        }
      }
    } else {
      // a tile of more than 64 entries (rare): its checks here, in rounds
      // of kQueue as wm_tile makes them (the previous tile has ended, so
      // `best` is this tile's); its end then only folds and stores
      pd.m = 0;
      uint32_t ent[kMaxTuples];
      wm_probe_tuples<Spec, KW>(a, tags, nbp, lane, k, ent);
      const uint64_t livemask = __builtin_amdgcn_ballot_w64(live);
      uint64_t mk[kMaxTuples];
#pragma unroll
      for (int tu = 0; tu < kMaxTuples; tu++)
        mk[tu] = __builtin_amdgcn_ballot_w64(ent[tu] != 0) & livemask;
      for (uint32_t r0 = 0; r0 < total; r0 += kQueue) {
        uint32_t base = 0;
#pragma unroll
        for (int tu = 0; tu < kMaxTuples; tu++) {
          const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
              (uint32_t)(mk[tu] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mk[tu], base));
          if (live && ent[tu] != 0 && pos - r0 < kQueue) q[pos - r0] = ent[tu];
          base += (uint32_t)__popcll(mk[tu]);
        }
        lds_fence();
        const uint32_t m = total - r0 < kQueue ? total - r0 : kQueue;
        wm_check<KW>(a, tags, mlds, best, q, m, lane, nbp, k);
        lds_fence();
      }
    }
    pending = true;
  }
  if (pending) wm_finish<Spec, KW>(a, tags, mlds, best, lane, nbp, pd);
}

// the producers' depth: kStreamDepthDeep tiles each when the ring has the
// slots for it (wm_stream_slots), else kStreamDepth (a uniform branch)
template <class Spec, int KW>
__device__ __forceinline__ void wm_tags_stream_body(const WmArgs &a) {
  if (a.ring_slots > (uint32_t)(kStreamProducers * kStreamDepthDeep + 4))
    wm_stream_impl<Spec, KW, kStreamDepthDeep>(a);
  else
    wm_stream_impl<Spec, KW, kStreamDepth>(a);
}

}  // namespace
}  // namespace bg

#endif  // BESS_AMD_BG_WM_BODY_H_
