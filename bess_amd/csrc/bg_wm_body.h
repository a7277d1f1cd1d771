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
__device__ __forceinline__ uint32_t wm_tile(const WmArgs &a, const uint32_t *tags,
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
  return bb ? (uint32_t)(uint16_t)bb : a.default_gate;
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


// Round 6: the gates of kWmGateHold tiles are held in LDS and stored
// together (C4 on the header slab 0.1502 -> 0.1435 ms, mean of 4 runs each,
// profiles/r06/wm_hold_ab_r06wm2.json; 16 tiles no better than 8).
// PAIR 1: the pair loads (lanes 2m / 2m+1 load slot m's two window chunks,
// one 32 B request per slot); 0: one slot per lane, NCH chunks.
template <class Spec, int KW, int NCH, int PAIR>
__device__ __forceinline__ void wm_tags_body(const WmArgs &a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tag_bytes = (a.t.nbp * 4 + 15) & ~15u;
  const uint64_t *mlds = wm_stage_tags<KW>(a, lds, tag_bytes);
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(lds);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t *wl = lds + tag_bytes + kMaxTuples * KW * 8 + kWmDirLds +
                wid * kWaveLds;
  uint64_t *best = reinterpret_cast<uint64_t *>(wl);
  uint32_t *q = reinterpret_cast<uint32_t *>(wl + 64 * 8);
  best[lane] = 0;
  __syncthreads();

  const uint32_t nbp = a.t.nbp;
  const uint64_t ntiles = (a.n + 63) / 64;
  const uint64_t nw = (uint64_t)gridDim.x * kWaves;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint32_t wn[PAIR ? 8 : NCH * 4 + 2];
  if constexpr (PAIR) {
    if (t < ntiles) load_pair(a.frames, a.n, t * 64, lane, a.fp.win_lo, (uint32_t)a.stride, wn);
  } else {
    if (t < ntiles && t * 64 + lane < a.n)
      load_window<NCH>(a.frames + (t * 64 + lane) * a.stride, a.fp, wn);
  }
  // the gates: held in LDS for hl tiles and stored 16 B per lane after
  // them (wm_hold_tiles: when the CU's LDS has room), else each tile's
  // stored after it (streaming)
  const uint32_t hl = wm_hold_tiles(nbp, KW);
  uint16_t *hold = reinterpret_cast<uint16_t *>(lds + wm_tags_lds_base(nbp, KW)) +
                   (size_t)wid * hl * 64;
  const uint32_t per_round = hl ? hl : 1u;
  for (uint64_t t0 = t; t0 < ntiles; t0 += nw * per_round) {
  for (uint32_t hh = 0; hh < per_round; hh++) {
    t = t0 + (uint64_t)hh * nw;
    if (t >= ntiles) break;
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
    const uint32_t g = wm_tile<Spec, KW, NCH>(a, tags, mlds, best, q, nbp, lane, idx, live, w, [&]() {
      if constexpr (PAIR) {
        if (t + nw < ntiles)
          load_pair(a.frames, a.n, (t + nw) * 64, lane, a.fp.win_lo, (uint32_t)a.stride, wn);
      } else {
        const uint64_t nidx = (t + nw) * 64 + lane;
        if (t + nw < ntiles && nidx < a.n)
          load_window<NCH>(a.frames + nidx * a.stride, a.fp, wn);
      }
    });
    if (hl)
      hold[hh * 64 + (uint32_t)(idx - t * 64)] = (uint16_t)g;
    else if (live)  // (a streaming store)
      __builtin_nontemporal_store((uint16_t)g, a.gates + idx);
  }
  if (hl) {
    lds_fence();
    store_held(hold, hl, t0, nw, lane, a.gates, a.n);
    lds_fence();  // the region's reads retire before the next round writes
  }
  }
}

}  // namespace
}  // namespace bg

#endif  // BESS_AMD_BG_WM_BODY_H_
