// bg_wm.hip -- WildcardMatch::ProcessBatch (core/modules/wildcard_match.cc:
// 159-203, LookupEntry 136-157) for tables whose tag words fit in LDS.
//
// The combined tuple table (bg_table.h: one table, a seed per tuple) keeps
// its tag words -- one u32 of four 8-bit fingerprints per bucket, <= 128 KB
// -- in LDS, so the per-(packet, tuple) probe of both candidate buckets is
// two LDS reads and a SWAR compare; nothing leaves the CU unless a
// fingerprint matches. Lane = packet, 64 packets per wave tile:
//
//   1. header window -> raw key (WildcardMatch's unmasked 8-byte loads,
//      P4), the next tile's window in flight;
//   2. per tuple (wave-uniform): key & mask, hash, both tag words from
//      LDS (all tuples' reads issued before any is used);
//   3. every fingerprint match goes into a per-wave LDS queue as (slot,
//      lane, tuple): each lane counts its matches, a bit-sliced wave prefix
//      sum (one ballot + mbcnt per count bit) gives each lane its first
//      queue position, and each lane writes its own entries -- so the key
//      checks run on dense lanes instead of on whichever lanes matched
//      (measured: the per-tuple ballot loop this replaces took a third of
//      the kernel);
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
#include <hip/hip_runtime.h>
#include <limits.h>

#include "bg_kernels.h"
#include "bg_keys_dev.h"

namespace bg {
namespace {

constexpr int kWmBlock = 1024;
constexpr int kWaves = kWmBlock / 64;
constexpr uint32_t kQueue = 256;        // entries per wave per round
constexpr int kPerLane = kQueue / 64;   // entries a lane checks per round
constexpr uint32_t kWaveLds = 64 * 8 + kQueue * 4;  // best[64] + queue

__device__ __forceinline__ uint32_t shfl32(uint32_t v, int src) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src << 2, (int)v);
}

// The owning lane's key for queue entry e (every lane takes part in the
// permutes)
template <int KW>
__device__ __forceinline__ void owner_key(uint32_t e, const uint64_t (&k)[KW],
                                          uint64_t (&kk)[KW]) {
  const int pl = (int)((e >> 20) & 63u);
#pragma unroll
  for (int j = 0; j < KW; j++) {
    const uint32_t lo = shfl32((uint32_t)k[j], pl);
    const uint32_t hi = shfl32((uint32_t)(k[j] >> 32), pl);
    kk[j] = (uint64_t)hi << 32 | lo;
  }
}

// fold a hit of entry e (slot value v) into its packet's best
__device__ __forceinline__ void wm_fold(uint64_t *best, uint32_t e, uint64_t v) {
  const uint32_t pl = (e >> 20) & 63u, tu = e >> 26;
  // (priority as unsigned order, valid bit, tuple, gate)
  const uint64_t comb = ((uint64_t)((uint32_t)v ^ 0x80000000u) << 32) |
                        (1u << 19) | (tu << 16) | ((uint32_t)(v >> 32) & 0xFFFFu);
  atomicMax(reinterpret_cast<unsigned long long *>(best + pl),
            (unsigned long long)comb);
}

template <int KW>
__device__ __forceinline__ bool wm_hit(const uint64_t *mlds, uint32_t e,
                                       uint64_t v, const uint64_t (&sk)[KW],
                                       const uint64_t (&kk)[KW]) {
  const uint32_t tu = e >> 26;
  bool hit = (uint32_t)(v >> 48) == tu;
#pragma unroll
  for (int j = 0; j < KW; j++) hit &= sk[j] == (kk[j] & mlds[tu * KW + j]);
  return hit;
}

// Check queue entries [0, m), m <= kQueue: lane l takes entries l, l + 64,
// ... (an entry is slot | lane << 20 | tuple << 26); every entry's key and
// value loads are issued before any is compared (one L2 round trip).
template <int KW>
__device__ __forceinline__ void wm_check(const WmArgs &a, const uint64_t *mlds,
                                         uint64_t *best, const uint32_t *q,
                                         uint32_t m, int lane,
                                         const uint64_t (&k)[KW]) {
  const uint64_t *vals = reinterpret_cast<const uint64_t *>(a.t.base + a.t.vals_off);
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(a.t.base + a.t.keys_off);
  uint32_t e[kPerLane];
  uint64_t v[kPerLane], sk[kPerLane][KW], kk[kPerLane][KW];
#pragma unroll
  for (int r = 0; r < kPerLane; r++) {
    const uint32_t i = (uint32_t)lane + 64u * r;
    e[r] = 0;
    v[r] = 0;
#pragma unroll
    for (int j = 0; j < KW; j++) sk[r][j] = kk[r][j] = 0;
    if (64u * r < m) {  // wave-uniform: the permutes need every lane
      e[r] = q[i];
      owner_key<KW>(e[r], k, kk[r]);
      if (i < m) {
        const uint32_t slot = e[r] & 0xFFFFFu;
        v[r] = vals[slot];
#pragma unroll
        for (int j = 0; j < KW; j++) sk[r][j] = keys[(uint64_t)slot * KW + j];
      }
    }
  }
#pragma unroll
  for (int r = 0; r < kPerLane; r++) {
    const uint32_t i = (uint32_t)lane + 64u * r;
    if (i < m && wm_hit<KW>(mlds, e[r], v[r], sk[r], kk[r])) wm_fold(best, e[r], v[r]);
  }
}

// Exclusive wave prefix sum of small per-lane counts (< 128): one ballot +
// mbcnt per bit. *total: the wave's sum.
__device__ __forceinline__ uint32_t wave_excl_scan7(uint32_t c, uint32_t *total) {
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int b = 0; b < 7; b++) {
    const uint64_t bal = __ballot((c >> b) & 1u);
    off += __builtin_amdgcn_mbcnt_hi((uint32_t)(bal >> 32),
                                     __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0))
           << b;
    tot += (uint32_t)__popcll(bal) << b;
  }
  *total = tot;
  return off;
}

template <int KW, int NCH>
__global__ __launch_bounds__(kWmBlock) void wm_tags_kernel(WmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const uint32_t tag_bytes = (a.t.nbp * 4 + 15) & ~15u;
  {  // stage the tag words
    const uint4 *src = reinterpret_cast<const uint4 *>(a.t.base);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    for (uint32_t i = threadIdx.x; i < tag_bytes / 16; i += kWmBlock) dst[i] = src[i];
  }
  uint64_t *mlds = reinterpret_cast<uint64_t *>(lds + tag_bytes);
  {
    const kconst_u64 tm = tuple_masks(a);
    if (threadIdx.x < kMaxTuples * KW)
      mlds[threadIdx.x] = tm[(threadIdx.x / KW) * kMaxKeyWords + threadIdx.x % KW];
  }
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(lds);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint8_t *wl = lds + tag_bytes + kMaxTuples * KW * 8 + wid * kWaveLds;
  uint64_t *best = reinterpret_cast<uint64_t *>(wl);
  uint32_t *q = reinterpret_cast<uint32_t *>(wl + 64 * 8);
  best[lane] = 0;
  __syncthreads();

  const uint32_t lg = 31 - __builtin_clz(a.t.nbp);
  const uint64_t ntiles = (a.n + 63) / 64;
  const uint64_t nw = (uint64_t)gridDim.x * kWaves;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint32_t wn[NCH * 4 + 2];
  if (t < ntiles && t * 64 + lane < a.n)
    load_window<NCH>(a.frames + (t * 64 + lane) * a.stride, a.fp, wn);
  for (; t < ntiles; t += nw) {
    const uint64_t idx = t * 64 + lane;
    const bool live = idx < a.n;
    uint32_t w[NCH * 4 + 2];
#pragma unroll
    for (int i = 0; i < NCH * 4 + 2; i++) w[i] = wn[i];
    const uint64_t nidx = (t + nw) * 64 + lane;
    if (t + nw < ntiles && nidx < a.n)
      load_window<NCH>(a.frames + nidx * a.stride, a.fp, wn);
    uint64_t k[KW];
    extract_key<KW, NCH>(w, a.fp, k);
#ifdef BG_AB  // phase timing (scripts/variants.py wmphase): header read only
    if (a.ab_phase == 1) {
      if (live) a.gates[idx] = (uint16_t)(k[0] ^ (k[KW - 1] >> 32));
      continue;
    }
#endif
    const kconst_u64 tm = tuple_masks(a);  // laundered per tile: no hoisting

    // A. every tuple's hash and both tag words (16 LDS reads in flight);
    // fingerprint matches as bit 7 of each matching tag byte
    uint32_t b1[kMaxTuples], b2[kMaxTuples], c1[kMaxTuples], c2[kMaxTuples];
#pragma unroll
    for (int tu = 0; tu < kMaxTuples; tu++) {
      b1[tu] = b2[tu] = c1[tu] = c2[tu] = 0;
      if (tu < (int)a.ntuples) {
        const Probe p = wm_probe(
            wm_tuple_hash<KW>(k, tm, tu, a.tcover[tu], a.tseed[tu]), lg);
        b1[tu] = p.b1;
        b2[tu] = p.b2;
        const uint32_t tb = __builtin_amdgcn_perm(0u, p.tag, 0u);  // tag in every byte
        c1[tu] = tags[p.b1] ^ tb;  // zero bytes = matches (below)
        c2[tu] = tags[p.b2] ^ tb;
      }
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int tu = 0; tu < kMaxTuples; tu++) {
      c1[tu] = zero_bytes(c1[tu]);
      c2[tu] = zero_bytes(c2[tu]);
      if (!live) c1[tu] = c2[tu] = 0;
      cnt += __popc(c1[tu]) + __popc(c2[tu]);
    }
#ifdef BG_AB  // phase timing: + hashes and tag reads
    if (a.ab_phase == 2) {
      if (live) a.gates[idx] = (uint16_t)cnt;
      continue;
    }
#endif
    // B. queue positions: a wave prefix sum of the per-lane match counts
    uint32_t total;
    const uint32_t off = wave_excl_scan7(cnt, &total);
    // C. in rounds of kQueue entries (one round unless the tile has more
    // than four candidates per packet): each lane writes its entries that
    // fall into the round, then the round is checked
    for (uint32_t r0 = 0; r0 < total; r0 += kQueue) {
      uint32_t pos = off;
#pragma unroll
      for (int tu = 0; tu < kMaxTuples; tu++) {
        uint32_t m1 = c1[tu], m2 = c2[tu];
        while (m1 | m2) {
          uint32_t slot;
          if (m1) {
            slot = b1[tu] * kSlots + (__builtin_ctz(m1) >> 3);
            m1 &= m1 - 1;
          } else {
            slot = b2[tu] * kSlots + (__builtin_ctz(m2) >> 3);
            m2 &= m2 - 1;
          }
          if (pos - r0 < kQueue)
            q[pos - r0] = slot | ((uint32_t)lane << 20) | ((uint32_t)tu << 26);
          pos++;
        }
      }
      lds_fence();
#ifdef BG_AB  // phase timing: queue built, no key checks
      if (a.ab_phase == 3) continue;
#endif
      const uint32_t m = total - r0 < kQueue ? total - r0 : kQueue;
      wm_check<KW>(a, mlds, best, q, m, lane, k);
      lds_fence();  // the queue is rewritten by the next round
    }
    lds_fence();
    const uint64_t bb = best[lane];
    best[lane] = 0;
    if (live) a.gates[idx] = bb ? (uint16_t)bb : (uint16_t)a.default_gate;
  }
}

template <int KW, int NCH>
hipError_t launch_tags(const WmArgs &a, int num_cus, hipStream_t s) {
  const size_t lds = ((a.t.nbp * 4 + 15) & ~(size_t)15) + kMaxTuples * KW * 8 +
                     (size_t)kWaves * kWaveLds;
  const uint64_t ntiles = (a.n + 63) / 64;
  uint64_t blocks = (ntiles + kWaves - 1) / kWaves;
  if (blocks > (uint64_t)num_cus) blocks = (uint64_t)num_cus;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((wm_tags_kernel<KW, NCH>), dim3((unsigned)blocks),
                     dim3(kWmBlock), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_wm_tags(const WmArgs &a, int num_cus, hipStream_t s) {
  const bool n2 = fits_nch2(a.fp);
  if (a.fp.direct || a.fp.nch > 4) return hipErrorInvalidValue;
#define BG_WT(KW)                                                          \
  if (a.t.kw == KW)                                                        \
    return n2 ? launch_tags<KW, 2>(a, num_cus, s) : launch_tags<KW, 4>(a, num_cus, s);
  BG_WT(1) BG_WT(2) BG_WT(4) BG_WT(8)
#undef BG_WT
  return hipErrorInvalidValue;
}

}  // namespace bg
