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
//      LDS (all tuples' reads issued before any is used); every
//      fingerprint match is appended to the tile's per-wave LDS queue as
//      (slot, lane, tuple) with a ballot + mbcnt prefix, so the key checks
//      run on dense lanes instead of on whichever lanes happen to match;
//   3. the tile's queued entries are checked two per lane: a lane loads
//      each entry's slot key and value from L2 and the owning lane's key
//      comes over with ds_bpermute. Those loads are software-pipelined: they
//      are issued at the end of tile t and consumed after steps 1-2 of tile
//      t + 1, so the L2 round trip overlaps the next tile's hashing. A hit
//      is folded into the packet's best with a 64-bit LDS atomic max over
//      (priority, tuple, gate) -- the highest priority wins and an equal
//      priority goes to the later tuple, LookupEntry's '>=' (P5). (A tile
//      with more than 128 candidates checks 64 of them at once.)
//   4. gate = the best's gate, or the default gate when nothing matched.
//
// One 960-thread workgroup per CU: tags <= 128 KB + per wave two queues of
// 128 entries and two best arrays (tiles t and t + 1), 2 KB.
#include <hip/hip_runtime.h>
#include <limits.h>

#include "bg_kernels.h"
#include "bg_keys_dev.h"

namespace bg {
namespace {

constexpr int kWmBlock = 960;           // 15 waves: LDS for the tags + 2 KB each
constexpr int kWaves = kWmBlock / 64;
constexpr uint32_t kQueue = 128;        // entries per wave per tile (ring)
constexpr uint32_t kWaveLds = 2 * (64 * 8 + kQueue * 4);  // 2 x (best + queue)

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

// Up to 128 queued entries of one tile in flight: lane l holds entries l
// and l + 64 (an entry is slot | lane << 20 | tuple << 26), the owning
// lanes' keys and the slots' keys and values being loaded.
template <int KW>
struct Pending {
  uint32_t e0, e1, m;  // m: entries (wave-uniform), 0 = none
  uint64_t v0, v1, sk0[KW], sk1[KW], kk0[KW], kk1[KW];
};

// Issue the loads of queue entries [head, head + m), m <= 128.
template <int KW>
__device__ __forceinline__ void wm_issue(const WmArgs &a, const uint32_t *q,
                                         uint32_t head, uint32_t m, int lane,
                                         const uint64_t (&k)[KW], Pending<KW> &p) {
  p.m = m;
  p.e0 = q[(head + lane) & (kQueue - 1)];
  p.e1 = q[(head + 64 + lane) & (kQueue - 1)];
  owner_key<KW>(p.e0, k, p.kk0);
  if (m > 64) owner_key<KW>(p.e1, k, p.kk1);  // wave-uniform
  const uint8_t *tab = a.t.base;
  const uint64_t *vals = reinterpret_cast<const uint64_t *>(tab + a.t.vals_off);
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(tab + a.t.keys_off);
  p.v0 = p.v1 = 0;
#pragma unroll
  for (int j = 0; j < KW; j++) p.sk0[j] = p.sk1[j] = 0;
  if ((uint32_t)lane < m) {
    const uint32_t slot = p.e0 & 0xFFFFFu;
    p.v0 = vals[slot];
#pragma unroll
    for (int j = 0; j < KW; j++) p.sk0[j] = keys[(uint64_t)slot * KW + j];
  }
  if ((uint32_t)lane + 64 < m) {
    const uint32_t slot = p.e1 & 0xFFFFFu;
    p.v1 = vals[slot];
#pragma unroll
    for (int j = 0; j < KW; j++) p.sk1[j] = keys[(uint64_t)slot * KW + j];
  }
}

// Compare the loaded entries and fold the hits into `best`.
template <int KW>
__device__ __forceinline__ void wm_resolve(const uint64_t *mlds, uint64_t *best,
                                           int lane, const Pending<KW> &p) {
  if ((uint32_t)lane < p.m && wm_hit<KW>(mlds, p.e0, p.v0, p.sk0, p.kk0))
    wm_fold(best, p.e0, p.v0);
  if ((uint32_t)lane + 64 < p.m && wm_hit<KW>(mlds, p.e1, p.v1, p.sk1, p.kk1))
    wm_fold(best, p.e1, p.v1);
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
  // two buffers: the tile being hashed (cur) and the one whose key checks
  // are in flight (cur ^ 1)
  uint64_t *bests = reinterpret_cast<uint64_t *>(wl);            // [2][64]
  uint32_t *queues = reinterpret_cast<uint32_t *>(wl + 2 * 64 * 8);  // [2][kQueue]
  bests[lane] = 0;
  bests[64 + lane] = 0;
  __syncthreads();

  const uint64_t ntiles = (a.n + 63) / 64;
  const uint64_t nw = (uint64_t)gridDim.x * kWaves;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint32_t wn[NCH * 4 + 2];
  if (t < ntiles && t * 64 + lane < a.n)
    load_window<NCH>(a.frames + (t * 64 + lane) * a.stride, a.fp, wn);
  Pending<KW> pend;
  pend.m = 0;
  int cur = 0;
  uint64_t prev_idx = 0;
  bool prev_live = false, have_prev = false;
  // the previous tile: its checks resolved, its gates out
  auto finish_prev = [&]() {
    uint64_t *best = bests + (cur ^ 1) * 64;
    wm_resolve<KW>(mlds, best, lane, pend);
    lds_fence();
    const uint64_t b = best[lane];
    best[lane] = 0;
    if (prev_live) a.gates[prev_idx] = b ? (uint16_t)b : (uint16_t)a.default_gate;
  };
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

    // A. every tuple's hash and both tag words (16 LDS reads in flight)
    uint32_t b1[kMaxTuples], b2[kMaxTuples], tw1[kMaxTuples], tw2[kMaxTuples],
        tb[kMaxTuples];
#pragma unroll
    for (int tu = 0; tu < kMaxTuples; tu++) {
      b1[tu] = b2[tu] = tw1[tu] = tw2[tu] = tb[tu] = 0;
      if (tu < (int)a.ntuples) {
        uint64_t km[KW];
#pragma unroll
        for (int j = 0; j < KW; j++) km[j] = k[j] & tm[tu * kMaxKeyWords + j];
        const Probe p = split_hash(
            hash_join(hash_words_h1(km, KW, tuple_seed(a.t.seed, tu))), 1, a.t.nbp);
        b1[tu] = p.b1;
        b2[tu] = p.b2;
        tb[tu] = __builtin_amdgcn_perm(0u, p.tag, 0u);  // tag in every byte
        tw1[tu] = tags[p.b1];
        tw2[tu] = tags[p.b2];
      }
    }
#ifdef BG_AB  // phase timing: + hashes and tag reads
    if (a.ab_phase == 2) {
      uint32_t x = 0;
#pragma unroll
      for (int tu = 0; tu < kMaxTuples; tu++) x ^= tw1[tu] ^ tw2[tu];
      if (live) a.gates[idx] = (uint16_t)x;
      continue;
    }
#endif
    // B. fingerprint matches -> this tile's queue (a full queue checks 64
    // entries at once)
    uint64_t *best = bests + cur * 64;
    const uint32_t *qc = queues + cur * kQueue;
    uint32_t *q = queues + cur * kQueue;
    uint32_t head = 0, qlen = 0;  // wave-uniform
#pragma unroll
    for (int tu = 0; tu < kMaxTuples; tu++) {
      if (tu < (int)a.ntuples) {
        // bytes of the tag words equal to the fingerprint: bit 7 of each
        uint32_t c1 = zero_bytes(tw1[tu] ^ tb[tu]);
        uint32_t c2 = zero_bytes(tw2[tu] ^ tb[tu]);
        if (!live) c1 = c2 = 0;
        for (;;) {
          const bool has = (c1 | c2) != 0;
          const uint64_t bal = __ballot(has);
          if (!bal) break;
          if (has) {
            uint32_t slot;
            if (c1) {
              slot = b1[tu] * kSlots + (__builtin_ctz(c1) >> 3);
              c1 &= c1 - 1;
            } else {
              slot = b2[tu] * kSlots + (__builtin_ctz(c2) >> 3);
              c2 &= c2 - 1;
            }
            const uint32_t rank = __builtin_amdgcn_mbcnt_hi(
                (uint32_t)(bal >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bal, 0));
            q[(head + qlen + rank) & (kQueue - 1)] =
                slot | ((uint32_t)lane << 20) | ((uint32_t)tu << 26);
          }
          qlen += (uint32_t)__popcll(bal);
          if (qlen > kQueue - 64) {  // room for one more ballot round
            lds_fence();
            Pending<KW> now;
            wm_issue<KW>(a, qc, head, 64, lane, k, now);
            wm_resolve<KW>(mlds, best, lane, now);
            head += 64;
            qlen -= 64;
          }
        }
      }
    }
    // C. the previous tile's checks (loads issued one tile ago) and gates
    if (have_prev) finish_prev();
    // D. this tile's checks go in flight
    lds_fence();
    wm_issue<KW>(a, qc, head, qlen, lane, k, pend);
    prev_idx = idx;
    prev_live = live;
    have_prev = true;
    cur ^= 1;
  }
  if (have_prev) finish_prev();
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
