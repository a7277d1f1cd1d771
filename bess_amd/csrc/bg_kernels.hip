// bg_kernels.hip -- gfx950 (CDNA4) kernels for the BESS classification path.
//
//   em_classify  : ExactMatch::ProcessBatch   (core/modules/exact_match.cc:224-244)
//   wm_classify  : WildcardMatch::ProcessBatch (core/modules/wildcard_match.cc:159-203)
//   cksum        : IPChecksum / L4Checksum::ProcessBatch (ip_checksum.cc:39-84,
//                  l4_checksum.cc:41-83) fused into one pass over the frame.
//
// All integer work; HBM-bound streaming over resident packet slabs (frame i
// at frames + i*stride). No MFMA: there is no contraction on this path.
#include <hip/hip_runtime.h>
#include <limits.h>
#include <stddef.h>

#include <algorithm>

#include "bg_kernels.h"
#include "bg_keys_dev.h"
#include "bg_launch.h"

namespace bg {
namespace {

constexpr int kEmBlock = 512;  // 8 waves; LDS tables <= 40 KB -> 4 blocks/CU
constexpr int kCkBlock = 256;
constexpr int kDefaultPpl = 1;

template <int KW>
__device__ __forceinline__ bool key_eq(const uint8_t *slot_key,
                                       const uint64_t (&k)[KW]) {
  if constexpr (KW % 2 == 0) {
    const uint4 *s = reinterpret_cast<const uint4 *>(slot_key);
    bool eq = true;
#pragma unroll
    for (int j = 0; j < KW / 2; j++) {
      uint4 v = s[j];
      eq &= (((uint64_t)v.y << 32 | v.x) == k[2 * j]) &
            (((uint64_t)v.w << 32 | v.z) == k[2 * j + 1]);
    }
    return eq;
  } else {
    const uint64_t *s = reinterpret_cast<const uint64_t *>(slot_key);
    bool eq = true;
#pragma unroll
    for (int j = 0; j < KW; j++) eq &= s[j] == k[j];
    return eq;
  }
}

template <int KW>
__device__ __forceinline__ void load_key(const uint8_t *p, uint64_t (&o)[KW]) {
  if constexpr (KW % 2 == 0) {
    const uint4 *s = reinterpret_cast<const uint4 *>(p);
#pragma unroll
    for (int j = 0; j < KW / 2; j++) {
      const uint4 v = s[j];
      o[2 * j] = (uint64_t)v.y << 32 | v.x;
      o[2 * j + 1] = (uint64_t)v.w << 32 | v.z;
    }
  } else {
    const uint64_t *s = reinterpret_cast<const uint64_t *>(p);
#pragma unroll
    for (int j = 0; j < KW; j++) o[j] = s[j];
  }
}


// Look one key up: the two tag words, then for each fingerprint match the
// slot's key AND value, loaded together (one dependent round trip per
// candidate instead of two). `tab` is either the global image or its LDS
// copy; inlined separately for each so address spaces stay concrete.
template <int KW>
__device__ __forceinline__ uint32_t em_lookup(const uint8_t *tab,
                                              const TableRef &t,
                                              const uint64_t (&k)[KW],
                                              uint32_t dflt) {
  const uint64_t h = hash_words(k, KW, t.seed);
  const Probe p = split_hash(h, t.nparts, t.nbp);
  const uint8_t *pb = tab + (uint64_t)p.part * t.part_bytes;
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(pb);
  uint32_t cand = tag_match(tags[p.b1], p.tag) |
                  (tag_match(tags[p.b2], p.tag) << 4);
  if (t.vik) {  // the gate rides in the key's top two bytes: one read
    while (cand) {
      const int s = __builtin_ctz(cand);
      cand &= cand - 1;
      const uint32_t slot = (s < 4 ? p.b1 : p.b2) * kSlots + (s & 3);
      uint64_t sk[KW];
      load_key<KW>(pb + t.keys_off + (uint64_t)slot * KW * 8, sk);
      const uint32_t v = (uint32_t)(sk[KW - 1] >> 48);
      sk[KW - 1] &= 0x0000FFFFFFFFFFFFULL;
      bool eq = true;
#pragma unroll
      for (int j = 0; j < KW; j++) eq &= sk[j] == k[j];
      if (eq) return v;
    }
    return dflt;
  }
  const uint16_t *vals = reinterpret_cast<const uint16_t *>(pb + t.vals_off);
  while (cand) {
    const int s = __builtin_ctz(cand);
    cand &= cand - 1;
    const uint32_t slot = (s < 4 ? p.b1 : p.b2) * kSlots + (s & 3);
    const uint32_t v = vals[slot];
    if (key_eq<KW>(pb + t.keys_off + (uint64_t)slot * KW * 8, k)) return v;
  }
  return dflt;
}

// em_lookup for a table in L2 / MALL with the second bucket's tag word
// read only when the first bucket does not hold the key (a miss reads
// both, a hit placed in its first bucket one): fewer L2 requests per
// packet, at one more dependent round trip for those that need b2.
template <int KW>
__device__ __forceinline__ uint32_t em_lookup_seq(const uint8_t *tab, const TableRef &t,
                                                  const uint64_t (&k)[KW], uint32_t dflt) {
  const uint64_t h = hash_words(k, KW, t.seed);
  const Probe p = split_hash(h, t.nparts, t.nbp);
  const uint8_t *pb = tab + (uint64_t)p.part * t.part_bytes;
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(pb);
  const uint16_t *vals = reinterpret_cast<const uint16_t *>(pb + t.vals_off);
  for (int pass = 0; pass < 2; pass++) {
    const uint32_t b = pass ? p.b2 : p.b1;
    uint32_t cand = tag_match(tags[b], p.tag);
    while (cand) {
      const int s = __builtin_ctz(cand);
      cand &= cand - 1;
      const uint32_t slot = b * kSlots + s;
      uint64_t sk[KW];
      load_key<KW>(pb + t.keys_off + (uint64_t)slot * KW * 8, sk);
      uint32_t v;
      if (t.vik) {
        v = (uint32_t)(sk[KW - 1] >> 48);
        sk[KW - 1] &= 0x0000FFFFFFFFFFFFULL;
      } else {
        v = vals[slot];
      }
      bool eq = true;
#pragma unroll
      for (int j = 0; j < KW; j++) eq &= sk[j] == k[j];
      if (eq) return v;
    }
  }
  return dflt;
}

// Table / filter fill: four 16-byte loads in flight per thread before
// their LDS writes (a 40 KB table is ~5 loads per thread of a 512-thread
// block; one round trip instead of five).
__device__ __forceinline__ void copy_to_lds(uint8_t *lds, const uint8_t *g,
                                            uint32_t bytes) {
  const uint4 *src = reinterpret_cast<const uint4 *>(g);
  uint4 *dst = reinterpret_cast<uint4 *>(lds);
  const uint32_t n = bytes / 16, step = blockDim.x;
  uint32_t i = threadIdx.x;
  for (; i + 3 * step < n; i += 4 * step) {
    const uint4 a = src[i], b = src[i + step], c = src[i + 2 * step],
                d = src[i + 3 * step];
    dst[i] = a;
    dst[i + step] = b;
    dst[i + 2 * step] = c;
    dst[i + 3 * step] = d;
  }
  for (; i < n; i += step) dst[i] = src[i];
  __syncthreads();
}

__device__ __forceinline__ void copy_table_to_lds(uint8_t *lds,
                                                  const TableRef &t) {
  if (t.lds == kLdsTable)
    copy_to_lds(lds, t.base, t.bytes_total);
  else if (t.lds == kLdsFilter)
    copy_to_lds(lds, t.base + t.filt_off, t.filt_words * 4);
}

// ---------------------------------------------------------------------------
// ExactMatch: one lane per packet (PPL packets per lane per iteration),
// grid-stride over the resident slab with a residency-sized grid.
// ---------------------------------------------------------------------------
template <int KW, int NCH, int PPL>
__device__ __forceinline__ void em_body(const EmArgs &a, uint8_t *lds) {
  if (a.t.lds) copy_table_to_lds(lds, a.t);
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x * PPL;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * PPL + threadIdx.x;
       base < a.n; base += step) {
    uint64_t k[PPL][KW];
    build_keys<KW, NCH, PPL>(a.frames, a.stride, a.n, base, a.fp, k);
#pragma unroll
    for (int j = 0; j < PPL; j++) {
      const uint64_t idx = base + (uint64_t)j * blockDim.x;
      uint32_t g;
      if (a.t.lds == kLdsTable)
        g = em_lookup<KW>(lds, a.t, k[j], a.default_gate);
      else
        g = em_lookup<KW>(a.t.base, a.t, k[j], a.default_gate);
      if (idx < a.n) a.gates[idx] = (uint16_t)g;
    }
  }
}

// <= 80 SGPRs: the hardware then admits the occupancy the runtime reports
// (MI355X_MICROARCH.md, residency), so a residency-sized grid has no tail.
template <int KW, int NCH, int PPL>
__global__ __launch_bounds__(kEmBlock) __attribute__((amdgpu_num_sgpr(80)))
void em_classify_kernel(EmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  em_body<KW, NCH, PPL>(a, lds);
}

// ExactMatch on strided slots (1500 B frames in 2 KB slots: SURVEY §8d's
// 1500 B point) whose key window is two chunks inside the slot's first
// 64 B: a wave takes 64-slot tiles and loads their windows with pair loads
// (bg_keys_dev.h: one 32 B request per slot instead of two 16 B ones, the
// L2 requests in flight per CU being what bounds a scattered-window read,
// DESIGN §3 C4), the next tile's issued before this tile's lookup.
template <int KW>
__global__ __launch_bounds__(kEmBlock) __attribute__((amdgpu_num_sgpr(80)))
void em_pair_kernel(EmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (a.t.lds) copy_table_to_lds(lds, a.t);
  const int lane = threadIdx.x & 63;
  constexpr int kWaves = kEmBlock / 64;
  const uint64_t nw = (uint64_t)gridDim.x * kWaves, ntiles = (a.n + 63) / 64;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  const uint32_t stride = (uint32_t)a.stride;
  uint32_t wn[8];
  if (t < ntiles) load_pair(a.frames, a.n, t * 64, lane, a.fp.win_lo, stride, wn);
  for (; t < ntiles; t += nw) {
    uint32_t w[10];
    pair_window<2>(wn, lane, w);
    if (t + nw < ntiles) load_pair(a.frames, a.n, (t + nw) * 64, lane, a.fp.win_lo, stride, wn);
    uint64_t k[KW];
    extract_key<KW, 2>(w, a.fp, k);
    const uint32_t g = a.t.lds == kLdsTable
                           ? em_lookup<KW>(lds, a.t, k, a.default_gate)
                           : em_lookup<KW>(a.t.base, a.t, k, a.default_gate);
    const uint64_t idx = t * 64 + pair_slot(lane);
    if (idx < a.n) __builtin_nontemporal_store((uint16_t)g, a.gates + idx);
  }
}


// ---------------------------------------------------------------------------
// ExactMatch over a dense 64-byte-slot slab (stride 64, key window inside
// the slot): the slab is read with fully coalesced 16 B/lane loads -- a
// wave's 64 slots are 4 KB contiguous, 4 loads per lane -- and transposed
// through a per-wave 4 KB LDS stage so that each lane then reads its own
// slot's window. Measured (scripts/hbm_probe.hip): lane-contiguous loads
// stream the slab at ~7.1 TB/s where one-slot-per-lane 16 B loads at a
// 64 B stride reach ~5.0 TB/s. The stage is swizzled (slot s keeps chunk q
// at unit 4s + ((q + s/4) & 3)) so both the writes and the per-slot reads
// of 16 lanes hit 16 distinct 16-byte bank groups.
// The next tile's four loads are issued before this tile is looked up (one
// tile ahead: measured against none and two, scripts/variants.py).
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t stage_unit(uint32_t slot, uint32_t q) {
  return slot * 4 + ((q + (slot >> 2)) & 3);
}


// A table in L2 / MALL is probed with em_lookup_seq (the second bucket's
// tag word only when the first does not hold the key: C5 0.382 -> 0.357 ms);
// the gates are stored nontemporally (streaming stores; C2 0.1896 -> 0.1825
// ms). Both measured in one process each (scripts/variants.py em / c5,
// profiles/r05/em_variants_r05m.json).
// Round 6: the 2-byte gate stores interleaved with the header stream cost
// the stream (scripts/gate_probe.hip, C2's shape with no lookup: 0.1690 ms
// with each tile's gates stored after it, 0.1649 with 16 tiles' held in
// registers, 0.1593 / 0.1568 with 64 / 128 tiles' held in LDS, 0.1501
// reading alone; profiles/r06/gate_probe_r06q.jsonl). A wave holds its
// tiles' gates and stores them together after those tiles' reads:
//  * table in LDS (C2; one workgroup per CU): in LDS, lds_hold_tiles() tiles
//    (up to 128: what the CU's LDS leaves after the table and the stages),
//    stored 16 B per lane. C2 0.1837 (per-tile stores) -> 0.1674 (32 tiles
//    in registers) -> 0.1615 ms (64 in LDS): 0.857 of the roofline
//    (profiles/r06/c2_ab_r06n.json, c2_ab_r06q.json);
//  * table in L2 / MALL (C5; two workgroups per CU): kGateHold tiles in
//    registers (0.3448 -> 0.3424 ms; LDS holding at one workgroup per CU
//    0.376). The register form unrolls the tile body kGateHold times: past
//    32 it spills (64: 0.333 ms, c2_ab_r06o.json).

template <int KW, int NCH>
__global__ __launch_bounds__(kEmBlock) __attribute__((amdgpu_num_sgpr(80)))
void em_slab_kernel(EmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  copy_table_to_lds(lds, a.t);
  const uint32_t stage_off =
      a.t.lds == kLdsTable ? ((a.t.bytes_total + 15) & ~15u) : 0u;
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  constexpr int kWaves = kEmBlock / 64;
  uint4 *stage = reinterpret_cast<uint4 *>(lds + stage_off) + wid * 256;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t ntiles = (a.n + 63) / 64;
  const uint4 *src = reinterpret_cast<const uint4 *>(a.frames);
  const uint32_t q0 = (uint32_t)a.fp.win_lo >> 4;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint4 v[4];
  auto load_tile = [&](uint64_t tile, uint4 (&o)[4]) {
    const uint64_t p0 = tile * 64;
    const uint64_t units = (a.n - p0 < 64 ? a.n - p0 : 64) * 4;
    const uint4 *g = src + p0 * 4;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      o[c] = u < units ? ld_stream(g + u) : make_uint4(0, 0, 0, 0);
    }
  };
  // tile tt (its loads in v): staged, the next tile's loads issued, this
  // lane's slot looked up; returns its gate
  auto tile_gate = [&](uint64_t tt) -> uint32_t {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[stage_unit(u >> 2, u & 3)] = v[c];
    }
    lds_fence();
    if (tt + nwaves < ntiles) load_tile(tt + nwaves, v);
    uint32_t w[NCH * 4 + 2];
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      uint4 x = make_uint4(0, 0, 0, 0);
      if (c < a.fp.nch) x = stage[stage_unit(lane, q0 + c)];
      w[4 * c] = x.x;
      w[4 * c + 1] = x.y;
      w[4 * c + 2] = x.z;
      w[4 * c + 3] = x.w;
    }
    w[NCH * 4] = 0;
    w[NCH * 4 + 1] = 0;
    uint64_t k[KW];
    extract_key<KW, NCH>(w, a.fp, k);
    const uint32_t g = a.t.lds == kLdsTable
                           ? em_lookup<KW>(lds, a.t, k, a.default_gate)
                           : em_lookup_seq<KW>(a.t.base, a.t, k, a.default_gate);
    lds_fence();  // this tile's stage reads retire before the next writes
    return g;
  };
  if (t < ntiles) load_tile(t, v);
  const uint32_t hl = a.t.lds == kLdsTable ? lds_hold_tiles(stage_off) : 0u;
  if (hl) {  // (a multiple of 8; the launch sized the LDS for it)
    uint16_t *hold = reinterpret_cast<uint16_t *>(lds + stage_off + kWaves * 4096) +
                     (size_t)wid * hl * 64;
    for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * hl) {
#pragma unroll 1
      for (uint32_t h = 0; h < hl; h++) {
        const uint64_t tt = t0 + (uint64_t)h * nwaves;
        if (tt >= ntiles) break;
        hold[h * 64 + lane] = (uint16_t)tile_gate(tt);
      }
      lds_fence();
      store_held(hold, hl, t0, nwaves, lane, a.gates, a.n);
      lds_fence();  // the region's reads retire before the next round writes
    }
    return;
  }
  for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * kGateHold) {
    uint16_t held[kGateHold];
#pragma unroll
    for (int h = 0; h < kGateHold; h++) {
      const uint64_t tt = t0 + (uint64_t)h * nwaves;
      held[h] = 0;
      if (tt >= ntiles) break;
      held[h] = (uint16_t)tile_gate(tt);
    }
#pragma unroll
    for (int h = 0; h < kGateHold; h++) {  // the held gates, streaming stores
      const uint64_t idx = (t0 + (uint64_t)h * nwaves) * 64 + lane;
      if (idx < a.n) __builtin_nontemporal_store(held[h], a.gates + idx);
    }
  }
}


// ---------------------------------------------------------------------------
// Persistent ExactMatch over a ring of batch descriptors (RingArgs,
// bg_kernels.h): BESS hands a module <= 32 packets per ProcessBatch
// (core/pktbatch.h:70); one launch drains any number of such batches.
// Lane = packet inside the batch; the table stays in LDS for the whole run.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t ld_sys(const uint64_t *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// all four words of the slot carry `tag`: the descriptor is complete
__device__ __forceinline__ bool ring_read(const uint64_t *d, uint64_t tag,
                                          uint64_t (&w)[4]) {
#pragma unroll
  for (int i = 0; i < 4; i++) w[i] = ld_sys(d + i);
  return (w[0] >> 48) == tag && (w[1] >> 48) == tag && (w[2] >> 48) == tag &&
         (w[3] >> 48) == tag;
}

__device__ __forceinline__ uint64_t ld_agent(const unsigned long long *p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(unsigned long long *p, uint64_t v) {
  __hip_atomic_store(p, (unsigned long long)v, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// Workgroup 0, its first wave (one wave lane per submission lane): lane l
// reads the host's published count of submission lane l (PCIe) and mirrors
// it in device memory (L2), where that lane's workgroups wait, until the
// grid has been idle for idle_ticks or the owner stops it. On its way out it
// raises the device stop word and tells the host which launch ended.
__device__ __forceinline__ void ring_dispatch(const RingArgs &a) {
  const uint32_t l = threadIdx.x;
  const bool mine = l < a.nlanes;
  unsigned long long *dl = a.dev + (size_t)l * kRingLaneWords;
  uint64_t last = mine ? ld_agent(dl + 1) : 0;
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    const uint64_t p = mine ? ld_sys(a.pub + (size_t)l * kRingLaneWords) : last;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    const bool moved = p != last;
    if (moved) {
      st_agent(dl + 1, p);
      last = p;
    }
    if (__ballot(moved)) t0 = now;
    const uint32_t st = __hip_atomic_load(a.stop, __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_SYSTEM);
    if (st || now - t0 > a.idle_ticks) {
      if (l == 0) {
        // the mirrors above are visible before the stop word
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        st_agent(a.dev + (size_t)a.nlanes * kRingLaneWords, 1);
        __hip_atomic_store(a.ended, a.launch_id, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_SYSTEM);
      }
      return;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// kPpl packets' keys of one round: packet j's frame at f[j] (null: none)
template <int KW, int NCH>
__device__ __forceinline__ void ring_key1(const uint8_t *f, const FieldPlan &fp,
                                          uint32_t (&w)[NCH * 4 + 2]) {
#pragma unroll
  for (int q = 0; q < NCH * 4 + 2; q++) w[q] = 0;
  if (f) load_window<NCH>(f, fp, w);
}

template <int KW, int NCH>
__device__ __forceinline__ void ring_keys(const uint8_t *const (&f)[4], const FieldPlan &fp,
                                          uint64_t (&k0)[KW], uint64_t (&k1)[KW],
                                          uint64_t (&k2)[KW], uint64_t (&k3)[KW]) {
  if constexpr (NCH > 0) {
    uint32_t w0[NCH * 4 + 2], w1[NCH * 4 + 2], w2[NCH * 4 + 2], w3[NCH * 4 + 2];
    ring_key1<KW, NCH>(f[0], fp, w0);
    ring_key1<KW, NCH>(f[1], fp, w1);
    ring_key1<KW, NCH>(f[2], fp, w2);
    ring_key1<KW, NCH>(f[3], fp, w3);
    extract_key<KW, NCH>(w0, fp, k0);
    extract_key<KW, NCH>(w1, fp, k1);
    extract_key<KW, NCH>(w2, fp, k2);
    extract_key<KW, NCH>(w3, fp, k3);
  } else {  // fields too far apart for a window: per-field loads
    uint64_t (*ks[4])[KW] = {&k0, &k1, &k2, &k3};
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (f[j]) {
        direct_key<KW>(f[j], fp, *ks[j]);
      } else {
#pragma unroll
        for (int q = 0; q < KW; q++) (*ks[j])[q] = 0;
      }
    }
  }
}

// The ticket loop's two barriers without __syncthreads' fences:
// __syncthreads' workgroup acquire waits for every outstanding vector memory
// operation of each wave (vmcnt(0)), which for the done wave is the done
// word still in flight to the host -- the stall the done wave exists to
// avoid. Each wave's LDS writes before it are complete (lgkmcnt).
__device__ __forceinline__ void ring_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// The done wave (threads kRingBlock.. of a worker workgroup): per run of
// tickets, after the first barrier it takes the run's first ticket and
// length, after the second (every wave's gate stores complete) its lanes
// 0..k-1 write the k done words (adjacent words: one or two lines) -- and
// never wait for those stores, so no claim or frame load of the next run
// waits behind the writes' trip to the host. Its barriers pair one to one
// with em_ring_kernel's.
__device__ __forceinline__ void ring_done_wave(const RingArgs &a, uint32_t *ldone,
                                            const uint64_t *sh_t, const uint32_t *sh_k,
                                            const uint32_t *sh_rel) {
  const uint32_t wl = threadIdx.x & 63;
  for (;;) {
    ring_barrier();  // B1: the run is in sh_*
    const uint32_t k = *sh_k;
    if (!k) return;
    const uint64_t t = *sh_t + wl;
    const bool release = *sh_rel != 0;
    ring_barrier();  // B2: the gates are stored (sh_* free for the next run)
    // every wave's gate stores (system-scope write-through stores,
    // completed by each wave's vmcnt(0) before B2) reach the host before
    // the done words; with kRingRelease the L2 is written back first
    // (one system-scope release fence for the run)
    if (release) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    if (wl < k)
      __hip_atomic_store(ldone + t % a.nslots, (uint32_t)(t + 1), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// Workgroup b >= 1 serves submission lane (b - 1) % nlanes. Its first wave
// claims a range of the lane's next tickets (one atomic; claims run ahead of
// publication, so the lane's workgroups queue up on its coming tickets),
// waits until the range's next ticket is published and takes every ticket
// of the range published by then as one run (<= kRingRunMax tickets: a
// 32-packet batch alone would leave 7/8 of the workgroup's lanes idle),
// reads the run's descriptors (one per lane, every word tagged with its
// ticket), acquires (no line of an earlier batch survives in L1, or in L2
// for non-coherently cached memory: kRingSysAcquire), and the workgroup
// classifies the run's packets, writes the gates through to memory (sc0 sc1
// stores) and marks the tickets done in host memory after them
// (kRingRelease: behind a system-scope release). The range length adapts to
// the batch size the lane sees: about kRingRunPackets packets per claim.
// Create a ring with as many lanes as workers submit on. (Round 6 measured
// workgroups claiming on another lane when their own had no unclaimed
// published ticket: the sweep's 4-submitter rows fell from ~40 to ~20 Gpps
// -- the scans and the extra claimers crowd the lanes' counter lines --
// profiles/r06/ring_ab_r06g.json.)
//
// The serving loop is shared by the table kinds: `look(key, default_gate)`
// is the classifier (em_ring_kernel: ExactMatch, wm_ring_kernel:
// WildcardMatch); the workgroup's table copy in LDS is made before.
template <int KW, int NCH, int PPL, class Look>
__device__ __forceinline__ void ring_serve(const RingArgs &a, Look look) {
  static_assert(PPL == 1 || PPL == 4, "packets per lane per round: 1 or 4");
  __shared__ uint64_t sh_w[kRingRunMax][4];
  __shared__ uint32_t sh_pre[kRingRunMax + 1];  // the run's packet prefix sums
  __shared__ uint64_t sh_t;
  __shared__ uint32_t sh_k, sh_rel;
  const uint32_t lane = (blockIdx.x - 1) % a.nlanes;
  unsigned long long *dl = a.dev + (size_t)lane * kRingLaneWords;
  const unsigned long long *dstop = a.dev + (size_t)a.nlanes * kRingLaneWords;
  const uint64_t *ldesc = a.desc + (size_t)lane * a.nslots * kRingDescWords;
  uint32_t *ldone = a.done + (size_t)lane * a.nslots;
  if (threadIdx.x >= kRingBlock) {  // wave-uniform
    ring_done_wave(a, ldone, &sh_t, &sh_k, &sh_rel);
    return;
  }
  const uint64_t mask48 = (1ull << 48) - 1;
  constexpr int kPpl = PPL;  // packets per lane per round, loads in flight
  const uint32_t wl = threadIdx.x & 63;
  // wave 0's claim state (uniform): the claimed range [next, end)
  uint64_t next = 0, end = 0;
  uint32_t claim = 1;  // tickets per claim
  bool fresh = false, backlog = false;  // the claim is new / was published whole
  for (;;) {
    if (threadIdx.x < 64) {  // wave 0
      if (next == end) {
        uint64_t t = 0;
        if (wl == 0) t = atomicAdd(dl, (unsigned long long)claim);
        next = __shfl(t, 0);
        end = next + claim;
        fresh = true;
      }
      uint64_t p = 0;
      if (wl == 0) {
        // The stop word is read relaxed: an acquire load per poll put a
        // cache invalidate (buffer_inv) in every iteration of every waiting
        // workgroup (the ring sweep +10-15 % without it, profiles/r06/
        // ring_ab_r06g.json); the acquire follows only once it is set.
        // (Backing the polls off, s_sleep 2 -> 32, measured no better.)
        for (;;) {
          p = ld_agent(dl + 1);
          if (p > next) break;
          // stopping (the dispatcher's mirrors precede its stop word):
          // published meanwhile?
          if (__hip_atomic_load(dstop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            p = ld_agent(dl + 1);
            break;
          }
          __builtin_amdgcn_s_sleep(2);
        }
      }
      p = __shfl(p, 0);
      if (fresh) backlog = p >= end;  // the whole claim was waiting for us
      fresh = false;
      const uint32_t k = p > next ? (uint32_t)((p < end ? p : end) - next) : 0u;
      const uint64_t t = next + wl;
      uint64_t w[4] = {0, 0, 0, 0};
      if (wl < k) {
        const uint64_t tag = (t + 1) & 0xFFFF;
        const uint64_t *d = ldesc + (t % a.nslots) * kRingDescWords;
        while (!ring_read(d, tag, w)) __builtin_amdgcn_s_sleep(1);
      }
      // acquire: the batches' frames were written (by the host or a copy)
      // before their descriptors were published, and this grid outlives
      // many batches, so lines of an earlier batch in the same buffer may
      // still sit in this CU's L1 (and, for memory the device caches
      // non-coherently, in the XCD's L2): invalidate them before any wave
      // reads the frames (after the barrier below)
      if (__ballot(wl < k && (w[3] & kRingSysAcquire)))
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
      else if (k)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      // the run's packet prefix sums (inclusive scan over the wave)
      uint32_t c = wl < k ? (uint32_t)w[2] : 0u;
#pragma unroll
      for (int o = 1; o < kRingRunMax; o <<= 1) {
        const uint32_t v = __shfl_up(c, o);
        if (wl >= (uint32_t)o) c += v;
      }
      if (wl < k) {
#pragma unroll
        for (int i = 0; i < 4; i++) sh_w[wl][i] = w[i];
        sh_pre[wl + 1] = c;
      }
      const uint32_t total = __shfl(c, (int)(k ? k - 1 : 0));
      const bool rel = __ballot(wl < k && (w[3] & kRingRelease)) != 0;
      if (wl == 0) {
        sh_pre[0] = 0;
        sh_t = next;
        sh_k = k;
        sh_rel = rel ? 1u : 0u;
      }
      next += k;
      // the next claim: about kRingRunPackets packets of this lane's
      // batches while the lane has a backlog (its tickets were all
      // published before this workgroup got to them), one round's worth
      // while it trickles (tickets a busy workgroup has claimed wait for
      // it, however many others are idle)
      if (k && next == end) {
        const uint32_t per = max(total / k, 1u);
        const uint32_t want = backlog ? kRingRunPackets : kRingRunPacketsIdle;
        claim = min(max(want / per, 1u), (uint32_t)kRingRunMax);
      }
    }
    // B1 (ring_barrier): the frames' freshness for every wave is the
    // system-scope acquire above (its invalidations are the CU's L1 and the
    // XCD's L2)
    ring_barrier();
    const uint32_t k = sh_k;
    if (!k) return;
    const uint32_t total = sh_pre[k];
    for (uint32_t base = threadIdx.x; base < total; base += kRingBlock * kPpl) {
      // kPpl packets per lane, their header windows loaded before any key
      // is built; one named window array per packet (a 2-D array indexed
      // by the plan's runtime dword index would live in scratch)
      const uint8_t *f[kPpl];
      uint16_t *g[kPpl];
      uint32_t dflt[kPpl];
#pragma unroll
      for (int j = 0; j < kPpl; j++) {
        const uint32_t i = base + j * kRingBlock;
        uint32_t q = 0;  // the run's ticket holding packet i
        if (k > 1) {
#pragma unroll
          for (uint32_t st = kRingRunMax / 2; st; st >>= 1)
            if (q + st < k && sh_pre[q + st] <= i) q += st;
        }
        const uint32_t x = i - sh_pre[q];
        const uint64_t w2 = sh_w[q][2];
        const bool in = i < total;
        f[j] = in ? reinterpret_cast<const uint8_t *>(sh_w[q][0] & mask48) +
                        (uint64_t)x * ((w2 >> 32) & 0xFFFF)
                  : nullptr;
        g[j] = reinterpret_cast<uint16_t *>(sh_w[q][1] & mask48) + x;
        dflt[j] = (uint32_t)(sh_w[q][3] & 0xFFFF);
      }
      uint64_t k0[KW], k1[KW], k2[KW], k3[KW];
      if constexpr (PPL == 4) {
        ring_keys<KW, NCH>(f, a.fp, k0, k1, k2, k3);
      } else if constexpr (NCH > 0) {
        uint32_t w0[NCH * 4 + 2];
        ring_key1<KW, NCH>(f[0], a.fp, w0);
        extract_key<KW, NCH>(w0, a.fp, k0);
      } else if (f[0]) {
        direct_key<KW>(f[0], a.fp, k0);
      } else {
#pragma unroll
        for (int q = 0; q < KW; q++) k0[q] = 0;
      }
      const uint64_t *kk[4] = {k0, k1, k2, k3};
#pragma unroll
      for (int j = 0; j < kPpl; j++) {
        uint64_t key[KW];
#pragma unroll
        for (int q = 0; q < KW; q++) key[q] = kk[j][q];
        const uint32_t gt = look(key, dflt[j]);
        // written through to memory (sc0 sc1): seen by any reader once
        // this wave's stores have drained
        if (f[j])
          __hip_atomic_store(g[j], (uint16_t)gt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's gates complete
    ring_barrier();  // B2 (then sh_* may be rewritten for the next run)
  }
}

template <int KW, int NCH>
__global__ __launch_bounds__(kRingThreads) __attribute__((amdgpu_num_sgpr(80)))
void em_ring_kernel(RingArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (blockIdx.x == 0) {
    if (threadIdx.x < 64) ring_dispatch(a);
    return;
  }
  copy_table_to_lds(lds, a.t);  // (ends with a barrier)
  ring_serve<KW, NCH, 4>(a, [&](const uint64_t(&key)[KW], uint32_t dflt) -> uint32_t {
    return a.t.lds == kLdsTable ? em_lookup<KW>(lds, a.t, key, dflt)
                                : em_lookup<KW>(a.t.base, a.t, key, dflt);
  });
}

// ---------------------------------------------------------------------------
// WildcardMatch: tuple-space search over <= 8 masks in one combined table;
// the best (priority, later-tuple-on-tie) entry wins (LookupEntry 136-157).
// ---------------------------------------------------------------------------
// WildcardMatch entry value: priority | gate << 32 | tuple << 48. A slot
// matches tuple `tu` when its tuple field is tu and its key is k & mask.
template <int KW>
__device__ __forceinline__ bool wm_slot_hit(uint64_t v, const uint64_t (&sk)[KW],
                                            const uint64_t (&km)[KW], int tu) {
  bool eq = (uint32_t)(v >> 48) == (uint32_t)tu;
#pragma unroll
  for (int j = 0; j < KW; j++) eq &= sk[j] == km[j];
  return eq;
}

// Sequential-resolve lookup (default): tag reads batched over all tuples,
// then each tuple's fingerprint matches probed in turn, the slot's key and
// value loaded together.
template <int KW, bool FILT>
__device__ __forceinline__ uint32_t wm_lookup_seq(const uint8_t *tab,
                                                  const WmArgs &a,
                                                  const uint64_t (&k)[KW],
                                                  const uint32_t *filt) {
  const kconst_u64 tm = tuple_masks(a);
    uint32_t b1[kMaxTuples], b2[kMaxTuples], tg[kMaxTuples];
  uint32_t w1[kMaxTuples], w2[kMaxTuples];
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(tab);
  uint64_t dv[kMaxDirect];  // direct tuples' values (global, issued first)
#pragma unroll
  for (int d = 0; d < kMaxDirect; d++) {
    dv[d] = ~0ull;
    if ((uint32_t)d < a.ndirect)
      dv[d] = reinterpret_cast<const uint64_t *>(a.t.base + a.doff[d])[direct_index_k<KW>(k, a.dspec[d])];
  }
#pragma unroll
  for (int tu = 0; tu < kMaxTuples; tu++) {
    b1[tu] = b2[tu] = 0;
    tg[tu] = 1;  // fingerprints are never 0, so empty (0) tag words never match
    w1[tu] = w2[tu] = 0;
    if (tu < (int)a.ntuples && direct_of(a, tu) < 0) {
      const uint32_t h = wm_tuple_hash<KW>(k, tm, tu, a);
      bool pass = true;
      if (FILT) {
        const FilterProbe q = filter_probe(h, a.t.filt_words);
        pass = (filt[q.word] & q.bits) == q.bits;
      }
      if (pass) {
        const Probe p = wm_probe(h, a.t.nbp);
        b1[tu] = p.b1;
        b2[tu] = p.b2;
        tg[tu] = p.tag;
        w1[tu] = tags[p.b1];
        w2[tu] = tags[p.b2];
      }
    }
  }
  int32_t best = INT_MIN;
  uint32_t gate = a.default_gate;
  const uint64_t *vals = reinterpret_cast<const uint64_t *>(tab + a.t.vals_off);
#pragma unroll
  for (int tu = 0; tu < kMaxTuples; tu++) {
    const int d = direct_of(a, tu);
    if (d >= 0) {  // direct tuple: its value or empty
#pragma unroll
      for (int e = 0; e < kMaxDirect; e++) {
        const uint64_t v = dv[e];
        if (e == d && (uint32_t)(v >> 48) == (uint32_t)tu && (int32_t)(uint32_t)v >= best) {
          best = (int32_t)(uint32_t)v;
          gate = (uint32_t)(v >> 32) & 0xFFFFu;
        }
      }
    } else if (tu < (int)a.ntuples) {
      uint32_t cand = tag_match(w1[tu], tg[tu]) | (tag_match(w2[tu], tg[tu]) << 4);
      if (cand) {
        uint64_t km[KW];
#pragma unroll
        for (int j = 0; j < KW; j++) km[j] = k[j] & tm[tu * kMaxKeyWords + j];
        while (cand) {
          const int sl = __builtin_ctz(cand);
          cand &= cand - 1;
          const uint32_t slot = (sl < 4 ? b1[tu] : b2[tu]) * kSlots + (sl & 3);
          // value and key of the slot in one round trip
          const uint64_t v = vals[(uint64_t)slot * wm_rec_words(KW)];
          uint64_t sk[KW];
          load_key<KW>(tab + a.t.keys_off + (uint64_t)slot * wm_rec_words(KW) * 8, sk);
          if (wm_slot_hit<KW>(v, sk, km, tu)) {
            const int32_t prio = (int32_t)(uint32_t)v;
            if (prio >= best) {  // '>=': the later tuple wins a tie (P5)
              best = prio;
              gate = (uint32_t)(v >> 32) & 0xFFFFu;
            }
            break;
          }
        }
      }
    }
  }
  return gate;
}

// the table in LDS, the key filter in LDS, or the table in L2 / MALL
template <int KW>
__device__ __forceinline__ uint32_t wm_lookup_any(const WmArgs &a,
                                                  const uint64_t (&k)[KW],
                                                  const uint8_t *lds) {
  if (a.t.lds == kLdsTable) return wm_lookup_seq<KW, false>(lds, a, k, nullptr);
  if (a.t.lds == kLdsFilter)
    return wm_lookup_seq<KW, true>(a.t.base, a, k, reinterpret_cast<const uint32_t *>(lds));
  return wm_lookup_seq<KW, false>(a.t.base, a, k, nullptr);
}

// measured on MI355X (scripts/variants.py, C4): the sequential resolve
// beats a batched-rounds lookup, which hashes every tuple twice; with one
// packet per lane the next packet's header is prefetched
template <int KW, int NCH, int PPL>
__device__ __forceinline__ void wm_body(const WmArgs &a, uint8_t *lds) {
  copy_table_to_lds(lds, a.t);
  if constexpr (NCH > 0 && PPL == 1) {
    // one packet per lane, the next grid-stride packet's header window
    // loaded while this one is looked up
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t wn[NCH * 4 + 2];
    if (idx < a.n) load_window<NCH>(a.frames + idx * a.stride, a.fp, wn);
    for (; idx < a.n; idx += step) {
      uint32_t w[NCH * 4 + 2];
#pragma unroll
      for (int q = 0; q < NCH * 4 + 2; q++) w[q] = wn[q];
      if (idx + step < a.n)
        load_window<NCH>(a.frames + (idx + step) * a.stride, a.fp, wn);
      uint64_t k[KW];
      extract_key<KW, NCH>(w, a.fp, k);
      a.gates[idx] = (uint16_t)wm_lookup_any<KW>(a, k, lds);
    }
    return;
  }
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x * PPL;
  for (uint64_t base = (uint64_t)blockIdx.x * blockDim.x * PPL + threadIdx.x;
       base < a.n; base += step) {
    uint64_t k[PPL][KW];
    build_keys<KW, NCH, PPL>(a.frames, a.stride, a.n, base, a.fp, k);
#pragma unroll
    for (int j = 0; j < PPL; j++) {
      const uint64_t idx = base + (uint64_t)j * blockDim.x;
      const uint32_t g = wm_lookup_any<KW>(a, k[j], lds);
      if (idx < a.n) a.gates[idx] = (uint16_t)g;
    }
  }
}

template <int KW, int NCH, int PPL>
__global__ __launch_bounds__(kEmBlock) __attribute__((amdgpu_num_sgpr(80)))
void wm_classify_kernel(WmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  wm_body<KW, NCH, PPL>(a, lds);
}

// The persistent ring over a WildcardMatch table (bg::wm_ring_create): the
// ring's own copy of the image, probed in L2/MALL (wm_lookup_seq) or, for a
// table of <= 40 KB, from LDS; w.default_gate is kRingNoGate, so a miss
// takes each ticket's own default gate. One packet per lane per round (the
// lookup's dependent L2 reads are the latency; four packets' lookups inlined
// in a row spilled). WmArgs is the FIRST argument: the
// lookup reads the tuple data at the kernarg segment's start (tuple_masks).
constexpr int kWmRingPpl = 1;
template <int KW, int NCH>
__global__ __launch_bounds__(kRingThreads) __attribute__((amdgpu_num_sgpr(80)))
void wm_ring_kernel(WmArgs w, RingArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (blockIdx.x == 0) {
    if (threadIdx.x < 64) ring_dispatch(a);
    return;
  }
  copy_table_to_lds(lds, w.t);  // (ends with a barrier)
  ring_serve<KW, NCH, kWmRingPpl>(a, [&](const uint64_t(&key)[KW], uint32_t dflt) -> uint32_t {
    const uint32_t g = wm_lookup_any<KW>(w, key, lds);
    return g == kRingNoGate ? dflt : g;
  });
}


// ---------------------------------------------------------------------------
// IPChecksum + L4Checksum, one wave per frame.
//
// One's-complement sums are accumulated as exact integer sums of the
// frame's little-endian 16-bit words (every summed range starts at an even
// frame offset, so frame dword halves ARE the reference's u16 words), then
// end-around folded once. The folded value is independent of reduction order
// and is 0 only for an all-zero input, exactly like CalculateSum's adc
// chains (checksum.h:52-181) -- so the wave-tree reduction is bit-exact.
//
// Frames of <= 2 KiB are software-pipelined across a wave's packets: while
// packet p is summed, packet p+1's tail and packet p+2's head are in flight.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  s = (s & 0xFFFFu) + (s >> 16);
  s = (s & 0xFFFFu) + (s >> 16);
  return s;
}

__device__ __forceinline__ uint32_t halves(uint32_t v) {
  return (v & 0xFFFFu) + (v >> 16);
}

// u16-halves sum of the bytes of dword `dw` (frame offset o) inside [lo,hi)
__device__ __forceinline__ uint32_t range_sum(uint32_t dw, int o, int lo,
                                              int hi) {
  int s = lo - o, e = hi - o;
  s = s < 0 ? 0 : (s > 4 ? 4 : s);
  e = e < 0 ? 0 : (e > 4 ? 4 : e);
  const uint64_t one = 1;
  uint32_t m = e > s ? (uint32_t)(((one << (8 * e)) - 1) ^ ((one << (8 * s)) - 1))
                     : 0u;
  return halves(dw & m);
}

// the 16-byte chunk at frame offset o restricted to [lo, hi)
__device__ __forceinline__ uint32_t chunk_sum(const uint4 &c, int o, int lo,
                                              int hi) {
  if (o >= lo && o + 16 <= hi)
    return halves(c.x) + halves(c.y) + halves(c.z) + halves(c.w);
  if (o + 16 <= lo || o >= hi) return 0;
  return range_sum(c.x, o, lo, hi) + range_sum(c.y, o + 4, lo, hi) +
         range_sum(c.z, o + 8, lo, hi) + range_sum(c.w, o + 12, lo, hi);
}

__device__ __forceinline__ uint32_t sel4(const uint4 &c, int comp) {
  return comp == 0 ? c.x : comp == 1 ? c.y : comp == 2 ? c.z : c.w;
}
// frame dword j (< 256) of the first 1 KiB chunk held across the wave
__device__ __forceinline__ uint32_t hdr_dw(const uint4 &c0, int j) {
  return __builtin_amdgcn_readlane(sel4(c0, j & 3), j >> 2);
}
__device__ __forceinline__ uint32_t hdr_u8(const uint4 &c0, int o) {
  return (hdr_dw(c0, o >> 2) >> ((o & 3) * 8)) & 0xFFu;
}
__device__ __forceinline__ uint32_t hdr_be16(const uint4 &c0, int o) {
  return (hdr_u8(c0, o) << 8) | hdr_u8(c0, o + 1);
}
__device__ __forceinline__ uint32_t hdr_le16(const uint4 &c0, int o) {
  return hdr_u8(c0, o) | (hdr_u8(c0, o + 1) << 8);
}

// Wave-wide sum, DPP row reductions (result valid in lane 63).
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  v += __builtin_amdgcn_update_dpp(0u, v, 0xb1, 0xf, 0xf, false);   // quad [1,0,3,2]
  v += __builtin_amdgcn_update_dpp(0u, v, 0x4e, 0xf, 0xf, false);   // quad [2,3,0,1]
  v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xf, 0xf, false);  // row_shr:4
  v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xf, 0xf, false);  // row_shr:8
  v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xa, 0xf, false);  // row_bcast:15
  v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return __builtin_amdgcn_readlane(v, 63);
}

// Per-frame header walk (wave-uniform results).
struct CkHdr {
  int ip_state;  // 0 forward untouched, 1 IPv4 processed
  int ip_off, ip_lo, ip_hi;
  int l4_kind;   // 0 forward, 1 udp, 2 tcp, 3 not emitted
  int l4_off, l4_len, l4_ck, l4_lo, l4_hi;
  int l4_valid;
  int end;       // bytes of the frame the sums need
};

__device__ __forceinline__ CkHdr ck_parse(const uint4 &c0, int mode,
                                          int stride) {
  CkHdr h;
  h.ip_state = 0;
  h.ip_off = 14;
  h.ip_lo = h.ip_hi = 0;
  // IPChecksum::ProcessBatch ethertype walk (ip_checksum.cc:50-74)
  if (mode & 1) {
    uint32_t et = hdr_be16(c0, 12);
    bool fwd = false;
    if (et == 0x88a8) {  // kQinQ: must be followed by 802.1Q
      et = hdr_be16(c0, h.ip_off + 2);
      h.ip_off += 4;
      if (et != 0x8100) fwd = true;
    }
    if (!fwd && et == 0x8100) {  // kVlan
      et = hdr_be16(c0, h.ip_off + 2);
      h.ip_off += 4;
    }
    if (!fwd && et == 0x0800) {
      h.ip_state = 1;
      const int hl = (int)(hdr_u8(c0, h.ip_off) & 15) * 4;
      if (hl >= 20) {
        h.ip_lo = h.ip_off;
        h.ip_hi = h.ip_off + hl;
      }
    }
  }
  // L4Checksum::ProcessBatch (l4_checksum.cc:53-82): untagged IPv4 only
  h.l4_kind = 0;
  h.l4_off = h.l4_len = h.l4_ck = h.l4_lo = h.l4_hi = 0;
  h.l4_valid = 0;
  if ((mode & 2) && hdr_be16(c0, 12) == 0x0800) {
    const int hl = (int)(hdr_u8(c0, 14) & 15) * 4;
    const uint32_t proto = hdr_u8(c0, 23);
    h.l4_off = 14 + hl;
    if (proto == 17) {
      h.l4_kind = 1;
      h.l4_len = (int)hdr_be16(c0, h.l4_off + 4);
      h.l4_valid = h.l4_len >= 8;
      h.l4_ck = h.l4_off + 6;
    } else if (proto == 6) {
      h.l4_kind = 2;
      const int ip_len = (int)hdr_be16(c0, 16);
      h.l4_valid = ip_len >= hl + 20;
      h.l4_len = (ip_len - hl) & 0xFFFF;
      h.l4_ck = h.l4_off + 16;
    } else {
      h.l4_kind = 3;
    }
    if (h.l4_valid) {
      h.l4_lo = h.l4_off;
      h.l4_hi = h.l4_off + h.l4_len;
      if (h.l4_hi > stride) h.l4_hi = stride;  // the reference reads past (UB)
    }
  }
  if (h.ip_hi > stride) h.ip_hi = stride;
  h.end = h.ip_hi > h.l4_hi ? h.ip_hi : h.l4_hi;
  return h;
}

// Sums of one frame given its chunks (c[k] = bytes [1024k + 16 lane, +16)).
// `l4_extra`: this lane's L4 partial sum of bytes beyond the NC chunks.
template <int NC>
__device__ __forceinline__ void ck_finish(uint8_t *f, uint64_t pkt,
                                          const uint4 (&c)[NC], const CkHdr &h,
                                          const CkArgs &a, int lane,
                                          uint32_t l4_extra) {
  const uint4 &c0 = c[0];
  uint32_t s_ip = 0, s_l4 = l4_extra;
  if (lane * 16 < h.ip_hi) s_ip = chunk_sum(c0, lane * 16, h.ip_lo, h.ip_hi);
#pragma unroll
  for (int k = 0; k < NC; k++)
    s_l4 += chunk_sum(c[k], k * 1024 + lane * 16, h.l4_lo, h.l4_hi);
  // the IPv4 header lies in lanes 0..5 (offset <= 22 + 60)
  uint32_t t_ip = 0;
#pragma unroll
  for (int l = 0; l < 6; l++) t_ip += __builtin_amdgcn_readlane(s_ip, l);
  s_ip = t_ip;
  s_l4 = wave_sum(s_l4);

  // ---- IPChecksum result (checksum.h:254-318)
  uint32_t ip_gate = 0;
  bool ip_wrote = false;
  uint32_t ip_new = 0;  // value written at ip_off+10 (LE u16)
  if (h.ip_state == 1) {
    if (h.ip_hi == 0) {  // IHL < 5: calc writes 0, verify fails
      if (a.verify) {
        ip_gate = 1;
      } else {
        ip_wrote = true;
        ip_new = 0;
      }
    } else if (a.verify) {
      ip_gate = fold16(s_ip) == 0xFFFFu ? 0u : 1u;
    } else {
      const uint32_t old = hdr_le16(c0, h.ip_off + 10);
      ip_wrote = true;
      ip_new = (~fold16(s_ip - old)) & 0xFFFFu;
    }
    if (ip_wrote && lane == 0)
      *reinterpret_cast<uint16_t *>(f + h.ip_off + 10) = (uint16_t)ip_new;
  }
  // ---- L4Checksum result (checksum.h:324-504)
  uint32_t l4_gate = kGateNone;
  const bool l4_runs = (a.mode & 2) && (!(a.mode & 1) || ip_gate == 0);
  if (l4_runs) {
    if (h.l4_kind == 0) {
      l4_gate = 0;
    } else if (h.l4_kind == 3) {
      l4_gate = kGateNone;
    } else {
      // pseudo header: src, dst (LE u16 words of the BE addresses),
      // bswap16(length), protocol word 0x1100 (UDP) / 0x0600 (TCP)
      const uint32_t len = (uint32_t)h.l4_len;
      const uint32_t ps = hdr_le16(c0, 26) + hdr_le16(c0, 28) +
                          hdr_le16(c0, 30) + hdr_le16(c0, 32) +
                          ((len >> 8) | ((len & 0xFF) << 8)) +
                          (h.l4_kind == 1 ? 0x1100u : 0x0600u);
      uint32_t old = h.l4_valid ? hdr_le16(c0, h.l4_ck) : 0u;
      // Pipeline order: L4Checksum sees IPChecksum's write. With IHL < 5
      // the "L4 header" overlaps the IP checksum bytes 24..25.
      if ((a.mode & 1) && ip_wrote && h.ip_off == 14) {
        const uint32_t old_ip = hdr_le16(c0, 24);
#pragma unroll
        for (int b = 24; b < 26; b++) {
          if (b >= h.l4_lo && b < h.l4_hi) {
            const int sh = (b & 1) * 8;
            s_l4 = s_l4 - (((old_ip >> sh) & 0xFFu) << sh) +
                   (((ip_new >> sh) & 0xFFu) << sh);
          }
        }
        if (h.l4_valid && h.l4_ck == 24) old = ip_new;
      }
      if (a.verify) {
        if (!h.l4_valid) {
          l4_gate = 1;
        } else if (h.l4_kind == 1 && old == 0) {
          l4_gate = 0;  // UDP checksum 0 = not computed (checksum.h:328-331)
        } else {
          l4_gate = fold16(s_l4 + ps) == 0xFFFFu ? 0u : 1u;
        }
      } else {
        uint32_t ck = 0;  // invalid UDP/TCP lengths write 0
        if (h.l4_valid) {
          ck = (~fold16(s_l4 - old + ps)) & 0xFFFFu;
          if (h.l4_kind == 1 && ck == 0) ck = 0xFFFFu;  // RFC 768
        }
        const int at = h.l4_kind == 1 ? h.l4_off + 6 : h.l4_off + 16;
        if (lane == 0 && at + 2 <= (int)a.stride)
          *reinterpret_cast<uint16_t *>(f + at) = (uint16_t)ck;
        l4_gate = h.l4_kind == 1 ? 0u : kGateNone;  // TCP: never emitted
      }
    }
  }
  if (lane == 0) {
    if (a.ip_gates) a.ip_gates[pkt] = (a.mode & 1) ? (uint16_t)ip_gate : kGateNone;
    if (a.l4_gates) a.l4_gates[pkt] = (uint16_t)l4_gate;
  }
}

__device__ __forceinline__ uint4 ld_chunk(const uint8_t *f, int k, int lane,
                                          int limit) {
  const int o = k * 1024 + lane * 16;
  if (o < limit) return ld_stream(reinterpret_cast<const uint4 *>(f + o));
  return make_uint4(0, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Tiled checksum kernel (128 <= stride <= 2048): a wave owns tiles of 64
// frames.
//   1. lane = frame: the first 128 bytes of the frame (one 128 B line) are
//      loaded to registers; header walk, the IPv4 header sum and the L4 sum
//      of bytes < 128 are computed there with static register indices.
//   2. frame by frame, all 64 lanes: coalesced 16 B/lane loads of bytes
//      [128, l4_end) (next frame prefetched), unmasked u16-halves sums with
//      one tail mask, DPP wave reduction; the sum goes back to the frame's
//      lane. Frames whose L4 range ends below 128 skip this phase.
//   3. lane = frame: fold, store the checksum words (the old words were
//      kept from phase 1: no second read of the header line), write the
//      gates.
// The scalar unit only handles the per-frame loop.
// ---------------------------------------------------------------------------
constexpr int kHdrDw = 32;  // 128-byte header line

__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p) {
  return *reinterpret_cast<const uint16_t *>(p);
}

// u16-halves sum of the bytes of h[d] (frame offset 4d) inside [lo, hi)
__device__ __forceinline__ uint32_t dw_range_sum(uint32_t w, int o, int lo,
                                                 int hi) {
  int a = lo - o, b = hi - o;
  a = a < 0 ? 0 : (a > 4 ? 4 : a);
  b = b < 0 ? 0 : (b > 4 ? 4 : b);
  const uint32_t m =
      b > a ? ((0xFFFFFFFFu >> (32 - 8 * (b - a))) << (8 * a)) : 0u;
  const uint32_t v = w & m;
  return (v & 0xFFFFu) + (v >> 16);
}

template <int N>
__device__ __forceinline__ uint32_t hb(const uint32_t (&h)[N], int o) {
  return (h[o >> 2] >> ((o & 3) * 8)) & 0xFFu;  // o compile-time constant
}
template <int N>
__device__ __forceinline__ uint32_t hbe16(const uint32_t (&h)[N], int o) {
  return (hb(h, o) << 8) | hb(h, o + 1);
}
template <int N>
__device__ __forceinline__ uint32_t hle16(const uint32_t (&h)[N], int o) {
  return hb(h, o) | (hb(h, o + 1) << 8);
}

struct CkLane {       // phase-1 state of this lane's frame
  uint32_t flags;     // bit0 ip_state, bit1 ihl<5, 2-3 l4_kind, 4 l4_valid
  uint32_t ip_off;    // 14 / 18 / 22
  uint32_t s_ip;      // IPv4 header sum (all header bytes)
  uint32_t s_l4;      // L4 range sum over bytes < 128
  uint32_t l4_lo, l4_hi;
  uint32_t l4_ck;     // frame offset of the L4 checksum word
  uint32_t ps;        // pseudo-header sum
};

// (Fields at per-lane offsets are read with per-lane 2-byte loads of the
// frame -- L1 hits -- never by indexing the register array dynamically,
// which would move it to scratch.)
__device__ __forceinline__ CkLane ck_walk(const uint8_t *f,
                                          const uint32_t (&h)[kHdrDw], int mode,
                                          int stride) {
  CkLane r;
  r.flags = 0;
  r.ip_off = 14;
  r.s_ip = 0;
  r.s_l4 = 0;
  r.l4_lo = r.l4_hi = 0;
  r.l4_ck = 0;
  r.ps = 0;
  const uint32_t et12 = hbe16(h, 12);
  // IPChecksum ethertype walk (ip_checksum.cc:50-74)
  if (mode & 1) {
    uint32_t et = et12, off = 14;
    bool fwd = false;
    if (et == 0x88a8) {  // kQinQ must carry an 802.1Q tag
      et = hbe16(h, 16);
      off = 18;
      if (et != 0x8100) fwd = true;
    }
    if (!fwd && et == 0x8100) {  // kVlan
      et = off == 14 ? hbe16(h, 16) : hbe16(h, 20);
      off += 4;
    }
    if (!fwd && et == 0x0800) {
      r.flags |= 1;
      r.ip_off = off;
      const uint32_t vihl =
          off == 14 ? hb(h, 14) : (off == 18 ? hb(h, 18) : hb(h, 22));
      const uint32_t hl = (vihl & 15) * 4;
      if (hl >= 20) {  // header <= 22 + 60 bytes: inside the 128 B line
        const int lo = (int)off, hi = (int)(off + hl);
#pragma unroll
        for (int d = 3; d < 21; d++) r.s_ip += dw_range_sum(h[d], 4 * d, lo, hi);
      } else {
        r.flags |= 2;  // IHL < 5: calc writes 0, verify fails
      }
    }
  }
  // L4Checksum (l4_checksum.cc:53-82): untagged IPv4 only
  if ((mode & 2) && et12 == 0x0800) {
    const uint32_t hl = (hb(h, 14) & 15) * 4;
    const uint32_t proto = hb(h, 23);
    const uint32_t l4_off = 14 + hl;
    uint32_t kind = 3, len = 0, valid = 0;
    if (proto == 17) {
      kind = 1;
      const uint32_t v = ld_u16(f + l4_off + 4);
      len = ((v & 0xFF) << 8) | (v >> 8);
      valid = len >= 8;
      r.l4_ck = l4_off + 6;
    } else if (proto == 6) {
      kind = 2;
      const uint32_t ip_len = hbe16(h, 16);
      valid = ip_len >= hl + 20;
      len = (ip_len - hl) & 0xFFFF;
      r.l4_ck = l4_off + 16;
    }
    r.flags |= kind << 2;
    if (kind != 3) {
      if (valid) {
        r.flags |= 16;
        uint32_t hi = l4_off + len;
        if (hi > (uint32_t)stride) hi = stride;  // reference reads past (UB)
        r.l4_lo = l4_off;
        r.l4_hi = hi;
#pragma unroll
        for (int d = 3; d < kHdrDw; d++)
          r.s_l4 += dw_range_sum(h[d], 4 * d, (int)l4_off, (int)hi);
      }
      r.ps = hle16(h, 26) + hle16(h, 28) + hle16(h, 30) + hle16(h, 32) +
             ((len >> 8) | ((len & 0xFF) << 8)) + (kind == 1 ? 0x1100u : 0x0600u);
    }
  }
  return r;
}

// 16 bytes at frame offset o >= 128 restricted to [., hi): whole dwords
// before hi, a byte mask on the one that straddles it
__device__ __forceinline__ uint32_t tail_sum(const uint4 &c, int o, int hi) {
  uint32_t s = 0;
  const uint32_t w[4] = {c.x, c.y, c.z, c.w};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    int b = hi - (o + 4 * k);
    b = b < 0 ? 0 : (b > 4 ? 4 : b);
    const uint32_t m = b >= 4 ? 0xFFFFFFFFu : ((1u << (8 * b)) - 1u);
    const uint32_t v = w[k] & m;
    s += (v & 0xFFFFu) + (v >> 16);
  }
  return s;
}

// Phase 1 keeps the two header words phase 3 needs (the old IPv4 checksum,
// bytes 24..25) and phase 3 stores the checksum words alone: no re-read of
// the header line and no line store. Measured against re-reading the line
// in phase 3, holding it in VGPRs through phase 2 and parking it in LDS
// (round 5, scripts/variants.py ck, profiles/r05/ck_variants_*.json).
template <int DEPTH>
__device__ __forceinline__ void cksum_body(const CkArgs &a) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(
      ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int stride = (int)a.stride;
  const uint64_t ntiles = (a.n + 63) / 64;
  for (uint64_t tile = wave0; tile < ntiles; tile += nw) {
    const uint64_t p0 = tile * 64;
    const int cnt = (int)((a.n - p0) < 64 ? (a.n - p0) : 64);
    // ---- phase 1: lane = frame
    uint8_t *mine = a.frames + (p0 + (uint64_t)lane) * a.stride;
    uint32_t h[kHdrDw];
    CkLane L;
    uint32_t ip_old = 0, w24 = 0, l4_old = 0;
    if (lane < cnt) {
      const uint4 *q = reinterpret_cast<const uint4 *>(mine);
#pragma unroll
      for (int c = 0; c < kHdrDw / 4; c++) {
        const uint4 v = q[c];
        h[4 * c] = v.x;
        h[4 * c + 1] = v.y;
        h[4 * c + 2] = v.z;
        h[4 * c + 3] = v.w;
      }
      L = ck_walk(mine, h, a.mode, stride);
      ip_old = L.ip_off == 14 ? hle16(h, 24) : (L.ip_off == 18 ? hle16(h, 28) : hle16(h, 32));
      w24 = hle16(h, 24);
      l4_old = (L.flags & 16) ? ld_u16(mine + L.l4_ck) : 0u;  // (in the line: an L1 hit)
    } else {
#pragma unroll
      for (int d = 0; d < kHdrDw; d++) h[d] = 0;
      L.flags = L.s_ip = L.s_l4 = L.l4_lo = L.l4_hi = L.l4_ck = L.ps = 0;
      L.ip_off = 14;
    }
    // ---- phase 2: bytes [128, l4_hi) of each frame across the wave,
    // DEPTH frames prefetched ahead
    uint32_t tail = 0;
    const uint8_t *f = a.frames + p0 * a.stride;
    uint4 q0[DEPTH + 1], q1[DEPTH + 1];
    int qh[DEPTH + 1];
#pragma unroll
    for (int d = 0; d <= DEPTH; d++) {
      q0[d] = q1[d] = make_uint4(0, 0, 0, 0);
      qh[d] = 0;
      if (d < DEPTH && d < cnt) {
        qh[d] = (int)__builtin_amdgcn_readlane(L.l4_hi, d);
        if (qh[d] > 128) {
          const uint8_t *fd = f + (size_t)d * a.stride + 128;
          q0[d] = ld_chunk(fd, 0, lane, qh[d] - 128);
          q1[d] = ld_chunk(fd, 1, lane, qh[d] - 128);
        }
      }
    }
    for (int j = 0; j < cnt; j++) {
      if (j + DEPTH < cnt) {  // prefetch frame j+DEPTH
        const int hn = (int)__builtin_amdgcn_readlane(L.l4_hi, j + DEPTH);
        qh[DEPTH] = hn;
        if (hn > 128) {
          const uint8_t *fn = f + (size_t)DEPTH * a.stride + 128;
          q0[DEPTH] = ld_chunk(fn, 0, lane, hn - 128);
          q1[DEPTH] = ld_chunk(fn, 1, lane, hn - 128);
        }
      }
      const int hi = qh[0];
      if (hi > 128) {  // wave-uniform
        const int o = 128 + lane * 16;
        uint32_t s = tail_sum(q0[0], o, hi);
        if (o + 1024 < hi) s += tail_sum(q1[0], o + 1024, hi);
        s = wave_sum(s);
        tail = lane == j ? s : tail;
      }
#pragma unroll
      for (int d = 0; d < DEPTH; d++) {
        q0[d] = q0[d + 1];
        q1[d] = q1[d + 1];
        qh[d] = qh[d + 1];
      }
      q0[DEPTH] = q1[DEPTH] = make_uint4(0, 0, 0, 0);
      qh[DEPTH] = 0;
      f += a.stride;
    }
    if (lane >= cnt) continue;
    // ---- phase 3: lane = frame
    uint32_t ip_gate = 0;
    bool ip_wrote = false;
    uint32_t ip_new = 0;
    if (L.flags & 1) {
      if (L.flags & 2) {  // IHL < 5: calc writes 0, verify fails
        if (a.verify) {
          ip_gate = 1;
        } else {
          ip_wrote = true;
        }
      } else if (a.verify) {
        ip_gate = fold16(L.s_ip) == 0xFFFFu ? 0u : 1u;
      } else {
        ip_new = (~fold16(L.s_ip - ip_old)) & 0xFFFFu;
        ip_wrote = true;
      }
    }
    uint32_t l4_gate = kGateNone, l4_new = 0;
    bool l4_wrote = false;
    const uint32_t kind = (L.flags >> 2) & 3;
    const bool valid = L.flags & 16;
    const bool l4_runs = (a.mode & 2) && (!(a.mode & 1) || ip_gate == 0);
    if (l4_runs) {
      if (kind == 0) {
        l4_gate = 0;
      } else if (kind == 3) {
        l4_gate = kGateNone;
      } else {
        uint32_t s = L.s_l4 + tail;
        uint32_t old = l4_old;
        // Pipeline order: L4Checksum sees IPChecksum's write. With IHL < 5
        // the "L4 header" overlaps the IP checksum bytes 24..25.
        if (ip_wrote && L.ip_off == 14 && valid) {
          const int lo2 = (int)L.l4_lo > 24 ? (int)L.l4_lo : 24;
          const int hi2 = (int)L.l4_hi < 26 ? (int)L.l4_hi : 26;
          s = s - dw_range_sum(w24, 24, lo2, hi2) +
              dw_range_sum(ip_new, 24, lo2, hi2);
          if (L.l4_ck == 24) old = ip_new;
        }
        if (a.verify) {
          if (!valid)
            l4_gate = 1;
          else if (kind == 1 && old == 0)
            l4_gate = 0;  // UDP checksum 0 = not computed
          else
            l4_gate = fold16(s + L.ps) == 0xFFFFu ? 0u : 1u;
        } else {
          if (valid) {  // invalid UDP/TCP lengths write 0
            l4_new = (~fold16(s - old + L.ps)) & 0xFFFFu;
            if (kind == 1 && l4_new == 0) l4_new = 0xFFFFu;  // RFC 768
          }
          l4_wrote = true;
          l4_gate = kind == 1 ? 0u : kGateNone;  // TCP: never emitted
        }
      }
    }
    // the checksum words, in the reference's order (IPChecksum first)
    if (ip_wrote) *reinterpret_cast<uint16_t *>(mine + L.ip_off + 10) = (uint16_t)ip_new;
    if (l4_wrote && L.l4_ck + 2 <= (uint32_t)stride)
      *reinterpret_cast<uint16_t *>(mine + L.l4_ck) = (uint16_t)l4_new;
    if (a.ip_gates) a.ip_gates[p0 + lane] = (a.mode & 1) ? (uint16_t)ip_gate : kGateNone;
    if (a.l4_gates) a.l4_gates[p0 + lane] = (uint16_t)l4_gate;
  }
}

template <int DEPTH>
__global__ __launch_bounds__(kCkBlock) __attribute__((amdgpu_num_sgpr(80)))
void cksum_kernel(CkArgs a) { cksum_body<DEPTH>(a); }


// any stride: frame chunks loaded after the header walk, one frame at a time
__global__ __launch_bounds__(kCkBlock) void cksum_kernel_generic(CkArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(
      ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint64_t nw = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int stride = (int)a.stride;
  for (uint64_t p = wave0; p < a.n; p += nw) {
    uint8_t *f = a.ptrs ? reinterpret_cast<uint8_t *>(a.ptrs[p]) : a.frames + p * a.stride;
    uint4 c[1];
    c[0] = ld_chunk(f, 0, lane, stride);
    const CkHdr h = ck_parse(c[0], a.mode, stride);
    uint32_t extra = 0;  // L4 bytes beyond the first KiB
    for (int k = 1; k * 1024 < h.end; k++)
      extra += chunk_sum(ld_chunk(f, k, lane, h.end), k * 1024 + lane * 16,
                         h.l4_lo, h.l4_hi);
    ck_finish<1>(f, p, c, h, a, lane, extra);
  }
}


// Packets per workgroup below which staging the table into LDS costs more
// than probing it in L2 (a 40 KB table fill vs. 64 B of header per packet).
constexpr uint64_t kLdsMinPktsPerBlock = 4096;

template <typename Args, typename K>
hipError_t launch_classify(K kernel, Args a, int num_cus, hipStream_t s,
                           int ppl, int block = kEmBlock) {
  if (a.n == 0) return hipSuccess;
  const uint32_t pf = path_flags();
  if (pf & kPathNoLds) a.t.lds = kLdsNone;
  const uint64_t need = (a.n + (uint64_t)block * ppl - 1) / ((uint64_t)block * ppl);
  // Measured on MI355X (scripts/variants.py): with the table in LDS two
  // 512-thread blocks per CU (16 waves) stream fastest -- fewer LDS table
  // fills; with the table in L2/MALL, twice the resident grid.
  for (int pass = 0; pass < 2; pass++) {
    const size_t lds = a.t.lds == kLdsTable    ? a.t.bytes_total
                       : a.t.lds == kLdsFilter ? (size_t)a.t.filt_words * 4
                                               : 0;
    const int occ = occupancy(reinterpret_cast<const void *>(kernel), block, lds, 2);
    const int pc = a.t.lds ? std::min(occ, 2) : occ * 2;
    const uint64_t cap = (uint64_t)num_cus * pc;
    const uint64_t blocks = need > cap ? cap : need;
    if (a.t.lds && pass == 0 && a.n < blocks * kLdsMinPktsPerBlock &&
        !(pf & kPathForceLds)) {
      a.t.lds = kLdsNone;  // small launch: probe the table in L2 instead
      continue;
    }
    hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(block), lds, s, a);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

template <template <int, int, int> class Sel, typename Args>
hipError_t dispatch(const Args &a, int num_cus, hipStream_t s, int dflt_ppl) {
  int maxops = 0;
  for (int q = 0; q < a.fp.nkd; q++) maxops = std::max(maxops, kd_nops_of(a.fp, q));
  const int nch = a.fp.direct ? 0 : (a.fp.nch <= 2 && maxops <= 2 ? 2 : 4);
  const int ppl = dflt_ppl;
#define BG_CASE(KW, NCH, PPL)                                                   \
  if (a.t.kw == KW && nch == NCH && ppl == PPL)                                 \
    return launch_classify(Sel<KW, NCH, PPL>::kernel(), a, num_cus, s, PPL);
#define BG_NCHS(KW) BG_CASE(KW, 0, 1) BG_CASE(KW, 2, 1) BG_CASE(KW, 4, 1)
  BG_NCHS(1) BG_NCHS(2) BG_NCHS(4) BG_NCHS(8)
#undef BG_NCHS
#undef BG_CASE
  return hipErrorInvalidValue;
}

template <int KW, int NCH, int PPL>
struct EmSel {
  static auto kernel() { return em_classify_kernel<KW, NCH, PPL>; }
};
template <int KW, int NCH, int PPL>
struct WmSel {
  static auto kernel() { return wm_classify_kernel<KW, NCH, PPL>; }
};

// Dense 64 B slots with the key window inside the slot: the coalesced slab
// kernel. LDS = table (if staged) + the per-wave stage.
template <typename K>
hipError_t launch_slab(K kern, EmArgs a, int num_cus, hipStream_t s, int block,
                       size_t stage) {
  const uint32_t pf = path_flags();
  if (pf & kPathNoLds) a.t.lds = kLdsNone;
  const uint64_t need = (a.n + block - 1) / block;
  for (int pass = 0; pass < 2; pass++) {
    const size_t tab = a.t.lds == kLdsTable ? (a.t.bytes_total + 15) & ~(size_t)15 : 0;
    // (em_slab_kernel's gates held in LDS beside an LDS table)
    const size_t hold = a.t.lds == kLdsTable
                            ? (size_t)lds_hold_tiles((uint32_t)tab) * (block / 64) * 128
                            : 0;
    const size_t lds = tab + stage + hold;
    int pc = occupancy(reinterpret_cast<const void *>(kern), block, lds, 1);
    // a table in L2 / MALL: 2 workgroups per CU (16 waves) probe faster
    // than the occupancy limit (C5: 0.3444 against 0.3557 ms,
    // scripts/variants.py c5, profiles/r05/c5_variants_r05q.json); the
    // table in LDS: one (8 waves, the table copied once per CU), with the
    // gates held (round 6: 0.1674 against 0.1757 ms at two, c2_ab_r06m/n)
    pc = std::min(pc, a.t.lds == kLdsNone ? 2 : 1);
    const uint64_t cap = (uint64_t)num_cus * pc;
    const uint64_t blocks = need > cap ? cap : need;
    if (a.t.lds == kLdsTable && pass == 0 && a.n < blocks * kLdsMinPktsPerBlock &&
        !(pf & kPathForceLds)) {
      a.t.lds = kLdsNone;  // small launch: probe the table in L2 instead
      continue;
    }
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(block), lds, s, a);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

template <int KW, int NCH>
hipError_t launch_em_slab(const EmArgs &a, int num_cus, hipStream_t s) {
  constexpr size_t kStage = (size_t)(kEmBlock / 64) * 4096;
  return launch_slab(em_slab_kernel<KW, NCH>, a, num_cus, s, kEmBlock, kStage);
}

}  // namespace

hipError_t launch_em_ring(const RingArgs &a, int blocks, hipStream_t s) {
  int maxops = 0;
  for (int q = 0; q < a.fp.nkd; q++) maxops = std::max(maxops, kd_nops_of(a.fp, q));
  const int nch = a.fp.direct ? 0 : (a.fp.nch <= 2 && maxops <= 2 ? 2 : 4);
  const size_t lds = a.t.lds == kLdsTable ? (a.t.bytes_total + 15) & ~(size_t)15 : 0;
#define BG_RING(KW, NCH)                                                     \
  if (a.t.kw == KW && nch == NCH) {                                          \
    hipLaunchKernelGGL((em_ring_kernel<KW, NCH>), dim3((unsigned)blocks),     \
                       dim3(kRingThreads), lds, s, a);                       \
    return hipGetLastError();                                                \
  }
#define BG_RINGS(KW) BG_RING(KW, 0) BG_RING(KW, 2) BG_RING(KW, 4)
  BG_RINGS(1) BG_RINGS(2) BG_RINGS(4) BG_RINGS(8)
#undef BG_RINGS
#undef BG_RING
  return hipErrorInvalidValue;
}

hipError_t launch_wm_ring(const RingArgs &a, const WmArgs &w, int blocks, hipStream_t s) {
  if (w.t.rec != wm_rec_words(w.t.kw)) return hipErrorInvalidValue;  // (slot records)
  int maxops = 0;
  for (int q = 0; q < a.fp.nkd; q++) maxops = std::max(maxops, kd_nops_of(a.fp, q));
  const int nch = a.fp.direct ? 0 : (a.fp.nch <= 2 && maxops <= 2 ? 2 : 4);
  const size_t lds = w.t.lds == kLdsTable ? (w.t.bytes_total + 15) & ~(size_t)15 : 0;
#define BG_WRING(KW, NCH)                                                    \
  if (w.t.kw == KW && nch == NCH) {                                          \
    hipLaunchKernelGGL((wm_ring_kernel<KW, NCH>), dim3((unsigned)blocks),     \
                       dim3(kRingThreads), lds, s, w, a);                    \
    return hipGetLastError();                                                \
  }
#define BG_WRINGS(KW) BG_WRING(KW, 0) BG_WRING(KW, 2) BG_WRING(KW, 4)
  BG_WRINGS(1) BG_WRINGS(2) BG_WRINGS(4) BG_WRINGS(8)
#undef BG_WRINGS
#undef BG_WRING
  return hipErrorInvalidValue;
}

bool fits_nch2(const FieldPlan &fp) {
  if (fp.direct || fp.nch > 2) return false;
  for (int q = 0; q < fp.nkd; q++)
    if (kd_nops_of(fp, q) > 2) return false;
  return true;
}

bool slab_ok(const EmArgs &a) {
  return a.stride == 64 && !a.fp.direct && a.fp.win_lo >= 0 &&
         a.fp.win_lo + 16 * a.fp.nch <= 64 && ((uintptr_t)a.frames & 15) == 0 &&
         !(path_flags() & kPathNoSlab);
}

hipError_t launch_em(const EmArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  if (slab_ok(a)) {
    const bool two = fits_nch2(a.fp);
#define BG_SLAB(KW)                                                        \
  if (a.t.kw == KW)                                                        \
    return two ? launch_em_slab<KW, 2>(a, num_cus, s)                      \
               : launch_em_slab<KW, 4>(a, num_cus, s);
    BG_SLAB(1) BG_SLAB(2) BG_SLAB(4) BG_SLAB(8)
#undef BG_SLAB
  }
  // strided slots with the window in the slot's first 64 B: pair loads
  // (measured: scripts/variants.py em1500)
  if (!a.fp.direct && fits_nch2(a.fp) && a.fp.win_lo % 16 == 0 && a.fp.win_lo + 32 <= 64 &&
      a.stride > 64 && a.stride <= 65536 && !(path_flags() & kPathNoSlab)) {
#define BG_PAIR(KW) \
  if (a.t.kw == KW) return launch_classify(em_pair_kernel<KW>, a, num_cus, s, 1);
    BG_PAIR(1) BG_PAIR(2) BG_PAIR(4) BG_PAIR(8)
#undef BG_PAIR
  }
  return dispatch<EmSel>(a, num_cus, s, kDefaultPpl);
}

hipError_t launch_wm(const WmArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  // the kernels read slot records of wm_rec_words(kw) words (bg_table.h)
  if (a.t.rec != wm_rec_words(a.t.kw)) return hipErrorInvalidValue;
  if (a.t.lds == kLdsTags) {
    if (!a.fp.direct && a.fp.nch <= 4 && !(path_flags() & kPathNoLds))
      return launch_wm_tags(a, num_cus, s);
    WmArgs b = a;  // fields too far apart for a window: probe in L2
    b.t.lds = kLdsNone;
    return dispatch<WmSel>(b, num_cus, s, 1);
  }
  return dispatch<WmSel>(a, num_cus, s, 1);
}

hipError_t launch_cksum(const CkArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  // (frames by pointer: one wave per frame wherever it lies)
  const bool tiled = !a.ptrs && a.stride >= 128 && a.stride <= 2048 &&
                     !(path_flags() & kPathNoSlab);
  using CkKern = void (*)(CkArgs);
  CkKern kfn = cksum_kernel_generic;
  if (tiled) {
    // measured on MI355X (scripts/variants.py ck, profiles/r05/): phase 1
    // keeping the two header words phase 3 needs and phase 3 storing the
    // checksum words alone (no re-read of the line, no line store) beats
    // re-reading the line (round 4's default, 0.2964 -> 0.2896 ms per 1 M
    // frames, 31 B/pkt less fetched), holding it in registers (0.362) or
    // parking it in LDS (0.368); prefetch depth 1
    kfn = cksum_kernel<1>;
  }
  const void *kern = reinterpret_cast<const void *>(kfn);
  // four residency-sized rounds of workgroups (scripts/variants.py ck)
  const int per_cu = occupancy(kern, kCkBlock, 0, 7) * 4;
  const uint64_t waves_per_block = kCkBlock / 64;
  const uint64_t max_waves = (uint64_t)num_cus * per_cu * waves_per_block;
  uint64_t waves;
  if (tiled) {
    // equal tile counts per wave: no tail from a partial last round
    const uint64_t ntiles = (a.n + 63) / 64;
    const uint64_t rounds = (ntiles + max_waves - 1) / max_waves;
    waves = (ntiles + rounds - 1) / rounds;
  } else {
    waves = std::min<uint64_t>(a.n, max_waves);
  }
  const uint64_t blocks = (waves + waves_per_block - 1) / waves_per_block;
  hipLaunchKernelGGL(kfn, dim3((unsigned)blocks), dim3(kCkBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bg
