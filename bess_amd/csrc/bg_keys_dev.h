// bg_keys_dev.h -- device-side key building shared by the classify kernels
// (ExactMatch, WildcardMatch, HashLB field mode). Included only from .hip
// translation units; everything lives in an anonymous namespace so each
// kernel file gets its own inlined copy.
#ifndef BESS_AMD_BG_KEYS_DEV_H_
#define BESS_AMD_BG_KEYS_DEV_H_

#ifndef __HIPCC_RTC__  // hiprtc (bg_wm_jit.cc) has its own
#include <hip/hip_runtime.h>
#endif

#include "bg_kernels.h"

namespace bg {
namespace {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint32_t compact_bytes(uint32_t m) {
  // bits 7, 15, 23, 31 -> bits 0..3
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) |
         ((m >> 28) & 8u);
}

// bit 7 of every byte of x that is zero -- exact (the carry-free form: no
// borrow crosses a byte), so an empty slot (fingerprint 0) never matches a
// fingerprint, which is never 0
__device__ __forceinline__ uint32_t zero_bytes(uint32_t x) {
  const uint32_t y = (x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu;
  return ~(y | x | 0x7F7F7F7Fu);
}

// SWAR "which tag bytes equal `tag`" -> bits 0..3
__device__ __forceinline__ uint32_t tag_match(uint32_t tags, uint32_t tag) {
  return compact_bytes(zero_bytes(tags ^ (tag * 0x01010101u)));
}

// The WildcardMatch tuple masks (up to 64 words) would otherwise be hoisted
// into scalar registers for the whole kernel and spilled; laundering the
// kernarg pointer per packet makes them cheap scalar-cache loads instead.
// (The WmArgs block is every WildcardMatch kernel's first argument, so it
// starts at the kernarg segment; taking the parameter's address instead
// would copy the whole block to scratch.)
typedef const uint64_t __attribute__((address_space(4))) *kconst_u64;
__device__ __forceinline__ kconst_u64 tuple_masks(const WmArgs &) {
  const __attribute__((address_space(4))) uint8_t *ka =
      (const __attribute__((address_space(4))) uint8_t *)
          __builtin_amdgcn_kernarg_segment_ptr();
  kconst_u64 p = (kconst_u64)(ka + offsetof(WmArgs, tmask));
  asm volatile("" : "+s"(p));
  return p;
}

typedef const uint32_t __attribute__((address_space(4))) *kconst_u32;
// tcover / tseed / ntuples the same way (read per tile: hoisted, the
// per-dword branch conditions would become lane masks spilled to VGPR lanes)
__device__ __forceinline__ kconst_u32 tuple_words(const WmArgs &, size_t off) {
  const __attribute__((address_space(4))) uint8_t *ka =
      (const __attribute__((address_space(4))) uint8_t *)
          __builtin_amdgcn_kernarg_segment_ptr();
  kconst_u32 p = (kconst_u32)(ka + off);
  asm volatile("" : "+s"(p));
  return p;
}

// The tuple's hash of packet key k (bg_table.h wm_hash over k & mask):
// uniform branches skip the dwords the tuple's mask clears.
template <int KW>
__device__ __forceinline__ uint32_t wm_tuple_hash(const uint64_t (&k)[KW],
                                                  kconst_u64 tm, int tu,
                                                  const WmArgs &a) {
  const uint32_t cover = tuple_words(a, offsetof(WmArgs, tcover))[tu];
  uint32_t h = tuple_words(a, offsetof(WmArgs, tseed))[tu];
#pragma unroll
  for (int d = 0; d < 2 * KW; d++) {
    if ((cover >> d) & 1u) {
      const uint64_t mw = tm[tu * kMaxKeyWords + d / 2];
      const uint32_t x = (uint32_t)(k[d / 2] >> (32 * (d & 1))) &
                         (uint32_t)(mw >> (32 * (d & 1)));
      h = (h ^ x) * 0x9E3779B1u;
      h ^= h >> 15;
    }
  }
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  return h;
}

// direct_index (bg_kernels.h) over a key held in registers: the key words
// are picked with selects on the uniform byte positions (no register-array
// indexing)
template <int KW>
__device__ __forceinline__ uint32_t direct_index_k(const uint64_t (&k)[KW], uint32_t spec) {
  const uint32_t pa = spec & 63, pb = (spec >> 8) & 63;
  uint64_t wa = 0, wb = 0;
#pragma unroll
  for (int j = 0; j < KW; j++) {
    if ((uint32_t)j == pa >> 3) wa = k[j];
    if ((uint32_t)j == pb >> 3) wb = k[j];
  }
  const uint32_t ba = (uint32_t)(wa >> ((pa & 7) * 8)) & (spec >> 16) & 0xFFu;
  const uint32_t bb = (uint32_t)(wb >> ((pb & 7) * 8)) & (spec >> 24) & 0xFFu;
  return ba | bb << 8;
}

// the direct-tuple slot of tuple tu (WmArgs::ndirect), or -1 (uniform)
__device__ __forceinline__ int direct_of(const WmArgs &a, int tu) {
  int r = -1;
#pragma unroll
  for (int d = 0; d < kMaxDirect; d++)
    if ((uint32_t)d < a.ndirect && a.dtu[d] == (uint32_t)tu) r = d;
  return r;
}

__device__ __forceinline__ void lds_fence() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}


// streaming (read-once) 16-byte load: nontemporal so packet bytes do not
// evict the flow table from L2
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
// a streaming (nontemporal) 16-byte store
__device__ __forceinline__ void st_stream(uint4 *p, const uint4 &v) {
  const u32x4 x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, reinterpret_cast<u32x4 *>(p));
}

// Tiles of 2-byte results a slab kernel's wave holds in LDS at one 512-
// thread workgroup per CU (8 waves, 4 KB stage each), beside tab_bytes of
// tables: a multiple of 8, at most kGateHoldLds; 0 when nothing fits.
__host__ __device__ constexpr uint32_t lds_hold_tiles(uint32_t tab_bytes) {
  constexpr uint32_t stage = 8 * 4096u, per_tile = 8 * 128u;
  const uint32_t room = tab_bytes + stage < kLdsPerCu ? kLdsPerCu - tab_bytes - stage : 0u;
  const uint32_t h = (room / per_tile) & ~7u;
  return h < (uint32_t)kGateHoldLds ? h : (uint32_t)kGateHoldLds;
}

// The wave's held results (hold[h * 64 + s] = tile t0 + h * nwaves's
// result for slot s, h < hl) to out[]: 16 B (8 results) per lane, 8
// lanes per tile, streaming; 2-byte stores for a partial last group or an
// out[] not 16 B aligned. Nothing at or past n is written.
__device__ __forceinline__ void store_held(const uint16_t *hold, uint32_t hl, uint64_t t0,
                                           uint64_t nwaves, int lane, uint16_t *out,
                                           uint64_t n) {
  const bool al16 = (reinterpret_cast<unsigned long long>(out) & 15) == 0;
#pragma unroll 1
  for (uint32_t i = 0; i < hl; i += 8) {
    const uint32_t h = i + (lane >> 3);
    const uint64_t idx = (t0 + (uint64_t)h * nwaves) * 64 + (lane & 7) * 8;
    if (idx >= n) continue;
    const uint4 x = reinterpret_cast<const uint4 *>(hold + h * 64)[lane & 7];
    if (al16 && idx + 8 <= n) {
      st_stream(reinterpret_cast<uint4 *>(out + idx), x);
    } else {
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
      for (int j = 0; j < 8 && idx + j < n; j++)
        out[idx + j] = (uint16_t)(xs[j >> 1] >> (16 * (j & 1)));
    }
  }
}

// Key building (ExactMatchTable::MakeKeys exact_match_table.h:239-263 /
// WildcardMatch::ProcessBatch wildcard_match.cc:169-197). The window
// [win_lo, win_lo + 16*nch) of a frame is staged in registers with 16-byte
// loads; each field is funnel-shifted out of it with a wave-uniform dword
// index (s_set_gpr_idx, no scratch) and OR-ed into its key word(s).
template <int NCH>
__device__ __forceinline__ void load_window(const uint8_t *__restrict__ frame,
                                            const FieldPlan &fp,
                                            uint32_t (&w)[NCH * 4 + 2]) {
  const uint4 *src = reinterpret_cast<const uint4 *>(frame + fp.win_lo);
#pragma unroll
  for (int c = 0; c < NCH; c++) {
    uint4 v = make_uint4(0, 0, 0, 0);
    if (c < fp.nch) v = ld_stream(src + c);
    w[4 * c + 0] = v.x;
    w[4 * c + 1] = v.y;
    w[4 * c + 2] = v.z;
    w[4 * c + 3] = v.w;
  }
  w[NCH * 4] = 0;
  w[NCH * 4 + 1] = 0;
}

template <int KW>
__device__ __forceinline__ void place_field(uint64_t v, int p,
                                            uint64_t (&k)[KW]) {
  const int pw = p >> 3, pb = (p & 7) * 8;
#pragma unroll
  for (int j = 0; j < KW; j++) {
    if (j == pw) k[j] |= v << pb;
    if (pb && j == pw + 1) k[j] |= v >> (64 - pb);
  }
}

// Key from the byte-permute plan (FieldPlan::kd_*): per key dword one
// v_perm_b32 per source dword pair (wave-uniform window index: s_set_gpr_idx,
// no scratch) and one AND. ExactMatchTable::MakeKeys semantics (mask per
// field, bytes past the key zero) are folded into selectors and masks.
template <int KW, int NCH>
__device__ __forceinline__ void extract_key(const uint32_t (&w)[NCH * 4 + 2],
                                            const FieldPlan &fp,
                                            uint64_t (&k)[KW]) {
  // NCH == 2 kernels are only dispatched for plans with <= 2 permutes per
  // key dword. Branch-free: unused permutes have all-zero selectors.
  constexpr int kMaxOps = NCH == 2 ? 2 : 4;
  uint32_t kd[2 * KW];
#pragma unroll
  for (int q = 0; q < 2 * KW; q++) {
    const uint32_t dws = fp.kd_dw[q];
    uint32_t x = 0;
#pragma unroll
    for (int o = 0; o < kMaxOps; o++) {
      const uint32_t d = (dws >> (8 * o)) & 0xFF;
      x |= __builtin_amdgcn_perm(w[d + 1], w[d], fp.kd_sel[o][q]);
    }
    kd[q] = x & fp.kd_mask[q];
  }
#pragma unroll
  for (int j = 0; j < KW; j++) k[j] = (uint64_t)kd[2 * j + 1] << 32 | kd[2 * j];
}

// fields too far apart for one window: per-field aligned dword loads
template <int KW>
__device__ __forceinline__ void direct_key(const uint8_t *__restrict__ frame,
                                           const FieldPlan &fp,
                                           uint64_t (&k)[KW]) {
#pragma unroll
  for (int j = 0; j < KW; j++) k[j] = 0;
#pragma unroll
  for (int f = 0; f < kMaxFields; f++) {
    if (f < fp.nf) {
      const uint32_t spec = fp.fspec[f];
      const uint32_t *q =
          reinterpret_cast<const uint32_t *>(frame) + fspec_d(spec);
      const int nd = fspec_nd(spec), sh = fspec_shift_bits(spec);
      uint32_t d0 = q[0];
      uint32_t d1 = nd > 1 ? q[1] : 0u;
      uint32_t d2 = nd > 2 ? q[2] : 0u;
      uint64_t lo = (uint64_t)d0 | ((uint64_t)d1 << 32);
      uint64_t v = sh ? ((lo >> sh) | ((uint64_t)d2 << (64 - sh))) : lo;
      place_field<KW>(v & fp.fmask[f], fspec_pos(spec), k);
    }
  }
}

// Keys of PPL packets handled by one lane (idx = base + j*blockDim.x): all
// window loads are issued before any key is built (memory-level parallelism).
template <int KW, int NCH, int PPL>
__device__ __forceinline__ void build_keys(const uint8_t *__restrict__ frames,
                                           uint64_t stride, uint64_t n,
                                           uint64_t base, const FieldPlan &fp,
                                           uint64_t (&k)[PPL][KW]) {
  if constexpr (NCH > 0) {
    uint32_t w[PPL][NCH * 4 + 2];
#pragma unroll
    for (int j = 0; j < PPL; j++) {
      const uint64_t idx = base + (uint64_t)j * blockDim.x;
      if (idx < n) {
        load_window<NCH>(frames + idx * stride, fp, w[j]);
      } else {
#pragma unroll
        for (int q = 0; q < NCH * 4 + 2; q++) w[j][q] = 0;
      }
    }
#pragma unroll
    for (int j = 0; j < PPL; j++) extract_key<KW, NCH>(w[j], fp, k[j]);
  } else {
#pragma unroll
    for (int j = 0; j < PPL; j++) {
      const uint64_t idx = base + (uint64_t)j * blockDim.x;
      if (idx < n) {
        direct_key<KW>(frames + idx * stride, fp, k[j]);
      } else {
#pragma unroll
        for (int q = 0; q < KW; q++) k[j][q] = 0;
      }
    }
  }
}

// Pair loads (the WildcardMatch tag-word kernels' PAIR mode, the
// ExactMatch pair kernel on strided slots): the two 16-byte window chunks of a slot
// are loaded by a lane pair -- load 0 of lanes 2m, 2m+1 holds chunks q0,
// q0+1 of slot m, load 1 those of slot 32+m -- so each load instruction
// covers 32 B of each of 32 adjacent slots (half the cache lines per
// instruction of one 16 B chunk per lane at a 64 B stride). One DPP swap
// per dword completes the windows: lane 2m takes slot m, lane 2m+1 slot
// 32+m.
__device__ __forceinline__ uint64_t pair_slot(int lane) {
  return (lane & 1) ? 32u + (lane >> 1) : (uint32_t)(lane >> 1);
}

__device__ __forceinline__ void load_pair(const uint8_t *__restrict__ frames,
                                          uint64_t n, uint64_t p0, int lane,
                                          uint32_t win_lo, uint32_t stride,
                                          uint32_t (&r)[8]) {
  const uint64_t s0 = p0 + (lane >> 1), s1 = s0 + 32;
  // a uniform base plus a 32-bit lane offset recomputed here (hoisted out
  // of the tile loop, the per-lane 64-bit addresses were spilled, and the
  // reload's wait retired every load issued before it)
  uint32_t ln = (uint32_t)lane;
  asm volatile("" : "+v"(ln));
  const uint32_t off = (ln >> 1) * stride + win_lo + (ln & 1) * 16;
  const uint8_t *base = frames + p0 * stride;
  uint4 x = make_uint4(0, 0, 0, 0), y = x;
  if (s0 < n) x = ld_stream(reinterpret_cast<const uint4 *>(base + off));
  if (s1 < n) y = ld_stream(reinterpret_cast<const uint4 *>(base + off + 32 * stride));
  r[0] = x.x; r[1] = x.y; r[2] = x.z; r[3] = x.w;
  r[4] = y.x; r[5] = y.y; r[6] = y.z; r[7] = y.w;
}

template <int NCH>
__device__ __forceinline__ void pair_window(const uint32_t (&r)[8], int lane,
                                            uint32_t (&w)[NCH * 4 + 2]) {
  static_assert(NCH == 2, "pair loads carry two chunks");
  const bool odd = lane & 1;
#pragma unroll
  for (int d = 0; d < 4; d++) {
    const uint32_t src = odd ? r[d] : r[4 + d];
    // quad_perm [1,0,3,2]: swap with the neighbouring lane
    const uint32_t recv = (uint32_t)__builtin_amdgcn_mov_dpp((int)src, 0xB1, 0xF, 0xF, false);
    w[d] = odd ? recv : r[d];
    w[4 + d] = odd ? r[4 + d] : recv;
  }
  w[8] = 0;
  w[9] = 0;
}

}  // namespace
}  // namespace bg

#endif  // BESS_AMD_BG_KEYS_DEV_H_
