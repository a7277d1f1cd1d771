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

#include "bg_kernels.h"

namespace bg {
namespace {

constexpr int kEmBlock = 512;  // 8 waves; LDS tables <= 40 KB -> 4 blocks/CU
constexpr int kCkBlock = 256;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// streaming (read-once) 16-byte load: nontemporal so packet bytes do not
// evict the flow table from L2
__device__ __forceinline__ uint4 ld_stream(const uint4 *p) {
  u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ uint32_t compact_bytes(uint32_t m) {
  // bits 7, 15, 23, 31 -> bits 0..3
  return ((m >> 7) & 1u) | ((m >> 14) & 2u) | ((m >> 21) & 4u) |
         ((m >> 28) & 8u);
}

// SWAR "which tag bytes equal `tag`": no false negatives; rare false
// positives only cost an extra key compare.
__device__ __forceinline__ uint32_t tag_match(uint32_t tags, uint32_t tag) {
  uint32_t x = tags ^ (tag * 0x01010101u);
  return compact_bytes((x - 0x01010101u) & ~x & 0x80808080u);
}

// Build the key of one frame. The window [win_lo, win_lo + 16*nch) is
// staged in registers with 16-byte loads; each field is funnel-shifted out
// of it with a wave-uniform dword index (s_set_gpr_idx, no scratch).
template <int KW>
__device__ __forceinline__ void build_key(const uint8_t *__restrict__ frame,
                                          const FieldPlan &fp,
                                          uint64_t (&k)[KW]) {
#pragma unroll
  for (int j = 0; j < KW; j++) k[j] = 0;
  if (!fp.direct) {
    uint32_t w[kMaxWindowChunks * 4 + 2];
    const uint4 *src = reinterpret_cast<const uint4 *>(frame + fp.win_lo);
#pragma unroll
    for (int c = 0; c < kMaxWindowChunks; c++) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c < fp.nch) v = ld_stream(src + c);
      w[4 * c + 0] = v.x;
      w[4 * c + 1] = v.y;
      w[4 * c + 2] = v.z;
      w[4 * c + 3] = v.w;
    }
    w[kMaxWindowChunks * 4] = 0;
    w[kMaxWindowChunks * 4 + 1] = 0;
#pragma unroll
    for (int f = 0; f < kMaxFields; f++) {
      if (f < fp.nf) {
        const int d = fp.fdw[f], sh = fp.fsh[f];
        uint64_t lo = (uint64_t)w[d] | ((uint64_t)w[d + 1] << 32);
        uint64_t v = sh ? ((lo >> sh) | ((uint64_t)w[d + 2] << (64 - sh))) : lo;
        v &= fp.fmask[f];
        const int p = fp.fpos[f], pw = p >> 3, pb = (p & 7) * 8;
#pragma unroll
        for (int j = 0; j < KW; j++) {
          if (j == pw) k[j] |= v << pb;
          if (pb && j == pw + 1) k[j] |= v >> (64 - pb);
        }
      }
    }
  } else {
#pragma unroll
    for (int f = 0; f < kMaxFields; f++) {
      if (f < fp.nf) {
        const uint32_t *q =
            reinterpret_cast<const uint32_t *>(frame + (fp.foff[f] & ~3));
        const int nd = fp.fnd[f], sh = fp.fsh[f];
        uint32_t d0 = q[0];
        uint32_t d1 = nd > 1 ? q[1] : 0u;
        uint32_t d2 = nd > 2 ? q[2] : 0u;
        uint64_t lo = (uint64_t)d0 | ((uint64_t)d1 << 32);
        uint64_t v = sh ? ((lo >> sh) | ((uint64_t)d2 << (64 - sh))) : lo;
        v &= fp.fmask[f];
        const int p = fp.fpos[f], pw = p >> 3, pb = (p & 7) * 8;
#pragma unroll
        for (int j = 0; j < KW; j++) {
          if (j == pw) k[j] |= v << pb;
          if (pb && j == pw + 1) k[j] |= v >> (64 - pb);
        }
      }
    }
  }
}

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

// Probe one key. Returns the slot index (bucket*4+s) of the match inside
// partition image `pb`, or -1. `tab` is either the global image or its LDS
// copy; inlined separately for each so address spaces stay concrete.
template <int KW>
__device__ __forceinline__ int probe(const uint8_t *tab, const TableRef &t,
                                     const uint64_t (&k)[KW], uint64_t seed,
                                     const uint8_t **pb_out) {
  const uint64_t h = hash_words(k, KW, seed);
  const Probe p = split_hash(h, t.nparts, t.nbp);
  const uint8_t *pb = tab + (uint64_t)p.part * t.part_bytes;
  *pb_out = pb;
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(pb);
  uint32_t cand = tag_match(tags[p.b1], p.tag) |
                  (tag_match(tags[p.b2], p.tag) << 4);
  while (cand) {
    const int s = __builtin_ctz(cand);
    cand &= cand - 1;
    const uint32_t slot = (s < 4 ? p.b1 : p.b2) * kSlots + (s & 3);
    if (key_eq<KW>(pb + t.keys_off + (uint64_t)slot * KW * 8, k)) return (int)slot;
  }
  return -1;
}

template <int KW>
__device__ __forceinline__ uint32_t em_lookup(const uint8_t *tab,
                                              const TableRef &t,
                                              const uint64_t (&k)[KW],
                                              uint32_t dflt) {
  const uint8_t *pb;
  int slot = probe<KW>(tab, t, k, t.seed, &pb);
  if (slot < 0) return dflt;
  return reinterpret_cast<const uint16_t *>(pb + t.vals_off)[slot];
}

__device__ __forceinline__ void copy_table_to_lds(uint8_t *lds,
                                                  const TableRef &t) {
  const uint4 *src = reinterpret_cast<const uint4 *>(t.base);
  uint4 *dst = reinterpret_cast<uint4 *>(lds);
  for (uint32_t i = threadIdx.x; i < t.bytes_total / 16; i += blockDim.x)
    dst[i] = src[i];
  __syncthreads();
}

// ---------------------------------------------------------------------------
// ExactMatch: one lane per packet, grid-stride over the resident slab.
// ---------------------------------------------------------------------------
template <int KW>
__global__ __launch_bounds__(kEmBlock) void em_classify_kernel(EmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (a.t.lds) copy_table_to_lds(lds, a.t);
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
       i += nthr) {
    uint64_t k[KW];
    build_key<KW>(a.frames + i * a.stride, a.fp, k);
    uint32_t g;
    if (a.t.lds)
      g = em_lookup<KW>(lds, a.t, k, a.default_gate);
    else
      g = em_lookup<KW>(a.t.base, a.t, k, a.default_gate);
    a.gates[i] = (uint16_t)g;
  }
}

// ---------------------------------------------------------------------------
// WildcardMatch: tuple-space search over <= 8 masks in one combined table;
// the best (priority, later-tuple-on-tie) entry wins (LookupEntry 136-157).
// ---------------------------------------------------------------------------
template <int KW>
__device__ __forceinline__ uint32_t wm_lookup(const uint8_t *tab,
                                              const WmArgs &a,
                                              const uint64_t (&k)[KW]) {
  int32_t best = INT_MIN;
  uint32_t gate = a.default_gate;
  for (uint32_t tu = 0; tu < a.ntuples; tu++) {
    uint64_t km[KW];
#pragma unroll
    for (int j = 0; j < KW; j++) km[j] = k[j] & a.tmask[tu][j];
    const uint8_t *pb;
    const uint64_t seed = tuple_seed(a.t.seed, tu);
    // the slot must also belong to this tuple: keys of different tuples
    // share the table, tagged in the value word
    const uint64_t h = hash_words(km, KW, seed);
    const Probe p = split_hash(h, a.t.nparts, a.t.nbp);
    pb = tab + (uint64_t)p.part * a.t.part_bytes;
    const uint32_t *tags = reinterpret_cast<const uint32_t *>(pb);
    uint32_t cand = tag_match(tags[p.b1], p.tag) |
                    (tag_match(tags[p.b2], p.tag) << 4);
    while (cand) {
      const int s = __builtin_ctz(cand);
      cand &= cand - 1;
      const uint32_t slot = (s < 4 ? p.b1 : p.b2) * kSlots + (s & 3);
      const uint64_t v =
          reinterpret_cast<const uint64_t *>(pb + a.t.vals_off)[slot];
      if ((uint32_t)(v >> 48) != tu) continue;
      if (key_eq<KW>(pb + a.t.keys_off + (uint64_t)slot * KW * 8, km)) {
        const int32_t prio = (int32_t)(uint32_t)v;
        if (prio >= best) {
          best = prio;
          gate = (uint32_t)(v >> 32) & 0xFFFFu;
        }
        break;
      }
    }
  }
  return gate;
}

template <int KW>
__global__ __launch_bounds__(kEmBlock) void wm_classify_kernel(WmArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  if (a.t.lds) copy_table_to_lds(lds, a.t);
  const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < a.n;
       i += nthr) {
    uint64_t k[KW];
    build_key<KW>(a.frames + i * a.stride, a.fp, k);
    uint32_t g;
    if (a.t.lds)
      g = wm_lookup<KW>(lds, a, k);
    else
      g = wm_lookup<KW>(a.t.base, a, k);
    a.gates[i] = (uint16_t)g;
  }
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
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t fold16(uint32_t s) {
  s = (s & 0xFFFFu) + (s >> 16);
  s = (s & 0xFFFFu) + (s >> 16);
  return s;
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
  const uint32_t v = dw & m;
  return (v & 0xFFFFu) + (v >> 16);
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

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__global__ __launch_bounds__(kCkBlock) void cksum_kernel(CkArgs a) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave0 = __builtin_amdgcn_readfirstlane(
      ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6);
  const uint64_t nwaves = ((uint64_t)gridDim.x * blockDim.x) >> 6;
  const int stride = (int)a.stride;
  for (uint64_t pkt = wave0; pkt < a.n; pkt += nwaves) {
    uint8_t *f = a.frames + pkt * a.stride;
    const uint4 *f16 = reinterpret_cast<const uint4 *>(f);
    uint4 c0 = make_uint4(0, 0, 0, 0);
    if (lane * 16 < stride) c0 = ld_stream(f16 + lane);

    // ---- IPChecksum header walk (ip_checksum.cc:50-74)
    int ip_lo = 0, ip_hi = 0;  // summed IPv4 header range
    int ip_state = 0;          // 0 forward untouched, 1 process IPv4
    int ip_off = 14;
    if (a.mode & 1) {
      uint32_t et = hdr_be16(c0, 12);
      bool fwd = false;
      if (et == 0x88a8) {
        et = hdr_be16(c0, ip_off + 2);
        ip_off += 4;
        if (et != 0x8100) fwd = true;
      }
      if (!fwd && et == 0x8100) {
        et = hdr_be16(c0, ip_off + 2);
        ip_off += 4;
      }
      if (!fwd && et == 0x0800) {
        ip_state = 1;
        const int hl = (int)(hdr_u8(c0, ip_off) & 15) * 4;
        if (hl >= 20) {
          ip_lo = ip_off;
          ip_hi = ip_off + hl;
        }
      }
    }
    // ---- L4Checksum header walk (l4_checksum.cc:53-82): untagged only
    int l4_lo = 0, l4_hi = 0, l4_kind = 0;  // 0 forward, 1 udp, 2 tcp, 3 none
    int l4_off = 0, l4_len = 0, l4_ck = 0;
    bool l4_valid = false;
    if (a.mode & 2) {
      if (hdr_be16(c0, 12) == 0x0800) {
        const int hl = (int)(hdr_u8(c0, 14) & 15) * 4;
        const uint32_t proto = hdr_u8(c0, 23);
        l4_off = 14 + hl;
        if (proto == 17) {
          l4_kind = 1;
          l4_len = (int)hdr_be16(c0, l4_off + 4);
          l4_valid = l4_len >= 8;
          l4_ck = l4_off + 6;
        } else if (proto == 6) {
          l4_kind = 2;
          const int ip_len = (int)hdr_be16(c0, 16);
          l4_valid = ip_len >= hl + 20;
          l4_len = (ip_len - hl) & 0xFFFF;
          l4_ck = l4_off + 16;
        } else {
          l4_kind = 3;
        }
        if (l4_valid) {
          l4_lo = l4_off;
          l4_hi = l4_off + l4_len;
          if (l4_hi > stride) l4_hi = stride;  // reference reads past (UB)
        }
      }
    }
    if (ip_hi > stride) ip_hi = stride;

    // ---- one pass over the frame: both range sums
    const int end = ip_hi > l4_hi ? ip_hi : l4_hi;
    uint32_t s_ip = 0, s_l4 = 0;
    for (int base = 0; base < end; base += 1024) {
      uint4 c;
      const int o = base + lane * 16;
      if (base == 0) {
        c = c0;
      } else {
        c = make_uint4(0, 0, 0, 0);
        if (o < end) c = ld_stream(f16 + (o >> 4));
      }
      s_ip += range_sum(c.x, o, ip_lo, ip_hi) + range_sum(c.y, o + 4, ip_lo, ip_hi) +
              range_sum(c.z, o + 8, ip_lo, ip_hi) + range_sum(c.w, o + 12, ip_lo, ip_hi);
      s_l4 += range_sum(c.x, o, l4_lo, l4_hi) + range_sum(c.y, o + 4, l4_lo, l4_hi) +
              range_sum(c.z, o + 8, l4_lo, l4_hi) + range_sum(c.w, o + 12, l4_lo, l4_hi);
    }
    s_ip = wave_sum(s_ip);
    s_l4 = wave_sum(s_l4);

    // ---- IPChecksum result (checksum.h:254-318)
    uint32_t ip_gate = 0;
    bool ip_wrote = false;
    uint32_t ip_new = 0;  // value written at ip_off+10 (LE u16)
    if (ip_state == 1) {
      if (ip_hi == 0) {  // IHL < 5
        if (a.verify) {
          ip_gate = 1;
        } else {
          ip_wrote = true;
          ip_new = 0;
        }
      } else if (a.verify) {
        ip_gate = fold16(s_ip) == 0xFFFFu ? 0u : 1u;
      } else {
        const uint32_t old = hdr_le16(c0, ip_off + 10);
        ip_wrote = true;
        ip_new = (~fold16(s_ip - old)) & 0xFFFFu;
      }
      if (ip_wrote && lane == 0) {
        f[ip_off + 10] = (uint8_t)ip_new;
        f[ip_off + 11] = (uint8_t)(ip_new >> 8);
      }
    }
    // ---- L4Checksum result (checksum.h:324-504)
    uint32_t l4_gate = kGateNone;
    const bool l4_runs = (a.mode & 2) && (!(a.mode & 1) || ip_gate == 0);
    if (l4_runs) {
      if (l4_kind == 0) {
        l4_gate = 0;
      } else if (l4_kind == 3) {
        l4_gate = kGateNone;
      } else {
        // pseudo header: src, dst (LE u16 words of the BE addresses),
        // bswap16(length), and the protocol word 0x1100 / 0x0600
        const uint32_t ps = hdr_le16(c0, 26) + hdr_le16(c0, 28) +
                            hdr_le16(c0, 30) + hdr_le16(c0, 32) +
                            (((uint32_t)l4_len >> 8) | (((uint32_t)l4_len & 0xFF) << 8)) +
                            (l4_kind == 1 ? 0x1100u : 0x0600u);
        uint32_t old = l4_valid ? hdr_le16(c0, l4_ck) : 0u;
        // Pipeline order: L4Checksum sees IPChecksum's write. With IHL < 5
        // the "L4 header" overlaps the IP checksum bytes 24..25.
        if ((a.mode & 1) && ip_wrote && ip_off == 14) {
          const uint32_t old_ip = hdr_le16(c0, 24);
#pragma unroll
          for (int b = 24; b < 26; b++) {
            if (b >= l4_lo && b < l4_hi) {
              const int sh = (b & 1) * 8;
              s_l4 = s_l4 - (((old_ip >> sh) & 0xFFu) << sh) +
                     (((ip_new >> sh) & 0xFFu) << sh);
            }
          }
          if (l4_valid && l4_ck == 24) old = ip_new;
        }
        if (a.verify) {
          if (!l4_valid) {
            l4_gate = 1;
          } else if (l4_kind == 1 && old == 0) {
            l4_gate = 0;  // UDP checksum 0 = not computed (checksum.h:328-331)
          } else {
            l4_gate = fold16(s_l4 + ps) == 0xFFFFu ? 0u : 1u;
          }
        } else {
          uint32_t ck = 0;
          if (l4_valid) {
            ck = (~fold16(s_l4 - old + ps)) & 0xFFFFu;
            if (l4_kind == 1 && ck == 0) ck = 0xFFFFu;  // RFC 768
          }
          // a UDP length < 8 / bad TCP length writes 0 at the field
          const int at = l4_kind == 1 ? l4_off + 6 : l4_off + 16;
          if (lane == 0 && at + 2 <= stride) {
            f[at] = (uint8_t)ck;
            f[at + 1] = (uint8_t)(ck >> 8);
          }
          l4_gate = l4_kind == 1 ? 0u : kGateNone;  // TCP: never emitted
        }
      }
    }
    if (lane == 0) {
      if (a.ip_gates) a.ip_gates[pkt] = (a.mode & 1) ? (uint16_t)ip_gate : kGateNone;
      if (a.l4_gates) a.l4_gates[pkt] = (uint16_t)l4_gate;
    }
  }
}

template <typename Args, typename K>
hipError_t launch_classify(K kernel, const Args &a, int num_cus,
                           hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  uint64_t blocks = (a.n + kEmBlock - 1) / kEmBlock;
  uint64_t cap = (uint64_t)num_cus * (a.t.lds ? 4 : 8);
  if (blocks > cap) blocks = cap;
  const size_t lds = a.t.lds ? a.t.bytes_total : 0;
  hipLaunchKernelGGL(kernel, dim3((unsigned)blocks), dim3(kEmBlock), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_em(const EmArgs &a, int num_cus, hipStream_t s) {
  switch (a.t.kw) {
    case 1: return launch_classify(em_classify_kernel<1>, a, num_cus, s);
    case 2: return launch_classify(em_classify_kernel<2>, a, num_cus, s);
    case 4: return launch_classify(em_classify_kernel<4>, a, num_cus, s);
    case 8: return launch_classify(em_classify_kernel<8>, a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_wm(const WmArgs &a, int num_cus, hipStream_t s) {
  switch (a.t.kw) {
    case 1: return launch_classify(wm_classify_kernel<1>, a, num_cus, s);
    case 2: return launch_classify(wm_classify_kernel<2>, a, num_cus, s);
    case 4: return launch_classify(wm_classify_kernel<4>, a, num_cus, s);
    case 8: return launch_classify(wm_classify_kernel<8>, a, num_cus, s);
    default: return hipErrorInvalidValue;
  }
}

hipError_t launch_cksum(const CkArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const uint64_t waves_per_block = kCkBlock / 64;
  uint64_t blocks = (a.n + waves_per_block - 1) / waves_per_block;
  const uint64_t cap = (uint64_t)num_cus * 8;  // 32 waves/CU
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(cksum_kernel, dim3((unsigned)blocks), dim3(kCkBlock), 0, s,
                     a);
  return hipGetLastError();
}

}  // namespace bg
