// bg_lb.hip -- gfx950 kernel for HashLB::ProcessBatch
// (core/modules/hash_lb.cc:155-236): per packet, the mode's hash input
//   l2     : XOR of the six LE u16 words of the MAC addresses (152-170),
//            CRC32C of those 2 bytes (hash_16, 35-41);
//   l3     : src IP ^ dst IP as LE u32 (174-190), CRC32C of 4 bytes (43-49);
//   l4     : l3 ^ src port ^ dst port (LE u16, at 14 + IHL*4) ^ ip proto
//            (194-219), CRC32C of 4 bytes;
//   fields : the ExactMatchTable::MakeKeys key (134-150), CRC32C over its
//            total_key_size / 8 u64 words (ExactMatchKeyHash,
//            exact_match_table.h:97-119);
// then EmitPacket(gates_[hash_range(crc, num_gates_)]), hash_range = the
// top bits of crc * num_gates (53-68: (1.b0..b31 - 1.0) * range is exact in
// double, so it equals (crc * range) >> 32).
//
// The GPU has no CRC instruction. With init 0 (every HashLB call site) a
// CRC is linear over GF(2) in its input bytes, so the CRC of an L-byte input
// is the XOR of one 256-entry table per byte position -- L independent LDS
// reads instead of a dependent byte-serial chain. The tables (L x 1 KiB)
// and the gate table are staged in LDS once per workgroup.
#include <hip/hip_runtime.h>

#include <stdlib.h>

#include <algorithm>

#include "bg_kernels.h"
#include "bg_keys_dev.h"

namespace bg {
namespace {

constexpr int kHlbBlock = 512;

__device__ __forceinline__ void hlb_stage_lds(uint32_t *lds, const HlbArgs &a) {
  const uint32_t nt = a.L * 256;  // crc table words
  const uint4 *src = reinterpret_cast<const uint4 *>(a.crc_tab);
  uint4 *dst = reinterpret_cast<uint4 *>(lds);
  for (uint32_t i = threadIdx.x; i < nt / 4; i += blockDim.x) dst[i] = src[i];
  uint16_t *g = reinterpret_cast<uint16_t *>(lds + nt);
  for (uint32_t i = threadIdx.x; i < a.ngtab; i += blockDim.x) g[i] = a.gtab[i];
  __syncthreads();
}

// CRC32C(init 0) of the 4 LE bytes of x: positions 0..3 of an L = 4 table
__device__ __forceinline__ uint32_t crc4(const uint32_t *T, uint32_t x) {
  return T[x & 0xFF] ^ T[256 + ((x >> 8) & 0xFF)] ^ T[512 + ((x >> 16) & 0xFF)] ^
         T[768 + (x >> 24)];
}

// Chunks (16 B) of the first 64 bytes each mode reads.
template <int MODE>
struct HlbChunks {
  static constexpr int lo = MODE == kHlbL3 ? 1 : 0;
  static constexpr int hi = MODE == kHlbL2 ? 1 : MODE == kHlbL3 ? 3 : 4;
};

// The mode's hash from the frame's first 64 bytes d[0..15] (only the
// HlbChunks of it need to be valid); `f` = the frame for the rare l4 read
// past the line.
template <int MODE>
__device__ __forceinline__ uint32_t hlb_crc_line(const HlbArgs &a,
                                                 const uint32_t *T,
                                                 const uint32_t (&d)[16],
                                                 const uint8_t *f) {
  if constexpr (MODE == kHlbL2) {
    const uint32_t x = d[0] ^ d[1] ^ d[2];  // bytes [0, 12): both MACs
    const uint32_t s = (x ^ (x >> 16)) & 0xFFFF;
    return T[s & 0xFF] ^ T[256 + (s >> 8)];
  } else if constexpr (MODE == kHlbL3) {
    // src IP = bytes 26..29, dst IP = bytes 30..33
    const uint32_t src = __builtin_amdgcn_alignbyte(d[7], d[6], 2);
    const uint32_t dst = __builtin_amdgcn_alignbyte(d[8], d[7], 2);
    return crc4(T, src ^ dst);
  } else {
    const uint32_t ihl = (d[3] >> 16) & 0x0F;  // byte 14, low nibble
    const uint32_t v0 = __builtin_amdgcn_alignbyte(d[7], d[6], 2) ^  // src IP
                        __builtin_amdgcn_alignbyte(d[8], d[7], 2) ^  // dst IP
                        (d[5] >> 24);                                // proto
    // ports at l4 = 14 + 4*IHL: src port = high half of dword 3 + IHL,
    // dst port = low half of dword 4 + IHL
    uint32_t sp = 0, dp = 0;
#pragma unroll
    for (int j = 0; j < 12; j++) {
      if (ihl == (uint32_t)j) {
        sp = d[3 + j] >> 16;
        dp = d[4 + j] & 0xFFFF;
      }
    }
    if (ihl >= 12) {  // ports past the 64-byte line (IHL 12..15), read
      // only inside the packet's slot (bytes past it read as zero)
      const uint32_t l4 = 14 + 4 * ihl;
      const uint16_t *q = reinterpret_cast<const uint16_t *>(f + l4);
      sp = l4 + 2 <= a.stride ? q[0] : 0u;
      dp = l4 + 4 <= a.stride ? q[1] : 0u;
    }
    return crc4(T, v0 ^ sp ^ dp);
  }
}

template <int MODE, int KW, int NCH>
__device__ __forceinline__ uint32_t hlb_crc(const HlbArgs &a, const uint32_t *T,
                                            uint64_t idx) {
  const uint8_t *f = a.frames + idx * a.stride;
  if constexpr (MODE != kHlbFields) {
    const uint4 *p = reinterpret_cast<const uint4 *>(f);
    uint32_t d[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c >= HlbChunks<MODE>::lo && c < HlbChunks<MODE>::hi) v = ld_stream(p + c);
      d[4 * c] = v.x;
      d[4 * c + 1] = v.y;
      d[4 * c + 2] = v.z;
      d[4 * c + 3] = v.w;
    }
    return hlb_crc_line<MODE>(a, T, d, f);
  } else {
    uint64_t k[1][KW];
    build_keys<KW, NCH, 1>(a.frames, a.stride, a.n, idx, a.fp, k);
    uint32_t crc = 0;
    const uint32_t nw = a.L / 8;
#pragma unroll
    for (int j = 0; j < KW; j++) {
      if ((uint32_t)j < nw) {
        const uint64_t w = k[0][j];
#pragma unroll
        for (int b = 0; b < 8; b++)
          crc ^= T[(8 * j + b) * 256 + (uint32_t)((w >> (8 * b)) & 0xFF)];
      }
    }
    return crc;
  }
}

template <int MODE, int KW, int NCH>
__global__ __launch_bounds__(kHlbBlock) void hlb_kernel(HlbArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  hlb_stage_lds(lds, a);
  const uint16_t *g = reinterpret_cast<const uint16_t *>(lds + a.L * 256);
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < a.n;
       idx += step) {
    const uint32_t crc = hlb_crc<MODE, KW, NCH>(a, lds, idx);
    a.out[idx] = g[(uint32_t)(((uint64_t)crc * a.num_gates) >> 32)];
  }
}

// Dense 64-byte slots (stride 64, l2/l3/l4): a wave reads 64 slots = 4 KB
// with lane-contiguous 16-byte loads (the coalesced shape that streams the
// slab fastest, see em_slab_kernel in bg_kernels.hip) into a swizzled
// per-wave LDS stage, then each lane takes its own slot's chunks from LDS.
// The next tile's loads are in flight while this one is hashed.
__device__ __forceinline__ uint32_t hlb_stage_unit(uint32_t slot, uint32_t q) {
  return slot * 4 + ((q + (slot >> 2)) & 3);
}

template <int MODE>
__global__ __launch_bounds__(kHlbBlock) void hlb_slab_kernel(HlbArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  hlb_stage_lds(lds, a);
  const uint32_t tab_words = (a.L * 256 + ((a.ngtab + 1) >> 1) + 3) & ~3u;
  const uint16_t *g = reinterpret_cast<const uint16_t *>(lds + a.L * 256);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kWaves = kHlbBlock / 64;
  uint4 *stage = reinterpret_cast<uint4 *>(lds + tab_words) + wid * 256;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t ntiles = (a.n + 63) / 64;
  const uint4 *src = reinterpret_cast<const uint4 *>(a.frames);
  constexpr int c0 = HlbChunks<MODE>::lo, c1 = HlbChunks<MODE>::hi;
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint4 v[4];
  auto load_tile = [&](uint64_t tile) {
    const uint64_t p0 = tile * 64;
    const uint64_t units = (a.n - p0 < 64 ? a.n - p0 : 64) * 4;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      const uint32_t q = u & 3;  // chunk of the slot this unit holds
      v[c] = (u < units && q >= (uint32_t)c0 && q < (uint32_t)c1)
                 ? ld_stream(src + p0 * 4 + u)
                 : make_uint4(0, 0, 0, 0);
    }
  };
  if (t < ntiles) load_tile(t);
  for (; t < ntiles; t += nwaves) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[hlb_stage_unit(u >> 2, u & 3)] = v[c];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (t + nwaves < ntiles) load_tile(t + nwaves);
    uint32_t d[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint4 x = make_uint4(0, 0, 0, 0);
      if (c >= c0 && c < c1) x = stage[hlb_stage_unit(lane, c)];
      d[4 * c] = x.x;
      d[4 * c + 1] = x.y;
      d[4 * c + 2] = x.z;
      d[4 * c + 3] = x.w;
    }
    const uint64_t idx = t * 64 + lane;
    if (idx < a.n) {
      const uint32_t crc = hlb_crc_line<MODE>(a, lds, d, a.frames + idx * 64);
      a.out[idx] = g[(uint32_t)(((uint64_t)crc * a.num_gates) >> 32)];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

template <int MODE>
hipError_t launch_hlb_slab(const HlbArgs &a, int num_cus, hipStream_t s) {
  auto kern = hlb_slab_kernel<MODE>;
  const size_t tab = ((size_t)a.L * 1024 + ((size_t)a.ngtab * 2 + 15) / 16 * 16);
  const size_t lds = tab + (size_t)(kHlbBlock / 64) * 4096;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &occ, reinterpret_cast<const void *>(kern), kHlbBlock, lds) != hipSuccess ||
      occ <= 0)
    occ = 1;
  const uint64_t need = (a.n + kHlbBlock - 1) / kHlbBlock;
  const uint64_t blocks = std::max<uint64_t>(1, std::min(need, (uint64_t)num_cus * occ));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kHlbBlock), lds, s, a);
  return hipGetLastError();
}

template <int MODE, int KW, int NCH>
hipError_t launch_hlb_t(const HlbArgs &a, int num_cus, hipStream_t s) {
  auto kern = hlb_kernel<MODE, KW, NCH>;
  const size_t lds = (size_t)a.L * 1024 + ((size_t)a.ngtab * 2 + 15) / 16 * 16;
  int occ = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &occ, reinterpret_cast<const void *>(kern), kHlbBlock, lds) != hipSuccess ||
      occ <= 0)
    occ = 1;
  const uint64_t need = (a.n + kHlbBlock - 1) / kHlbBlock;
  const uint64_t cap = (uint64_t)num_cus * occ;
  const uint64_t blocks = std::max<uint64_t>(1, std::min(need, cap));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kHlbBlock), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_hlb(const HlbArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const bool slab = a.stride == 64 && ((uintptr_t)a.frames & 15) == 0 &&
                    !getenv("BG_NO_SLAB");
  if (slab) {
    switch (a.mode) {
      case kHlbL2: return launch_hlb_slab<kHlbL2>(a, num_cus, s);
      case kHlbL3: return launch_hlb_slab<kHlbL3>(a, num_cus, s);
      case kHlbL4: return launch_hlb_slab<kHlbL4>(a, num_cus, s);
      default: break;
    }
  }
  switch (a.mode) {
    case kHlbL2: return launch_hlb_t<kHlbL2, 1, 0>(a, num_cus, s);
    case kHlbL3: return launch_hlb_t<kHlbL3, 1, 0>(a, num_cus, s);
    case kHlbL4: return launch_hlb_t<kHlbL4, 1, 0>(a, num_cus, s);
    default: break;
  }
  int maxops = 0;
  for (int q = 0; q < a.fp.nkd; q++) maxops = std::max(maxops, kd_nops_of(a.fp, q));
  const int nch = a.fp.direct ? 0 : (a.fp.nch <= 2 && maxops <= 2 ? 2 : 4);
  const int w8 = (int)(a.L + 7) / 8;
  const int kw = w8 <= 1 ? 1 : w8 <= 2 ? 2 : w8 <= 4 ? 4 : 8;
#define BG_HLB(KW, NCH) \
  if (kw == KW && nch == NCH) return launch_hlb_t<kHlbFields, KW, NCH>(a, num_cus, s);
#define BG_HLB_K(KW) BG_HLB(KW, 0) BG_HLB(KW, 2) BG_HLB(KW, 4)
  BG_HLB_K(1) BG_HLB_K(2) BG_HLB_K(4) BG_HLB_K(8)
#undef BG_HLB_K
#undef BG_HLB
  return hipErrorInvalidValue;
}

}  // namespace bg
