// bg_lb.hip -- gfx950 kernels for HashLB::ProcessBatch
// (core/modules/hash_lb.cc:140-236): per packet, the mode's hash input
//   l2     : XOR of the six LE u16 words of the MAC addresses (152-170),
//            CRC32C of those 2 bytes (hash_16, 35-41);
//   l3     : src IP ^ dst IP as LE u32 (174-190), CRC32C of 4 bytes (43-49);
//   l4     : l3 ^ src port ^ dst port (LE u16, at 14 + IHL*4) ^ ip proto
//            (194-219), CRC32C of 4 bytes;
//   fields : the ExactMatchTable::MakeKeys key (140-150), CRC32C over its
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
// and the gate table are staged in LDS once per workgroup. l2/l3/l4 run as
// header-line ops (bg_line_dev.h: coalesced slab kernel for 64 B slots).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bg_kernels.h"
#include "bg_keys_dev.h"
#include "bg_line_dev.h"

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
}

// CRC32C(init 0) of the 4 LE bytes of x: positions 0..3 of an L = 4 table
__device__ __forceinline__ uint32_t crc4(const uint32_t *T, uint32_t x) {
  return T[x & 0xFF] ^ T[256 + ((x >> 8) & 0xFF)] ^ T[512 + ((x >> 16) & 0xFF)] ^
         T[768 + (x >> 24)];
}

// l2/l3/l4 as header-line ops
template <int MODE>
struct HlbOp {
  using Args = HlbArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 1;
  // 16-byte chunks of the first 64 bytes each mode reads
  static constexpr int c0 = MODE == kHlbL3 ? 1 : 0;
  static constexpr int c1 = MODE == kHlbL2 ? 1 : MODE == kHlbL3 ? 3 : 4;
  static size_t lds_bytes(const HlbArgs &x) {
    return (size_t)x.L * 1024 + ((size_t)x.ngtab * 2 + 15) / 16 * 16;
  }
  __device__ static void stage(uint32_t *lds, const HlbArgs &x) {
    hlb_stage_lds(lds, x);
  }
  __device__ static uint32_t decide(const HlbArgs &x, const uint32_t *T,
                                    uint32_t (&d)[16], uint8_t *f) {
    uint32_t crc;
    if constexpr (MODE == kHlbL2) {
      const uint32_t v = d[0] ^ d[1] ^ d[2];  // bytes [0, 12): both MACs
      const uint32_t s = (v ^ (v >> 16)) & 0xFFFF;
      crc = T[s & 0xFF] ^ T[256 + (s >> 8)];
    } else if constexpr (MODE == kHlbL3) {
      crc = crc4(T, ip_src_le(d) ^ ip_dst_le(d));
    } else {
      const uint32_t p = l4_ports(d, f, x.stride);
      crc = crc4(T, ip_src_le(d) ^ ip_dst_le(d) ^ (d[5] >> 24) /* proto */ ^
                        (p & 0xFFFF) ^ (p >> 16));
    }
    const uint16_t *g = reinterpret_cast<const uint16_t *>(T + x.L * 256);
    return g[(uint32_t)(((uint64_t)crc * x.num_gates) >> 32)];
  }
};

// fields mode as a header-line op (the fields inside the frame's first 64
// bytes): the line arrives through the slab kernel's lane-contiguous loads,
// the key window is cut from it at the plan's (16-byte aligned) start --
// a uniform branch per possible start, so every register index is a
// constant -- then MakeKeys and the byte-table CRC as below
template <int KW, int NCH>
struct HlbFieldsOp {
  using Args = HlbArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 1;
  static constexpr int c0 = 0, c1 = 4;
  static size_t lds_bytes(const HlbArgs &x) { return HlbOp<kHlbL4>::lds_bytes(x); }
  __device__ static void stage(uint32_t *lds, const HlbArgs &x) { hlb_stage_lds(lds, x); }
  __device__ static uint32_t decide(const HlbArgs &x, const uint32_t *T,
                                    uint32_t (&d)[16], uint8_t *) {
    uint32_t w[NCH * 4 + 2];
    const uint32_t c = (uint32_t)x.fp.win_lo >> 4;  // wave-uniform
#pragma unroll
    for (int cc = 0; cc < 4; cc++) {
      if (c == (uint32_t)cc) {
#pragma unroll
        for (int i = 0; i < NCH * 4; i++) w[i] = 4 * cc + i < 16 ? d[4 * cc + i] : 0u;
      }
    }
    w[NCH * 4] = 0;
    w[NCH * 4 + 1] = 0;
    uint64_t k[KW];
    extract_key<KW, NCH>(w, x.fp, k);
    const uint32_t nw = x.L / 8;
    uint32_t crc = 0;
#pragma unroll
    for (int j = 0; j < KW; j++) {
      if ((uint32_t)j < nw) {
#pragma unroll
        for (int b = 0; b < 8; b++)
          crc ^= T[(8 * j + b) * 256 + (uint32_t)((k[j] >> (8 * b)) & 0xFF)];
      }
    }
    const uint16_t *g = reinterpret_cast<const uint16_t *>(T + x.L * 256);
    return g[(uint32_t)(((uint64_t)crc * x.num_gates) >> 32)];
  }
};

// fields mode: MakeKeys key, CRC over its first L bytes
template <int KW, int NCH>
__global__ __launch_bounds__(kHlbBlock) void hlb_fields_kernel(HlbArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  hlb_stage_lds(lds, a);
  __syncthreads();
  const uint16_t *g = reinterpret_cast<const uint16_t *>(lds + a.L * 256);
  const uint32_t nw = a.L / 8;
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t idx = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < a.n;
       idx += step) {
    uint64_t k[1][KW];
    build_keys<KW, NCH, 1>(a.frames, a.stride, a.n, idx, a.fp, k);
    uint32_t crc = 0;
#pragma unroll
    for (int j = 0; j < KW; j++) {
      if ((uint32_t)j < nw) {
        const uint64_t w = k[0][j];
#pragma unroll
        for (int b = 0; b < 8; b++)
          crc ^= lds[(8 * j + b) * 256 + (uint32_t)((w >> (8 * b)) & 0xFF)];
      }
    }
    a.out[idx] = g[(uint32_t)(((uint64_t)crc * a.num_gates) >> 32)];
  }
}

template <int KW, int NCH>
hipError_t launch_hlb_fields(const HlbArgs &a, int num_cus, hipStream_t s) {
  auto kern = hlb_fields_kernel<KW, NCH>;
  const size_t lds = HlbOp<kHlbL4>::lds_bytes(a);
  const int occ = line_occupancy(reinterpret_cast<const void *>(kern), lds);
  const uint64_t need = (a.n + kHlbBlock - 1) / kHlbBlock;
  const uint64_t blocks = std::max<uint64_t>(1, std::min(need, (uint64_t)num_cus * occ));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kHlbBlock), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_hlb(const HlbArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  switch (a.mode) {
    case kHlbL2: return launch_line<HlbOp<kHlbL2>>(a, num_cus, s);
    case kHlbL3: return launch_line<HlbOp<kHlbL3>>(a, num_cus, s);
    case kHlbL4: return launch_line<HlbOp<kHlbL4>>(a, num_cus, s);
    default: break;
  }
  int maxops = 0;
  for (int q = 0; q < a.fp.nkd; q++) maxops = std::max(maxops, kd_nops_of(a.fp, q));
  const int nch = a.fp.direct ? 0 : (a.fp.nch <= 2 && maxops <= 2 ? 2 : 4);
  const int w8 = (int)(a.L + 7) / 8;
  const int kw = w8 <= 1 ? 1 : w8 <= 2 ? 2 : w8 <= 4 ? 4 : 8;
  // the fields inside the first 64 bytes of dense 64 B slots: a line op on
  // the slab kernel's lane-contiguous loads (wider strides keep the
  // lane-per-packet kernel, which loads only the window's chunks)
  const bool line = nch > 0 && a.fp.win_lo + 16 * nch <= 64 && a.stride == 64 &&
                    ((uintptr_t)a.frames & 15) == 0 && !(path_flags() & kPathNoSlab);
#define BG_HLB(KW, NCH)                                                       \
  if (kw == KW && nch == NCH)                                                 \
    return line && NCH > 0 ? launch_line<HlbFieldsOp<KW, (NCH > 0 ? NCH : 2)>>(a, num_cus, s) \
                           : launch_hlb_fields<KW, NCH>(a, num_cus, s);
#define BG_HLB_K(KW) BG_HLB(KW, 0) BG_HLB(KW, 2) BG_HLB(KW, 4)
  BG_HLB_K(1) BG_HLB_K(2) BG_HLB_K(4) BG_HLB_K(8)
#undef BG_HLB_K
#undef BG_HLB
  return hipErrorInvalidValue;
}

}  // namespace bg
