// bg_line_dev.h -- generic "header-line" packet kernels: one decision per
// packet from the frame's first 64 bytes (HashLB l2/l3/l4, ACL, IPLookup,
// UpdateTTL). Included only from .hip translation units.
//
// An Op provides
//   using Args = ...;   // with frames, stride, n, out (uint16_t per packet)
//   static constexpr int c0, c1;   // 16-byte chunks [c0, c1) of the line used
//   static constexpr bool kWrites;  // d[] chunks [c0, c1) are written back
//   static constexpr int kSlabPerCu;  // line_slab_kernel workgroups per CU
//   static size_t lds_bytes(const Args &);            (host) tables in LDS
//   __device__ static void stage(uint32_t *lds, const Args &);   fill them
//   __device__ static uint32_t decide(const Args &, const uint32_t *lds,
//                                     uint32_t (&d)[16], uint8_t *f);
// d[] holds the line's dwords (only chunks [c0, c1) valid; a writing op
// updates them in place); f is the frame (for rare reads past the line).
// Writing ops store the chunks back whole -- through the LDS stage as
// lane-contiguous 16-byte stores in the slab kernel -- never partial dwords.
//
// Two launch shapes:
//   line_kernel      one packet per lane, its chunks loaded directly (any
//                    16-byte-multiple stride >= 64);
//   line_slab_kernel dense 64-byte slots (stride 64): a wave reads 64 slots
//                    = 4 KB with lane-contiguous 16-byte loads into a
//                    swizzled per-wave LDS stage (slot s keeps chunk q at
//                    unit 4s + ((q + s/4) & 3): conflict-free writes and
//                    per-slot reads), each lane then takes its own slot from
//                    LDS; the next tile's loads are in flight meanwhile.
//                    Lane-contiguous loads stream the slab at ~7.1 TB/s where
//                    slot-per-lane 16-byte loads reach ~5 TB/s
//                    (scripts/hbm_probe.hip).
#ifndef BESS_AMD_BG_LINE_DEV_H_
#define BESS_AMD_BG_LINE_DEV_H_

#include <hip/hip_runtime.h>

#include <algorithm>

#include "bg_kernels.h"
#include "bg_keys_dev.h"
#include "bg_launch.h"

namespace bg {
namespace {

constexpr int kLineBlock = 512;

__device__ __forceinline__ uint32_t line_stage_unit(uint32_t slot, uint32_t q) {
  return slot * 4 + ((q + (slot >> 2)) & 3);
}

// A reading op's lane holds kLineHold grid-stride results in registers and
// stores them together, nontemporally, after their lookups (as the slab
// kernels' held gates; round 6: IPLookup with tbl16 in LDS 0.2148 -> 0.1770
// ms, 8 held 0.1810, profiles/r06/lpm_ab_r06q.json).
constexpr int kLineHold = 16;

template <class Op, int kBlock = kLineBlock>
__global__ __launch_bounds__(kBlock) void line_kernel(typename Op::Args a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  Op::stage(lds, a);
  __syncthreads();
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  constexpr int H = Op::kWrites ? 1 : kLineHold;
  for (uint64_t i0 = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i0 < a.n;
       i0 += step * H) {
  uint16_t held[H];
#pragma unroll
  for (int h = 0; h < H; h++) {
    const uint64_t idx = i0 + (uint64_t)h * step;
    held[h] = 0;
    if (idx >= a.n) break;
    uint8_t *f = const_cast<uint8_t *>(a.frames) + idx * a.stride;
    const uint4 *p = reinterpret_cast<const uint4 *>(f);
    uint32_t d[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint4 v = make_uint4(0, 0, 0, 0);
      if (c >= Op::c0 && c < Op::c1) v = ld_stream(p + c);
      d[4 * c] = v.x;
      d[4 * c + 1] = v.y;
      d[4 * c + 2] = v.z;
      d[4 * c + 3] = v.w;
    }
    held[h] = (uint16_t)Op::decide(a, lds, d, f);
    if constexpr (Op::kWrites) {
      uint4 *q = reinterpret_cast<uint4 *>(f);
#pragma unroll
      for (int c = Op::c0; c < Op::c1; c++)
        q[c] = make_uint4(d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]);
    }
  }
#pragma unroll
  for (int h = 0; h < H; h++) {
    const uint64_t idx = i0 + (uint64_t)h * step;
    if (idx < a.n) __builtin_nontemporal_store(held[h], a.out + idx);
  }
  }
}

// The written-back lines are stored nontemporally (streaming stores:
// UpdateTTL 0.4093 -> 0.3879 ms, StaticNAT 0.4131 -> 0.3908 per 16 M
// packets, scripts/variants.py linew, profiles/r05/linew_r05n.json).
// A reading op's wave holds its tiles' results and stores them together
// after those tiles' reads (as em_slab_kernel): at one workgroup per CU
// (kSlabPerCu 1) in LDS, line_hold_tiles() tiles (HashLB l4 0.1653 ->
// 0.1605 ms, profiles/r06/legs_ab_r06r.json), otherwise kGateHold tiles in
// registers (HashLB l4 0.1811 -> 0.1635 ms at one workgroup per CU, ACL
// 0.2157 -> 0.1910 at two, legs_ab_r06o.json; ACL holding in LDS at two
// measured slower, 0.2019 against 0.1978; ACL at three or four workgroups
// per CU 0.209-0.212 against 0.192-0.196, acl_occ_ab_r06ao.json). A
// writing op stores each tile's
// (its line stores are per tile anyway: holding measured no better).
template <class Op>
__host__ __device__ constexpr uint32_t line_hold_tiles(uint32_t tab_bytes) {
  return Op::kWrites || Op::kSlabPerCu != 1 ? 0u : lds_hold_tiles(tab_bytes);
}

template <class Op>
__global__ __launch_bounds__(kLineBlock) void line_slab_kernel(typename Op::Args a,
                                                              uint32_t stage_words) {
  static_assert(kLineBlock == 512, "lds_hold_tiles sizes 8 waves' stages");
  extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
  Op::stage(lds, a);
  __syncthreads();
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kWaves = kLineBlock / 64;
  uint4 *stage = reinterpret_cast<uint4 *>(lds + stage_words) + wid * 256;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t ntiles = (a.n + 63) / 64;
  const uint4 *src = reinterpret_cast<const uint4 *>(a.frames);
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint4 v[4];
  auto load_tile = [&](uint64_t tile) {
    const uint64_t p0 = tile * 64;
    const uint64_t units = (a.n - p0 < 64 ? a.n - p0 : 64) * 4;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      const uint32_t q = u & 3;  // chunk of the slot this unit holds
      v[c] = (u < units && q >= (uint32_t)Op::c0 && q < (uint32_t)Op::c1)
                 ? ld_stream(src + p0 * 4 + u)
                 : make_uint4(0, 0, 0, 0);
    }
  };
  // tile tt (its loads in v): staged, the next tile's loads issued, this
  // lane's slot decided (a writing op's tile written back); returns the
  // lane's result (0 past n)
  auto tile_result = [&](uint64_t tt) -> uint32_t {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[line_stage_unit(u >> 2, u & 3)] = v[c];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (tt + nwaves < ntiles) load_tile(tt + nwaves);
    uint32_t d[16];
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint4 x = make_uint4(0, 0, 0, 0);
      if (c >= Op::c0 && c < Op::c1) x = stage[line_stage_unit(lane, c)];
      d[4 * c] = x.x;
      d[4 * c + 1] = x.y;
      d[4 * c + 2] = x.z;
      d[4 * c + 3] = x.w;
    }
    const uint64_t idx = tt * 64 + lane;
    uint32_t r = 0;
    if (idx < a.n) {
      uint8_t *f = const_cast<uint8_t *>(a.frames) + idx * 64;
      r = Op::decide(a, lds, d, f);
    }
    if constexpr (Op::kWrites) {
      // updated chunks back into this lane's slot of the stage, then the
      // tile leaves with lane-contiguous 16-byte stores (whole chunks) of
      // the slots the op changed: a slot left as it was is not written back
      // (StaticNAT with half its packets translated 0.3700-0.3712 -> 0.3214-
      // 0.3229 ms per 16 M packets, UpdateTTL unchanged, bit-exact;
      // profiles/r06/line_clean_ab_r06aq.json)
      bool mod = false;
#pragma unroll
      for (int c = Op::c0; c < Op::c1; c++) {
        const uint4 o = stage[line_stage_unit(lane, c)];
        mod |= o.x != d[4 * c] || o.y != d[4 * c + 1] || o.z != d[4 * c + 2] ||
               o.w != d[4 * c + 3];
        stage[line_stage_unit(lane, c)] =
            make_uint4(d[4 * c], d[4 * c + 1], d[4 * c + 2], d[4 * c + 3]);
      }
      const uint64_t dirty = __ballot(mod);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      const uint64_t p0 = tt * 64;
      const uint64_t units = (a.n - p0 < 64 ? a.n - p0 : 64) * 4;
      uint4 *dst = reinterpret_cast<uint4 *>(const_cast<uint8_t *>(a.frames));
#pragma unroll
      for (int c = 0; c < 4; c++) {
        const uint32_t u = c * 64 + lane;
        const uint32_t q = u & 3;
        if (u < units && q >= (uint32_t)Op::c0 && q < (uint32_t)Op::c1 &&
            ((dirty >> (u >> 2)) & 1))
          st_stream(dst + p0 * 4 + u, stage[line_stage_unit(u >> 2, q)]);
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return r;
  };
  if (t < ntiles) load_tile(t);
  const uint32_t hl = line_hold_tiles<Op>(stage_words * 4);
  if (hl) {  // (a multiple of 8; the launch sized the LDS for it)
    uint16_t *hold = reinterpret_cast<uint16_t *>(lds + stage_words + kWaves * 1024) +
                     (size_t)wid * hl * 64;
    for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * hl) {
#pragma unroll 1
      for (uint32_t h = 0; h < hl; h++) {
        const uint64_t tt = t0 + (uint64_t)h * nwaves;
        if (tt >= ntiles) break;
        hold[h * 64 + lane] = (uint16_t)tile_result(tt);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      store_held(hold, hl, t0, nwaves, lane, a.out, a.n);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    return;
  }
  // (an op at one workgroup per CU holds in LDS above unless its tables
  // leave no room: then per-tile stores, and no unrolled register hold)
  constexpr int H = Op::kWrites || Op::kSlabPerCu == 1 ? 1 : kGateHold;
  for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * H) {
    uint16_t held[H];
#pragma unroll
    for (int h = 0; h < H; h++) {
      const uint64_t tt = t0 + (uint64_t)h * nwaves;
      held[h] = 0;
      if (tt >= ntiles) break;
      held[h] = (uint16_t)tile_result(tt);
    }
#pragma unroll
    for (int h = 0; h < H; h++) {  // streaming stores, as em_slab_kernel's gates
      const uint64_t idx = (t0 + (uint64_t)h * nwaves) * 64 + lane;
      if (idx < a.n) __builtin_nontemporal_store(held[h], a.out + idx);
    }
  }
}

// The 4 bytes at l4 = 14 + 4*IHL (untagged IPv4: src port, dst port) as a
// LE dword, from the line d[] (IHL = low nibble of byte 14). l4 = 4*(3+IHL)
// + 2, so they are the high half of dword 3+IHL and the low half of dword
// 4+IHL; IHL 12..15 reach past the line and are read from the frame, only
// inside its slot (bytes past `stride` read as zero).
__device__ __forceinline__ uint32_t l4_ports(uint32_t (&d)[16],
                                             const uint8_t *f, uint64_t stride) {
  const uint32_t ihl = (d[3] >> 16) & 0x0F;
  uint32_t p = 0;
#pragma unroll
  for (int j = 0; j < 12; j++)
    if (ihl == (uint32_t)j) p = (d[3 + j] >> 16) | (d[4 + j] << 16);
  if (ihl >= 12) {
    const uint32_t l4 = 14 + 4 * ihl;
    const uint16_t *q = reinterpret_cast<const uint16_t *>(f + l4);
    const uint32_t sp = l4 + 2 <= stride ? q[0] : 0u;
    const uint32_t dp = l4 + 4 <= stride ? q[1] : 0u;
    p = sp | (dp << 16);
  }
  return p;
}

// IPv4 src / dst address (bytes 26..29 / 30..33) as LE dwords
__device__ __forceinline__ uint32_t ip_src_le(uint32_t (&d)[16]) {
  return __builtin_amdgcn_alignbyte(d[7], d[6], 2);
}
__device__ __forceinline__ uint32_t ip_dst_le(uint32_t (&d)[16]) {
  return __builtin_amdgcn_alignbyte(d[8], d[7], 2);
}

inline int line_occupancy(const void *kern, size_t lds) {
  return occupancy(kern, kLineBlock, lds, 1);
}

// Residency-sized grid; the slab shape for dense 64-byte slots.
template <class Op>
hipError_t launch_line(const typename Op::Args &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const size_t tab = (Op::lds_bytes(a) + 15) & ~(size_t)15;
  const uint64_t need = (a.n + kLineBlock - 1) / kLineBlock;
  if (a.stride == 64 && ((uintptr_t)a.frames & 15) == 0 &&
      !(path_flags() & kPathNoSlab)) {
    auto kern = line_slab_kernel<Op>;
    const size_t lds = tab + (size_t)(kLineBlock / 64) * 4096 +
                       (size_t)line_hold_tiles<Op>((uint32_t)tab) * (kLineBlock / 64) * 128;
    int occ = line_occupancy(reinterpret_cast<const void *>(kern), lds);
    // 2 workgroups per CU (16 waves) rather than the occupancy limit:
    // HashLB l4 0.1906 -> 0.1809 ms, fields 0.1917 -> 0.1814, StaticNAT
    // 0.3761 -> 0.3627, UpdateTTL 0.3738 -> 0.3721 (profiles/r05/
    // lineocc_r05v.json, linew_r05u.json); HashLB with held gates at one
    // (round 6, above): the op's kSlabPerCu
    occ = std::min(occ, Op::kSlabPerCu);
    const uint64_t blocks = std::max<uint64_t>(1, std::min(need, (uint64_t)num_cus * occ));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kLineBlock), lds, s, a,
                       (uint32_t)(tab / 4));
    return hipGetLastError();
  }
  auto kern = line_kernel<Op>;
  const int occ = line_occupancy(reinterpret_cast<const void *>(kern), tab);
  const uint64_t blocks = std::max<uint64_t>(1, std::min(need, (uint64_t)num_cus * occ));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kLineBlock), tab, s, a);
  return hipGetLastError();
}

// One packet per lane in 1024-thread workgroups, for ops whose LDS tables
// leave room for one workgroup per CU and no slab stage: 16 waves per CU
template <class Op>
hipError_t launch_line_wide(const typename Op::Args &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  const size_t tab = (Op::lds_bytes(a) + 15) & ~(size_t)15;
  auto kern = line_kernel<Op, 1024>;
  const int occ = occupancy(reinterpret_cast<const void *>(kern), 1024, tab, 1);
  const uint64_t need = (a.n + 1023) / 1024;
  const uint64_t blocks = std::max<uint64_t>(1, std::min(need, (uint64_t)num_cus * occ));
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(1024), tab, s, a);
  return hipGetLastError();
}

}  // namespace
}  // namespace bg

#endif  // BESS_AMD_BG_LINE_DEV_H_
