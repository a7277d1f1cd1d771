// bg_lpm.hip -- gfx950 kernel for IPLookup::ProcessBatch
// (core/modules/ip_lookup.cc:76-150): longest-prefix match of each packet's
// IPv4 destination (bytes 30..33) over the route table, emit on the route's
// gate, default_gate_ when no prefix matches (rte_lpm_lookup / _lookupx4).
//
// The tables are DIR-24-8 (the structure rte_lpm itself uses): a
// 2^24-entry u16 tbl24 (32 MB, resident in MALL) indexed by the top 24
// address bits, extended into 256-entry tbl8 groups for /24 blocks that
// carry longer prefixes; and the same entries folded into DIR-16-8-8 (a
// 2^16-entry tbl16 staged in LDS, 256-entry tbl2 groups in L2 for the /16
// blocks whose /24s differ), the default. The packet side is the header
// line's chunks 1..2 via bg_line_dev.h.
#include <hip/hip_runtime.h>

#include "bg_kernels.h"
#include "bg_line_dev.h"

namespace bg {
namespace {

// DIR-24-8: one dependent read of the 32 MB tbl24 (MALL)
struct LpmOp {
  using Args = LpmArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 1, c1 = 3;  // bytes [16, 48): dst IP at 30..33
  static size_t lds_bytes(const LpmArgs &) { return 0; }
  __device__ static void stage(uint32_t *, const LpmArgs &) {}
  __device__ static uint32_t decide(const LpmArgs &x, const uint32_t *,
                                    uint32_t (&d)[16], uint8_t *) {
    const uint32_t ip = __builtin_bswap32(ip_dst_le(d));  // host order
    uint32_t e = x.tbl24[ip >> 8];
    if (e & 0x8000u) e = x.tbl8[(e & 0x7FFFu) * 256u + (ip & 0xFFu)];
    return e ? e - 1u : x.default_gate;
  }
};

// DIR-16-8-8: tbl24 folded into a 128 KB tbl16 and the 256-entry tbl2
// groups of the /16 blocks whose /24s differ, so the tables stay in L2
// (bench routes: 10 K, 2.4 MB) and a packet makes two dependent L2 reads
// (three for /25../32 routes) instead of a tbl24 sector from MALL
struct Lpm16Op {
  using Args = LpmArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 1, c1 = 3;
  static size_t lds_bytes(const LpmArgs &) { return 0; }
  __device__ static void stage(uint32_t *, const LpmArgs &) {}
  __device__ static uint32_t decide(const LpmArgs &x, const uint32_t *,
                                    uint32_t (&d)[16], uint8_t *) {
    const uint32_t ip = __builtin_bswap32(ip_dst_le(d));
    uint32_t e = x.tbl16[ip >> 16];
    if (e & 0x8000u) e = x.tbl2[(e & 0x7FFFu) * 256u + ((ip >> 8) & 0xFFu)];
    if (e & 0x8000u) e = x.tbl8[(e & 0x7FFFu) * 256u + (ip & 0xFFu)];
    return e ? e - 1u : x.default_gate;
  }
};

// the same with tbl16 staged in LDS (128 KB: one workgroup per CU, so
// 1024 threads with a packet per lane and no slab stage): one L2 request
// per packet in a /16 block with longer routes, none otherwise
struct Lpm16LdsOp {  // (line_kernel only: launch_line_wide)
  using Args = LpmArgs;
  static constexpr bool kWrites = false;
  static constexpr int c0 = 1, c1 = 3;
  static size_t lds_bytes(const LpmArgs &) { return (1u << 16) * 2; }
  __device__ static void stage(uint32_t *lds, const LpmArgs &a) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a.tbl16);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    for (uint32_t i = threadIdx.x; i < (1u << 16) * 2 / 16; i += blockDim.x) dst[i] = src[i];
  }
  __device__ static uint32_t decide(const LpmArgs &x, const uint32_t *lds,
                                    uint32_t (&d)[16], uint8_t *) {
    const uint32_t ip = __builtin_bswap32(ip_dst_le(d));
    uint32_t e = reinterpret_cast<const uint16_t *>(lds)[ip >> 16];
    if (e & 0x8000u) e = x.tbl2[(e & 0x7FFFu) * 256u + ((ip >> 8) & 0xFFu)];
    if (e & 0x8000u) e = x.tbl8[(e & 0x7FFFu) * 256u + (ip & 0xFFu)];
    return e ? e - 1u : x.default_gate;
  }
};

}  // namespace

hipError_t launch_lpm(const LpmArgs &a, int num_cus, hipStream_t s) {
  const uint32_t pf = path_flags();
  if (!a.tbl16 || (pf & kPathLpmDir24)) return launch_line<LpmOp>(a, num_cus, s);
  // measured (scripts/lpm_paths.py, 16 M packets, 10 K routes): tbl16 in
  // LDS with 1024-thread lane-per-packet workgroups 0.214 ms; in LDS with
  // the slab stage (one 512-thread workgroup per CU) 0.242; tbl16 in L2
  // 0.279 (two L2 requests per packet); DIR-24-8 0.327
  if (pf & kPathNoLds) return launch_line<Lpm16Op>(a, num_cus, s);
  return launch_line_wide<Lpm16LdsOp>(a, num_cus, s);
}

}  // namespace bg
