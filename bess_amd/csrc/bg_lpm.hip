// bg_lpm.hip -- gfx950 kernel for IPLookup::ProcessBatch
// (core/modules/ip_lookup.cc:76-150): longest-prefix match of each packet's
// IPv4 destination (bytes 30..33) over the route table, emit on the route's
// gate, default_gate_ when no prefix matches (rte_lpm_lookup / _lookupx4).
//
// The table is DIR-24-8 (the structure rte_lpm itself uses): a 2^24-entry
// u16 tbl24 (32 MB, resident in MALL/L2) indexed by the top 24 address bits,
// extended into 256-entry tbl8 groups for /24 blocks that carry longer
// prefixes -- one dependent table read per packet (two for extended
// blocks). The packet side is the header line's chunks 1..2 via
// bg_line_dev.h (coalesced slab kernel for 64 B slots).
#include <hip/hip_runtime.h>

#include "bg_kernels.h"
#include "bg_line_dev.h"

namespace bg {
namespace {

struct LpmOp {
  using Args = LpmArgs;
  static constexpr bool kWrites = false;
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

}  // namespace

hipError_t launch_lpm(const LpmArgs &a, int num_cus, hipStream_t s) {
  return launch_line<LpmOp>(a, num_cus, s);
}

}  // namespace bg
