// bg_acl.hip -- gfx950 kernel for ACL::ProcessBatch (core/modules/acl.cc:
// 63-95, ACLRule::Match acl.h:45-50): per packet, the first rule (in order)
// whose src/dst prefixes and non-zero ports match decides -- emit on the
// input gate unless the rule drops; no match drops.
//
// The rule list is the same for every packet, so rules are read with
// wave-uniform (scalar) loads and each rule costs a handful of VALU ops per
// 64 packets; a wave stops scanning once all its lanes have matched. The
// packet side comes from the header line (IHL at byte 14, addresses at
// 26..33, ports at 14 + 4*IHL), via bg_line_dev.h (coalesced slab kernel
// for 64 B slots).
#include <hip/hip_runtime.h>

#include "bg_kernels.h"
#include "bg_line_dev.h"

namespace bg {
namespace {

struct AclOp {
  using Args = AclArgs;
  static constexpr bool kWrites = false;
  static constexpr int c0 = 0, c1 = 4;
  static size_t lds_bytes(const AclArgs &) { return 0; }
  __device__ static void stage(uint32_t *, const AclArgs &) {}
  __device__ static uint32_t decide(const AclArgs &x, const uint32_t *,
                                    uint32_t (&d)[16], uint8_t *f) {
    const uint32_t sip = ip_src_le(d), dip = ip_dst_le(d);
    const uint32_t ports = l4_ports(d, f, x.stride);
    // the rule list through the constant address space: wave-uniform
    // addresses become scalar loads (s_load_dwordx8 per rule)
    typedef const __attribute__((address_space(4))) u32x4 *kv4;
    const kv4 R = (kv4)(x.rules);
    uint32_t res = kDropGateDev;
    bool done = false;
    // nrules is padded to a multiple of 4 with never-valid rules (dword 7
    // = valid), so groups of 4 rules load together without bounds checks
    for (uint32_t r = 0; r < x.nrules; r += 4) {
      u32x4 A[4], B[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        A[j] = R[2 * (r + j)];
        B[j] = R[2 * (r + j) + 1];
      }
      // branch-free first-match update (a per-rule branch costs more than
      // the rule itself)
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t miss = ((sip ^ A[j].x) & A[j].y) | ((dip ^ A[j].z) & A[j].w) |
                              ((ports ^ B[j].x) & B[j].y);
        const bool take = (miss == 0) & (B[j].w != 0) & !done;
        res = take ? (B[j].z ? kDropGateDev : x.igate) : res;
        done |= take;
      }
      if (__all(done)) break;
    }
    return res;
  }
  static constexpr uint32_t kDropGateDev = 8192;  // DROP_GATE
};

}  // namespace

hipError_t launch_acl(const AclArgs &a, int num_cus, hipStream_t s) {
  return launch_line<AclOp>(a, num_cus, s);
}

}  // namespace bg
