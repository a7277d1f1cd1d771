// bg_nat.hip -- gfx950 kernel for StaticNAT::ProcessBatch
// (core/modules/static_nat.cc:146-181): the first address pair whose range
// holds the packet's source (forward, input gate 0) or destination (reverse,
// input gate 1) rewrites that address and updates the IPv4 checksum and the
// TCP / UDP checksum incrementally (UpdateChecksum 118-144, RFC 1624:
// ChecksumIncrement32 + UpdateChecksumWithIncrement, checksum.h:520-549;
// a UDP checksum of 0 stays 0, a result of 0 becomes 0xFFFF). Every packet
// is emitted: forward on gate 1, reverse on gate 0.
//
// Pairs are wave-uniform (scalar loads through the constant address space,
// like ACL rules). The header line is a writing op of bg_line_dev.h: the
// updated line goes back whole. An L4 checksum past the line (TCP with
// IHL >= 9, UDP with IHL >= 11) is read and written in the frame directly,
// only inside the packet's slot.
#include <hip/hip_runtime.h>

#include "bg_kernels.h"
#include "bg_line_dev.h"

namespace bg {
namespace {

// fold(~ck + incr) (UpdateChecksumWithIncrement)
__device__ __forceinline__ uint32_t upd_ck(uint32_t ck, uint32_t incr) {
  uint32_t s = (~ck & 0xFFFFu) + incr;
  s = (s >> 16) + (s & 0xFFFFu);
  s += s >> 16;
  return ~s & 0xFFFFu;
}

// The L4 checksum word sits at line byte l4 + 16 (TCP) or l4 + 6 (UDP),
// l4 = 14 + 4 * IHL: inside the 64-byte line for TCP with IHL <= 8 (the
// upper half of dword 7 + IHL) and UDP with IHL <= 10 (the lower half of
// dword 5 + IHL). Per-lane positions differ, so the word is picked and put
// back with constant-index selects over those dwords (a variable index into
// d[] would put the line in scratch memory).
constexpr int kL4Lo = 10, kL4Hi = 15;

__device__ __forceinline__ bool l4_hi_at(int j, uint32_t ihl, bool tcp) {
  return tcp && (uint32_t)j == 7u + ihl;
}
__device__ __forceinline__ bool l4_lo_at(int j, uint32_t ihl, bool udp) {
  return udp && (uint32_t)j == 5u + ihl;
}

struct NatOp {
  using Args = NatArgs;
  static constexpr bool kWrites = true;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 0, c1 = 4;
  static size_t lds_bytes(const NatArgs &) { return 0; }
  __device__ static void stage(uint32_t *, const NatArgs &) {}
  __device__ static uint32_t decide(const NatArgs &x, const uint32_t *,
                                    uint32_t (&d)[16], uint8_t *f) {
    const uint32_t gate = x.dir == 0 ? 1u : 0u;
    const uint32_t old_raw = x.dir == 0 ? ip_src_le(d) : ip_dst_le(d);
    const uint32_t addr = __builtin_bswap32(old_raw);
    typedef const __attribute__((address_space(4))) u32x4 *kv4;
    const kv4 P = (kv4)(x.pairs);
    uint32_t diff = 0;
    bool hit = false;
    for (uint32_t r = 0; r < x.npairs; r += 4) {
      u32x4 q[4];
#pragma unroll
      for (int j = 0; j < 4; j++) q[j] = P[r + j];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const bool in = !hit && q[j].x <= addr && addr - q[j].x < q[j].z;
        diff = in ? q[j].y - q[j].x : diff;
        hit |= in;
      }
      if (__all(hit)) break;
    }
    if (!hit) return gate;  // no pair: forward without NAT
    const uint32_t new_raw = __builtin_bswap32(addr + diff);
    // ChecksumIncrement32(old, new)
    const uint32_t incr = (~old_raw >> 16) + (~old_raw & 0xFFFFu) +
                          (new_raw >> 16) + (new_raw & 0xFFFFu);
    // IP checksum (bytes 24..25)
    d[6] = (d[6] & 0xFFFF0000u) | upd_ck(d[6] & 0xFFFFu, incr);
    const uint32_t ihl = (d[3] >> 16) & 0x0F, proto = d[5] >> 24;
    const uint32_t l4 = 14 + 4 * ihl;
    const bool tcp = proto == 6, udp = proto == 17;
    if (tcp || udp) {
      const uint32_t pos = l4 + (tcp ? 16u : 6u);
      const bool in_line = pos + 2 <= 64;
      const bool in_slot = pos + 2 <= x.stride;
      uint32_t ck = 0;
#pragma unroll
      for (int j = kL4Lo; j <= kL4Hi; j++) {
        ck = l4_hi_at(j, ihl, tcp) ? d[j] >> 16 : ck;
        ck = l4_lo_at(j, ihl, udp) ? d[j] & 0xFFFFu : ck;
      }
      if (!in_line) ck = in_slot ? *reinterpret_cast<const uint16_t *>(f + pos) : 0u;
      if (tcp || ck != 0) {
        uint32_t nck = upd_ck(ck, incr);
        if (udp && nck == 0) nck = 0xFFFF;
        if (in_line) {
#pragma unroll
          for (int j = kL4Lo; j <= kL4Hi; j++) {
            d[j] = l4_hi_at(j, ihl, tcp) ? (d[j] & 0xFFFFu) | (nck << 16) : d[j];
            d[j] = l4_lo_at(j, ihl, udp) ? (d[j] & 0xFFFF0000u) | nck : d[j];
          }
        } else if (in_slot) {
          *reinterpret_cast<uint16_t *>(f + pos) = (uint16_t)nck;
        }
      }
    }
    // the address itself (src 26..29 / dst 30..33)
    if (x.dir == 0) {
      d[6] = (d[6] & 0x0000FFFFu) | (new_raw << 16);
      d[7] = (d[7] & 0xFFFF0000u) | (new_raw >> 16);
    } else {
      d[7] = (d[7] & 0x0000FFFFu) | (new_raw << 16);
      d[8] = (d[8] & 0xFFFF0000u) | (new_raw >> 16);
    }
    return gate;
  }
};

}  // namespace

hipError_t launch_nat(const NatArgs &a, int num_cus, hipStream_t s) {
  return launch_line<NatOp>(a, num_cus, s);
}

}  // namespace bg
