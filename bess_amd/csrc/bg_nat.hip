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

// the u16 at even line byte offset `pos` (< 64) of d[], read / replaced
__device__ __forceinline__ uint32_t get16(const uint32_t (&d)[16], uint32_t pos) {
  uint32_t v = 0;
#pragma unroll
  for (int j = 0; j < 16; j++)
    if ((pos >> 2) == (uint32_t)j) v = (d[j] >> ((pos & 2) * 8)) & 0xFFFFu;
  return v;
}
__device__ __forceinline__ void set16(uint32_t (&d)[16], uint32_t pos, uint32_t v) {
#pragma unroll
  for (int j = 0; j < 16; j++)
    if ((pos >> 2) == (uint32_t)j) {
      const uint32_t sh = (pos & 2) * 8;
      d[j] = (d[j] & ~(0xFFFFu << sh)) | (v << sh);
    }
}

struct NatOp {
  using Args = NatArgs;
  static constexpr bool kWrites = true;
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
    if (proto == 6 || proto == 17) {
      const uint32_t pos = l4 + (proto == 6 ? 16u : 6u);
      uint32_t ck;
      const bool in_line = pos + 2 <= 64;
      const bool in_slot = pos + 2 <= x.stride;
      if (in_line) ck = get16(d, pos);
      else ck = in_slot ? *reinterpret_cast<const uint16_t *>(f + pos) : 0u;
      if (proto == 6 || ck != 0) {
        uint32_t nck = upd_ck(ck, incr);
        if (proto == 17 && nck == 0) nck = 0xFFFF;
        if (in_line) set16(d, pos, nck);
        else if (in_slot) *reinterpret_cast<uint16_t *>(f + pos) = (uint16_t)nck;
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
