// bg_encap.hip -- gfx950 kernel for IPEncap::ProcessBatch
// (core/modules/ip_encap.cc:40-80): prepend a 20-byte IPv4 header built from
// the packet's metadata attributes ip_src / ip_dst / ip_proto, with
// total_len + 20 as its length, DF, TTL 64 and the header checksum
// (CalculateIpv4NoOptChecksum: the id bytes are whatever the headroom held,
// the checksum bytes are skipped), then write the ip_nexthop and
// ether_type attributes. prepend() (packet.h:145-154) fails when the
// headroom is < 20 bytes: such a packet is left alone. Lane = packet; a
// dword-aligned new head (the usual 128-byte headroom) is written with
// dword stores, any other with byte stores.
#include <hip/hip_runtime.h>

#include "bg_kernels.h"

namespace bg {
namespace {

constexpr int kEncapBlock = 256;

__device__ __forceinline__ uint32_t ld_bytes4(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
         (uint32_t)p[3] << 24;
}

__global__ __launch_bounds__(kEncapBlock) void encap_kernel(EncapArgs a) {
  const uint64_t step = (uint64_t)gridDim.x * kEncapBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kEncapBlock + threadIdx.x; i < a.n;
       i += step) {
    uint8_t *slot = a.slots + i * a.stride, *meta = slot + a.meta_off;
    // get_attr: 0 for an invalid offset (core/module.h:686-698)
    const uint32_t src = a.offs[0] >= 0 ? ld_bytes4(meta + a.offs[0]) : 0u;
    const uint32_t dst = a.offs[1] >= 0 ? ld_bytes4(meta + a.offs[1]) : 0u;
    const uint32_t proto = a.offs[2] >= 0 ? meta[a.offs[2]] : 0u;
    const uint32_t h = a.head[i], len = a.len[i];
    const uint32_t tl = (len + 20) & 0xFFFFu;  // uint16_t total_len
    a.out[i] = 0;                              // RunNextModule
    if (h < 20) continue;                      // prepend() == nullptr
    const uint32_t nh = h - 20;
    a.head[i] = (uint16_t)nh;
    a.len[i] = len + 20;
    uint8_t *ip = slot + nh;
    uint32_t w[5];
    w[0] = 0x45u | (tl >> 8) << 16 | (tl & 0xFFu) << 24;
    w[1] = (uint32_t)ip[4] | (uint32_t)ip[5] << 8 | 0x40u << 16;  // id kept, DF
    w[2] = 64u | proto << 8;
    w[3] = src;
    w[4] = dst;
    // one's-complement sum of the five words, checksum bytes excluded
    uint64_t s = (uint64_t)w[0] + w[1] + w[2] + w[3] + w[4];
    s = (s & 0xFFFFFFFFu) + (s >> 32);
    uint32_t c = (uint32_t)((s & 0xFFFFFFFFu) + (s >> 32));
    c = (c >> 16) + (c & 0xFFFFu);
    c += c >> 16;
    w[2] |= (~c & 0xFFFFu) << 16;
    if (((uintptr_t)ip & 3) == 0) {
      uint32_t *d = reinterpret_cast<uint32_t *>(ip);
#pragma unroll
      for (int j = 0; j < 5; j++) d[j] = w[j];
    } else {
#pragma unroll
      for (int j = 0; j < 20; j++) ip[j] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
    }
    if (a.offs[3] >= 0) {  // ip_nexthop = ip_dst
      uint8_t *p = meta + a.offs[3];
#pragma unroll
      for (int j = 0; j < 4; j++) p[j] = (uint8_t)(dst >> (8 * j));
    }
    if (a.offs[4] >= 0) {  // ether_type = be16(0x0800)
      meta[a.offs[4]] = 0x08;
      meta[a.offs[4] + 1] = 0x00;
    }
  }
}

}  // namespace

hipError_t launch_encap(const EncapArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  uint64_t blocks = (a.n + kEncapBlock - 1) / kEncapBlock;
  const uint64_t cap = (uint64_t)num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(encap_kernel, dim3((unsigned)blocks), dim3(kEncapBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bg
