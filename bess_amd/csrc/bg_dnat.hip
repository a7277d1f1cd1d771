// bg_dnat.hip -- gfx950 kernels for NAT::ProcessBatch (core/modules/nat.cc:
// 321-363): per packet, ExtractEndpoint (120-160: TCP/UDP ports, ICMP
// query identifiers), the endpoint -> entry lookup in the device copy of
// the NAT map, then Stamp<dir> (262-319): the address and port rewritten,
// IPv4 and TCP/UDP/ICMP checksums updated incrementally (RFC 1624).
//
// dnat_find_kernel classifies a batch (entry index, or a miss / an
// invalid protocol) and counts the forward misses, which need a new
// mapping; dnat_apply_kernel rewrites every packet from a per-packet entry
// index (the lookup result itself when there was no forward miss, else the
// host's in-order walk, bg_dnat_api.cc) and refreshes forward timestamps.
// Lane = packet; header fields past the first bytes are reached through
// the frame pointer (any IHL).
#include <hip/hip_runtime.h>

#include "bg_kernels.h"
#include "bg_keys_dev.h"

namespace bg {
namespace {

constexpr int kNatBlock = 256;

__device__ __forceinline__ uint32_t ld_u16(const uint8_t *p) {
  return (uint32_t)p[0] | (uint32_t)p[1] << 8;
}
__device__ __forceinline__ void st_u16(uint8_t *p, uint32_t v) {
  p[0] = (uint8_t)v;
  p[1] = (uint8_t)(v >> 8);
}
__device__ __forceinline__ uint32_t ld_u32(const uint8_t *p) {
  return ld_u16(p) | ld_u16(p + 2) << 16;
}

// fold(~ck + incr) (UpdateChecksumWithIncrement, checksum.h:535-538)
__device__ __forceinline__ uint32_t upd_ck(uint32_t ck, uint32_t incr) {
  uint32_t s = (~ck & 0xFFFFu) + incr;
  s = (s >> 16) + (s & 0xFFFFu);
  s += s >> 16;
  return ~s & 0xFFFFu;
}

// ExtractEndpoint: the endpoint key (addr raw | port raw << 32 | proto <<
// 48) or ~0 for a protocol NAT does not handle
__device__ __forceinline__ uint64_t endpoint(const uint8_t *ip, int dir) {
  const uint8_t *l4 = ip + ((ip[0] & 0x0Fu) << 2);
  const uint32_t proto = ip[9];
  uint32_t port;
  if (proto == 6 || proto == 17) {
    port = ld_u16(l4 + (dir == 0 ? 0 : 2));
  } else if (proto == 1) {
    const uint32_t t = l4[0];
    if (!(t == 0 || t == 8 || t == 13 || t == 15 || t == 16)) return ~0ull;
    port = ld_u16(l4 + 4);  // icmp->ident
  } else {
    return ~0ull;
  }
  const uint32_t addr = ld_u32(ip + (dir == 0 ? 12 : 16));
  return (uint64_t)addr | (uint64_t)port << 32 | (uint64_t)proto << 48;
}

__global__ __launch_bounds__(kNatBlock) void dnat_find_kernel(DnatArgs a) {
  const uint64_t step = (uint64_t)gridDim.x * kNatBlock;
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(a.t.base);
  const uint64_t *keys = reinterpret_cast<const uint64_t *>(a.t.base + a.t.keys_off);
  const uint32_t *vals = reinterpret_cast<const uint32_t *>(a.t.base + a.t.vals_off);
  for (uint64_t i = (uint64_t)blockIdx.x * kNatBlock + threadIdx.x; i < a.n;
       i += step) {
    const uint8_t *ip = a.frames + i * a.stride + 14;
    const uint64_t key = endpoint(ip, a.dir);
    a.keys[i] = key;
    uint32_t r = kDnatInvalid;
    if (key != ~0ull) {
      r = kDnatMiss;
      const Probe p = split_hash(hash_words(&key, 1, a.t.seed), 1, a.t.nbp);
      uint32_t c = tag_match(tags[p.b1], p.tag) | (tag_match(tags[p.b2], p.tag) << 4);
      while (c) {
        const int s = __builtin_ctz(c);
        c &= c - 1;
        const uint32_t slot = (s < 4 ? p.b1 : p.b2) * kSlots + (s & 3);
        if (keys[slot] == key) {
          r = vals[slot];
          break;
        }
      }
      // a forward miss needs a new mapping (CreateNewEntry); a reverse
      // miss is dropped
      if (r == kDnatMiss && a.dir == 0) atomicAdd(a.nmiss, 1u);
    }
    a.res[i] = r;
  }
}

__global__ __launch_bounds__(kNatBlock) void dnat_apply_kernel(DnatArgs a) {
  const uint64_t step = (uint64_t)gridDim.x * kNatBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kNatBlock + threadIdx.x; i < a.n;
       i += step) {
    const uint32_t e = a.res[i];
    if (e >= kDnatInvalid || e >= a.nent) {  // drop codes (bound: never)
      a.out[i] = kDropGate;
      continue;
    }
    if (a.refresh) a.ts[e] = a.now;  // forward packets only (rfc4787 REQ-6)
    uint8_t *ip = a.frames + i * a.stride + 14;
    uint8_t *l4 = ip + ((ip[0] & 0x0Fu) << 2);
    const uint64_t before = a.keys[i], after = a.ent[e];
    const uint32_t oa = (uint32_t)before, na = (uint32_t)after;
    const uint32_t op = (uint32_t)(before >> 32) & 0xFFFFu, np = (uint32_t)(after >> 32) & 0xFFFFu;
    const uint32_t proto = ip[9];
    uint8_t *pa = ip + (a.dir == 0 ? 12 : 16);
    st_u16(pa, na & 0xFFFFu);
    st_u16(pa + 2, na >> 16);
    // ChecksumIncrement32(before.addr, after.addr)
    const uint32_t l3 = (~oa >> 16) + (~oa & 0xFFFFu) + (na >> 16) + (na & 0xFFFFu);
    st_u16(ip + 10, upd_ck(ld_u16(ip + 10), l3));
    const uint32_t inc16 = (~op & 0xFFFFu) + np;  // ChecksumIncrement16
    if (proto == 6 || proto == 17) {
      st_u16(l4 + (a.dir == 0 ? 0 : 2), np);
      if (proto == 6) {
        st_u16(l4 + 16, upd_ck(ld_u16(l4 + 16), l3 + inc16));
      } else {
        const uint32_t ck = ld_u16(l4 + 6);
        if (ck != 0) {
          const uint32_t nck = upd_ck(ck, l3 + inc16);
          st_u16(l4 + 6, nck ? nck : 0xFFFFu);
        }
      }
    } else {  // ICMP: ident, checksum over the ICMP message only
      st_u16(l4 + 4, np);
      st_u16(l4 + 2, upd_ck(ld_u16(l4 + 2), inc16));
    }
    a.out[i] = a.dir == 0 ? 1 : 0;
  }
}

uint64_t grid_of(uint64_t n, int num_cus) {
  uint64_t b = (n + kNatBlock - 1) / kNatBlock;
  const uint64_t cap = (uint64_t)num_cus * 8;
  return b > cap ? cap : b;
}

}  // namespace

hipError_t launch_dnat_find(const DnatArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(dnat_find_kernel, dim3((unsigned)grid_of(a.n, num_cus)),
                     dim3(kNatBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_dnat_apply(const DnatArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0) return hipSuccess;
  hipLaunchKernelGGL(dnat_apply_kernel, dim3((unsigned)grid_of(a.n, num_cus)),
                     dim3(kNatBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bg
