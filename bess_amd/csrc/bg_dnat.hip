// bg_dnat.hip -- gfx950 kernels for NAT::ProcessBatch (core/modules/nat.cc:
// 321-363): per packet, ExtractEndpoint (120-160: TCP/UDP ports, ICMP
// query identifiers), the endpoint -> entry lookup in the device copy of
// the NAT map, then Stamp<dir> (262-319): the address and port rewritten,
// IPv4 and TCP/UDP/ICMP checksums updated incrementally (RFC 1624).
//
// dnat_fused_*_kernel look every packet up and Stamp the final hits (any
// reverse hit; a forward hit on a mapping that has not expired at `now`),
// refreshing forward timestamps, and list the rest of the forward packets
// (misses, hits on expired mappings) for the host's in-order walk
// (bg_dnat_api.cc); dnat_apply_kernel then rewrites the listed packets from
// the walk's entry indices.
// Lane = packet; header fields past the first bytes are reached through
// the frame pointer (any IHL).
#include <hip/hip_runtime.h>
#include <algorithm>

#include "bg_kernels.h"
#include "bg_keys_dev.h"
#include "bg_launch.h"

namespace bg {
namespace {

constexpr int kNatBlock = 256;

// Frame byte access. Header fields sit at even offsets (the IPv4 header
// starts at 14, L4 at 14 + 4 * IHL), so a u16 never straddles a dword or a
// 16-byte stage chunk. Bytes past the slot read as 0 and writes to them are
// dropped (the reference reads on into its 2 KB buffer; a slot holds the
// frame only).
struct GlobalFrame {  // the frame in HBM (any stride)
  uint8_t *p;
  uint32_t lim;
  __device__ uint32_t u8(uint32_t o) const { return o < lim ? p[o] : 0u; }
  __device__ uint32_t u16(uint32_t o) const {
    return o + 2 <= lim ? (uint32_t)p[o] | (uint32_t)p[o + 1] << 8 : 0u;
  }
  __device__ void put16(uint32_t o, uint32_t v) const {
    if (o + 2 > lim) return;
    p[o] = (uint8_t)v;
    p[o + 1] = (uint8_t)(v >> 8);
  }
};

// This lane's 64-byte slot in the wave's swizzled LDS stage (slot s keeps
// chunk q at unit 4s + ((q + s/4) & 3), as line_slab_kernel)
struct StageSlot {
  uint8_t *stage;  // the wave's 4 KB stage
  uint32_t slot;
  __device__ uint32_t at(uint32_t o) const {
    return (slot * 4 + (((o >> 4) + (slot >> 2)) & 3)) * 16 + (o & 15);
  }
  __device__ uint32_t u8(uint32_t o) const { return o < 64 ? stage[at(o)] : 0u; }
  __device__ uint32_t u16(uint32_t o) const {
    return o + 2 <= 64 ? *reinterpret_cast<const uint16_t *>(stage + at(o)) : 0u;
  }
  __device__ void put16(uint32_t o, uint32_t v) const {
    if (o + 2 <= 64) *reinterpret_cast<uint16_t *>(stage + at(o)) = (uint16_t)v;
  }
};

// fold(~ck + incr) (UpdateChecksumWithIncrement, checksum.h:535-538)
__device__ __forceinline__ uint32_t upd_ck(uint32_t ck, uint32_t incr) {
  uint32_t s = (~ck & 0xFFFFu) + incr;
  s = (s >> 16) + (s & 0xFFFFu);
  s += s >> 16;
  return ~s & 0xFFFFu;
}

// ExtractEndpoint (nat.cc:120-160): the endpoint key (addr raw | port raw
// << 32 | proto << 48) or ~0 for a protocol NAT does not handle
template <class F>
__device__ __forceinline__ uint64_t endpoint(const F &f, uint32_t dir) {
  const uint32_t l4 = 14 + ((f.u8(14) & 0x0Fu) << 2);
  const uint32_t proto = f.u8(23);
  uint32_t port;
  if (proto == 6 || proto == 17) {
    port = f.u16(l4 + (dir == 0 ? 0 : 2));
  } else if (proto == 1) {
    const uint32_t t = f.u8(l4);
    if (!(t == 0 || t == 8 || t == 13 || t == 15 || t == 16)) return ~0ull;
    port = f.u16(l4 + 4);  // icmp->ident
  } else {
    return ~0ull;
  }
  const uint32_t ao = dir == 0 ? 26 : 30;
  const uint32_t addr = f.u16(ao) | f.u16(ao + 2) << 16;
  return (uint64_t)addr | (uint64_t)port << 32 | (uint64_t)proto << 48;
}

// endpoint -> table slot, or ~0u. A slot's key is two words: the
// endpoint and its translated endpoint (so a hit needs no entry read), and
// their spare top bits carry the entry index (for the timestamp): bits
// 16-23 of it in the endpoint word's top byte, bits 0-15 in the translated
// word's top half (its protocol byte is the endpoint's). A hit is one
// 16-byte key read after the tag words (a separate value array read cost
// 0.13 ms per 16 M packets: one more random line per packet).
struct SlotHit {
  uint32_t slot, entry;
  uint64_t ep;
};
__device__ __forceinline__ SlotHit lookup_in(const TableRef &t, uint64_t key) {
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(t.base);
  const u32x4 *kv = reinterpret_cast<const u32x4 *>(t.base + t.keys_off);
  const Probe p = split_hash(hash_words(&key, 1, t.seed), 1, t.nbp);
  uint32_t c = tag_match(tags[p.b1], p.tag) | (tag_match(tags[p.b2], p.tag) << 4);
  SlotHit h;
  h.slot = ~0u;
  h.entry = 0;
  h.ep = 0;
  while (c) {
    const int s = __builtin_ctz(c);
    c &= c - 1;
    const uint32_t slot = (s < 4 ? p.b1 : p.b2) * kSlots + (s & 3);
    const u32x4 k = kv[slot];
    if ((k.x | (uint64_t)(k.y & 0x00FFFFFFu) << 32) == key) {
      h.slot = slot;
      h.entry = (k.w >> 16) | ((k.y >> 24) << 16);
      h.ep = k.z | (uint64_t)(k.w & 0xFFFFu) << 32;
      break;
    }
  }
  return h;
}
// lookup_in with the second bucket's tag word read only when the first
// bucket does not hold the endpoint (em_lookup_seq's probe order: fewer L2
// requests per packet, one more dependent round trip for those in b2)
__device__ __forceinline__ SlotHit lookup_in_seq(const TableRef &t, uint64_t key) {
  const uint32_t *tags = reinterpret_cast<const uint32_t *>(t.base);
  const u32x4 *kv = reinterpret_cast<const u32x4 *>(t.base + t.keys_off);
  const Probe p = split_hash(hash_words(&key, 1, t.seed), 1, t.nbp);
  SlotHit h;
  h.slot = ~0u;
  h.entry = 0;
  h.ep = 0;
  for (int pass = 0; pass < 2 && h.slot == ~0u; pass++) {
    const uint32_t b = pass ? p.b2 : p.b1;
    uint32_t c = tag_match(tags[b], p.tag);
    while (c) {
      const int s = __builtin_ctz(c);
      c &= c - 1;
      const uint32_t slot = b * kSlots + s;
      const u32x4 k = kv[slot];
      if ((k.x | (uint64_t)(k.y & 0x00FFFFFFu) << 32) == key) {
        h.slot = slot;
        h.entry = (k.w >> 16) | ((k.y >> 24) << 16);
        h.ep = k.z | (uint64_t)(k.w & 0xFFFFu) << 32;
        break;
      }
    }
  }
  return h;
}
// the second bucket read only when the first does not hold the key
// (0.6097 -> 0.5443 ms per 16 M packets, scripts/variants.py natphase,
// profiles/r05/natphase_r05n.json)
__device__ __forceinline__ SlotHit lookup_hit(const DnatArgs &a, uint64_t key) {
  return lookup_in_seq(a.t, key);
}
// endpoint -> entry index, or kDnatMiss
__device__ __forceinline__ uint32_t lookup(const DnatArgs &a, uint64_t key) {
  const SlotHit h = lookup_hit(a, key);
  return h.slot == ~0u ? kDnatMiss : h.entry;
}

// Stamp<dir> (nat.cc:262-319): `before` -> `after` endpoint, IPv4 and
// TCP / UDP / ICMP checksums updated incrementally (RFC 1624)
template <class F>
__device__ __forceinline__ void stamp(const F &f, uint64_t before, uint64_t after,
                                      uint32_t dir) {
  const uint32_t l4 = 14 + ((f.u8(14) & 0x0Fu) << 2);
  const uint32_t oa = (uint32_t)before, na = (uint32_t)after;
  const uint32_t op = (uint32_t)(before >> 32) & 0xFFFFu,
                 np = (uint32_t)(after >> 32) & 0xFFFFu;
  const uint32_t proto = f.u8(23);
  const uint32_t ao = dir == 0 ? 26 : 30;
  f.put16(ao, na & 0xFFFFu);
  f.put16(ao + 2, na >> 16);
  // ChecksumIncrement32(before.addr, after.addr)
  const uint32_t l3 = (~oa >> 16) + (~oa & 0xFFFFu) + (na >> 16) + (na & 0xFFFFu);
  f.put16(24, upd_ck(f.u16(24), l3));
  const uint32_t inc16 = (~op & 0xFFFFu) + np;  // ChecksumIncrement16
  if (proto == 6 || proto == 17) {
    f.put16(l4 + (dir == 0 ? 0 : 2), np);
    if (proto == 6) {
      f.put16(l4 + 16, upd_ck(f.u16(l4 + 16), l3 + inc16));
    } else {
      const uint32_t ck = f.u16(l4 + 6);
      if (ck != 0) {
        const uint32_t nck = upd_ck(ck, l3 + inc16);
        f.put16(l4 + 6, nck ? nck : 0xFFFFu);
      }
    }
  } else {  // ICMP: ident, checksum over the ICMP message only
    f.put16(l4 + 4, np);
    f.put16(l4 + 2, upd_ck(f.u16(l4 + 2), inc16));
  }
}

__device__ __forceinline__ GlobalFrame frame_of(const DnatArgs &a, uint64_t i) {
  GlobalFrame f;
  f.p = a.frames + i * a.stride;
  f.lim = (uint32_t)(a.stride < 4096 ? a.stride : 4096);
  return f;
}

// Rewrites packets from entry indices: every packet of the batch (n > 0,
// res[i] per packet) or, with a.list, the nlist packets idx[k] = res[k]
// with entries mres[k] and endpoints keys[k].
__global__ __launch_bounds__(kNatBlock) void dnat_apply_kernel(DnatArgs a) {
  const uint64_t step = (uint64_t)gridDim.x * kNatBlock;
  const uint64_t cnt = a.list ? a.nlist : a.n;
  for (uint64_t k = (uint64_t)blockIdx.x * kNatBlock + threadIdx.x; k < cnt;
       k += step) {
    const uint64_t i = a.list ? a.res[k] : k;
    const uint32_t e = a.list ? a.mres[k] : a.res[k];
    if (e >= kDnatInvalid || e >= a.nent) {  // drop codes (bound: never)
      a.out[i] = kDropGate;
      continue;
    }
    if (a.refresh) a.ts[e] = a.now;  // forward packets only (rfc4787 REQ-6)
    stamp(frame_of(a, i), a.keys[k], a.list ? a.meps[k] : a.ent[e], a.dir);
    a.out[i] = a.dir == 0 ? 1 : 0;
  }
}

// One packet's decision (bg_dnat_process): lookup; a final hit is stamped
// and its forward timestamp refreshed; an invalid protocol or a reverse
// miss drops; a forward miss, or a forward hit on an expired mapping (a new
// flow earlier in the batch may evict it: CreateNewEntry, nat.cc:224-231),
// is appended to the list (wave-aggregated) for the host's in-order walk.
template <class F>
__device__ __forceinline__ void fused_one(const DnatArgs &a, const F &f,
                                          uint64_t i, bool live) {
  uint64_t key = ~0ull;
  SlotHit h;
  h.slot = ~0u;
  uint64_t ts = 0;
  if (live) {
    key = endpoint(f, a.dir);
    if (key != ~0ull) h = lookup_hit(a, key);
    // a reverse miss: the forward entries are in the same map (nat.cc Find)
    if (h.slot == ~0u && key != ~0ull && a.dir == 1 && a.t2.base) h = lookup_in(a.t2, key);
    if (h.slot != ~0u && a.dir == 0) ts = a.ts[h.entry];
  }
  // only a forward entry's timestamp decides expiry (nat.cc:222-226)
  bool expired = h.slot != ~0u && a.dir == 0 && a.now - ts > a.timeout;
  // a forward packet from an external address: an earlier packet of the
  // batch may create an entry under its endpoint -- the host decides
  if (a.dir == 0 && h.slot != ~0u) {
    bool ext = a.list_fwd != 0;
    for (uint32_t j = 0; j < a.next; j++) ext |= (uint32_t)key == a.ext[j];
    expired |= ext;
  }
  const bool fmiss =
      live && key != ~0ull && a.dir == 0 && (h.slot == ~0u || expired);
  const uint64_t m = __ballot(fmiss);
  if (m) {
    const int lead = __builtin_ctzll(m);
    uint32_t base = 0;
    if ((int)(threadIdx.x & 63) == lead) base = atomicAdd(a.nmiss, (uint32_t)__popcll(m));
    base = __shfl(base, lead);
    if (fmiss) {
      const uint32_t pos = base + __builtin_amdgcn_mbcnt_hi(
                                      (uint32_t)(m >> 32),
                                      __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
      a.res[pos] = (uint32_t)i;
      a.keys[pos] = key;
    }
  }
  if (!live) return;
  if (h.slot == ~0u || expired) {
    a.out[i] = kDropGate;  // the host's walk decides listed packets
    return;
  }
  stamp(f, key, h.ep, a.dir);
  a.out[i] = a.dir == 0 ? 1 : 0;
  // forward timestamp refresh. A scattered 8-byte store is a partial-line
  // write; an entry an earlier packet of the flow already stamped with
  // `now` is left alone (measured: 0.73-0.80 -> 0.69 ms per 16 M packets)
  if (a.dir == 0 && ts != a.now) a.ts[h.entry] = a.now;
}

// the entries a host walk changed: ent[idx] = ep, ts[idx] = ts
__global__ __launch_bounds__(kNatBlock) void dnat_scatter_kernel(
    const uint64_t *up, uint64_t k, uint64_t *ent, uint64_t *ts) {
  const uint64_t step = (uint64_t)gridDim.x * kNatBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kNatBlock + threadIdx.x; i < k; i += step) {
    const uint64_t e = up[i];
    ent[e] = up[k + i];
    ts[e] = up[2 * k + i];
  }
}

// the lookup-image words a host walk changed: img[up[i]] = up[k + i]
__global__ __launch_bounds__(kNatBlock) void dnat_image_kernel(
    const uint64_t *up, uint64_t k, uint64_t *img) {
  const uint64_t step = (uint64_t)gridDim.x * kNatBlock;
  for (uint64_t i = (uint64_t)blockIdx.x * kNatBlock + threadIdx.x; i < k; i += step)
    img[up[i]] = up[k + i];
}

// any stride: lane = packet, header bytes straight from HBM
__global__ __launch_bounds__(kNatBlock) void dnat_fused_kernel(DnatArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.nmiss_next) *a.nmiss_next = 0;
  const uint64_t step = (uint64_t)gridDim.x * kNatBlock;
  const uint64_t n_pad = (a.n + 63) & ~63ull;  // whole waves reach the ballot
  for (uint64_t i = (uint64_t)blockIdx.x * kNatBlock + threadIdx.x; i < n_pad;
       i += step)
    fused_one(a, frame_of(a, i < a.n ? i : 0), i, i < a.n);
}

// dense 64-byte slots: a wave's 64 slots (4 KB) come in with lane-contiguous
// 16-byte loads into its swizzled LDS stage (next tile in flight), each lane
// decides and stamps its slot in LDS, and the tile goes back whole with
// lane-contiguous 16-byte stores (no partial-line writes).
constexpr int kNatSlabBlock = 512;
// The tile is written back with streaming stores (as the line ops').
__global__ __launch_bounds__(kNatSlabBlock) void dnat_fused_slab_kernel(DnatArgs a) {
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.nmiss_next) *a.nmiss_next = 0;
  extern __shared__ __attribute__((aligned(16))) uint8_t lds[];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  constexpr int kWaves = kNatSlabBlock / 64;
  uint4 *stage = reinterpret_cast<uint4 *>(lds) + wid * 256;
  const uint64_t nwaves = (uint64_t)gridDim.x * kWaves;
  const uint64_t ntiles = (a.n + 63) / 64;
  uint4 *src = reinterpret_cast<uint4 *>(a.frames);
  uint64_t t = (uint64_t)blockIdx.x * kWaves + wid;
  uint4 v[4];
  auto units_of = [&](uint64_t tile) {
    const uint64_t p0 = tile * 64;
    return (uint32_t)((a.n - p0 < 64 ? a.n - p0 : 64) * 4);
  };
  auto load_tile = [&](uint64_t tile) {
    const uint32_t units = units_of(tile);
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      v[c] = u < units ? ld_stream(src + tile * 256 + u) : make_uint4(0, 0, 0, 0);
    }
  };
  StageSlot me;
  me.stage = reinterpret_cast<uint8_t *>(stage);
  me.slot = (uint32_t)lane;
  if (t < ntiles) load_tile(t);
  for (; t < ntiles; t += nwaves) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[(u >> 2) * 4 + (((u & 3) + (u >> 4)) & 3)] = v[c];
    }
    lds_fence();
    const uint32_t units = units_of(t);
    if (t + nwaves < ntiles) load_tile(t + nwaves);
    const uint64_t idx = t * 64 + lane;
    fused_one(a, me, idx, idx < a.n);
    lds_fence();
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      if (u < units) {
        st_stream(src + t * 256 + u, stage[(u >> 2) * 4 + (((u & 3) + (u >> 4)) & 3)]);
      }
    }
    lds_fence();  // stage reads retire before the next tile's writes
  }
}

uint64_t grid_of(uint64_t n, int num_cus) {
  uint64_t b = (n + kNatBlock - 1) / kNatBlock;
  const uint64_t cap = (uint64_t)num_cus * 8;
  return b > cap ? cap : b;
}

}  // namespace

hipError_t launch_dnat_scatter(const uint64_t *d_up, size_t k, uint64_t *ent,
                               uint64_t *ts, hipStream_t s) {
  if (k == 0) return hipSuccess;
  hipLaunchKernelGGL(dnat_scatter_kernel, dim3((unsigned)grid_of(k, 256)),
                     dim3(kNatBlock), 0, s, d_up, (uint64_t)k, ent, ts);
  return hipGetLastError();
}

hipError_t launch_dnat_image(const uint64_t *d_up, size_t k, uint64_t *img,
                             hipStream_t s) {
  if (k == 0) return hipSuccess;
  hipLaunchKernelGGL(dnat_image_kernel, dim3((unsigned)grid_of(k, 256)),
                     dim3(kNatBlock), 0, s, d_up, (uint64_t)k, img);
  return hipGetLastError();
}

hipError_t launch_dnat_apply(const DnatArgs &a, int num_cus, hipStream_t s) {
  const uint64_t cnt = a.list ? a.nlist : a.n;
  if (cnt == 0) return hipSuccess;
  hipLaunchKernelGGL(dnat_apply_kernel, dim3((unsigned)grid_of(cnt, num_cus)),
                     dim3(kNatBlock), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_dnat_fused(const DnatArgs &a0, int num_cus, hipStream_t s) {
  if (a0.n == 0) return hipSuccess;
  const DnatArgs &a = a0;
  if (a.stride == 64 && ((uintptr_t)a.frames & 15) == 0 &&
      !(path_flags() & kPathNoSlab)) {
    const size_t lds = (size_t)(kNatSlabBlock / 64) * 4096;
    auto kern = dnat_fused_slab_kernel;
    int occ = occupancy(reinterpret_cast<const void *>(kern), kNatSlabBlock, lds, 1);
    // 2 workgroups per CU (16 waves) rather than the occupancy limit (3):
    // 0.5395 -> 0.5017 ms per 16 M packets (profiles/r05/natphase_r05u.json)
    occ = std::max(1, std::min(occ, 2));
    const uint64_t need = (a.n + kNatSlabBlock - 1) / kNatSlabBlock;
    const uint64_t blocks = std::max<uint64_t>(1, std::min(need, (uint64_t)num_cus * occ));
    hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kNatSlabBlock), lds, s, a);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(dnat_fused_kernel, dim3((unsigned)grid_of(a.n, num_cus)),
                     dim3(kNatBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bg
