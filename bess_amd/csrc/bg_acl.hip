// bg_acl.hip -- gfx950 kernel for ACL::ProcessBatch (core/modules/acl.cc:
// 63-95, ACLRule::Match acl.h:45-50): per packet, the first rule (in order)
// whose src/dst prefixes and non-zero ports match decides -- emit on the
// input gate unless the rule drops; no match drops.
//
// Four forms (launch_acl picks): decision trees in LDS (AclTreeOp, the
// default), per-dimension bit vectors (AclBvOp), and the ordered rule scan
// from LDS (AclLdsOp) or with scalar loads (AclOp). The packet side comes
// from the header line (IHL at byte 14, addresses at 26..33, ports at
// 14 + 4*IHL), via bg_line_dev.h (coalesced slab kernel for 64 B slots).
#include <hip/hip_runtime.h>

#include "bg_kernels.h"
#include "bg_line_dev.h"

namespace bg {
namespace {

// The rule scan with scalar loads: the rule list is the same for every
// packet, so rules are read with wave-uniform (scalar) loads and each rule
// costs a handful of VALU ops per 64 packets; a wave stops scanning once
// all its lanes have matched.
struct AclOp {
  using Args = AclArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;
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

// (v ^ a) & m in one instruction (v_bitop3_b32, truth table 0x48 over
// (a, m, v)); the compiler otherwise spends an xor and an and
__device__ __forceinline__ uint32_t masked_ne(uint32_t v, uint32_t a, uint32_t m) {
  uint32_t r;
  asm("v_bitop3_b32 %0, %1, %2, %3 bitop3:0x48" : "=v"(r) : "v"(a), "v"(m), "v"(v));
  return r;
}

// The rule scan with the rule list in LDS: each rule reaches the lanes as
// two broadcast ds_read_b128 (no bank conflicts), so its three masked
// compares are single v_bitop3 instructions on VGPRs -- from scalar
// registers each needed a v_mov first (one scalar operand per VOP3). The
// first match is kept as a minimum over keys (rule index, plus bit 31 when
// the rule misses): no lane-mask bookkeeping per rule, whose scalar
// instructions share one scalar unit per CU. Per rule: 3 bitop3, or3, min,
// lshl_or, min; a wave leaves the scan once every lane has matched.
struct AclLdsOp {
  using Args = AclArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 0, c1 = 4;
  static size_t lds_bytes(const AclArgs &a) { return (size_t)a.nrules * 32; }
  __device__ static void stage(uint32_t *lds, const AclArgs &a) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a.rules);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    for (uint32_t i = threadIdx.x; i < a.nrules * 2; i += blockDim.x) dst[i] = src[i];
  }
  __device__ static uint32_t decide(const AclArgs &x, const uint32_t *lds,
                                    uint32_t (&d)[16], uint8_t *f) {
    const uint32_t sip = ip_src_le(d), dip = ip_dst_le(d);
    const uint32_t ports = l4_ports(d, f, x.stride);
    const uint4 *R = reinterpret_cast<const uint4 *>(lds);
    uint32_t best = 0xFFFFFFFFu;
    // nrules is a multiple of 4; the padding repeats the last rule, which
    // can never be a first match the rule before it was not
    for (uint32_t r = 0; r < x.nrules; r += 4) {
      uint4 A[4], B[4];
#pragma unroll
      for (int j = 0; j < 4; j++) {
        A[j] = R[2 * (r + j)];
        B[j] = R[2 * (r + j) + 1];
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const uint32_t miss = masked_ne(sip, A[j].x, A[j].y) | masked_ne(dip, A[j].z, A[j].w) |
                              masked_ne(ports, B[j].x, B[j].y);
        best = min(best, (min(miss, 1u) << 31) | (r + (uint32_t)j));
      }
      if ((r & 12) == 12 && __all(best < 0x80000000u)) break;  // every 16 rules
    }
    if (best >= 0x80000000u) return kDropGateDev;
    return R[2 * best + 1].z ? kDropGateDev : x.igate;
  }
  static constexpr uint32_t kDropGateDev = 8192;  // DROP_GATE
};

// LDS the scan may take for its rule list (32 B per rule)
constexpr size_t kAclLdsRules = 48 << 10;

// The same decision from per-dimension bit vectors (Lakshman-Stiliadis
// style, with a summary word per interval): a packet finds its interval in
// each of the four dimensions -- two binary searches over the address
// interval starts in LDS, two 64 K-entry port tables -- ANDs the four
// summary words, and for each set summary bit (lowest first) ANDs the
// four rule words of that group: the lowest set bit is the first rule, in
// list order, that matches in all four dimensions, which is the rule the
// ordered scan stops at. A summary bit that no single rule backs only
// costs one more group (rare). The work per packet no longer grows with
// the rule count, beyond the searches' log2 steps.
struct AclBvOp {
  using Args = AclArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 0, c1 = 4;
  static size_t lds_bytes(const AclArgs &a) { return (size_t)(a.k0 + a.k1) * 4; }
  __device__ static void stage(uint32_t *lds, const AclArgs &a) {
    const uint32_t nb = a.k0 + a.k1;  // B_0 then B_1, adjacent in bv
    const uint32_t *src = a.bv + a.b_off[0];
    for (uint32_t i = threadIdx.x; i < nb; i += blockDim.x) lds[i] = src[i];
  }
  // the last interval start <= v (B[0] == 0)
  __device__ static uint32_t search(const uint32_t *B, uint32_t k, uint32_t lg,
                                    uint32_t v) {
    uint32_t lo = 0;
    for (uint32_t step = lg ? 1u << (lg - 1) : 0u; step; step >>= 1) {
      const uint32_t j = lo + step;
      lo = (j < k && B[j] <= v) ? j : lo;
    }
    return lo;
  }
  __device__ static uint32_t decide(const AclArgs &x, const uint32_t *lds,
                                    uint32_t (&d)[16], uint8_t *f) {
    const uint32_t sip = __builtin_bswap32(ip_src_le(d));
    const uint32_t dip = __builtin_bswap32(ip_dst_le(d));
    const uint32_t ports = l4_ports(d, f, x.stride);  // raw frame bytes
    const uint32_t i0 = search(lds, x.k0, x.lg0, sip);
    const uint32_t i1 = search(lds + x.k0, x.k1, x.lg1, dip);
    const uint16_t *P2 = reinterpret_cast<const uint16_t *>(x.bv + x.p_off[0]);
    const uint16_t *P3 = reinterpret_cast<const uint16_t *>(x.bv + x.p_off[1]);
    const uint32_t i2 = P2[ports & 0xFFFFu], i3 = P3[ports >> 16];
    const uint32_t *bv = x.bv;
    uint32_t s = bv[x.s_off[0] + i0] & bv[x.s_off[1] + i1] & bv[x.s_off[2] + i2] &
                 bv[x.s_off[3] + i3];
    const uint32_t *V0 = bv + x.v_off[0] + (size_t)i0 * x.nw;
    const uint32_t *V1 = bv + x.v_off[1] + (size_t)i1 * x.nw;
    const uint32_t *V2 = bv + x.v_off[2] + (size_t)i2 * x.nw;
    const uint32_t *V3 = bv + x.v_off[3] + (size_t)i3 * x.nw;
    uint32_t res = kDropGateDev;
    while (s) {
      const uint32_t g = __builtin_ctz(s);
      s &= s - 1;
      const uint32_t w1 = min((g + 1) * x.grp, x.nw);
      for (uint32_t w = g * x.grp; w < w1; w++) {
        const uint32_t m = V0[w] & V1[w] & V2[w] & V3[w];
        if (m) {
          const uint32_t b = __builtin_ctz(m);
          res = ((bv[x.d_off + w] >> b) & 1u) ? kDropGateDev : x.igate;
          s = 0;
          break;
        }
      }
    }
    return res;
  }
  static constexpr uint32_t kDropGateDev = 8192;  // DROP_GATE
};

// The same decision from a decision tree in LDS (bit cuts, HiCuts-style;
// built by bg_acl_api.cc build_tree, layout in AclArgs): a lane walks from
// the root, each internal node taking a bit field of one dimension of its
// packet as the index into the node's child array (one LDS read per level),
// to a leaf of a few rule records that it checks in order. A leaf holds, in
// list order, only the rules that intersect its box, cut after the first
// one that covers the whole box, so the first of them to match is the
// reference's first match (acl.cc:80-88) for every packet in the box.
struct AclTreeOp {
  using Args = AclArgs;
  static constexpr bool kWrites = false;
  static constexpr int kSlabPerCu = 2;
  static constexpr int c0 = 0, c1 = 4;
  static size_t lds_bytes(const AclArgs &a) { return (size_t)a.tree_words * 4; }
  __device__ static void stage(uint32_t *lds, const AclArgs &a) {
    const uint4 *src = reinterpret_cast<const uint4 *>(a.tree);
    uint4 *dst = reinterpret_cast<uint4 *>(lds);
    for (uint32_t i = threadIdx.x; i < a.tree_words / 4; i += blockDim.x) dst[i] = src[i];
  }
  __device__ static uint32_t decide(const AclArgs &x, const uint32_t *lds,
                                    uint32_t (&d)[16], uint8_t *f) {
    const uint32_t sip = __builtin_bswap32(ip_src_le(d));
    const uint32_t dip = __builtin_bswap32(ip_dst_le(d));
    const uint32_t raw = l4_ports(d, f, x.stride);
    // host-order src port in the low half, dst port in the high half
    const uint32_t ports = ((raw & 0x00FF00FFu) << 8) | ((raw >> 8) & 0x00FF00FFu);
    // best: the matched record's last word (rule index in the top bits)
    uint32_t best = 0xFFFFFFFFu;
    for (uint32_t t = 0; t < x.ntrees; t++) {
      uint32_t ref = x.roots[t];
      while (!(ref >> 31)) {
        const uint32_t dim = ref >> 25;
        const uint32_t v = dim == 0 ? sip : (dim == 1 ? dip : ports);
        ref = lds[(ref & 0xFFFFu) +
                  __builtin_amdgcn_ubfe(v, (ref >> 16) & 31u, (ref >> 21) & 15u)];
      }
      const uint4 *rec = reinterpret_cast<const uint4 *>(lds) + (ref & 0xFFFFu);
      const uint32_t cnt = (ref >> 16) & 0xFFu;
      for (uint32_t i = 0; i < cnt; i++) {
        const uint4 r = rec[i];
        if (r.w >= best) break;  // records ascend by rule index
        const uint32_t pmask = ((0u - ((r.w >> 12) & 1u)) & 0xFFFFu) |
                               ((0u - ((r.w >> 13) & 1u)) << 16);
        // the top len bits of (value ^ rule): zero iff the prefix matches
        // (len 0 shifts every bit out)
        const uint32_t miss =
            (uint32_t)(((uint64_t)(sip ^ r.x) << (r.w & 63u)) >> 32) |
            (uint32_t)(((uint64_t)(dip ^ r.y) << ((r.w >> 6) & 63u)) >> 32) |
            ((ports ^ r.z) & pmask);
        if (miss == 0) {
          best = r.w;
          break;
        }
      }
    }
    if (best == 0xFFFFFFFFu || ((best >> 14) & 1u)) return kDropGateDev;
    return x.igate;
  }
  static constexpr uint32_t kDropGateDev = 8192;  // DROP_GATE
};

}  // namespace

hipError_t launch_acl(const AclArgs &a, int num_cus, hipStream_t s) {
  const uint32_t pf = path_flags();
  if (pf & (kPathAclScan | kPathNoLds)) return launch_line<AclOp>(a, num_cus, s);
  if (a.bv && (pf & kPathAclBv)) return launch_line<AclBvOp>(a, num_cus, s);
  if (a.tree && !(pf & kPathAclLds)) {
    // trees past 48 KB would leave one 512-thread slab workgroup per CU;
    // 1024-thread lane-per-packet workgroups keep 16 waves (3000 rules
    // without catch-alls: 0.36 ms against 0.68)
    if ((size_t)a.tree_words * 4 > kAclLdsRules && !(pf & kPathNoSlab))
      return launch_line_wide<AclTreeOp>(a, num_cus, s);
    return launch_line<AclTreeOp>(a, num_cus, s);
  }
  // measured (scripts/acl_paths.py, 16 M packets): bit vectors 0.41 ms at
  // 100 rules (4 words per vector) against 0.50 for the LDS scan; at 1000
  // rules (32 words) 0.77 against 0.49 -- wildcards fill the summaries, so
  // a packet that matches late or not at all ANDs every word
  if (a.bv && a.nw <= 4 && !(pf & kPathAclLds)) return launch_line<AclBvOp>(a, num_cus, s);
  if ((size_t)a.nrules * 32 <= kAclLdsRules) return launch_line<AclLdsOp>(a, num_cus, s);
  return launch_line<AclOp>(a, num_cus, s);
}

}  // namespace bg
