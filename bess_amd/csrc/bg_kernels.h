// bg_kernels.h -- kernel argument blocks and launchers (host <-> device).
#ifndef BESS_AMD_BG_KERNELS_H_
#define BESS_AMD_BG_KERNELS_H_

#ifndef __HIPCC_RTC__  // hiprtc (bg_wm_jit.cc) has its own
#include <hip/hip_runtime.h>
#include <stdint.h>
#endif

#include "bg_table.h"

namespace bg {

constexpr int kMaxFields = 8;
constexpr int kMaxTuples = 8;
constexpr int kMaxDirect = 2;  // direct tuples per WildcardMatch image (WmArgs)
constexpr int kMaxWindowChunks = 4;      // 16-byte chunks staged per packet
constexpr uint32_t kLdsTableMax = 40960;  // tables up to this size go to LDS
// tiles whose 2-byte results a slab kernel's wave holds in registers before
// it stores them (em_slab_kernel, line_slab_kernel; bg_kernels.hip)
constexpr int kGateHold = 32;
// A slab kernel at one workgroup per CU (em_slab_kernel with its table in
// LDS, line_slab_kernel for a reading op whose kSlabPerCu is 1) holds the
// results in LDS instead: up to kGateHoldLds tiles per wave, as many as the
// CU's LDS (kLdsPerCu) leaves after the tables and the per-wave stages
constexpr int kGateHoldLds = 64;
constexpr uint32_t kLdsPerCu = 163840;
constexpr uint16_t kGateNone = 0xFFFF;

// How a packet's key is built from its frame bytes. Field f contributes
// frame[off_f .. off_f+size_f) & mask_f at key byte pos_f
// (ExactMatchTable::MakeKeys, exact_match_table.h:239-263; WildcardMatch::
// ProcessBatch, wildcard_match.cc:169-197 -- there the mask is all-ones over
// the field and the tuple mask is applied per probe).
struct FieldPlan {
  int32_t nf;      // number of fields
  int32_t direct;  // 1: fields too far apart for one window -> per-field loads
  int32_t win_lo;  // 16-byte aligned frame offset of the staged window
  int32_t nch;     // 16-byte chunks in the window (1..4)
  // per field, packed to keep the kernels' scalar registers low:
  // bits 0-8 window dword index (direct: frame dword index), 9-10 byte shift
  // inside that dword, 11-16 key byte position, 17-18 dwords spanned
  uint32_t fspec[kMaxFields];
  uint64_t fmask[kMaxFields];  // mask in key byte order (low `size` bytes)
  // Byte-permute form of the key build, used by every window-mode kernel:
  //   key dword q = (OR over o < nops(q) of perm(w[d+1], w[d], kd_sel[o][q]),
  //                  d = byte o of kd_dw[q]) & kd_mask[q]
  // nops(q) = byte q of kd_nops (0..4). v_perm_b32 selectors pick byte 0..7
  // of {w[d+1]:w[d]}; 0x0C gives a zero byte.
  int32_t nkd;  // key dwords that carry bytes
  uint32_t kd_nops[2 * kMaxKeyWords / 4];
  uint32_t kd_dw[2 * kMaxKeyWords];
  uint32_t kd_sel[4][2 * kMaxKeyWords];
  uint32_t kd_mask[2 * kMaxKeyWords];
};

BG_HD int kd_nops_of(const FieldPlan &p, int q) {
  return (int)((p.kd_nops[q >> 2] >> (8 * (q & 3))) & 0xFF);
}

constexpr uint32_t kPermZero = 0x0C0C0C0Cu;  // v_perm_b32: four zero bytes

// v_perm_b32 semantics on the host (plan checks, bg_debug_key)
inline uint32_t perm_host(uint32_t s0, uint32_t s1, uint32_t sel) {
  const uint64_t d = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; i++) {
    const uint32_t b = (sel >> (8 * i)) & 0xFF;
    uint32_t v = 0;
    if (b < 8) v = (uint32_t)(d >> (8 * b)) & 0xFF;
    else if (b >= 0x0D) v = 0xFF;
    r |= v << (8 * i);
  }
  return r;
}

BG_HD uint32_t pack_fspec(int d, int byte_shift, int pos, int nd) {
  return (uint32_t)(d & 0x1FF) | ((uint32_t)(byte_shift & 3) << 9) |
         ((uint32_t)(pos & 0x3F) << 11) | ((uint32_t)(nd & 3) << 17);
}
BG_HD int fspec_d(uint32_t s) { return (int)(s & 0x1FF); }
BG_HD int fspec_shift_bits(uint32_t s) { return (int)((s >> 9) & 3) * 8; }
BG_HD int fspec_pos(uint32_t s) { return (int)((s >> 11) & 0x3F); }
BG_HD int fspec_nd(uint32_t s) { return (int)((s >> 17) & 3); }

// TableRef::lds values
constexpr uint32_t kLdsNone = 0;    // table probed in L2 / MALL
constexpr uint32_t kLdsTable = 1;   // whole image copied into LDS
constexpr uint32_t kLdsFilter = 2;  // only the key filter copied into LDS
constexpr uint32_t kFilterMaxWords = 32768;  // 128 KB of LDS
constexpr uint32_t kLdsTags = 3;    // only the tag words in LDS (bg_wm.hip)
constexpr uint64_t kTagsLdsMax = 131072;  // tag bytes staged by bg_wm.hip

struct TableRef {
  const uint8_t *base;  // device image (nparts * part_bytes [+ filter])
  uint64_t part_bytes, keys_off, vals_off, seed;
  uint32_t nparts, nbp, kw, lds;  // lds: kLds* above
  uint32_t bytes_total;           // table bytes (LDS copy length)
  uint32_t filt_words;            // 0: no filter
  uint32_t vik;                   // EM value in the key's top 2 bytes
  uint64_t filt_off;              // byte offset of the filter in the image
  // words per slot record (bg_table.h; 0: separate key / value arrays).
  // WildcardMatch kernels take wm_rec_words(kw) as a constant and their
  // launchers refuse an image laid out otherwise.
  uint32_t rec;
};

struct EmArgs {
  const uint8_t *frames;
  uint64_t stride, n;
  uint16_t *gates;
  uint32_t default_gate, pad;
  FieldPlan fp;
  TableRef t;
};

// a direct tuple's table index: the masked key bytes a and b (WmArgs::dspec)
BG_HD uint32_t direct_index(const uint64_t *k, uint32_t spec) {
  const uint32_t pa = spec & 63, pb = (spec >> 8) & 63;
  const uint32_t ba = (uint32_t)(k[pa >> 3] >> ((pa & 7) * 8)) & (spec >> 16) & 0xFFu;
  const uint32_t bb = (uint32_t)(k[pb >> 3] >> ((pb & 7) * 8)) & (spec >> 24) & 0xFFu;
  return ba | bb << 8;
}

struct WmArgs {
  const uint8_t *frames;
  uint64_t stride, n;
  uint16_t *gates;
  uint32_t default_gate, ntuples;
  FieldPlan fp;
  TableRef t;
  uint64_t tmask[kMaxTuples][kMaxKeyWords];
  uint32_t tcover[kMaxTuples];  // per tuple: the dwords wm_hash covers
  uint32_t tseed[kMaxTuples];   // per tuple: wm_seed32(tuple_seed(seed, tu))
  // Direct tuples (tag-word images only, <= kMaxDirect): a tuple whose mask
  // covers one or two key bytes is not in the hashed table; its entries sit
  // in a table indexed by those masked bytes (256 or 65536 values of the
  // hashed table's format, empty = all ones), one read per packet, no hash,
  // no fingerprint, no key compare.
  uint32_t ndirect;
  uint32_t hmask;  // bit tu: tuple tu is probed by hash (tu < ntuples, not direct)
  uint32_t dtu[kMaxDirect];    // tuple index
  uint32_t dspec[kMaxDirect];  // key byte a | byte b << 8 | mask a << 16 | mask b << 24
  uint64_t doff[kMaxDirect];   // the table's byte offset in the image
};

// WildcardMatch tag-word kernels (bg_wm_body.h): one 1024-thread workgroup
// per CU; LDS = the tag words, the tuple masks, and per wave best[64] plus
// a queue of kWmQueue entries
constexpr int kWmBlock = 1024;
constexpr int kWmWaves = kWmBlock / 64;
constexpr uint32_t kWmQueue = 256;
constexpr uint32_t kWmWaveLds = 64 * 8 + kWmQueue * 4;
// (after the tuple masks: the one-byte direct tuples' 256-entry tables,
// kMaxDirect x 2 KB, read from LDS instead of one L2 request per packet)
constexpr uint32_t kWmDirLds = 2048u * 2;
// ... and, when the CU's LDS has room for them after all that, each wave's
// gates of up to kWmGateHold tiles (stored together after those tiles,
// as the slab kernels hold theirs; bg_wm_body.h)
constexpr uint32_t kWmGateHold = 8;
BG_HD uint64_t wm_tags_lds_base(uint32_t nbp, uint32_t kw) {
  return ((uint64_t)nbp * 4 + 15) / 16 * 16 + (uint64_t)kMaxTuples * kw * 8 + kWmDirLds +
         (uint64_t)kWmWaves * kWmWaveLds;
}
BG_HD uint32_t wm_hold_tiles(uint32_t nbp, uint32_t kw) {
  const uint64_t base = wm_tags_lds_base(nbp, kw);
  const uint64_t room = base < kLdsPerCu ? kLdsPerCu - base : 0;
  const uint32_t h = (uint32_t)(room / ((uint64_t)kWmWaves * 128)) & ~7u;
  return h < kWmGateHold ? h : kWmGateHold;
}
BG_HD uint64_t wm_tags_lds_bytes(uint32_t nbp, uint32_t kw) {
  return wm_tags_lds_base(nbp, kw) + (uint64_t)kWmWaves * 128 * wm_hold_tiles(nbp, kw);
}

struct CkArgs {
  uint8_t *frames;
  uint64_t stride, n;
  // non-null: frame i at ptrs[i] (device addresses of host-registered or
  // device memory, bg_cksum_ptrs), `stride` bytes readable / writable each
  const uint64_t *ptrs;
  uint16_t *ip_gates;  // may be null
  uint16_t *l4_gates;  // may be null
  int32_t mode;        // bit0 IPChecksum, bit1 L4Checksum
  int32_t verify;
};

// HashLB (core/modules/hash_lb.cc): CRC32C of the mode's hash input, then
// gates[(crc * num_gates) >> 32]. The CRC of an L-byte input with init 0 is
// linear in the input bytes, so it is the XOR of one table entry per byte
// position: crc = XOR_i crc_tab[i*256 + byte_i] (tables built on the host).
constexpr int kHlbL2 = 0, kHlbL3 = 1, kHlbL4 = 2, kHlbFields = 3;
struct HlbArgs {
  const uint8_t *frames;
  uint64_t stride, n;
  uint16_t *out;
  const uint32_t *crc_tab;  // L x 256
  const uint16_t *gtab;     // max(num_gates, 1) entries
  uint32_t mode, L, num_gates, ngtab;
  FieldPlan fp;             // kHlbFields
};

// ACL (core/modules/acl.cc): first matching rule in order; rule r is 8
// dwords {src addr, src mask, dst addr, dst mask, ports, port mask, drop,
// valid} in the packet's LE byte order (addresses / ports as loaded from the
// frame); nrules is padded to a multiple of 4 with valid = 0 rules.
struct AclArgs {
  const uint8_t *frames;
  uint64_t stride, n;
  uint16_t *out;
  const uint32_t *rules;
  uint32_t nrules, igate;
  // Bit-vector form (bg_acl.hip AclBvOp; bv == nullptr: the rule scan).
  // Per dimension d (0 src addr, 1 dst addr, 2 src port, 3 dst port) the
  // values fall into elementary intervals; interval i of dimension d has a
  // bit vector V_d[i] of the rules that match there (nw words, bit r = rule
  // r) and a summary word S_d[i] (bit g: some rule of words [gG, gG + G)).
  // Addresses: the interval is found by binary search over the sorted
  // interval starts B_0 / B_1 (staged in LDS, k0 / k1 entries, host byte
  // order); ports: a 64 K-entry u16 table indexed by the port's raw frame
  // bytes. Word offsets into bv:
  const uint32_t *bv;
  uint32_t k0, k1, lg0, lg1, nw, grp;
  uint32_t b_off[2], s_off[4], v_off[4], p_off[2], d_off;
  // Decision-tree form (AclTreeOp; tree == nullptr: none): ntrees trees
  // (one per class of rules, bg_acl_api.cc build_tree) in one image of
  // tree_words dwords, staged whole in LDS: 16-byte leaf rule records, then
  // the internal nodes' child arrays. A node reference (roots, children):
  //   leaf      bit 31 | count << 16 | first record (16-byte units)
  //   internal  dim << 25 | k << 21 | shift << 16 | child array (dword)
  // where the child taken is bits [shift, shift + k) of the dimension's
  // value: 0 src addr, 1 dst addr (host order), 2 the ports (src port in
  // the low half, dst port in the high half, host order).
  // A record: {src addr, dst addr, ports (as above), src prefix length |
  // dst prefix length << 6 | src port exact << 12 | dst port exact << 13 |
  // drop << 14 | rule index << 16}; a leaf's records are, in list order,
  // the class's rules that can still be the first match in its box, cut
  // after one that covers it. The packet's rule: the lowest index matched.
  const uint32_t *tree;
  uint32_t tree_words, ntrees;
  uint32_t roots[4];
};

// IPLookup (core/modules/ip_lookup.cc): DIR-24-8 longest-prefix match on
// the destination address. Entries (u16): 0 = no route, 0x8000 | g = the
// /24 is extended into tbl8 group g, else next hop + 1.
struct LpmArgs {
  const uint8_t *frames;
  uint64_t stride, n;
  uint16_t *out;
  const uint16_t *tbl24;  // 2^24 entries
  const uint16_t *tbl8;   // groups x 256 entries
  uint32_t default_gate, pad;
  // DIR-16-8-8, the same entries with tbl24 folded (null: DIR-24-8): tbl16
  // (2^16 entries) per /16 block either the value every /24 of the block
  // has in tbl24, or 0x8000 | g for tbl2 group g (256 entries: the block's
  // tbl24 entries, which may extend into tbl8 as before)
  const uint16_t *tbl16;
  const uint16_t *tbl2;
};

// UpdateTTL (core/modules/update_ttl.cc): in place on the frames.
struct TtlArgs {
  uint8_t *frames;
  uint64_t stride, n;
  uint16_t *out;  // 0 (emitted) or DROP_GATE
};

// StaticNAT (core/modules/static_nat.cc): pairs of 4 dwords {start in
// the matched direction, start on the other side, size, 0} (host order),
// padded to a multiple of 4 with size-0 pairs; dir 0 rewrites the source
// (input gate 0 -> output gate 1), dir 1 the destination (1 -> 0).
struct NatArgs {
  uint8_t *frames;
  uint64_t stride, n;
  uint16_t *out;
  const uint32_t *pairs;
  uint32_t npairs, dir;
};

// IPEncap (core/modules/ip_encap.cc): slot i at slots + i*stride, its data
// at + head[i], metadata area at + meta_off; offs: attr offsets of ip_src,
// ip_dst, ip_proto, ip_nexthop, ether_type (< 0: invalid).
struct EncapArgs {
  uint8_t *slots;
  uint64_t stride, n;
  int32_t meta_off, offs[5];
  uint16_t *head;  // data_off, in/out
  uint32_t *len;   // pkt_len, in/out
  uint16_t *out;
};

// Rewrite (core/modules/rewrite.cc): packet i becomes template (start + i) %
// ntempl: its bytes at slot + headroom in whole 16-byte chunks up to the
// size rounded to 32 (the reference's sloppy 32-byte block copy; the
// template buffer is zero past its size), head[i] = headroom, len[i] = size
constexpr uint32_t kRwMaxTemplates = 32;   // PacketBatch::kMaxBurst
constexpr uint32_t kRwMaxSize = 1536;      // Rewrite::kMaxTemplateSize
struct RewriteArgs {
  uint8_t *slots;
  uint64_t stride, n;
  const uint8_t *tmpl;    // ntempl x kRwMaxSize, zero past each size
  const uint16_t *tsize;  // ntempl
  uint32_t ntempl, start, headroom;
  uint32_t lpp_log2;      // lanes per packet = 2^lpp_log2 (<= 64)
  uint32_t units;         // 16-byte chunks of the largest rounded template
  uint32_t pad;
  uint16_t *head;         // data_off, out
  uint32_t *len;          // pkt_len, out
};

// NAT (core/modules/nat.cc): endpoint keys (addr raw | port raw << 32 |
// proto << 48), per-packet entry indices (or kDnatMiss / kDnatInvalid),
// the entries' translated endpoints and forward timestamps.
constexpr uint32_t kDnatMiss = 0xFFFFFFFFu;
constexpr uint32_t kDnatInvalid = 0xFFFFFFFEu;  // every code >= this drops
constexpr uint16_t kDropGate = 8192;
struct DnatArgs {
  uint8_t *frames;
  uint64_t stride, n;
  uint32_t dir, refresh;
  uint64_t now, timeout;  // a forward hit with now - ts > timeout is listed
  TableRef t;        // endpoint -> entry index (u32 values), KW = 1
  uint64_t *keys;    // per packet: the endpoint key
  uint32_t *res;     // per packet: entry / kDnatMiss / kDnatInvalid
  uint32_t *nmiss;   // forward misses of the batch
  uint32_t *nmiss_next;  // the next call's counter: zeroed by this launch
  const uint64_t *ent;  // per entry: translated endpoint
  uint64_t *ts;      // per entry: last_refresh
  uint64_t nent;     // entries the two arrays hold
  uint16_t *out;
  // apply over a packet list: res[k] = packet, mres[k] = entry, keys[k] =
  // its endpoint, k < nlist (the fused kernel's forward misses)
  uint32_t list, pad;
  uint64_t nlist;
  const uint32_t *mres;
  // per listed packet: the translated endpoint as the walk found it when it
  // reached the packet (a later packet of the batch may overwrite the
  // entry: Stamp uses the value of its own moment, nat.cc:353-360)
  const uint64_t *meps;
  // The reference's map holds both directions' entries (nat.h: one
  // HashTable): a reverse packet whose destination is an internal endpoint
  // finds that forward entry (t2 = the forward image, probed on a reverse
  // miss), and a forward packet whose source address is one of the NAT's
  // external addresses may meet an entry an earlier packet of the batch
  // creates (CreateNewEntry inserts ext_addr:port keys): such forward
  // packets are listed for the host's in-order walk (next addresses, raw
  // be32; list_fwd: more than kDnatMaxExt, list every forward packet).
  TableRef t2;
  uint32_t next, list_fwd;
  uint32_t ext[16];
};
constexpr int kDnatMaxExt = 16;

// Persistent ExactMatch kernel fed by a ring of batch descriptors
// (bg_ring.cc). Descriptor of ticket t at desc + (t % nslots) * 4: four
// 8-byte words, each carrying the tag (t + 1) & 0xFFFF in its top 16 bits
// (one untorn 8-byte store each, so a reader that sees four matching tags
// sees the whole descriptor, no fence):
//   w0 frames address | tag << 48     w1 gates address | tag << 48
//   w2 n | stride << 32 | tag << 48   w3 default gate | tag << 48
// The host then raises *pub (host memory) to t + 1. Workgroup 0 is the
// dispatcher: one lane polls *pub over PCIe and mirrors it into dev[1]
// (device memory), so the other workgroups poll L2, not PCIe. A worker
// workgroup claims a ticket from dev[0] (one atomic add), waits until
// dev[1] > t, reads the descriptor, classifies the batch and publishes
// done[t % nslots] = t + 1 (system scope, after a system release of its
// gate stores). When *pub has not moved for idle_ticks (s_memrealtime,
// 100 MHz), or the host sets *stop, the dispatcher sets dev[2]: every
// worker re-checks dev[1] once and exits if its ticket is still
// unpublished, and the grid ends. The host relaunches from its oldest
// unfinished ticket (re-classifying a finished batch is harmless).
// Submission lanes (one per worker thread), each its own ring of nslots
// descriptors, done words and published count; lane l's words at
// l * kRingLaneWords (128 bytes apart: an L2 line and a host line pair of
// their own, so lanes' claim atomics and submitters never share a line).
struct RingArgs {
  const uint64_t *desc;   // nlanes x nslots x kRingDescWords (4 used)
  uint32_t *done;         // host memory (mapped): nlanes x nslots
  const uint64_t *pub;    // host memory: tickets published, per lane
  const uint32_t *stop;   // host memory: the owner stops the grid
  uint32_t *ended;        // host memory: launch_id of the grid that ended
  unsigned long long *dev;  // device memory, per lane: [0] next ticket to
                            // claim, [1] published (mirror); then the stop word
  uint32_t nslots, nlanes;
  uint32_t launch_id, pad;
  uint64_t idle_ticks;
  FieldPlan fp;
  TableRef t;
};
// four waves: a ticket's packets are spread over 256 lanes (4 per lane per
// round), so a 1024-packet batch takes one round of loads and lookups
// rather than four on one wave (a ticket's latency is its rounds')
constexpr int kRingBlock = 256;
// + one wave that only writes the done words: a store's completion is
// waited for by the next load or atomic of the wave that issued it (vector
// memory operations retire in order), and a done word bound for host memory
// takes microseconds to complete under load, so the wave that claims the
// next ticket must not be the one that wrote the last done word
constexpr int kRingThreads = kRingBlock + 64;
constexpr int kRingLaneWords = 16;
// A worker workgroup takes up to kRingRunMax published tickets of its lane
// as one run, and claims about kRingRunPackets packets' worth of tickets at
// a time while its lane has a backlog: four rounds of its 256 lanes x 4
// packets (kRingRunPacketsIdle, one round, while the lane's tickets arrive
// slower than they are served). Claims of one round (round 5) left a run's
// fixed costs -- the claim, the publication wait, the descriptor reads, the
// acquire, the done words -- on 1024 packets, and 512 / 1024-packet tickets
// ran at 25-36 Gpps from 16 submitters against 48 at 256; claims of four
// rounds: 58-62 Gpps at every size from 256 up, 16 submitters above 4
// (profiles/r06/ring_ab_r06h.json: claims of 1, 2 and 4 rounds measured)
constexpr uint32_t kRingRunMax = 16;
constexpr uint32_t kRingRunPackets = kRingBlock * 16;
constexpr uint32_t kRingRunPacketsIdle = kRingBlock * 4;
// a descriptor slot: 4 tagged words + 4 of padding, one 64-byte line, so a
// host writing it through write-combining buffers fills a whole buffer,
// which leaves for the device at once (a half-written line can wait in the
// buffer until the next descriptor's stores)
constexpr int kRingDescWords = 8;

// descriptor word 3, bits 16..: how the ticket's frames and gates meet the
// host (bg_ring_set_coherence). kRingSysAcquire: the frames may sit in
// memory the device caches non-coherently (mapped host memory that is not
// uncached, or device memory a copy engine wrote): acquire at system scope
// (invalidates L2's non-coherent lines) instead of agent scope (the CU's
// L1 only). kRingRelease: the done word is a system-scope release (writes
// L2 back) instead of a relaxed store after every wave's gate stores have
// completed (the gates are system-scope write-through stores).
// a WildcardMatch ring's table default gate: "no rule matched" (each
// ticket's own default gate applies)
constexpr uint32_t kRingNoGate = 0x10000;
constexpr uint64_t kRingSysAcquire = 1ull << 16;
constexpr uint64_t kRingRelease = 1ull << 17;
constexpr int kRingMaxLanes = 64;  // one dispatcher wave lane each

#ifndef __HIPCC_RTC__  // host launchers: not part of a run-time compile
// Launchers (grid sizing from the device's CU count). Return hipSuccess or
// the launch error.
hipError_t launch_em(const EmArgs &a, int num_cus, hipStream_t s);
hipError_t launch_wm(const WmArgs &a, int num_cus, hipStream_t s);
hipError_t launch_cksum(const CkArgs &a, int num_cus, hipStream_t s);
hipError_t launch_hlb(const HlbArgs &a, int num_cus, hipStream_t s);
hipError_t launch_acl(const AclArgs &a, int num_cus, hipStream_t s);
hipError_t launch_lpm(const LpmArgs &a, int num_cus, hipStream_t s);
hipError_t launch_ttl(const TtlArgs &a, int num_cus, hipStream_t s);
hipError_t launch_nat(const NatArgs &a, int num_cus, hipStream_t s);
hipError_t launch_encap(const EncapArgs &a, int num_cus, hipStream_t s);
hipError_t launch_rewrite(const RewriteArgs &a, int num_cus, hipStream_t s);
hipError_t launch_dnat_apply(const DnatArgs &a, int num_cus, hipStream_t s);
hipError_t launch_dnat_image(const uint64_t *d_up, size_t k, uint64_t *img,
                             hipStream_t s);
// lookup + stamp of the final hits in one pass; forward misses and forward
// hits on expired mappings listed in res/keys (count in *nmiss)
hipError_t launch_dnat_fused(const DnatArgs &a, int num_cus, hipStream_t s);
// up = [idx x k | ep x k | ts x k]: ent[idx[i]] = ep[i], ts[idx[i]] = ts[i]
hipError_t launch_dnat_scatter(const uint64_t *d_up, size_t k, uint64_t *ent,
                               uint64_t *ts, hipStream_t s);
// the persistent ring kernel: `blocks` workgroups
hipError_t launch_em_ring(const RingArgs &a, int blocks, hipStream_t s);
hipError_t launch_wm_ring(const RingArgs &a, const WmArgs &w, int blocks, hipStream_t s);
// WildcardMatch with the tag words in LDS (t.lds == kLdsTags)
hipError_t launch_wm_tags(const WmArgs &a, int num_cus, hipStream_t s);
// all key fields within two 16-byte chunks, <= 2 byte-permutes per key dword
#endif
bool fits_nch2(const FieldPlan &fp);

}  // namespace bg

#endif  // BESS_AMD_BG_KERNELS_H_
