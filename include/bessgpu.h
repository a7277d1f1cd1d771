/*
 * bessgpu.h -- C ABI of libbessgpu.so, the MI355X (gfx950) implementation of
 * BESS's per-batch packet-classification hot path.
 *
 * Plain C: pointers, sizes, integers. Every entry point returns 0 on success
 * or a negative errno (-EINVAL, -ENOENT, -ENOSPC, -ENODEV, -EIO, ...), the
 * way the reference reports CommandFailure(errno, ...) (core/message.h:44-53);
 * bg_last_error() returns the message of the calling thread's last failure.
 *
 * Which reference interface each group replaces (NetSys/bess paths):
 *   bg_em_*   ExactMatchTable<gate_idx_t> (core/utils/exact_match_table.h:
 *             146-458) and the datapath of ExactMatch::ProcessBatch
 *             (core/modules/exact_match.cc:224-244)
 *   bg_wm_*   WildcardMatch tuple tables + LookupEntry / ProcessBatch
 *             (core/modules/wildcard_match.cc:136-203, 278-315)
 *   bg_cksum  IPChecksum::ProcessBatch (core/modules/ip_checksum.cc:39-84)
 *             and L4Checksum::ProcessBatch (core/modules/l4_checksum.cc:41-83)
 *   bg_module_*  the module surface BESS's control plane drives: create with
 *             an <Class>Arg protobuf (core/module.h:93-102 MODULE_INIT_FUNC,
 *             core/bessctl.cc:1205 CreateModule), run a command by name with
 *             its protobuf argument (core/module.cc:92-116 RunCommand,
 *             core/bessctl.cc:1760 ModuleCommand), and ProcessBatch over a
 *             batch of packet head pointers (core/module.h:226) returning the
 *             per-packet EmitPacket gate (core/module.h:543).
 *
 * Device pointers (d_*) are HIP device memory on the handle's device;
 * `stream` is a hipStream_t. NULL means the legacy default stream for the
 * device-slab calls, and the calling thread's own non-blocking stream for
 * the synchronous host paths (*_process_host, bg_module_process), so that
 * worker threads never serialise on one stream.
 * Frame slabs: frame i starts at d_frames + i*stride (= Packet::head_data(),
 * core/packet.h:84-94); stride must be a multiple of 16 and d_frames 16-byte
 * aligned.
 */
#ifndef BESSGPU_H_
#define BESSGPU_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BG_MAX_GATES 8192   /* core/gate.h:57 */
#define BG_DROP_GATE 8192   /* core/gate.h:58 */
#define BG_GATE_NONE 0xFFFF /* packet not emitted (L4Checksum) */
#define BG_MAX_FIELDS 8     /* exact_match_table.h:50 */
#define BG_MAX_TUPLES 8     /* wildcard_match.h:45 */
#define BG_KEY_BYTES 64     /* sizeof(ExactMatchKey) */

#define BG_CK_IP 1 /* IPChecksum */
#define BG_CK_L4 2 /* L4Checksum */

typedef void *bg_stream_t; /* hipStream_t */

/* A field as resolved by ExactMatchTable::DoAddField (exact_match_table.h:
 * 391-443) or WildcardMatch::Init (wildcard_match.cc:111-134). */
typedef struct bg_field {
  int32_t offset; /* bytes from head_data() */
  int32_t size;   /* 1..8 */
  int32_t pos;    /* byte position in the key */
  int32_t attr_id; /* -1: offset field (metadata fields: not on the device) */
  uint64_t mask;  /* EM: ExactMatchField::mask (key byte order); WM: unused */
} bg_field;

/* ---- runtime ---------------------------------------------------------- */
const char *bg_version(void);
const char *bg_last_error(void);
int bg_device_count(void);
/* allocate / free / copy device memory (convenience for C callers) */
int bg_malloc(int device, size_t bytes, void **d_ptr);
int bg_free(void *d_ptr);
int bg_memcpy_h2d(void *d_dst, const void *src, size_t bytes, bg_stream_t s);
int bg_memcpy_d2h(void *dst, const void *d_src, size_t bytes, bg_stream_t s);
int bg_stream_sync(bg_stream_t s);

/* ---- ExactMatch -------------------------------------------------------- */
typedef struct bg_em bg_em;
int bg_em_create(const bg_field *fields, int nfields, bg_em **out);
void bg_em_destroy(bg_em *em);
size_t bg_em_key_size(const bg_em *em); /* total_key_size_ */
/* key: total_key_size bytes, as ExactMatchTable::gather_key lays it out
 * (exact_match_table.h:332-357). Insert-or-overwrite (cuckoo_map.h:182-187). */
int bg_em_add(bg_em *em, const uint8_t *key, uint16_t gate);
int bg_em_delete(bg_em *em, const uint8_t *key); /* -ENOENT if absent */
void bg_em_clear(bg_em *em);
size_t bg_em_count(const bg_em *em);
/* iterate rules (unspecified order); returns 1 with a rule, 0 at the end */
int bg_em_iter(const bg_em *em, size_t *cursor, uint8_t *key_out,
               uint16_t *gate_out);
/* Rebuild/upload the device table if rules changed (control path). */
int bg_em_sync(bg_em *em, int device, bg_stream_t stream);
/* attr_name fields (exact_match.cc:230-236 reads
 * ptr_attr(this, attr_id, pkt) = the packet's metadata area + the
 * attribute's offset that bessd's metadata allocator assigned,
 * core/module.h:679-684). On the device each slot carries that metadata
 * area at byte meta_off; attr_offsets[attr_id] is attr_offset(attr_id)
 * (nattrs entries, < 0: none -> EINVAL, where the reference would
 * dereference a null attribute pointer). meta_off -1: the attribute offsets
 * only (staged rows, bg_em_classify_staged; the device-slab calls are
 * unbound, including a slab layout an earlier call bound). Until bound,
 * classify returns ENOTSUP for tables with attr fields; bg_em_process_host
 * (head pointers only) never carries metadata and keeps returning ENOTSUP.
 * A bind is a table change: pipes' rings built on the old offsets retire. */
int bg_em_bind_meta(bg_em *em, int meta_off, const int32_t *attr_offsets,
                    int nattrs);
/* Device-resident classify: d_gates[i] = gate for frame i (default_gate on
 * a miss). Calls bg_em_sync implicitly when needed (not capturable then). */
int bg_em_classify(bg_em *em, const void *d_frames, size_t stride, size_t n,
                   uint16_t default_gate, uint16_t *d_gates, bg_stream_t stream);
/* Host batch (PacketBatch-style head pointers): stage the key window of
 * each frame into pinned memory, classify, copy gates back; synchronous. */
int bg_em_process_host(bg_em *em, const uint8_t *const *heads, size_t n,
                       uint16_t default_gate, uint16_t *gates,
                       bg_stream_t stream);
/* n rules at once: rule i's key at keys + i*key_stride, its gate gates[i]
 * (bg_em_add each). part >= 0: only the rules that fall into partition
 * `part` of an nparts-way sharded table are kept (a rank of a multi-GPU
 * build inserts its own share only). */
int bg_em_add_many(bg_em *em, const uint8_t *keys, size_t n, size_t key_stride,
                   const uint16_t *gates, int part, int nparts);
/* Sharded table build (multi-GPU): fix a layout of `nparts` partitions for
 * the current rules, export the host image of one partition, and attach an
 * externally assembled (all-gathered) device image. bg_em_plan_count fixes
 * the layout from the largest partition's entry count, which a rank that
 * holds only its own partition learns from the other ranks (all-reduce
 * MAX of bg_em_part_count). A partition image depends only on the rule
 * set, not on insertion order. */
int bg_em_plan(bg_em *em, int nparts, uint64_t *part_bytes);
int bg_em_part_count(const bg_em *em, int part, int nparts, uint64_t *count);
int bg_em_plan_count(bg_em *em, int nparts, uint64_t max_part_entries,
                     uint64_t *part_bytes);
int bg_em_build_part(bg_em *em, int part, void *host_dst);
int bg_em_attach(bg_em *em, int device, const void *d_image);
/* The sharded build over RCCL (xGMI), with no torch: see bg_comm below. */
/* bytes of the current device table image and whether it lives in LDS */
int bg_em_table_info(const bg_em *em, uint64_t *bytes, int *in_lds);
/* Classify staged windows: byte 0 of window i (at d_win + i*stride) is frame
 * offset win_off of packet i (the host path stages only the field window). */
int bg_em_classify_window(bg_em *em, const void *d_win, size_t stride,
                          size_t n, int win_off, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream);
/* [lo, hi): the frame bytes the fields cover (MakeKeys reads) */
void bg_em_window(const bg_em *em, int *lo, int *hi);
/* Staged rows with metadata (the aggregation queue, host packets): byte 0
 * of row i (d_win + i*stride) is frame byte win_off of packet i, and row
 * offset meta_row + a is byte a of packet i's metadata area, so an attr
 * field reads the row at meta_row + attr_offset (offsets as bound by
 * bg_em_bind_meta, whose meta_off may then be -1: offsets only). */
int bg_em_classify_staged(bg_em *em, const void *d_win, size_t stride, size_t n,
                          int win_off, int meta_row, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream);
/* [lo, hi): the metadata bytes the attr fields read (lo == hi: none);
 * -ENOTSUP while attr offsets are unbound */
int bg_em_meta_window(const bg_em *em, int *lo, int *hi);

/* ---- Rule-table collective (RCCL over xGMI) -----------------
 * The only exchange of the multi-GPU path: the ExactMatch image of a rule
 * set too large to build on every GPU (C5). A communicator spans the GPUs
 * that share one rule set, one rank per GPU:
 *   bg_comm_init_all   every listed GPU of this process at once (a bessd
 *                      with workers on several GPUs; ncclCommInitAll);
 *   bg_comm_unique_id + bg_comm_init_rank   one rank per process (the id
 *                      travels by the caller's own means).
 * bg_em_allgather (one rank; collective: every rank calls it): the ranks
 * agree on the layout with one all-reduce MAX of their partition sizes,
 * build their own partition (the table may hold only partition `rank`'s
 * rules: bg_em_add_many part = rank) and one all-gather assembles the image,
 * which becomes the table's image on the rank's device. nranks: 1, 2, 4 or
 * 8. bg_em_allgather_all: the same for all ranks of an init_all set from
 * one thread (grouped calls), the table holding all rules. */
#define BG_COMM_ID_BYTES 128
typedef struct bg_comm bg_comm;
int bg_comm_unique_id(uint8_t *id /* BG_COMM_ID_BYTES */);
int bg_comm_init_rank(const uint8_t *id, int nranks, int rank, int device,
                      bg_comm **out);
int bg_comm_init_all(const int *devices, int ndev, bg_comm **comms);
void bg_comm_destroy(bg_comm *c);
int bg_comm_info(const bg_comm *c, int *rank, int *nranks, int *device);
int bg_em_allgather(bg_em *em, bg_comm *comm, bg_stream_t stream);
/* the rank's last bg_em_allgather: ns3 = {size all-reduce, partition build
 * on the host, upload + all-gather} in ns; bytes = the gathered image */
int bg_comm_last_stats(const bg_comm *c, uint64_t *ns3, uint64_t *bytes);
int bg_em_allgather_all(bg_em *em, bg_comm *const *comms, int ncomm);

/* ---- WildcardMatch ----------------------------------------------------- */
typedef struct bg_wm bg_wm;
int bg_wm_create(const bg_field *fields, int nfields, bg_wm **out);
void bg_wm_destroy(bg_wm *wm);
size_t bg_wm_key_size(const bg_wm *wm);
/* key/mask: 64-byte keys as ExtractKeyMask builds them (wildcard_match.cc:
 * 215-276). FindTuple/AddTuple/Insert of CommandAdd (317-354); -ENOSPC on
 * a 9th distinct mask. */
int bg_wm_add(bg_wm *wm, const uint8_t *key, const uint8_t *mask,
              int32_t priority, uint16_t gate);
/* CommandDelete/DelEntry (357-377, 302-315), including the reference's
 * "failed remove on an empty tuple erases it and succeeds" behaviour. */
int bg_wm_delete(bg_wm *wm, const uint8_t *key, const uint8_t *mask);
void bg_wm_clear(bg_wm *wm); /* Clear(): tables emptied, tuples kept */
int bg_wm_num_tuples(const bg_wm *wm);
int bg_wm_tuple_mask(const bg_wm *wm, int t, uint8_t *mask_out);
size_t bg_wm_tuple_count(const bg_wm *wm, int t);
int bg_wm_iter(const bg_wm *wm, int t, size_t *cursor, uint8_t *key_out,
               int32_t *priority, uint16_t *gate);
int bg_wm_sync(bg_wm *wm, int device, bg_stream_t stream);
/* as bg_em_bind_meta (wildcard_match.cc:177-195: buffer +
 * mt_offset_to_databuf_offset(attr_offset(attr_id)), packet.h:189-191) */
int bg_wm_bind_meta(bg_wm *wm, int meta_off, const int32_t *attr_offsets,
                    int nattrs);
int bg_wm_classify(bg_wm *wm, const void *d_frames, size_t stride, size_t n,
                   uint16_t default_gate, uint16_t *d_gates, bg_stream_t stream);
int bg_wm_process_host(bg_wm *wm, const uint8_t *const *heads, size_t n,
                       uint16_t default_gate, uint16_t *gates,
                       bg_stream_t stream);
/* in_lds: 0 table probed in L2/MALL, 1 table in LDS, 2 key filter in LDS,
 * 3 tag words in LDS; bits 8 and up: the image's direct tuples (one- or
 * two-byte masks read by index, not hashed) */
int bg_wm_table_info(const bg_wm *wm, uint64_t *bytes, int *in_lds);
int bg_wm_classify_window(bg_wm *wm, const void *d_win, size_t stride,
                          size_t n, int win_off, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream);
void bg_wm_window(const bg_wm *wm, int *lo, int *hi);
/* as bg_em_classify_staged / bg_em_meta_window */
int bg_wm_classify_staged(bg_wm *wm, const void *d_win, size_t stride, size_t n,
                          int win_off, int meta_row, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream);
int bg_wm_meta_window(const bg_wm *wm, int *lo, int *hi);
/* Run-time compiled kernels (bess_amd/csrc/bg_wm_jit.cc). A tag-word image's
 * tuple data (masks, seeds, direct tuples) and its key plan are compiled
 * into a specialised kernel with hiprtc on a background thread; launches use
 * it once ready and the ahead-of-time kernel until then (same results).
 * bg_wm_jit_wait syncs the table on `device` and blocks until that kernel
 * is ready: 0, -ETIMEDOUT, -ENOEXEC (compile failed; the ahead-of-time kernel
 * stays in use) or -ENOENT (the image has no tag words: nothing to compile).
 * bg_wm_jit_source copies the generated source (*need: bytes incl. NUL;
 * device < 0: the source for the current rules' host image, no device). */
int bg_wm_jit_wait(bg_wm *wm, int device, int timeout_ms);
int bg_wm_jit_source(bg_wm *wm, int device, char *buf, size_t len, size_t *need);
/* Build the host image of the current rules and compile its specialised
 * kernel on the calling thread; no device needed (0, -ENOENT: no tag-word
 * image, -ENOEXEC: compile failed, log in `log`). */
int bg_wm_jit_check(bg_wm *wm, char *log, size_t len, size_t *code_bytes);
/* Before a process exits: stop the background compiler (a compile in
 * progress in the bg_rtc helper process is killed). Idempotent; later
 * tables keep the ahead-of-time kernels. (bess_amd/_lib.py registers it with
 * Python's atexit; a C process gets it registered at its first compile.) */
void bg_shutdown(void);

/* A caller's stream the library may fence lazily. A table image replaced by
 * a rule change is freed only after every launch that reads it has
 * finished; on a stream the library does not know, each launch records an
 * event to prove that (a few microseconds per launch: the HIP runtime
 * cannot be asked about a stream handle that may have been destroyed). An
 * attached stream is fenced once, when an image retires, instead. Detach
 * before destroying the stream: detach synchronizes it. 0 or -errno. */
int bg_stream_attach(bg_stream_t stream);
int bg_stream_detach(bg_stream_t stream);

/* ---- IPChecksum / L4Checksum ------------------------------------------ */
/* mode: BG_CK_IP, BG_CK_L4 or both (= IPChecksum -> L4Checksum pipeline:
 * only frames IPChecksum emits on gate 0 reach L4Checksum). Checksums are
 * written in place into the frames; gates: 0 forward, 1 fail, BG_GATE_NONE
 * not emitted / not reached. d_ip_gates / d_l4_gates may be NULL. */
int bg_cksum(int device, void *d_frames, size_t stride, size_t n, int mode,
             int verify, uint16_t *d_ip_gates, uint16_t *d_l4_gates,
             bg_stream_t stream);
/* Frames by pointer: frame i at d_ptrs[i] (the device address of host memory
 * registered with bg_host_register, or device memory), each with `span`
 * readable / writable bytes; the checksum words are written there in place.
 * d_ptrs itself may be mapped host memory. */
int bg_cksum_ptrs(int device, const uint64_t *d_ptrs, size_t span, size_t n, int mode,
                  int verify, uint16_t *d_ip_gates, uint16_t *d_l4_gates,
                  bg_stream_t stream);
/* host frames (head pointers, each with >= `span` readable/writable bytes):
 * staged to the device, processed, written back; synchronous. */
int bg_cksum_process_host(int device, uint8_t *const *heads, size_t n,
                          size_t span, int mode, int verify,
                          uint16_t *ip_gates, uint16_t *l4_gates,
                          bg_stream_t stream);

/* ---- host memory the device works on in place --------------------------- */
/* Register host memory (BESS's packet pool: core/packet_pool.h, the DPDK
 * mempool's memory chunks, rte_mempool_mem_iter) for device access in place
 * (hipHostRegister, mapped on every device). Then a bg_pipe of a module that
 * works on whole frames (IPChecksum, L4Checksum) hands the device each
 * packet's head pointer instead of a copy of its bytes: the kernel reads the
 * frame over PCIe and writes the checksum words into the packet buffer.
 * Unregister only with no packet of the region in flight. -EEXIST: overlaps
 * a registered region. */
int bg_host_register(void *base, size_t bytes);
int bg_host_unregister(void *base);
/* the device address of host bytes [p, p + len) in a registered region */
int bg_host_dev_addr(const void *p, size_t len, uint64_t *dev);

/* ---- kernel paths (parity tests) ---------------------------------------- */
/* Several kernels compute each result (flow table staged in LDS or probed in
 * L2; coalesced 64-byte-slot slab shape or one packet per lane; for
 * WildcardMatch tag words in LDS or a key filter). bg_set_path_flags picks
 * among them process-wide so the parity tests can run every path against
 * the oracle; no result depends on the flags. 0 = the measured defaults.
 * The product library reads no environment variable. */
#define BG_PATH_FORCE_LDS 1
#define BG_PATH_NO_LDS 2
#define BG_PATH_NO_SLAB 4
#define BG_PATH_WM_NO_TAGS 8
#define BG_PATH_ACL_SCAN 16 /* ACL: rule scan with scalar loads (not LDS) */
#define BG_PATH_ACL_BV 32   /* ACL: per-dimension bit vectors */
#define BG_PATH_ACL_LDS 64  /* ACL: rule scan from LDS (not the decision tree) */
#define BG_PATH_LPM_DIR24 128 /* IPLookup: DIR-24-8 tables (not DIR-16-8-8) */
#define BG_PATH_PIPE_NO_RING 256 /* pipes launch per slot (not via a ring) */
#define BG_PATH_WM_NO_JIT 512 /* WildcardMatch: the ahead-of-time kernel, never the
                                run-time compiled one (bg_wm_jit_wait) */
#define BG_PATH_RING_HOST_DESC 1024 /* rings created now keep their descriptors in
                                       pinned host memory (not device memory
                                       through the BAR) */
int bg_set_path_flags(uint32_t flags);
uint32_t bg_get_path_flags(void);

/* ---- diagnostics ------------------------------------------------------- */
/* The key the classify kernels build for `frame` from `fields` (em_masks 1:
 * ExactMatch field masks applied; 0: WildcardMatch raw field bytes), run on
 * the host with the kernels' own field plan (byte-permute or direct form).
 * key_out: 64 bytes. No device needed. */
int bg_debug_key(const bg_field *fields, int nfields, int em_masks,
                 const uint8_t *frame, uint8_t *key_out);

/* ---- HashLB (core/modules/hash_lb.cc) --------------------------------- */
/* ProcessBatch 155-236: CRC32C of the mode's hash input (l2: MAC words,
 * l3: IPs, l4: IPs + ports + proto, fields: MakeKeys key over
 * total_key_size), gate = gates[(crc * num_gates) >> 32] (hash_range 53-68).
 * l2/l3/l4 read the frame from offset 0 (slots of >= 16/64 bytes). */
#define BG_HLB_L2 0
#define BG_HLB_L3 1
#define BG_HLB_L4 2
#define BG_HLB_FIELDS 3
#define BG_HLB_MAX_GATES 16384 /* hash_lb.h kMaxGates */
typedef struct bg_hlb bg_hlb;
int bg_hlb_create(int mode, const bg_field *fields, int nfields, bg_hlb **out);
void bg_hlb_destroy(bg_hlb *h);
/* hash_len: bytes hashed (fields mode); -1 = total_key_size of the fields */
int bg_hlb_set_mode(bg_hlb *h, int mode, const bg_field *fields, int nfields,
                    int hash_len);
/* gate table gates[0..n) (n >= 1: the reference's gates_ prefix) and
 * num_gates <= n. num_gates == 0: every packet takes gates[0]. */
int bg_hlb_set_gates(bg_hlb *h, const uint16_t *gates, size_t n,
                     size_t num_gates);
void bg_hlb_window(const bg_hlb *h, int *lo, int *hi);
int bg_hlb_classify(bg_hlb *h, const void *d_frames, size_t stride, size_t n,
                    int win_off, uint16_t *d_gates, bg_stream_t stream);

/* ---- ACL (core/modules/acl.cc) ----------------------------------------- */
/* ACL::ACLRule (acl.h:43-57) in host byte order: Ipv4Prefix addr / mask
 * values, be16_t port values (0 = wildcard). */
typedef struct bg_acl_rule {
  uint32_t src_addr, src_mask, dst_addr, dst_mask;
  uint16_t src_port, dst_port;
  uint8_t drop, pad[3];
} bg_acl_rule;
typedef struct bg_acl bg_acl;
int bg_acl_create(bg_acl **out);
void bg_acl_destroy(bg_acl *h);
/* append rules in order (ACL::CommandAdd -> Init, acl.cc:42-58) */
int bg_acl_add(bg_acl *h, const bg_acl_rule *rules, size_t n);
void bg_acl_clear(bg_acl *h);
size_t bg_acl_count(const bg_acl *h);
/* ProcessBatch 63-95: out[i] = igate (first matching rule forwards) or
 * BG_DROP_GATE (it drops, or no rule matches). Stride >= 64. */
int bg_acl_classify(bg_acl *h, const void *d_frames, size_t stride, size_t n,
                    uint16_t igate, uint16_t *d_out, bg_stream_t stream);
/* Diagnostic (host only, no device): the decision-tree image the classify
 * kernel stages in LDS for the current rule list (layout: AclArgs in
 * bess_amd/csrc/bg_kernels.h) into img (capacity cap words; *words = its
 * size) and the roots of its *ntrees (<= 4) trees. -ENOENT when the list
 * gets no trees (masks that are not prefixes, > 8192 rules, or an image
 * past 112 KB). */
int bg_acl_tree(bg_acl *h, uint32_t *img, size_t cap, size_t *words, uint32_t *roots,
                int *ntrees);

/* ---- IPLookup (core/modules/ip_lookup.cc) ----------------------------- */
/* Longest-prefix match on the IPv4 destination with rte_lpm's table
 * semantics (DPDK 19.11, as ip_lookup.cc:54-241 uses it): add replaces the
 * next hop of an existing (prefix, depth); a new rule fails with -ENOSPC
 * when max_rules rules exist or, deeper than /24, when its /24 block needs a
 * tbl8 group and max_tbl8s are in use; delete of an absent rule -EINVAL.
 * Addresses in host byte order; depth 1..32; next hop <= 0x7FFE. */
typedef struct bg_lpm bg_lpm;
int bg_lpm_create(uint32_t max_rules, uint32_t max_tbl8s, bg_lpm **out);
void bg_lpm_destroy(bg_lpm *h);
int bg_lpm_add(bg_lpm *h, uint32_t ip, int depth, uint32_t next_hop);
int bg_lpm_delete(bg_lpm *h, uint32_t ip, int depth);
void bg_lpm_clear(bg_lpm *h); /* rte_lpm_delete_all */
size_t bg_lpm_count(const bg_lpm *h);
/* ProcessBatch 76-150: out[i] = next hop of the longest matching prefix of
 * packet i's destination (bytes 30..33), else default_gate. Stride >= 64. */
int bg_lpm_classify(bg_lpm *h, const void *d_frames, size_t stride, size_t n,
                    uint16_t default_gate, uint16_t *d_out, bg_stream_t stream);

/* ---- UpdateTTL (core/modules/update_ttl.cc) --------------------------- */
/* ProcessBatch 39-58 in place on a device slab: ttl > 1 -> ttl - 1 and the
 * IPv4 checksum updated incrementally (UpdateChecksum16(csum, 2, 1)), out[i]
 * = 0; ttl <= 1 -> out[i] = BG_DROP_GATE, frame untouched. Stride >= 32. */
int bg_update_ttl(int device, void *d_frames, size_t stride, size_t n,
                  uint16_t *d_out, bg_stream_t stream);

/* ---- StaticNAT (core/modules/static_nat.cc) --------------------------- */
/* Address pairs [int_addr, +size) <-> [ext_addr, +size), host byte order,
 * in order. ProcessBatch 146-181 in place: dir 0 (input gate 0) maps the
 * source of the first pair whose internal range holds it and emits on gate
 * 1; dir 1 maps the destination from the external range and emits on gate
 * 0; IPv4 and TCP/UDP checksums updated incrementally (RFC 1624). */
typedef struct bg_snat bg_snat;
int bg_snat_create(bg_snat **out);
void bg_snat_destroy(bg_snat *h);
int bg_snat_add(bg_snat *h, uint32_t int_addr, uint32_t ext_addr, uint32_t size);
size_t bg_snat_count(const bg_snat *h);
int bg_snat_classify(bg_snat *h, void *d_frames, size_t stride, size_t n,
                     int dir, uint16_t *d_out, bg_stream_t stream);

/* ---- NAT (core/modules/nat.{h,cc}): dynamic address/port translation --- */
/* Init (nat.cc:46-96): naddr external addresses (dotted strings) with
 * nranges[i] port ranges each, flattened in begin / end / suspended (end
 * exclusive as in PortRange; no ranges = [0, 65535)); errors and messages as
 * the reference. seed: the Random the port search draws from (the
 * reference seeds it from rdtsc). */
typedef struct bg_dnat bg_dnat;
int bg_dnat_create(const char *const *addrs, int naddr, const int32_t *nranges,
                   const int64_t *begin, const int64_t *end,
                   const uint8_t *suspended, uint64_t seed, bg_dnat **out);
void bg_dnat_destroy(bg_dnat *h);
/* GetDesc: mappings (map entries / 2) */
size_t bg_dnat_count(const bg_dnat *h);
/* DoProcessBatch<dir> (nat.cc:321-363) on a device slab in place: dir 0
 * (input gate 0) maps internal sources, creating mappings, and emits on
 * gate 1; dir 1 maps external destinations and emits on 0; unknown
 * endpoints and other protocols: DROP_GATE. now: ctx->current_ns. A batch
 * with new forward flows is decided on the host in packet order (the port
 * search is sequential); synchronous, on `stream` as given (NULL: the legacy
 * default stream). */
int bg_dnat_process(bg_dnat *h, void *d_frames, size_t stride, size_t n,
                    int dir, uint64_t now, uint16_t *d_out, bg_stream_t stream);

/* ---- Rewrite (core/modules/rewrite.{h,cc}) ----------------------------- */
/* The template set and the round-robin turn. add = CommandAdd (25-61):
 * all or nothing, -EINVAL "max 32 packet templates can be used %zu %d" /
 * "template is too big" (> 1536 bytes); clear = CommandClear (63-67).
 * Init(arg) is add(arg.templates). */
typedef struct bg_rewrite bg_rewrite;
int bg_rewrite_create(bg_rewrite **out);
void bg_rewrite_destroy(bg_rewrite *h);
int bg_rewrite_add(bg_rewrite *h, const uint8_t *const *templates,
                   const uint32_t *lens, int n);
void bg_rewrite_clear(bg_rewrite *h);
size_t bg_rewrite_count(const bg_rewrite *h);
/* add() from a serialized bess.pb.RewriteArg (repeated bytes templates = 1),
 * as a bessd plugin receives its Init / add argument */
int bg_rewrite_add_pb(bg_rewrite *h, const void *arg, size_t len);
/* ProcessBatch (72-113) over n packets in one call, as consecutive batches:
 * asynchronous on `stream` as given (NULL: the legacy default stream, so
 * the kernel runs after the caller's earlier work there):
 * packet i (slot d_slots + i*stride) gets template (turn + i) % count at
 * slot + headroom, d_head[i] = headroom (data_off), d_len[i] = its size;
 * the turn advances by n. Whole 32-byte blocks are written, as the
 * reference's sloppy copy does (bytes past the size are the template's
 * zero padding), so headroom + the largest size rounded up to 32 must fit
 * the slot. No template: packets untouched. */
int bg_rewrite_process(bg_rewrite *h, int device, void *d_slots, size_t stride,
                       size_t n, uint32_t headroom, uint16_t *d_head, uint32_t *d_len,
                       bg_stream_t stream);
/* Host packets: slots[i] = packet i's buffer (slot_bytes each); written at
 * headroom through the calling thread's pinned staging. Synchronous. */
int bg_rewrite_process_host(bg_rewrite *h, int device, uint8_t *const *slots,
                            size_t slot_bytes, size_t n, uint32_t headroom,
                            uint16_t *head, uint32_t *len, bg_stream_t stream);

/* ---- IPEncap (core/modules/ip_encap.cc) -------------------------------- */
/* ProcessBatch 40-80 on a device slab: packet i's slot at d_slots +
 * i*stride, its data at slot + d_head[i] (the mbuf's data_off), pkt_len
 * d_len[i], its metadata area at slot + meta_off. attr_offsets[5]: the
 * attr_offset() of ip_src, ip_dst, ip_proto (read) and ip_nexthop,
 * ether_type (written); < 0 = invalid (reads give 0, writes are skipped).
 * A 20-byte IPv4 header is prepended in place (d_head -= 20, d_len += 20)
 * unless the headroom is < 20; d_out[i] = 0 for every packet. */
int bg_ip_encap(int device, void *d_slots, size_t stride, size_t n,
                int meta_off, const int32_t *attr_offsets, uint16_t *d_head,
                uint32_t *d_len, uint16_t *d_out, bg_stream_t stream);
/* Host packets: slots[i] = packet i's buffer (metadata area at meta_off,
 * data at slots[i] + head[i], len[i] bytes; all within slot_bytes), staged
 * through the calling thread's pinned buffers and written back with the
 * updated head / len. Synchronous; stream as the other host paths. */
int bg_ip_encap_host(int device, uint8_t *const *slots, size_t slot_bytes, size_t n,
                     int meta_off, const int32_t *attr_offsets, uint16_t *head,
                     uint32_t *len, uint16_t *out, bg_stream_t stream);

/* ---- BESS module surface (protobuf arguments) -------------------------- */
typedef struct bg_module bg_module;

/* The per-call context of a ProcessBatch: what bessd's Context
 * (core/module.h:59-75) carries into Module::ProcessBatch(ctx, batch) --
 * the input gate the batch arrived on (ctx->current_igate: ACL emits on it,
 * acl.cc:70; StaticNAT and NAT pick their direction by it, static_nat.cc:
 * 146-181, nat.cc:321-363), the worker's clock (ctx->current_ns: NAT's
 * mapping timestamps) and the worker (ctx->wid). It is passed with every
 * datapath call and never stored in the module, so workers that feed one
 * module through different input gates at the same time cannot see each
 * other's values. `device`: the HIP device this call's work runs on (the
 * module keeps a table replica per device); -1 = the module's device
 * (bg_module_set_device, default 0). A NULL bg_ctx means igate 0, now =
 * CLOCK_MONOTONIC at the call, device -1. */
typedef struct bg_ctx {
  uint64_t now_ns;
  uint16_t igate;
  int16_t device;
  uint32_t wid;
} bg_ctx;
/* mclass: "ExactMatch", "WildcardMatch", "IPChecksum", "L4Checksum",
 * "HashLB", "ACL", "IPLookup", "UpdateTTL", "StaticNAT", "NAT".
 * arg: serialized bess.pb.<mclass>Arg. On failure returns -errno and the
 * reference's message via bg_last_error(). */
int bg_module_create(const char *mclass, const void *arg, size_t arg_len,
                     bg_module **out);
/* Releases the caller's handle. Pipes still open on the module keep it
 * alive: it is freed when the last of them is destroyed. */
void bg_module_destroy(bg_module *m);
/* cmd by name with its serialized argument (arg type per the module's cmds
 * table). The serialized response message (e.g. ExactMatchConfig for
 * get_runtime_config, empty for add) goes to out (capacity *out_len; on
 * return *out_len = bytes needed). */
int bg_module_command(bg_module *m, const char *cmd, const void *arg,
                      size_t arg_len, void *out, size_t *out_len);
/* ProcessBatch over cnt <= any packets: heads[i] = head_data() of packet i;
 * ogates[i] = the output gate packet i left on, BG_DROP_GATE if it was
 * dropped (DropPacket, or EmitPacket to a gate that is out of range or not
 * connected, core/module.h:546-549), BG_GATE_NONE if it was not emitted.
 * Synchronous; may be called from many worker threads at once (each stages
 * into its own pinned buffers on its own HIP stream; core/module.h:485),
 * each with its own ctx. */
int bg_module_process(bg_module *m, const bg_ctx *ctx, uint8_t *const *heads,
                      size_t cnt, uint16_t *ogates);
/* bg_module_process with each packet's metadata area (metas[i], as
 * bg_pipe_submit_meta): the synchronous path of a module with attr_name
 * fields (bg_module_process on one: every packet dropped, -EINVAL). */
int bg_module_process_meta(bg_module *m, const bg_ctx *ctx, uint8_t *const *heads,
                           uint8_t *const *metas, size_t cnt, uint16_t *ogates);
/* bg_module_process plus the batches the Task would run next
 * (core/module.h:543-618): per output gate, packets in emission order cut
 * into batches of <= 32 (PacketBatch::kMaxBurst), in the order the batches
 * were started (Task::AddToRun). batch_gate / batch_len get *nbatches
 * entries; pkt_idx lists the batches' packet indices back to back, then the
 * *ndead dropped packets in drop order. Capacities: cnt each. */
int bg_module_process_batches(bg_module *m, const bg_ctx *ctx,
                              uint8_t *const *heads, size_t cnt,
                              uint16_t *ogates, uint16_t *batch_gate,
                              uint32_t *batch_len, uint32_t *pkt_idx,
                              size_t *nbatches, size_t *ndead);
/* A worker's loop with the synchronous path: bg_module_process on each
 * `burst` packets of heads[0..n) in turn (ogates as bg_module_process). */
int bg_module_run(bg_module *m, const bg_ctx *ctx, uint8_t *const *heads,
                  size_t n, size_t burst, uint16_t *ogates);
/* Output gate `ogate` connected (1) or not (0) to a next module
 * (ConnectModules). Until the first call every gate < BG_MAX_GATES counts
 * as connected. EmitPacket to an unconnected gate drops the packet. */
int bg_module_connect(bg_module *m, uint16_t ogate, int connected);
/* Device-resident ProcessBatch over a slab on ctx->device (the slab and
 * gates must live there). */
int bg_module_process_device(bg_module *m, const bg_ctx *ctx, void *d_frames,
                             size_t stride, size_t n, uint16_t *d_ogates,
                             bg_stream_t stream);
/* the device of calls whose ctx says -1 (default 0); control path */
int bg_module_set_device(bg_module *m, int device);
/* Metadata layout for attr_name fields (ExactMatch, WildcardMatch): the
 * slot offset of each packet's metadata area in a device slab (-1: no
 * device-slab layout; the host paths stage each packet's metadata bytes
 * themselves) and, by attribute name, the offsets the pipeline assigned
 * (Module::attr_offset, core/module.h). */
int bg_module_bind_meta(bg_module *m, int meta_off, const char *const *names,
                        const int32_t *offsets, int n);
/* The module's i-th metadata attribute (the attr_name fields of ExactMatch
 * and WildcardMatch, in field order: AddMetadataAttr, core/module.h:294) --
 * what a bessd wrapper registers with bessd so its pipeline assigns the
 * offset. Returns 1 (name, size filled) or 0 past the last. */
int bg_module_attr(const bg_module *m, int i, char *name, size_t cap, uint32_t *size);
/* GetDesc() (exact_match.cc:246-249, wildcard_match.cc:205-213) */
int bg_module_desc(const bg_module *m, char *buf, size_t len);

/* ---- Asynchronous host ingress/egress: the aggregation queue ------------
 * Replaces the per-call synchronous host path for BESS pipelines, where a
 * module receives <= 32 packets per ProcessBatch (core/pktbatch.h:70). Like
 * the Queue module (core/modules/queue.cc:173 enqueue in ProcessBatch, 190
 * emit from RunTask), submit() enqueues and poll() returns finished packets:
 *   submit: gathers each packet's device bytes (the field window for
 *           ExactMatch/WildcardMatch; the frame for IP/L4Checksum, span
 *           bytes at most, data_len when lens != NULL) into a pinned slot;
 *           a full slot (batch packets) is launched on its own HIP stream:
 *           H2D -> device ProcessBatch -> D2H (gates [+ header lines]);
 *           on an ExactMatch / WildcardMatch module a slot of <= 8192
 *           packets is instead one ticket of the module's persistent ring
 *           (no HIP call; BG_PATH_PIPE_NO_RING: launches).
 *           Blocks only when all `depth` slots are in flight. ctx: the
 *           ProcessBatch's context (NULL as for bg_module_process; its
 *           device is ignored: the pipe's device is fixed at create). A
 *           slot holds packets of one context as far as the module reads
 *           it on the device (ACL, StaticNAT: the input gate; NAT: the
 *           gate and the clock): a submit whose context differs there
 *           launches the filling slot first.
 *   flush:  launches the partially filled slot (a RunTask deadline).
 *   poll:   completed packets in submission order: cookie (default: the
 *           head pointer) and the gate EmitPacket would get (BG_GATE_NONE:
 *           not emitted); checksum modules' recomputed header lines are
 *           written back into the packet buffers first. wait != 0 blocks
 *           until a launched slot completes (returns 0 if none in flight).
 * Packets stay owned by the caller until poll returns them, their bytes
 * unchanged: a submit's windows are copied by the pipe's next call (by then
 * the caller's prefetch of their lines has landed) or when their slot
 * launches. One pipe per worker thread; pipes may share a module. */
typedef struct bg_pipe bg_pipe;
int bg_pipe_create(bg_module *m, int device, size_t batch, int depth,
                   size_t span, bg_pipe **out);
void bg_pipe_destroy(bg_pipe *p); /* waits for in-flight slots */
int bg_pipe_window(const bg_pipe *p, int *lo, int *hi, size_t *stride);
int bg_pipe_submit(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                   const uint16_t *lens, void *const *cookies, size_t cnt);
/* submit for a module with attr_name fields (ExactMatch / WildcardMatch,
 * exact_match.cc:230-236, wildcard_match.cc:177-195): metas[i] = packet i's
 * metadata area (Packet::metadata(): the snbuf's SNBUF_METADATA bytes); the
 * bytes the fields read (bg_em_meta_window, attribute offsets bound with
 * bg_module_bind_meta, meta_off -1 will do) travel in the packet's staged
 * row after its field window. bg_pipe_submit on such a module: -EINVAL. */
int bg_pipe_submit_meta(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                        uint8_t *const *metas, const uint16_t *lens,
                        void *const *cookies, size_t cnt);
int bg_pipe_flush(bg_pipe *p);
long bg_pipe_poll(bg_pipe *p, int wait, void **cookies, uint16_t *gates,
                  size_t cap);
size_t bg_pipe_pending(const bg_pipe *p);
/* counters (first n of): submits, packets, slot launches, ns spent in
 * launches (HIP calls), ns submits waited for a free slot, ns polls
 * waited, the slot size, TSC cycles inside submit, inside poll, TSC cycles
 * from slot launches to their completion being seen (sum, max), and the
 * launch ns by HIP call (launch mode): H2D copy, module kernel, gates D2H,
 * header lines D2H, completion write */
int bg_pipe_stats(const bg_pipe *p, uint64_t *out, int n);
/* A worker loop (Source -> module -> Sink): n packets submitted in bursts of
 * `burst`, completions polled after each submit; ogates[i] = packet i's
 * gate. Returns when all n are back. */
int bg_pipe_run(bg_pipe *p, const bg_ctx *ctx, uint8_t *const *heads,
                const uint16_t *lens, size_t n, size_t burst, uint16_t *ogates);

/* ---- Persistent classify kernel: rings of batch descriptors -------------
 * (A pipe on an ExactMatch / WildcardMatch module submits its slots to
 * such a ring: see bg_pipe_create.)
 * BESS hands a module <= 32 packets per ProcessBatch (core/pktbatch.h:70);
 * a kernel launch per batch costs more than the batch. A ring is ONE
 * running ExactMatch kernel that drains batch descriptors the workers write
 * into pinned host memory (the Queue split, core/modules/queue.cc:173,190).
 * Each worker thread submits on its own lane (0 .. lanes-1: its own ring of
 * `slots` descriptors, done words and published count, so workers never
 * share a cache line or a lock): submit enqueues a batch (frames at
 * `frames` + i*stride (n <= 2^27), device or mapped host memory, each slot holding the
 * frame from byte win_off on -- 0: whole frames, the field window's start:
 * staged windows; gates written to `gates`) and returns the lane's ticket; wait blocks until that ticket's
 * gates are written; completed returns the number of the lane's tickets
 * finished in order. Create it with as many lanes as workers submit on (one
 * thread per lane: wait / completed claim the lane and return -EBUSY to a
 * second thread; submit only detects one on a best-effort basis). The
 * kernel keeps the table in LDS for its whole run and classifies with the
 * rule set as of bg_em_ring_create (it holds its own copy of the table
 * image: re-create the ring after rule changes, which bessd makes with
 * workers paused). slots: a power of two <= 32768 (submit blocks while
 * `slots` of the lane's tickets are unfinished); blocks: 256-thread workgroups
 * (0: 4 per CU), spread evenly over the lanes; idle_us: the kernel exits after this long without work and is
 * relaunched by the next submit or wait (so it never outlives its work); a
 * submit makes no HIP call while the kernel runs. */
typedef struct bg_ring bg_ring;
int bg_em_ring_create(bg_em *em, int device, int lanes, int slots, int blocks,
                      uint32_t idle_us, int win_off, bg_ring **out);
/* The same ring over a WildcardMatch table (WildcardMatch::ProcessBatch,
 * wildcard_match.cc:159-203, per ticket): the kernel probes its own copy of
 * the table image in L2 (in LDS when the image is <= 40 KB); a ticket's
 * default gate applies where no rule matches. */
int bg_wm_ring_create(bg_wm *wm, int device, int lanes, int slots, int blocks,
                      uint32_t idle_us, int win_off, bg_ring **out);
void bg_ring_destroy(bg_ring *r); /* stops the kernel and waits for it */
int64_t bg_ring_submit(bg_ring *r, int lane, const void *frames, size_t stride,
                       size_t n, uint16_t default_gate, uint16_t *gates);
int bg_ring_wait(bg_ring *r, int lane, int64_t ticket);
int64_t bg_ring_completed(bg_ring *r, int lane);
/* A worker loop on one lane: n packets in batches of `burst` submitted back
 * to back, then waits for the last (the persistent series of the C2 sweep). */
int bg_ring_run(bg_ring *r, int lane, const void *frames, size_t stride,
                size_t n, size_t burst, uint16_t default_gate, uint16_t *gates);
/* `threads` such workers at once (native threads, released together),
 * worker i on lane i over packets [i n / threads, (i + 1) n / threads),
 * `reps` passes each; returns the wall seconds per pass (from the release
 * to the last worker's end), or -errno. */
double bg_ring_run_lanes(bg_ring *r, int threads, const void *frames, size_t stride,
                         size_t n, size_t burst, uint16_t default_gate, uint16_t *gates,
                         int reps);
/* kernel launches so far (1 + relaunches after idle exits), workgroups */
int bg_ring_info(const bg_ring *r, uint64_t *launches, int *blocks);
/* 1: the descriptors live in device memory the host writes through the
 * PCIe BAR (workers read them from HBM); 0: in pinned host memory (read
 * over PCIe; no CPU mapping of device memory, or BG_PATH_RING_HOST_DESC). */
int bg_ring_desc_in_device(const bg_ring *r);
/* How the kernel meets the memory of later submits (one thread, before or
 * between submits). frames 1 (default): the frames may be memory the
 * device caches non-coherently -- mapped host memory that is not uncached
 * (hipHostMallocUncached), or device memory rewritten by a copy between
 * tickets -- so each ticket acquires at system scope (invalidating L2's
 * non-coherent lines); 0: frames in device memory written by kernels, or in
 * uncached host memory (each ticket invalidates its CU's L1 only). done 1
 * (default): the done word is a system-scope release; 0: a system-scope
 * store after the ticket's gate stores (themselves system-scope
 * write-through stores) have completed. */
int bg_ring_set_coherence(bg_ring *r, int frames, int done);

#ifdef __cplusplus
}
#endif
#endif /* BESSGPU_H_ */
