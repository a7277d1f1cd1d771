/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the BESS per-batch packet-classification hot path
 * (reference: NetSys/bess, all citations relative to its tree). Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this
 * library, and only as the checker / CPU baseline -- never as the thing that is
 * measured or shipped. The product path (bess_amd/libbessgpu.so) never links
 * or calls it.
 *
 * Pinning: see oracle/README.md (golden vectors transcribed from the reference's
 * own tests, plus oracle/_ref built from core/utils/endian.cc).
 */
#ifndef BESS_ORACLE_H_
#define BESS_ORACLE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_FIELDS 8     /* exact_match_table.h:50, wildcard_match.h:46 */
#define OR_MAX_FIELD_SIZE 8 /* exact_match_table.h:51 */
#define OR_MAX_TUPLES 8     /* wildcard_match.h:45 */
#define OR_KEY_BYTES 64     /* sizeof(ExactMatchKey) / sizeof(wm_hkey_t) */
#define OR_MAX_BURST 32     /* pktbatch.h:70 kMaxBurst */
#define OR_GATE_NONE 0xFFFFu /* "packet was not emitted" (L4Checksum quirk) */

/* ---- utils ---------------------------------------------------------- */
/* endian.cc:36-58 */
int or_uint64_to_bin(void *ptr, uint64_t val, size_t size, int big_endian);
/* ExactMatchKeyHash exact_match_table.h:101-119 / wm_hash wildcard_match.h:106-129 */
uint32_t or_key_hash(const uint64_t *key, size_t len);

/* ---- CuckooMap restatement (cuckoo_map.h) ----------------------------- */
typedef struct or_cuckoo or_cuckoo;

/* ---- ExactMatch -------------------------------------------------------- */
typedef struct or_em or_em;
or_em *or_em_new(void);
void or_em_free(or_em *em);
/* ExactMatchTable::AddField(offset,...) -> DoAddField, exact_match_table.h:303-307,
 * 391-443. Returns 0 or errno; msg (may be NULL) gets the reference's text. */
int or_em_add_field(or_em *em, int offset, int size, uint64_t mask, int idx,
                    char *msg, size_t msglen);
size_t or_em_num_fields(const or_em *em);
/* get_field: mask, offset, pos, size */
void or_em_get_field(const or_em *em, size_t i, uint64_t *mask, int *offset,
                     int *pos, int *size);
size_t or_em_total_key_size(const or_em *em);
/* ExactMatchTable::AddRule / DeleteRule (exact_match_table.h:175-217) */
int or_em_add_rule(or_em *em, uint16_t gate, const uint8_t *const *vals,
                   const size_t *lens, size_t nvals, char *msg, size_t msglen);
int or_em_add_rules(or_em *em, const uint8_t *keys, size_t n, size_t key_stride,
                    const uint16_t *gates);
int or_em_delete_rule(or_em *em, const uint8_t *const *vals, const size_t *lens,
                      size_t nvals, char *msg, size_t msglen);
void or_em_clear(or_em *em);
size_t or_em_count(const or_em *em);
/* iteration in CuckooMap order (cuckoo_map.h:70-150); returns 0 at end */
int or_em_iter(const or_em *em, size_t *cursor, uint8_t key_out[OR_KEY_BYTES],
               uint16_t *gate_out);
/* ExactMatch::ProcessBatch (exact_match.cc:224-244) for one batch of <= 32
 * packets given their head_data() pointers. gates[i] = EmitPacket gate. */
void or_em_process_batch(const or_em *em, const uint8_t *const *heads, int cnt,
                         uint16_t default_gate, uint16_t *gates);
/* MakeKeys for one packet (key zero-filled past the fields) */
void or_em_make_key(const or_em *em, const uint8_t *head, uint64_t key[8]);
/* the same over n packets at base + i*stride, in kMaxBurst batches */
void or_em_process(const or_em *em, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates);
void or_em_bind_attr(or_em *em, int idx, int mt_offset);
void or_em_process_meta(const or_em *em, const uint8_t *base, size_t stride,
                        const uint8_t *meta, size_t meta_stride, size_t n,
                        uint16_t default_gate, uint16_t *gates);

/* ---- WildcardMatch ----------------------------------------------------- */
typedef struct or_wm or_wm;
or_wm *or_wm_new(void);
void or_wm_free(or_wm *wm);
/* WildcardMatch::Init + AddFieldOne (wildcard_match.cc:75-134), offset
 * fields; call once per field in order then or_wm_init_done(). */
int or_wm_add_field(or_wm *wm, int offset, int size, char *msg, size_t msglen);
void or_wm_init_done(or_wm *wm);
size_t or_wm_total_key_size(const or_wm *wm);
size_t or_wm_num_fields(const or_wm *wm);
void or_wm_get_field(const or_wm *wm, size_t i, int *offset, int *pos,
                     int *size);
/* CommandAdd after ExtractKeyMask (wildcard_match.cc:317-354): key/mask are
 * 64-byte gathered keys. Returns 0 or errno. */
int or_wm_add(or_wm *wm, const uint8_t key[OR_KEY_BYTES],
              const uint8_t mask[OR_KEY_BYTES], int32_t priority,
              uint16_t gate);
/* CommandDelete after ExtractKeyMask (wildcard_match.cc:357-377) */
int or_wm_delete(or_wm *wm, const uint8_t key[OR_KEY_BYTES],
                 const uint8_t mask[OR_KEY_BYTES]);
void or_wm_clear(or_wm *wm);
int or_wm_num_tuples(const or_wm *wm);
void or_wm_tuple_mask(const or_wm *wm, int t, uint8_t mask_out[OR_KEY_BYTES]);
size_t or_wm_tuple_count(const or_wm *wm, int t);
int or_wm_iter(const or_wm *wm, int t, size_t *cursor,
               uint8_t key_out[OR_KEY_BYTES], int32_t *prio, uint16_t *gate);
/* WildcardMatch::ProcessBatch (wildcard_match.cc:159-203) */
void or_wm_process_batch(const or_wm *wm, const uint8_t *const *heads, int cnt,
                         uint16_t default_gate, uint16_t *gates);
void or_wm_process(const or_wm *wm, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates);
void or_wm_bind_attr(or_wm *wm, int idx, int mt_offset);
void or_wm_process_meta(const or_wm *wm, const uint8_t *base, size_t stride,
                        const uint8_t *meta, size_t meta_stride, size_t n,
                        uint16_t default_gate, uint16_t *gates);

/* ---- checksums (checksum.h) ------------------------------------------- */
uint32_t or_calculate_sum(const void *buf, size_t len);           /* 52-181 */
uint16_t or_fold_checksum(uint32_t cksum);                        /* 185-189 */
uint16_t or_generic_checksum(const void *buf, size_t len);        /* 193-195 */
uint16_t or_ipv4_checksum(const uint8_t *ip);                     /* 288-318 */
int or_ipv4_verify(const uint8_t *ip);                            /* 254-283 */
uint16_t or_udp_checksum(const uint8_t *ip, const uint8_t *udp);  /* 398-407 */
int or_udp_verify(const uint8_t *ip, const uint8_t *udp);         /* 352-362 */
uint16_t or_tcp_checksum(const uint8_t *ip, const uint8_t *tcp);  /* 492-504 */
int or_tcp_verify(const uint8_t *ip, const uint8_t *tcp);         /* 442-452 */
/* RFC 1624 incremental update (checksum.h:520-560) */
uint16_t or_update_checksum16(uint16_t old_ck, uint16_t old_v, uint16_t new_v);
uint16_t or_update_checksum32(uint16_t old_ck, uint32_t old_v, uint32_t new_v);

/* IPChecksum::ProcessBatch (ip_checksum.cc:39-84): in place; gates 0/1 */
void or_ip_checksum_batch(uint8_t *const *heads, int cnt, int verify,
                          uint16_t *gates);
/* L4Checksum::ProcessBatch (l4_checksum.cc:41-83): gates 0/1/OR_GATE_NONE */
void or_l4_checksum_batch(uint8_t *const *heads, int cnt, int verify,
                          uint16_t *gates);
/* n frames at base + i*stride, 32-packet batches.
 * mode bit0 = IPChecksum, bit1 = L4Checksum (bit0|bit1 = IPChecksum ->
 * L4Checksum pipeline: only packets IPChecksum emitted on gate 0 reach
 * L4Checksum). ip_gates / l4_gates may be NULL. */
void or_cksum_process(uint8_t *base, size_t stride, size_t n, int mode,
                      int verify, uint16_t *ip_gates, uint16_t *l4_gates);

/* ---- HashLB (core/modules/hash_lb.cc) -- oracle_more.c ----------------- */
#define OR_HLB_L2 0
#define OR_HLB_L3 1
#define OR_HLB_L4 2
#define OR_HLB_FIELDS 3
/* hash_range 53-68 */
uint16_t or_hash_range(uint32_t hashval, uint16_t range);
/* HashLB::DoProcessBatch<mode> 140-236: out[i] = gates[hash_range(hash,
 * num_gates)]; fields mode: MakeKeys of `fields` (an or_em whose fields were
 * added with mask 0) hashed over hash_len bytes (ExactMatchKeyHash). */
void or_hashlb_process(int mode, const or_em *fields, size_t hash_len,
                       const uint16_t *gates, size_t num_gates,
                       const uint8_t *base, size_t stride, size_t n,
                       uint16_t *out);
double or_hashlb_bench(int mode, const or_em *fields, size_t hash_len,
                       const uint16_t *gates, size_t num_gates,
                       const uint8_t *base, size_t stride, size_t n,
                       uint16_t *out, int nthreads, int reps);

/* ---- ACL (core/modules/acl.cc) -- oracle_more.c ------------------------- */
#define OR_DROP_GATE 8192
typedef struct or_acl_rule { /* ACLRule, host byte order */
  uint32_t src_addr, src_mask, dst_addr, dst_mask;
  uint16_t src_port, dst_port;
  uint8_t drop, pad[3];
} or_acl_rule;
/* ParseIpv4Address (ip.cc:40-51): 1 on success */
int or_ipv4_address(const char *str, uint32_t *addr);
/* Ipv4Prefix(string) (ip.cc:63-79); -1 where std::stoi would throw */
int or_ipv4_prefix(const char *prefix, uint32_t *addr, uint32_t *mask);
void or_acl_process(const or_acl_rule *rules, size_t nrules, const uint8_t *base,
                    size_t stride, size_t n, uint16_t igate, uint16_t *out);
double or_acl_bench(const or_acl_rule *rules, size_t nrules, const uint8_t *base,
                    size_t stride, size_t n, uint16_t igate, uint16_t *out,
                    int nthreads, int reps);

/* ---- IPLookup (core/modules/ip_lookup.cc) -- oracle_more.c ------------ */
/* longest-prefix match of each packet's IPv4 dst over (ip, depth, next hop)
 * rules; default_gate when none matches */
void or_lpm_process(const uint32_t *ips, const uint8_t *depths,
                    const uint32_t *nhs, size_t nrules, const uint8_t *base,
                    size_t stride, size_t n, uint16_t default_gate,
                    uint16_t *out);

/* ---- UpdateTTL (core/modules/update_ttl.cc) -- oracle_more.c ---------- */
/* in place; out[i] = 0 (emitted) or OR_DROP_GATE */
void or_update_ttl_process(uint8_t *base, size_t stride, size_t n, uint16_t *out);

/* ---- multi-threaded CPU baseline drivers ------------------------------ */
/* Each thread owns a contiguous slice of the n packets (pointer batches of
 * 32 over base + i*stride) and sweeps it `reps` times; threads are pinned to
 * the first `nthreads` CPUs of the process affinity mask. Returns wall
 * seconds of the timed region. */
/* C1: Source -> ExactMatch -> Sink (gates 0..63 bitmap `connected`); the
 * packets the sink received in *sunk */
double or_c1_bench(const or_em *em, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint64_t connected,
                   uint16_t *gates, int nthreads, int reps, uint64_t *sunk);
double or_em_bench(const or_em *em, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates,
                   int nthreads, int reps);
double or_wm_bench(const or_wm *wm, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates,
                   int nthreads, int reps);
double or_cksum_bench(uint8_t *base, size_t stride, size_t n, int mode,
                      int verify, uint16_t *l4_gates, int nthreads, int reps);
int or_num_cpus(void);

#ifdef __cplusplus
}
#endif
#endif /* BESS_ORACLE_H_ */
