/*
 * oracle_more.c -- TEST INFRASTRUCTURE ONLY (see oracle.h): CPU
 * restatements of the SURVEY §8f modules that sit beside the
 * classification path -- HashLB, ACL, IPLookup, UpdateTTL. Only tests/,
 * smoke() and bench.py's cpu_baseline leg load it.
 *
 * Each function cites the reference file:line it follows. CRC32C is computed
 * with the same SSE4.2 instructions the reference's DPDK helpers compile to
 * (rte_hash_crc.h crc32c_sse42_u16/u32/u64 = _mm_crc32_u16/u32/u64).
 */
#define _GNU_SOURCE
#include <nmmintrin.h>
#include <pthread.h>
#include <sched.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "oracle.h"

static inline uint16_t ld16(const uint8_t *p) {
  uint16_t v;
  memcpy(&v, p, 2);
  return v;
}
static inline uint32_t ld32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}

/* ====================================================================== */
/* HashLB (core/modules/hash_lb.cc)                                        */
/* ====================================================================== */

/* hash_range 53-68: 1.(b0)..(b31) as a double, minus 1, times range */
uint16_t or_hash_range(uint32_t hashval, uint16_t range) {
  union {
    uint64_t i;
    double d;
  } tmp;
  tmp.i = 0x3ff0000000000000ull | ((uint64_t)hashval << 20);
  return (uint16_t)((tmp.d - 1.0) * range);
}

static uint32_t hlb_hash(int mode, const or_em *fields, size_t hash_len,
                         const uint8_t *head) {
  switch (mode) {
    case OR_HLB_L2: { /* 152-170 */
      uint16_t sum = 0;
      for (int j = 0; j < 6; j++) sum ^= ld16(head + 2 * j);
      return _mm_crc32_u16(0, sum); /* hash_16(sum, 0) */
    }
    case OR_HLB_L3: { /* 174-190 */
      const int ip = 14;
      uint32_t v0 = ld32(head + ip + 12) ^ ld32(head + ip + 16);
      return _mm_crc32_u32(0, v0);
    }
    case OR_HLB_L4: { /* 194-219 */
      const int ip = 14;
      uint32_t l4 = ip + ((head[ip] & 0x0F) << 2);
      uint32_t v0 = ld32(head + ip + 12);
      v0 ^= ld32(head + ip + 16);
      v0 ^= ld16(head + l4);
      v0 ^= ld16(head + l4 + 2);
      v0 ^= head[ip + 9];
      return _mm_crc32_u32(0, v0);
    }
    default: { /* 140-150: MakeKeys + ExactMatchKeyHash (exact_match_table.h:101-119) */
      uint64_t key[8];
      or_em_make_key(fields, head, key);
      uint64_t h = 0;
      for (size_t i = 0; i < hash_len / 8; i++) h = _mm_crc32_u64(h, key[i]);
      return (uint32_t)h;
    }
  }
}

void or_hashlb_process(int mode, const or_em *fields, size_t hash_len,
                       const uint16_t *gates, size_t num_gates,
                       const uint8_t *base, size_t stride, size_t n,
                       uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    uint32_t h = hlb_hash(mode, fields, hash_len, base + i * stride);
    out[i] = gates[or_hash_range(h, (uint16_t)num_gates)];
  }
}

/* ====================================================================== */
/* threaded CPU-baseline driver                                            */
/* ====================================================================== */

typedef void (*slice_fn)(void *ctx, size_t begin, size_t end);

typedef struct {
  slice_fn fn;
  void *ctx;
  size_t begin, end;
  int reps, cpu;
  pthread_barrier_t *bar;
} slice_arg;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

static void *slice_thread(void *p) {
  slice_arg *a = (slice_arg *)p;
  if (a->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(a->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  pthread_barrier_wait(a->bar);
  for (int r = 0; r < a->reps; r++) a->fn(a->ctx, a->begin, a->end);
  pthread_barrier_wait(a->bar);
  return NULL;
}

/* each thread (pinned to the next CPU of the affinity mask) owns a
 * contiguous, 32-packet aligned slice; returns the wall seconds */
static double run_slices(slice_fn fn, void *ctx, size_t n, int nthreads,
                         int reps) {
  if (nthreads < 1) nthreads = 1;
  cpu_set_t set;
  int cpus[1024], ncpu = 0;
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; c++)
      if (CPU_ISSET(c, &set)) cpus[ncpu++] = c;
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads + 1);
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  slice_arg *args = (slice_arg *)calloc((size_t)nthreads, sizeof(slice_arg));
  size_t nb = (n + OR_MAX_BURST - 1) / OR_MAX_BURST;
  for (int t = 0; t < nthreads; t++) {
    slice_arg *a = &args[t];
    size_t b0 = nb * (size_t)t / (size_t)nthreads,
           b1 = nb * (size_t)(t + 1) / (size_t)nthreads;
    a->fn = fn;
    a->ctx = ctx;
    a->begin = b0 * OR_MAX_BURST;
    a->end = b1 * OR_MAX_BURST < n ? b1 * OR_MAX_BURST : n;
    if (a->begin > a->end) a->begin = a->end;
    a->reps = reps;
    a->cpu = ncpu ? cpus[t % ncpu] : -1;
    a->bar = &bar;
    pthread_create(&th[t], NULL, slice_thread, a);
  }
  pthread_barrier_wait(&bar);
  double t0 = now_s();
  pthread_barrier_wait(&bar);
  double t1 = now_s();
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  pthread_barrier_destroy(&bar);
  free(th);
  free(args);
  return t1 - t0;
}

typedef struct {
  int mode;
  const or_em *fields;
  size_t hash_len;
  const uint16_t *gates;
  size_t num_gates;
  const uint8_t *base;
  size_t stride;
  uint16_t *out;
} hlb_ctx;

static void hlb_slice(void *p, size_t b, size_t e) {
  hlb_ctx *c = (hlb_ctx *)p;
  or_hashlb_process(c->mode, c->fields, c->hash_len, c->gates, c->num_gates,
                    c->base + b * c->stride, c->stride, e - b, c->out + b);
}

double or_hashlb_bench(int mode, const or_em *fields, size_t hash_len,
                       const uint16_t *gates, size_t num_gates,
                       const uint8_t *base, size_t stride, size_t n,
                       uint16_t *out, int nthreads, int reps) {
  hlb_ctx c = {mode, fields, hash_len, gates, num_gates, base, stride, out};
  return run_slices(hlb_slice, &c, n, nthreads, reps);
}

/* ====================================================================== */
/* ACL (core/modules/acl.{h,cc})                                           */
/* ====================================================================== */

#include <errno.h>
#include <limits.h>
#include <stdio.h>

static uint32_t be32(const uint8_t *p) {
  return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) |
         p[3];
}
static uint16_t be16(const uint8_t *p) { return (uint16_t)((p[0] << 8) | p[1]); }

/* ParseIpv4Address (core/utils/ip.cc:40-51): 1 on success */
int or_ipv4_address(const char *str, uint32_t *addr) {
  unsigned a, b, c, d;
  if (sscanf(str, "%u.%u.%u.%u", &a, &b, &c, &d) != 4 || a >= 256 || b >= 256 ||
      c >= 256 || d >= 256)
    return 0;
  *addr = (a << 24) | (b << 16) | (c << 8) | d;
  return 1;
}

/* Ipv4Prefix::Ipv4Prefix (core/utils/ip.cc:63-79) + ParseIpv4Address
 * (40-51) + SetBitsLow (bits.h:193-198). Returns 0, or -1 where std::stoi
 * would throw (no digits / out of int range). */
int or_ipv4_prefix(const char *prefix, uint32_t *addr, uint32_t *mask) {
  *addr = 0;
  *mask = 0;
  const char *slash = strchr(prefix, '/');
  if (!*prefix || !slash) return 0;
  char ip[256];
  size_t il = (size_t)(slash - prefix);
  if (il >= sizeof(ip)) il = sizeof(ip) - 1;
  memcpy(ip, prefix, il);
  ip[il] = 0;
  unsigned a, b, c, d;
  if (sscanf(ip, "%u.%u.%u.%u", &a, &b, &c, &d) == 4 && a < 256 && b < 256 &&
      c < 256 && d < 256)
    *addr = (a << 24) | (b << 16) | (c << 8) | d;
  char *end;
  errno = 0;
  long v = strtol(slash + 1, &end, 10);
  if (end == slash + 1 || errno == ERANGE || v > INT_MAX || v < INT_MIN) return -1;
  size_t n = (size_t)(long)(int)v;
  *mask = n == 0 ? 0u : n >= 32 ? 0xFFFFFFFFu : ~((1u << (32 - n)) - 1u);
  return 0;
}

/* ACL::ProcessBatch (acl.cc:63-95) with ACLRule::Match (acl.h:45-50) */
void or_acl_process(const or_acl_rule *rules, size_t nrules, const uint8_t *base,
                    size_t stride, size_t n, uint16_t igate, uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    const uint8_t *eth = base + i * stride;
    const uint8_t *ip = eth + 14;
    size_t ip_bytes = (size_t)(ip[0] & 0x0F) << 2; /* header_length << 2 */
    const uint8_t *udp = ip + ip_bytes;
    uint32_t src = be32(ip + 12), dst = be32(ip + 16);
    uint16_t sp = be16(udp), dp = be16(udp + 2);
    uint16_t g = OR_DROP_GATE;
    for (size_t r = 0; r < nrules; r++) {
      const or_acl_rule *R = &rules[r];
      if ((R->src_addr & R->src_mask) == (src & R->src_mask) &&
          (R->dst_addr & R->dst_mask) == (dst & R->dst_mask) &&
          (R->src_port == 0 || R->src_port == sp) &&
          (R->dst_port == 0 || R->dst_port == dp)) {
        if (!R->drop) g = igate;
        break; /* stop matching other rules */
      }
    }
    out[i] = g;
  }
}

typedef struct {
  const or_acl_rule *rules;
  size_t nrules;
  const uint8_t *base;
  size_t stride;
  uint16_t igate;
  uint16_t *out;
} acl_ctx;

static void acl_slice(void *p, size_t b, size_t e) {
  acl_ctx *c = (acl_ctx *)p;
  or_acl_process(c->rules, c->nrules, c->base + b * c->stride, c->stride, e - b,
                 c->igate, c->out + b);
}

double or_acl_bench(const or_acl_rule *rules, size_t nrules, const uint8_t *base,
                    size_t stride, size_t n, uint16_t igate, uint16_t *out,
                    int nthreads, int reps) {
  acl_ctx c = {rules, nrules, base, stride, igate, out};
  return run_slices(acl_slice, &c, n, nthreads, reps);
}

/* ====================================================================== */
/* IPLookup (core/modules/ip_lookup.cc) -- longest-prefix match            */
/* ====================================================================== */
/* The reference delegates to DPDK 19.11 rte_lpm (DIR-24-8); its lookup
 * result is the next hop of the longest rule (ip & mask(depth) == rule ip)
 * or the module's default gate (ip_lookup.cc:76-150). Restated here as a
 * search over per-depth sorted rule arrays, longest depth first -- an
 * independent formulation of the same function (no DIR-24-8). */

typedef struct {
  uint32_t ip, nh;
} lpm_ent;

static int lpm_cmp(const void *a, const void *b) {
  uint32_t x = ((const lpm_ent *)a)->ip, y = ((const lpm_ent *)b)->ip;
  return x < y ? -1 : x > y;
}

static uint32_t lpm_mask(int d) {
  return d == 0 ? 0u : d >= 32 ? 0xFFFFFFFFu : ~((1u << (32 - d)) - 1u);
}

void or_lpm_process(const uint32_t *ips, const uint8_t *depths,
                    const uint32_t *nhs, size_t nrules, const uint8_t *base,
                    size_t stride, size_t n, uint16_t default_gate,
                    uint16_t *out) {
  lpm_ent *by[33];
  size_t cnt[33] = {0};
  for (size_t r = 0; r < nrules; r++) cnt[depths[r]]++;
  for (int d = 0; d <= 32; d++) by[d] = (lpm_ent *)malloc((cnt[d] + 1) * sizeof(lpm_ent));
  size_t fill[33] = {0};
  for (size_t r = 0; r < nrules; r++) {
    int d = depths[r];
    by[d][fill[d]].ip = ips[r] & lpm_mask(d);
    by[d][fill[d]].nh = nhs[r];
    fill[d]++;
  }
  for (int d = 0; d <= 32; d++) qsort(by[d], cnt[d], sizeof(lpm_ent), lpm_cmp);
  for (size_t i = 0; i < n; i++) {
    const uint8_t *ip = base + i * stride + 14;
    uint32_t dst = be32(ip + 16); /* ip->dst.value() */
    uint16_t g = default_gate;
    for (int d = 32; d >= 1; d--) {
      if (!cnt[d]) continue;
      lpm_ent key = {dst & lpm_mask(d), 0};
      lpm_ent *e = (lpm_ent *)bsearch(&key, by[d], cnt[d], sizeof(lpm_ent), lpm_cmp);
      if (e) {
        g = (uint16_t)e->nh;
        break;
      }
    }
    out[i] = g;
  }
  for (int d = 0; d <= 32; d++) free(by[d]);
}

/* ====================================================================== */
/* UpdateTTL (core/modules/update_ttl.cc:39-58)                            */
/* ====================================================================== */
void or_update_ttl_process(uint8_t *base, size_t stride, size_t n, uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    uint8_t *ip = base + i * stride + 14;
    if (ip[8] > 1) { /* ip->ttl */
      uint16_t ck;
      memcpy(&ck, ip + 10, 2);
      ck = or_update_checksum16(ck, 2, 1);
      memcpy(ip + 10, &ck, 2);
      ip[8] -= 1;
      out[i] = 0;
    } else {
      out[i] = OR_DROP_GATE;
    }
  }
}

/* ====================================================================== */
/* StaticNAT (core/modules/static_nat.cc)                                  */
/* ====================================================================== */
/* UpdateChecksumWithIncrement (checksum.h:535-538) */
static uint16_t upd_ck(uint16_t ck, uint32_t incr) {
  return or_fold_checksum((uint32_t)(~ck & 0xFFFF) + incr);
}

/* UpdateChecksum 118-144 */
static void snat_update_checksum(uint8_t *ip, uint32_t incr) {
  size_t ip_bytes = (size_t)(ip[0] & 0x0F) << 2;
  uint8_t *l4 = ip + ip_bytes;
  uint8_t proto = ip[9];
  uint16_t ck;
  memcpy(&ck, ip + 10, 2);
  ck = upd_ck(ck, incr);
  memcpy(ip + 10, &ck, 2);
  if (proto == 6) {
    memcpy(&ck, l4 + 16, 2);
    ck = upd_ck(ck, incr);
    memcpy(l4 + 16, &ck, 2);
  } else if (proto == 17) {
    memcpy(&ck, l4 + 6, 2);
    if (ck != 0) {
      ck = upd_ck(ck, incr);
      if (ck == 0) ck = 0xFFFF;
      memcpy(l4 + 6, &ck, 2);
    }
  }
}

/* DoProcessBatch<dir> 146-181: dir 0 forward (src, emit on 1), 1 reverse */
void or_static_nat_process(const uint32_t *int_addr, const uint32_t *ext_addr,
                           const uint32_t *size, size_t npairs, uint8_t *base,
                           size_t stride, size_t n, int dir, uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    uint8_t *ip = base + i * stride + 14;
    uint8_t *a = dir == 0 ? ip + 12 : ip + 16;
    uint32_t raw;
    memcpy(&raw, a, 4);
    uint32_t addr = be32(a);
    for (size_t p = 0; p < npairs; p++) {
      uint32_t start = dir == 0 ? int_addr[p] : ext_addr[p];
      if (start <= addr && addr < start + size[p]) {
        uint32_t diff = dir == 0 ? ext_addr[p] - int_addr[p] : int_addr[p] - ext_addr[p];
        uint32_t na = addr + diff;
        uint8_t nb[4] = {(uint8_t)(na >> 24), (uint8_t)(na >> 16), (uint8_t)(na >> 8),
                         (uint8_t)na};
        uint32_t nraw;
        memcpy(&nraw, nb, 4);
        /* ChecksumIncrement32(old raw, new raw) 520-525 */
        uint32_t incr = (~raw >> 16) + (~raw & 0xFFFF);
        incr += (nraw >> 16) + (nraw & 0xFFFF);
        snat_update_checksum(ip, incr);
        memcpy(a, nb, 4);
        break;
      }
    }
    out[i] = dir == 0 ? 1 : 0;
  }
}

/* ====================================================================== */
/* IPEncap (core/modules/ip_encap.cc)                                      */
/* ====================================================================== */
/* ProcessBatch 40-80 over a slab: slot i at base + i*stride; the packet's
 * data at slot + head[i] (data_off), pkt_len len[i]; its metadata area at
 * slot + meta_off; offs[0..4] = attr_offset() of ip_src, ip_dst, ip_proto
 * (read), ip_nexthop, ether_type (write), < 0 when invalid (get_attr gives
 * 0, set_attr does nothing: core/module.h:686-705). head/len are updated as
 * Packet::prepend does (packet.h:145-154); a packet whose headroom is < 20
 * is left alone. Every packet goes on (RunNextModule: gate 0). */
void or_ip_encap_process(uint8_t *base, size_t stride, size_t n, int meta_off,
                         const int32_t *offs, uint16_t *head, uint32_t *len,
                         uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    uint8_t *slot = base + i * stride, *meta = slot + meta_off;
    uint8_t src[4] = {0}, dst[4] = {0}, proto = 0;
    if (offs[0] >= 0) memcpy(src, meta + offs[0], 4);
    if (offs[1] >= 0) memcpy(dst, meta + offs[1], 4);
    if (offs[2] >= 0) proto = meta[offs[2]];
    uint16_t total_len = (uint16_t)(len[i] + 20);
    out[i] = 0;
    if (head[i] < 20) continue; /* prepend() returned nullptr */
    head[i] -= 20;
    len[i] += 20;
    uint8_t *ip = slot + head[i];
    ip[0] = 0x45;              /* version 4, header_length 5 */
    ip[1] = 0;                 /* type_of_service */
    ip[2] = (uint8_t)(total_len >> 8);
    ip[3] = (uint8_t)total_len;
    /* id (4-5) is not written: the headroom's bytes stay */
    ip[6] = 0x40;              /* fragment_offset = kDF */
    ip[7] = 0;
    ip[8] = 64;                /* ttl */
    ip[9] = proto;
    memcpy(ip + 12, src, 4);
    memcpy(ip + 16, dst, 4);
    uint16_t ck = or_ipv4_checksum(ip); /* CalculateIpv4NoOptChecksum */
    memcpy(ip + 10, &ck, 2);
    if (offs[3] >= 0) memcpy(meta + offs[3], dst, 4);
    if (offs[4] >= 0) {
      meta[offs[4]] = 0x08;    /* be16(Ethernet::Type::kIpv4) */
      meta[offs[4] + 1] = 0x00;
    }
  }
}

/* ====================================================================== */
/* NAT (core/modules/nat.{h,cc}): dynamic address/port translation         */
/* ====================================================================== */
/* Endpoint (nat.h:48-78) as its 8 bytes: addr raw be32 | port raw be16 <<
 * 32 | protocol << 48; NatEntry {endpoint, last_refresh}. CuckooMap lookup
 * semantics only (a key maps to one entry; Insert overwrites). The port
 * search draws from bess::utils::Random (random.h:38-70), seeded here
 * (the reference seeds it from rdtsc). */
typedef struct {
  uint64_t key, ep, ts;
  int used;
} or_nat_slot;

typedef struct or_nat {
  uint32_t naddr;
  uint32_t addrs[64];          /* ext_addrs_ (raw be32), sorted by value */
  uint32_t nranges[64];
  uint16_t rbeg[64][16], rend[64][16];
  uint8_t rsusp[64][16];       /* port_ranges_[i] (Init order, not sorted) */
  uint64_t seed;               /* Random::seed_ */
  size_t cap, count, tomb;
  or_nat_slot *tab;            /* open addressing, power-of-two capacity */
} or_nat;

static uint64_t nat_mix(uint64_t x) {
  x ^= x >> 33; x *= 0xff51afd7ed558ccdULL; x ^= x >> 33;
  return x;
}

static or_nat_slot *nat_find(or_nat *m, uint64_t key) {
  size_t i = nat_mix(key) & (m->cap - 1);
  for (;;) {
    or_nat_slot *s = &m->tab[i];
    if (s->used == 0) return NULL;
    if (s->used == 1 && s->key == key) return s;
    i = (i + 1) & (m->cap - 1);
  }
}

static void nat_grow(or_nat *m);
/* HashTable::Insert: overwrite or add */
static or_nat_slot *nat_insert(or_nat *m, uint64_t key, uint64_t ep) {
  or_nat_slot *s = nat_find(m, key);
  if (s) { s->ep = ep; return s; }
  if ((m->count + m->tomb + 1) * 2 > m->cap) nat_grow(m);
  size_t i = nat_mix(key) & (m->cap - 1);
  while (m->tab[i].used == 1) i = (i + 1) & (m->cap - 1);
  if (m->tab[i].used == 2) m->tomb--;
  m->tab[i].used = 1;
  m->tab[i].key = key;
  m->tab[i].ep = ep;
  m->tab[i].ts = 0;
  m->count++;
  return &m->tab[i];
}

static void nat_grow(or_nat *m) {
  size_t oc = m->cap;
  or_nat_slot *ot = m->tab;
  m->cap = oc ? (m->count * 4 > oc ? oc * 2 : oc) : 1024;
  m->tab = (or_nat_slot *)calloc(m->cap, sizeof(or_nat_slot));
  m->count = 0;
  m->tomb = 0;
  for (size_t i = 0; i < oc; i++)
    if (ot[i].used == 1) {
      or_nat_slot *s = nat_insert(m, ot[i].key, ot[i].ep);
      s->ts = ot[i].ts;
    }
  free(ot);
}

/* HashTable::Remove: tombstone (used = 2) */
static void nat_remove(or_nat *m, uint64_t key) {
  or_nat_slot *s = nat_find(m, key);
  if (s) { s->used = 2; m->count--; m->tomb++; }
}

or_nat *or_nat_new(uint64_t seed) {
  or_nat *m = (or_nat *)calloc(1, sizeof(or_nat));
  m->seed = seed;
  nat_grow(m);
  return m;
}
void or_nat_free(or_nat *m) { if (m) { free(m->tab); free(m); } }
size_t or_nat_count(const or_nat *m) { return m->count; }

/* Init 46-96 after validation: addresses in the argument's order with their
 * range lists; ext_addrs_ is then sorted (be32_t compares values) while
 * port_ranges_ keeps the argument's order. */
void or_nat_init(or_nat *m, const uint32_t *addrs_host, uint32_t naddr,
                 const uint32_t *nranges, const uint16_t *beg, const uint16_t *end,
                 const uint8_t *susp) {
  uint32_t k = 0;
  for (uint32_t i = 0; i < naddr; i++) {
    if (nranges[i] == 0) {
      m->nranges[i] = 1;
      m->rbeg[i][0] = 0; m->rend[i][0] = 65535; m->rsusp[i][0] = 0;
    } else {
      m->nranges[i] = nranges[i];
      for (uint32_t r = 0; r < nranges[i]; r++, k++) {
        m->rbeg[i][r] = beg[k]; m->rend[i][r] = end[k]; m->rsusp[i][r] = susp[k];
      }
    }
  }
  uint32_t v[64];
  memcpy(v, addrs_host, naddr * 4);
  for (uint32_t i = 1; i < naddr; i++)   /* insertion sort by value */
    for (uint32_t j = i; j > 0 && v[j - 1] > v[j]; j--) {
      uint32_t t = v[j]; v[j] = v[j - 1]; v[j - 1] = t;
    }
  for (uint32_t i = 0; i < naddr; i++) m->addrs[i] = __builtin_bswap32(v[i]);
  m->naddr = naddr;
}

/* Random::GetRange (random.h:58-75) */
static uint32_t nat_get_range(or_nat *m, uint32_t range) {
  m->seed = m->seed * 1103515245 + 12345;
  union { uint64_t i; double d; } t;
  t.i = (m->seed >> 12) | 0x3ff0000000000000ULL;
  return (uint32_t)((t.d - 1.0) * range);
}

static uint64_t ep_make(uint32_t addr_raw, uint16_t port_raw, uint16_t proto) {
  return (uint64_t)addr_raw | (uint64_t)port_raw << 32 | (uint64_t)proto << 48;
}

/* CreateNewEntry 180-258 -> the forward entry, or NULL */
static or_nat_slot *nat_create(or_nat *m, uint64_t in, uint64_t now) {
  const uint32_t in_addr = (uint32_t)in;
  const uint16_t in_port = (uint16_t)(in >> 32), proto = (uint16_t)(in >> 48);
  const uint32_t hashed = _mm_crc32_u32(0, in_addr); /* rte_hash_crc(&addr, 4, 0) */
  const uint32_t idx = hashed % m->naddr;
  const uint16_t in_port_host = __builtin_bswap16(in_port);
  for (uint32_t r = 0; r < m->nranges[idx]; r++) {
    uint16_t min, range;
    if (m->rsusp[idx][r]) continue;
    if (proto == 1) {
      min = m->rbeg[idx][r];
      range = (uint16_t)(m->rend[idx][r] - m->rbeg[idx][r]);
    } else if (in_port_host == 0) {
      return NULL;
    } else if (in_port_host & ~1023u) {
      if (m->rend[idx][r] <= 1024u) continue;
      min = m->rbeg[idx][r] > 1024 ? m->rbeg[idx][r] : 1024;
      range = (uint16_t)(m->rend[idx][r] - min + 1);
    } else {
      if (m->rbeg[idx][r] >= 1023u) continue;
      min = m->rbeg[idx][r];
      range = (uint16_t)((m->rend[idx][r] < 1023 ? m->rend[idx][r] : 1023) - min);
    }
    const uint16_t start = (uint16_t)(min + nat_get_range(m, range));
    uint16_t port = start;
    int trials = 0;
    do {
      const uint64_t ext = ep_make(m->addrs[idx], __builtin_bswap16(port), proto);
      or_nat_slot *rev = nat_find(m, ext);
      int take = rev == NULL;
      if (!take) {
        or_nat_slot *fwd = nat_find(m, rev->ep);
        if (now - fwd->ts > 300ull * 1000 * 1000 * 1000) { /* kTimeOutNs */
          nat_remove(m, fwd->key);
          nat_remove(m, rev->key);
          take = 1;
        }
      }
      if (take) {
        nat_insert(m, ext, in);
        return nat_insert(m, in, ext);
      }
      port++;
      trials++;
      if (port == 0 || port >= min + range) port = min;
    } while (port != start && trials < 128); /* kMaxTrials */
  }
  return NULL;
}

/* UpdateChecksumWithIncrement / ChecksumIncrement16/32 (checksum.h:520-549) */
static uint16_t nat_upd(uint16_t ck, uint32_t incr) {
  return or_fold_checksum((uint32_t)(~ck & 0xFFFF) + incr);
}
static uint32_t nat_inc32(uint32_t o, uint32_t n) {
  return (~o >> 16) + (~o & 0xFFFF) + (n >> 16) + (n & 0xFFFF);
}
static uint32_t nat_inc16(uint16_t o, uint16_t n) { return (uint32_t)(~o & 0xFFFF) + n; }

/* DoProcessBatch<dir> 321-363 with ExtractEndpoint 120-160 and Stamp
 * 262-319, over n packets (32-packet batches give the same result: every
 * packet is decided in order) */
void or_nat_process(or_nat *m, uint8_t *base, size_t stride, size_t n, int dir,
                    uint64_t now, uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    uint8_t *ip = base + i * stride + 14;
    uint8_t *l4 = ip + ((ip[0] & 0x0F) << 2);
    const uint8_t proto = ip[9];
    uint16_t port;
    int valid = 0;
    if (proto == 6 || proto == 17) {
      memcpy(&port, l4 + (dir == 0 ? 0 : 2), 2);
      valid = 1;
    } else if (proto == 1) {
      const uint8_t t = l4[0];
      if (t == 0 || t == 8 || t == 13 || t == 15 || t == 16) {
        memcpy(&port, l4 + 4, 2); /* icmp->ident */
        valid = 1;
      }
    }
    if (!valid) { out[i] = 8192; continue; } /* DropPacket */
    uint32_t addr;
    memcpy(&addr, ip + (dir == 0 ? 12 : 16), 4);
    const uint64_t before = ep_make(addr, port, proto);
    or_nat_slot *e = nat_find(m, before);
    if (!e) {
      if (dir != 0 || !(e = nat_create(m, before, now))) { out[i] = 8192; continue; }
    }
    if (dir == 0) e->ts = now;
    /* Stamp<dir> */
    const uint32_t na = (uint32_t)e->ep;
    const uint16_t np = (uint16_t)(e->ep >> 32);
    memcpy(ip + (dir == 0 ? 12 : 16), &na, 4);
    const uint32_t l3 = nat_inc32(addr, na);
    uint16_t ck;
    memcpy(&ck, ip + 10, 2);
    ck = nat_upd(ck, l3);
    memcpy(ip + 10, &ck, 2);
    const uint32_t l4inc = l3 + nat_inc16(port, np);
    if (proto == 6 || proto == 17) {
      memcpy(l4 + (dir == 0 ? 0 : 2), &np, 2);
      if (proto == 6) {
        memcpy(&ck, l4 + 16, 2);
        ck = nat_upd(ck, l4inc);
        memcpy(l4 + 16, &ck, 2);
      } else {
        memcpy(&ck, l4 + 6, 2);
        if (ck != 0) {
          ck = nat_upd(ck, l4inc);
          if (ck == 0) ck = 0xFFFF;
          memcpy(l4 + 6, &ck, 2);
        }
      }
    } else {
      memcpy(l4 + 4, &np, 2);
      memcpy(&ck, l4 + 2, 2);
      ck = nat_upd(ck, nat_inc16(port, np)); /* UpdateChecksum16 */
      memcpy(l4 + 2, &ck, 2);
    }
    out[i] = dir == 0 ? 1 : 0;
  }
}

/* ====================================================================== */
/* CPU baselines (bench.py cpu_baseline legs)                              */
/* ====================================================================== */

/* IPLookup's CPU cost is rte_lpm's lookup (DPDK 19.11, absent here):
 * DIR-24-8 -- one 2^24-entry table indexed by the top 24 address bits,
 * and 256-entry groups for /24 blocks that hold deeper rules. This is a
 * restatement of that structure (rte_lpm.c's rte_lpm_lookup_bulk fast
 * path), used only to time the reference's lookup on the host; results are
 * checked equal to or_lpm_process. Entry: 0 none, 0x80000000 | group, else
 * next hop + 1. Rules are applied in ascending depth (deeper overrides). */
typedef struct or_dir24 {
  uint32_t *tbl24;
  uint32_t *tbl8;
  size_t ngroups;
} or_dir24;

static int dir24_cmp_depth(const void *a, const void *b) {
  return (int)((const uint32_t *)a)[1] - (int)((const uint32_t *)b)[1];
}

or_dir24 *or_dir24_build(const uint32_t *ips, const uint8_t *depths,
                         const uint32_t *nhs, size_t nrules) {
  or_dir24 *t = (or_dir24 *)calloc(1, sizeof(or_dir24));
  t->tbl24 = (uint32_t *)calloc((size_t)1 << 24, 4);
  uint32_t(*r)[3] = (uint32_t(*)[3])malloc((nrules + 1) * sizeof(*r));
  for (size_t i = 0; i < nrules; i++) {
    r[i][0] = ips[i] & lpm_mask(depths[i]);
    r[i][1] = depths[i];
    r[i][2] = nhs[i];
  }
  qsort(r, nrules, sizeof(*r), dir24_cmp_depth);  /* stable enough: distinct (ip, depth) */
  size_t cap = 0;
  for (size_t i = 0; i < nrules; i++) {
    const uint32_t ip = r[i][0], d = r[i][1], v = r[i][2] + 1;
    if (d <= 24) {
      const uint32_t b = ip >> 8, cnt = 1u << (24 - d);
      for (uint32_t k = b; k < b + cnt; k++) {
        if (t->tbl24[k] & 0x80000000u) {  /* deeper block: fill its group */
          uint32_t *g = t->tbl8 + (size_t)(t->tbl24[k] & 0x7FFFFFFFu) * 256;
          for (int j = 0; j < 256; j++) g[j] = v;  /* rules come by depth */
        } else {
          t->tbl24[k] = v;
        }
      }
    } else {
      const uint32_t b = ip >> 8;
      if (!(t->tbl24[b] & 0x80000000u)) {
        if (t->ngroups == cap) {
          cap = cap ? cap * 2 : 64;
          t->tbl8 = (uint32_t *)realloc(t->tbl8, cap * 256 * 4);
        }
        uint32_t *g = t->tbl8 + t->ngroups * 256;
        for (int j = 0; j < 256; j++) g[j] = t->tbl24[b];
        t->tbl24[b] = 0x80000000u | (uint32_t)t->ngroups++;
      }
      uint32_t *g = t->tbl8 + (size_t)(t->tbl24[b] & 0x7FFFFFFFu) * 256;
      const uint32_t lo = ip & 0xFF, cnt = 1u << (32 - d);
      for (uint32_t j = lo; j < lo + cnt; j++) g[j] = v;
    }
  }
  free(r);
  return t;
}

void or_dir24_free(or_dir24 *t) {
  if (!t) return;
  free(t->tbl24);
  free(t->tbl8);
  free(t);
}

void or_dir24_process(const or_dir24 *t, const uint8_t *base, size_t stride,
                      size_t n, uint16_t default_gate, uint16_t *out) {
  for (size_t i = 0; i < n; i++) {
    const uint32_t dst = be32(base + i * stride + 30);
    uint32_t e = t->tbl24[dst >> 8];
    if (e & 0x80000000u) e = t->tbl8[(size_t)(e & 0x7FFFFFFFu) * 256 + (dst & 0xFF)];
    out[i] = e ? (uint16_t)(e - 1) : default_gate;
  }
}

typedef struct {
  const or_dir24 *t;
  const uint8_t *base;
  size_t stride;
  uint16_t dg;
  uint16_t *out;
} dir24_ctx;

static void dir24_slice(void *p, size_t b, size_t e) {
  dir24_ctx *c = (dir24_ctx *)p;
  or_dir24_process(c->t, c->base + b * c->stride, c->stride, e - b, c->dg, c->out + b);
}

double or_dir24_bench(const or_dir24 *t, const uint8_t *base, size_t stride,
                      size_t n, uint16_t default_gate, uint16_t *out,
                      int nthreads, int reps) {
  dir24_ctx c = {t, base, stride, default_gate, out};
  return run_slices(dir24_slice, &c, n, nthreads, reps);
}

typedef struct {
  uint8_t *base;
  size_t stride;
  uint16_t *out;
} ttl_ctx;

static void ttl_slice(void *p, size_t b, size_t e) {
  ttl_ctx *c = (ttl_ctx *)p;
  or_update_ttl_process(c->base + b * c->stride, c->stride, e - b, c->out + b);
}

double or_update_ttl_bench(uint8_t *base, size_t stride, size_t n, uint16_t *out,
                           int nthreads, int reps) {
  ttl_ctx c = {base, stride, out};
  return run_slices(ttl_slice, &c, n, nthreads, reps);
}

typedef struct {
  const uint32_t *ia, *ea, *sz;
  size_t np;
  uint8_t *base;
  size_t stride;
  uint16_t *out;
} snat_ctx;

static void snat_slice(void *p, size_t b, size_t e) {
  snat_ctx *c = (snat_ctx *)p;
  or_static_nat_process(c->ia, c->ea, c->sz, c->np, c->base + b * c->stride,
                        c->stride, e - b, 0, c->out + b);
}

double or_static_nat_bench(const uint32_t *int_addr, const uint32_t *ext_addr,
                           const uint32_t *size, size_t npairs, uint8_t *base,
                           size_t stride, size_t n, uint16_t *out, int nthreads,
                           int reps) {
  snat_ctx c = {int_addr, ext_addr, size, npairs, base, stride, out};
  return run_slices(snat_slice, &c, n, nthreads, reps);
}

/* ------------------------------------------------------------------------
 * Rewrite (core/modules/rewrite.{h,cc}): kNumSlots = 2 * kMaxBurst - 1 = 63
 * template slots of kMaxTemplateSize = 1536 bytes; CommandAdd (25-61) fills
 * slots [curr, curr + k) and replicates template i % n into every later
 * slot so that a batch reads templates_[start + i] without a modulo;
 * ProcessBatch (105-113) -> DoRewriteSingle (72-86) / DoRewrite (88-103)
 * per batch of <= kMaxBurst packets: data_off = SNBUF_HEADROOM, lengths =
 * the template's size, CopyInlined(..., sloppy = true) -- whole 32-byte
 * AVX2 blocks (copy.h:145-231), so up to 31 bytes past the size come from
 * the template slot too. next_turn_ = jump_[start + cnt]: jump_[i] is
 * written only for i >= n (its value i % n), so for start + cnt < n the
 * reference reads an unset entry; restated as start + cnt (its meaning).
 * ------------------------------------------------------------------------ */
#define OR_RW_SLOTS 63
#define OR_RW_MAX 1536
#define OR_RW_BURST 32

typedef struct {
  uint8_t t[OR_RW_SLOTS][OR_RW_MAX];
  uint16_t size[OR_RW_SLOTS];
  size_t jump[OR_RW_SLOTS + 1];
  size_t n, next;
} or_rewrite;

or_rewrite *or_rewrite_new(void) { return (or_rewrite *)calloc(1, sizeof(or_rewrite)); }
void or_rewrite_free(or_rewrite *r) { free(r); }

/* CommandAdd: 0, -EINVAL with the reference's message in msg */
int or_rewrite_add(or_rewrite *r, const uint8_t *const *tmpl, const uint32_t *len,
                   int k, char *msg, size_t msglen) {
  size_t curr = r->n;
  if (curr + (size_t)k > OR_RW_BURST) {
    snprintf(msg, msglen, "max %zu packet templates can be used %zu %d",
             (size_t)OR_RW_BURST, curr, k);
    return -EINVAL;
  }
  for (int i = 0; i < k; i++) {
    if (len[i] > OR_RW_MAX) {
      snprintf(msg, msglen, "template is too big");
      return -EINVAL;
    }
    memset(r->t[curr + i], 0, OR_RW_MAX);
    memcpy(r->t[curr + i], tmpl[i], len[i]);
    r->size[curr + i] = (uint16_t)len[i];
  }
  r->n = curr + (size_t)k;
  if (r->n == 0) return 0;
  for (size_t i = r->n; i < OR_RW_SLOTS; i++) {
    size_t j = i % r->n;
    memcpy(r->t[i], r->t[j], r->size[j]);
    r->size[i] = r->size[j];
    r->jump[i] = j;
  }
  r->jump[OR_RW_SLOTS] = OR_RW_SLOTS % r->n;
  return 0;
}

void or_rewrite_clear(or_rewrite *r) {
  r->next = 0;
  r->n = 0;
}

/* n packets in slots of `stride` bytes (data at slot + head[i]), processed
 * as consecutive batches of <= 32: head[i] = headroom, len[i] = size */
void or_rewrite_process(or_rewrite *r, uint8_t *slots, size_t stride, size_t n,
                        uint32_t headroom, uint16_t *head, uint32_t *len) {
  for (size_t b = 0; b < n; b += OR_RW_BURST) {
    const size_t cnt = n - b < OR_RW_BURST ? n - b : OR_RW_BURST;
    if (r->n == 0) continue;
    const size_t start = r->n == 1 ? 0 : r->next;
    for (size_t i = 0; i < cnt; i++) {
      const size_t s = start + i;
      const uint16_t size = r->size[s];
      uint8_t *dst = slots + (b + i) * stride + headroom;
      size_t blocks = ((size_t)size + 31) / 32;  /* sloppy: whole 32 B blocks */
      memcpy(dst, r->t[s], blocks * 32);
      head[b + i] = (uint16_t)headroom;
      len[b + i] = size;
    }
    if (r->n > 1) r->next = start + cnt < r->n ? start + cnt : r->jump[start + cnt];
  }
}
