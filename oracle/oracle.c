/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h / oracle/README.md).
 *
 * A plain-C restatement of the reference (NetSys/bess) algorithms on the
 * packet-classification hot path. Every function cites the reference
 * file:line it follows. It is used by tests/ as the parity checker and by
 * bench.py as the timed CPU baseline ("kind": "port"); the shipped library
 * bess_amd/libbessgpu.so never links or calls it.
 *
 * Build: oracle/Makefile (gcc -O3 -mavx2 -msse4.2 -fPIC -shared -pthread).
 */
#define _GNU_SOURCE
#include "oracle.h"

#include <errno.h>
#include <pthread.h>
#include <sched.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

/* ====================================================================== */
/* utils                                                                   */
/* ====================================================================== */

/* endian.cc:36-58 uint64_to_bin */
int or_uint64_to_bin(void *ptr, uint64_t val, size_t size, int big_endian) {
  uint8_t *const p8 = (uint8_t *)ptr;
  if (big_endian) {
    for (size_t i = size; i-- > 0;) {
      p8[i] = val & 0xff;
      val >>= 8;
    }
  } else {
    for (size_t i = 0; i < size; i++) {
      p8[i] = val & 0xff;
      val >>= 8;
    }
  }
  return val == 0;
}

static inline uint64_t ld64(const uint8_t *p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return v;
}
static inline uint32_t ld32(const uint8_t *p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return v;
}
static inline uint16_t ld16(const uint8_t *p) {
  uint16_t v;
  memcpy(&v, p, 2);
  return v;
}
static inline uint16_t be16(const uint8_t *p) {
  return (uint16_t)((p[0] << 8) | p[1]);
}

/* ExactMatchKeyHash (exact_match_table.h:97-119) and wm_hash
 * (wildcard_match.h:106-129): CRC32C over len/8 u64 words, init 0, using
 * DPDK rte_hash_crc.h crc32c_sse42_u64(data, init) == _mm_crc32_u64(init,
 * data) (DPDK 19.11.4). */
uint32_t or_key_hash(const uint64_t *key, size_t len) {
  uint64_t h = 0;
  for (size_t i = 0; i < len / 8; i++) h = _mm_crc32_u64(h, key[i]);
  return (uint32_t)h;
}

/* ====================================================================== */
/* CuckooMap restatement (core/utils/cuckoo_map.h)                         */
/* ====================================================================== */

#define CK_SLOTS 4        /* kEntriesPerBucket, cuckoo_map.h:291 */
#define CK_INIT_BUCKETS 4 /* kInitNumBucket 289 */
#define CK_INIT_ENTRIES 16 /* kInitNumEntries 290 */
#define CK_MAX_PATH 3      /* kMaxCuckooPath 297 */
#define CK_INVALID 0xFFFFFFFFu

typedef struct {
  uint32_t hash[CK_SLOTS]; /* Bucket::hash_values, 307-312 */
  uint32_t idx[CK_SLOTS];  /* Bucket::entry_indices */
} ck_bucket;

typedef struct {
  uint64_t key[8]; /* Entry::first (ExactMatchKey / wm_hkey_t) */
  uint8_t val[8];  /* Entry::second (gate_idx_t / WmData) */
} ck_entry;

struct or_cuckoo {
  uint32_t bucket_mask;
  size_t num_entries;
  size_t nbuckets;
  ck_bucket *buckets;
  size_t nentries;
  ck_entry *entries;
  uint32_t *stack; /* free_entry_indices_ (std::stack, top = last) */
  size_t stack_n, stack_cap;
  size_t key_len; /* the len_ handed to hasher/eq by the caller */
  size_t val_len;
};

static void ck_push(struct or_cuckoo *m, uint32_t idx) {
  if (m->stack_n == m->stack_cap) {
    m->stack_cap = m->stack_cap ? m->stack_cap * 2 : 64;
    m->stack = (uint32_t *)realloc(m->stack, m->stack_cap * sizeof(uint32_t));
  }
  m->stack[m->stack_n++] = idx;
}

/* CuckooMap(reserve_buckets, reserve_entries) cuckoo_map.h:152-164 */
static void ck_init(struct or_cuckoo *m, size_t nb, size_t ne, size_t key_len,
                    size_t val_len) {
  memset(m, 0, sizeof(*m));
  m->bucket_mask = (uint32_t)(nb - 1);
  m->nbuckets = nb;
  m->buckets = (ck_bucket *)calloc(nb, sizeof(ck_bucket));
  m->nentries = ne;
  m->entries = (ck_entry *)calloc(ne, sizeof(ck_entry));
  m->key_len = key_len;
  m->val_len = val_len;
  for (size_t i = ne; i-- > 0;) ck_push(m, (uint32_t)i);
}

static void ck_destroy(struct or_cuckoo *m) {
  free(m->buckets);
  free(m->entries);
  free(m->stack);
  memset(m, 0, sizeof(*m));
}

/* Hash() 508-510: never 0 (bit 31 forced) */
static inline uint32_t ck_hash(const struct or_cuckoo *m, const uint64_t *key) {
  return or_key_hash(key, m->key_len) | (1u << 31);
}
/* HashSecondary() 502-505 */
static inline uint32_t ck_hash2(uint32_t primary) {
  uint32_t tag = primary >> 12;
  return primary ^ ((tag + 1) * 0x5bd1e995u);
}
/* ExactMatchKeyEq 76-94 / wm_eq */
static inline int ck_eq(const struct or_cuckoo *m, const uint64_t *a,
                        const uint64_t *b) {
  for (size_t i = 0; i < m->key_len / 8; i++)
    if (a[i] != b[i]) return 0;
  return 1;
}

/* FindSlot 432-445 */
static int ck_find_slot(const struct or_cuckoo *m, const ck_bucket *b,
                        uint32_t primary, const uint64_t *key) {
  for (int i = 0; i < CK_SLOTS; i++) {
    if (b->hash[i] == primary) {
      const ck_entry *e = &m->entries[b->idx[i]];
      if (ck_eq(m, e->key, key)) return i;
    }
  }
  return -1;
}

/* GetFromBucket 374-387 */
static uint32_t ck_get_from_bucket(const struct or_cuckoo *m, uint32_t primary,
                                   uint32_t bidx, const uint64_t *key) {
  const ck_bucket *b = &m->buckets[bidx];
  int s = ck_find_slot(m, b, primary, key);
  return s < 0 ? CK_INVALID : b->idx[s];
}

/* FindWithHash 492-499 */
static uint32_t ck_find_with_hash(const struct or_cuckoo *m, uint32_t primary,
                                  const uint64_t *key) {
  uint32_t r = ck_get_from_bucket(m, primary, primary & m->bucket_mask, key);
  if (r != CK_INVALID) return r;
  return ck_get_from_bucket(m, primary, ck_hash2(primary) & m->bucket_mask,
                            key);
}

/* Find 243-253 */
static const ck_entry *ck_find(const struct or_cuckoo *m, const uint64_t *key) {
  uint32_t idx = ck_find_with_hash(m, ck_hash(m, key), key);
  return idx == CK_INVALID ? NULL : &m->entries[idx];
}

/* ExpandEntries 513-523 */
static void ck_expand_entries(struct or_cuckoo *m) {
  size_t old_size = m->nentries;
  size_t new_size = old_size + old_size / 2;
  m->entries = (ck_entry *)realloc(m->entries, new_size * sizeof(ck_entry));
  memset(m->entries + old_size, 0, (new_size - old_size) * sizeof(ck_entry));
  m->nentries = new_size;
  for (size_t i = new_size; i-- > old_size;) ck_push(m, (uint32_t)i);
}

/* PopFreeEntryIndex 318-325 */
static uint32_t ck_pop_free(struct or_cuckoo *m) {
  if (m->stack_n == 0) ck_expand_entries(m);
  return m->stack[--m->stack_n];
}

/* FindEmptySlot 422-429 */
static int ck_find_empty(const ck_bucket *b) {
  for (int i = 0; i < CK_SLOTS; i++)
    if (b->hash[i] == 0) return i;
  return -1;
}

/* EmplaceInBucket 329-350 */
static ck_entry *ck_emplace_in_bucket(struct or_cuckoo *m, uint32_t bidx,
                                      const uint64_t *key, const void *val) {
  ck_bucket *b = &m->buckets[bidx];
  int slot = ck_find_empty(b);
  if (slot == -1) return NULL;
  uint32_t free_idx = ck_pop_free(m);
  b = &m->buckets[bidx];
  b->hash[slot] = ck_hash(m, key);
  b->idx[slot] = free_idx;
  ck_entry *e = &m->entries[free_idx];
  memcpy(e->key, key, OR_KEY_BYTES);
  memset(e->val, 0, sizeof(e->val));
  memcpy(e->val, val, m->val_len);
  m->num_entries++;
  return e;
}

/* MakeSpace 450-488 */
static int ck_make_space(struct or_cuckoo *m, uint32_t index, int depth) {
  if (depth >= CK_MAX_PATH) return -1;
  ck_bucket *b = &m->buckets[index];
  for (int i = 0; i < CK_SLOTS; i++) {
    uint32_t idx = b->idx[i];
    const uint64_t *key = m->entries[idx].key;
    uint32_t pri = ck_hash(m, key);
    uint32_t sec = ck_hash2(pri);
    uint32_t alt;
    if (pri == b->hash[i]) {
      alt = sec & m->bucket_mask;
    } else if (sec == b->hash[i]) {
      alt = pri & m->bucket_mask;
    } else {
      return -1;
    }
    int j = ck_find_empty(&m->buckets[alt]);
    if (j == -1) j = ck_make_space(m, alt, depth + 1);
    if (j >= 0) {
      ck_bucket *ab = &m->buckets[alt];
      ab->hash[j] = b->hash[i];
      ab->idx[j] = b->idx[i];
      b->hash[i] = 0;
      return i;
    }
  }
  return -1;
}

/* EmplaceEntry 392-418 */
static ck_entry *ck_emplace_entry(struct or_cuckoo *m, uint32_t primary,
                                  uint32_t secondary, const uint64_t *key,
                                  const void *val) {
  ck_entry *e;
  uint32_t pb, sb;
again:
  pb = primary & m->bucket_mask;
  if ((e = ck_emplace_in_bucket(m, pb, key, val)) != NULL) return e;
  sb = secondary & m->bucket_mask;
  if ((e = ck_emplace_in_bucket(m, sb, key, val)) != NULL) return e;
  if (ck_make_space(m, pb, 0) >= 0) goto again;
  if (ck_make_space(m, sb, 0) >= 0) goto again;
  return NULL;
}

static ck_entry *ck_do_emplace(struct or_cuckoo *m, const uint64_t *key,
                               const void *val);

/* ExpandBuckets 530-547 */
static void ck_expand_buckets(struct or_cuckoo *m) {
  struct or_cuckoo bigger;
  ck_init(&bigger, m->nbuckets * 2, m->nentries, m->key_len, m->val_len);
  for (size_t bi = 0; bi < m->nbuckets; bi++) {
    for (int s = 0; s < CK_SLOTS; s++) {
      if (m->buckets[bi].hash[s] == 0) continue;
      const ck_entry *e = &m->entries[m->buckets[bi].idx[s]];
      if (!ck_do_emplace(&bigger, e->key, e->val)) {
        ck_destroy(&bigger);
        return;
      }
    }
  }
  ck_destroy(m);
  *m = bigger;
}

/* DoEmplace 178-207 (Insert 213-222): insert or overwrite */
static ck_entry *ck_do_emplace(struct or_cuckoo *m, const uint64_t *key,
                               const void *val) {
  uint32_t primary = ck_hash(m, key);
  uint32_t idx = ck_find_with_hash(m, primary, key);
  if (idx != CK_INVALID) {
    ck_entry *e = &m->entries[idx];
    memset(e->val, 0, sizeof(e->val));
    memcpy(e->val, val, m->val_len);
    return e;
  }
  uint32_t secondary = ck_hash2(primary);
  int trials = 0;
  ck_entry *e;
  while ((e = ck_emplace_entry(m, primary, secondary, key, val)) == NULL) {
    if (++trials >= 3) return NULL; /* "Excessive hash colision" */
    ck_expand_buckets(m);
  }
  return e;
}

/* RemoveFromBucket 355-371 */
static int ck_remove_from_bucket(struct or_cuckoo *m, uint32_t primary,
                                 uint32_t bidx, const uint64_t *key) {
  ck_bucket *b = &m->buckets[bidx];
  int slot = ck_find_slot(m, b, primary, key);
  if (slot == -1) return 0;
  b->hash[slot] = 0;
  uint32_t idx = b->idx[slot];
  memset(&m->entries[idx], 0, sizeof(ck_entry));
  ck_push(m, idx);
  m->num_entries--;
  return 1;
}

/* Remove 257-267 */
static int ck_remove(struct or_cuckoo *m, const uint64_t *key) {
  uint32_t pri = ck_hash(m, key);
  if (ck_remove_from_bucket(m, pri, pri & m->bucket_mask, key)) return 1;
  uint32_t sec = ck_hash2(pri);
  if (ck_remove_from_bucket(m, pri, sec & m->bucket_mask, key)) return 1;
  return 0;
}

/* Clear 269-286 */
static void ck_clear(struct or_cuckoo *m) {
  size_t kl = m->key_len, vl = m->val_len;
  ck_destroy(m);
  ck_init(m, CK_INIT_BUCKETS, CK_INIT_ENTRIES, kl, vl);
}

/* iterator 70-150: bucket-major, slot-minor, skipping hash == 0 */
static const ck_entry *ck_iter(const struct or_cuckoo *m, size_t *cursor) {
  while (*cursor < m->nbuckets * CK_SLOTS) {
    size_t b = *cursor / CK_SLOTS, s = *cursor % CK_SLOTS;
    (*cursor)++;
    if (m->buckets[b].hash[s] != 0) return &m->entries[m->buckets[b].idx[s]];
  }
  return NULL;
}

static void set_msg(char *msg, size_t msglen, const char *fmt, ...)
    __attribute__((format(printf, 3, 4)));
#include <stdarg.h>
static void set_msg(char *msg, size_t msglen, const char *fmt, ...) {
  if (!msg || !msglen) return;
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, msglen, fmt, ap);
  va_end(ap);
}

/* ====================================================================== */
/* ExactMatch (core/utils/exact_match_table.h, core/modules/exact_match.cc) */
/* ====================================================================== */

typedef struct {
  uint64_t mask;
  int attr_id;
  int offset;
  int pos;
  int size;
} em_field; /* ExactMatchField 126-140 */

struct or_em {
  size_t raw_key_size;
  size_t total_key_size;
  size_t num_fields;
  em_field fields[OR_MAX_FIELDS];
  struct or_cuckoo table; /* CuckooMap<ExactMatchKey, gate_idx_t> */
};

or_em *or_em_new(void) {
  or_em *em = (or_em *)calloc(1, sizeof(or_em));
  /* key_len is set as fields are added (hasher(total_key_size_)) */
  ck_init(&em->table, CK_INIT_BUCKETS, CK_INIT_ENTRIES, 0, 2);
  return em;
}

void or_em_free(or_em *em) {
  if (!em) return;
  ck_destroy(&em->table);
  free(em);
}

/* DoAddField 391-443 (offset-based fields; attr fields are out of scope) */
int or_em_add_field(or_em *em, int offset, int size, uint64_t mask, int idx,
                    char *msg, size_t msglen) {
  if (idx >= OR_MAX_FIELDS) {
    set_msg(msg, msglen, "idx %d is not in [0,%d)", idx, OR_MAX_FIELDS);
    return EINVAL;
  }
  em_field *f = &em->fields[idx];
  f->size = size;
  if (f->size < 1 || f->size > OR_MAX_FIELD_SIZE) {
    set_msg(msg, msglen, "idx %d: 'size' must be in [1,%d]", idx,
            OR_MAX_FIELD_SIZE);
    return EINVAL;
  }
  f->attr_id = -1;
  f->offset = offset;
  if (f->offset < 0 || f->offset > 1024) {
    set_msg(msg, msglen, "idx %d: invalid 'offset'", idx);
    return EINVAL;
  }
  int force_be = 1; /* attr_id < 0 */
  if (mask == 0) {
    /* SetBitsHigh<uint64_t>(size*8), bits.h:180-185: the LOW n bits */
    f->mask = (f->size * 8 >= 64) ? ~0ULL : ((1ULL << (f->size * 8)) - 1);
  } else {
    if (!or_uint64_to_bin(&f->mask, mask, (size_t)f->size, force_be)) {
      set_msg(msg, msglen, "idx %d: not a valid %d-byte mask", idx, f->size);
      return EINVAL;
    }
  }
  if (f->mask == 0) {
    set_msg(msg, msglen, "idx %d: empty mask", idx);
    return EINVAL;
  }
  em->num_fields++;
  f->pos = (int)em->raw_key_size;
  em->raw_key_size += (size_t)f->size;
  em->total_key_size = (em->raw_key_size + 7) / 8 * 8; /* align_ceil */
  em->table.key_len = em->total_key_size;
  return 0;
}

size_t or_em_num_fields(const or_em *em) { return em->num_fields; }
size_t or_em_total_key_size(const or_em *em) { return em->total_key_size; }

void or_em_get_field(const or_em *em, size_t i, uint64_t *mask, int *offset,
                     int *pos, int *size) {
  const em_field *f = &em->fields[i];
  if (mask) *mask = f->mask;
  if (offset) *offset = f->offset;
  if (pos) *pos = f->pos;
  if (size) *size = f->size;
}

/* gather_key 332-357 */
static int em_gather_key(const or_em *em, const uint8_t *const *vals,
                         const size_t *lens, size_t n, uint64_t *key,
                         char *msg, size_t msglen) {
  if (n != em->num_fields) {
    set_msg(msg, msglen, "rule should have %zu fields (has %zu)",
            em->num_fields, n);
    return EINVAL;
  }
  memset(key, 0, OR_KEY_BYTES);
  for (size_t i = 0; i < n; i++) {
    int field_size = em->fields[i].size;
    int field_pos = em->fields[i].pos;
    if ((size_t)field_size != lens[i]) {
      set_msg(msg, msglen, "rule field %zu should have size %d (has %zu)", i,
              field_size, lens[i]);
      return EINVAL;
    }
    memcpy((uint8_t *)key + field_pos, vals[i], (size_t)field_size);
  }
  return 0;
}

/* AddRule 175-191 (Insert failure ignored, 187-190) */
int or_em_add_rule(or_em *em, uint16_t gate, const uint8_t *const *vals,
                   const size_t *lens, size_t nvals, char *msg,
                   size_t msglen) {
  uint64_t key[8];
  if (nvals == 0) {
    set_msg(msg, msglen, "rule has no fields");
    return EINVAL;
  }
  int err = em_gather_key(em, vals, lens, nvals, key, msg, msglen);
  if (err) return err;
  ck_do_emplace(&em->table, key, &gate);
  return 0;
}

/* n rules at once (test helper): rule i's field values are the
 * raw_key_size bytes at keys + i * key_stride, cut at the fields' sizes in
 * field order, i.e. or_em_add_rule with value_bin fields. */
int or_em_add_rules(or_em *em, const uint8_t *keys, size_t n, size_t key_stride,
                    const uint16_t *gates) {
  const uint8_t *vals[OR_MAX_FIELDS];
  size_t lens[OR_MAX_FIELDS];
  for (size_t i = 0; i < n; i++) {
    const uint8_t *k = keys + i * key_stride;
    size_t pos = 0;
    for (size_t f = 0; f < em->num_fields; f++) {
      vals[f] = k + pos;
      lens[f] = (size_t)em->fields[f].size;
      pos += lens[f];
    }
    int err = or_em_add_rule(em, gates[i], vals, lens, em->num_fields, NULL, 0);
    if (err) return err;
  }
  return 0;
}

/* DeleteRule 198-217 */
int or_em_delete_rule(or_em *em, const uint8_t *const *vals, const size_t *lens,
                      size_t nvals, char *msg, size_t msglen) {
  uint64_t key[8];
  if (nvals == 0) {
    set_msg(msg, msglen, "rule has no fields");
    return EINVAL;
  }
  int err = em_gather_key(em, vals, lens, nvals, key, msg, msglen);
  if (err) return err;
  if (!ck_remove(&em->table, key)) {
    set_msg(msg, msglen, "rule doesn't exist");
    return ENOENT;
  }
  return 0;
}

void or_em_clear(or_em *em) { ck_clear(&em->table); } /* ClearRules 220 */
size_t or_em_count(const or_em *em) { return em->table.num_entries; }

int or_em_iter(const or_em *em, size_t *cursor, uint8_t key_out[OR_KEY_BYTES],
               uint16_t *gate_out) {
  const ck_entry *e = ck_iter(&em->table, cursor);
  if (!e) return 0;
  memcpy(key_out, e->key, OR_KEY_BYTES);
  memcpy(gate_out, e->val, 2);
  return 1;
}

/* ExactMatchTable::MakeKeys (exact_match_table.h:239-263) for one packet;
 * the key is zeroed first (the reference zeroes only the last key word;
 * words past total_key_size are never read by its callers). */
void or_em_make_key(const or_em *em, const uint8_t *head, uint64_t key[8]) {
  memset(key, 0, 64);
  for (size_t f = 0; f < em->num_fields; f++) {
    uint64_t v = ld64(head + em->fields[f].offset) & em->fields[f].mask;
    uint8_t tmp[16];
    memcpy(tmp, &v, 8);
    int pos = em->fields[f].pos;
    memcpy((uint8_t *)key + pos, tmp, (size_t)(pos + 8 <= 64 ? 8 : 64 - pos));
  }
}

/* An attr_name field reads its metadata attribute: ExactMatch::ProcessBatch's
 * buffer_fn (exact_match.cc:230-236) returns ptr_attr(this, attr_id, pkt) =
 * the packet's metadata + attr_offset(attr_id) (module.h:679-684). The
 * offset is whatever the pipeline's metadata allocator assigned; it is
 * bound here. */
void or_em_bind_attr(or_em *em, int idx, int mt_offset) {
  em->fields[idx].attr_id = 0;
  em->fields[idx].offset = mt_offset;
}

/* MakeKeys 239-263 + ExactMatch::ProcessBatch 224-244 + Find 273-278;
 * metas[j]: packet j's metadata area (attr fields), may be NULL without
 * attr fields */
static void em_process_batch_meta(const or_em *em, const uint8_t *const *heads,
                                  const uint8_t *const *metas, int cnt,
                                  uint16_t default_gate, uint16_t *gates) {
  uint64_t keys[OR_MAX_BURST][8];
  if (em->total_key_size == 0) {
    /* no fields: the reference indexes u64_arr[(0-1)/8] (UB); with no
     * fields no rule can exist, so every packet takes the default gate. */
    for (int i = 0; i < cnt; i++) gates[i] = default_gate;
    return;
  }
  size_t last = (em->total_key_size - 1) / 8;
  for (int i = 0; i < cnt; i++) keys[i][last] = 0;
  for (size_t f = 0; f < em->num_fields; f++) {
    uint64_t mask = em->fields[f].mask;
    int pos = em->fields[f].pos;
    int off = em->fields[f].offset;
    const int attr = em->fields[f].attr_id >= 0;
    for (int j = 0; j < cnt; j++) {
      uint64_t v = ld64((attr ? metas[j] : heads[j]) + off) & mask;
      memcpy((uint8_t *)keys[j] + pos, &v, 8);
    }
  }
  for (int i = 0; i < cnt; i++) {
    const ck_entry *e = ck_find(&em->table, keys[i]);
    uint16_t g;
    if (e) {
      memcpy(&g, e->val, 2);
    } else {
      g = default_gate;
    }
    gates[i] = g;
  }
}

void or_em_process_batch(const or_em *em, const uint8_t *const *heads, int cnt,
                         uint16_t default_gate, uint16_t *gates) {
  em_process_batch_meta(em, heads, NULL, cnt, default_gate, gates);
}

/* n packets: frame i at base + i*stride, its metadata area at
 * meta + i*meta_stride (meta may be NULL without attr fields) */
void or_em_process_meta(const or_em *em, const uint8_t *base, size_t stride,
                        const uint8_t *meta, size_t meta_stride, size_t n,
                        uint16_t default_gate, uint16_t *gates) {
  const uint8_t *heads[OR_MAX_BURST], *metas[OR_MAX_BURST];
  for (size_t i = 0; i < n; i += OR_MAX_BURST) {
    int cnt = (int)((n - i) < OR_MAX_BURST ? (n - i) : OR_MAX_BURST);
    for (int j = 0; j < cnt; j++) {
      heads[j] = base + (i + (size_t)j) * stride;
      metas[j] = meta ? meta + (i + (size_t)j) * meta_stride : NULL;
    }
    em_process_batch_meta(em, heads, metas, cnt, default_gate, gates + i);
  }
}

void or_em_process(const or_em *em, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates) {
  or_em_process_meta(em, base, stride, NULL, 0, n, default_gate, gates);
}

/* ====================================================================== */
/* WildcardMatch (core/modules/wildcard_match.{h,cc})                      */
/* ====================================================================== */

typedef struct {
  int attr_id, offset, pos, size;
} wm_field; /* WmField wildcard_match.h:62-72 */

typedef struct {
  int32_t priority;
  uint16_t ogate;
} wm_data; /* WmData .h:57-60 */

typedef struct {
  struct or_cuckoo ht;
  uint64_t mask[8];
} wm_tuple; /* WmTuple .h:166-169 */

struct or_wm {
  size_t total_key_size;
  int size_acc;
  int nfields;
  wm_field fields[64];
  int ntuples;
  wm_tuple tuples[OR_MAX_TUPLES];
};

or_wm *or_wm_new(void) { return (or_wm *)calloc(1, sizeof(or_wm)); }

void or_wm_free(or_wm *wm) {
  if (!wm) return;
  for (int t = 0; t < wm->ntuples; t++) ck_destroy(&wm->tuples[t].ht);
  free(wm);
}

/* Init 111-134 / AddFieldOne 75-100 (offset fields) */
int or_wm_add_field(or_wm *wm, int offset, int size, char *msg,
                    size_t msglen) {
  if (wm->nfields >= 64) {
    set_msg(msg, msglen, "too many fields");
    return EINVAL;
  }
  wm_field *f = &wm->fields[wm->nfields++];
  f->pos = wm->size_acc;
  f->size = size;
  if (f->size < 1 || f->size > OR_MAX_FIELD_SIZE) {
    set_msg(msg, msglen, "'size' must be 1-%d", OR_MAX_FIELD_SIZE);
    return EINVAL;
  }
  f->attr_id = -1;
  f->offset = offset;
  if (f->offset < 0 || f->offset > 1024) {
    set_msg(msg, msglen, "too small 'offset'");
    return EINVAL;
  }
  wm->size_acc += f->size;
  return 0;
}

void or_wm_init_done(or_wm *wm) {
  wm->total_key_size = ((size_t)wm->size_acc + 7) / 8 * 8;
}

size_t or_wm_total_key_size(const or_wm *wm) { return wm->total_key_size; }
size_t or_wm_num_fields(const or_wm *wm) { return (size_t)wm->nfields; }
void or_wm_get_field(const or_wm *wm, size_t i, int *offset, int *pos,
                     int *size) {
  if (offset) *offset = wm->fields[i].offset;
  if (pos) *pos = wm->fields[i].pos;
  if (size) *size = wm->fields[i].size;
}

/* FindTuple 278-288 */
static int wm_find_tuple(const or_wm *wm, const uint8_t *mask) {
  for (int i = 0; i < wm->ntuples; i++)
    if (memcmp(wm->tuples[i].mask, mask, wm->total_key_size) == 0) return i;
  return -ENOENT;
}

/* AddTuple 290-300 */
static int wm_add_tuple(or_wm *wm, const uint8_t *mask) {
  if (wm->ntuples >= OR_MAX_TUPLES) return -ENOSPC;
  wm_tuple *t = &wm->tuples[wm->ntuples];
  ck_init(&t->ht, CK_INIT_BUCKETS, CK_INIT_ENTRIES, wm->total_key_size,
          sizeof(wm_data));
  memcpy(t->mask, mask, OR_KEY_BYTES);
  return wm->ntuples++;
}

/* CommandAdd 317-354 after ExtractKeyMask + is_valid_gate */
int or_wm_add(or_wm *wm, const uint8_t key[OR_KEY_BYTES],
              const uint8_t mask[OR_KEY_BYTES], int32_t priority,
              uint16_t gate) {
  wm_data data;
  memset(&data, 0, sizeof(data));
  data.priority = priority;
  data.ogate = gate;
  int idx = wm_find_tuple(wm, mask);
  if (idx < 0) {
    idx = wm_add_tuple(wm, mask);
    if (idx < 0) return -idx; /* ENOSPC */
  }
  uint64_t k[8];
  memcpy(k, key, OR_KEY_BYTES);
  if (ck_do_emplace(&wm->tuples[idx].ht, k, &data) == NULL) return EINVAL;
  return 0;
}

/* CommandDelete 357-377 + DelEntry 302-315 (a successful Remove returns 1,
 * so an emptied tuple is erased only when Remove FAILS on an empty tuple). */
int or_wm_delete(or_wm *wm, const uint8_t key[OR_KEY_BYTES],
                 const uint8_t mask[OR_KEY_BYTES]) {
  int idx = wm_find_tuple(wm, mask);
  if (idx < 0) return -idx; /* ENOENT */
  uint64_t k[8];
  memcpy(k, key, OR_KEY_BYTES);
  wm_tuple *t = &wm->tuples[idx];
  int ret = ck_remove(&t->ht, k);
  if (ret) return 0; /* DelEntry returned 1 (> 0): success */
  if (t->ht.num_entries == 0) {
    ck_destroy(&t->ht);
    memmove(&wm->tuples[idx], &wm->tuples[idx + 1],
            (size_t)(wm->ntuples - idx - 1) * sizeof(wm_tuple));
    wm->ntuples--;
    memset(&wm->tuples[wm->ntuples], 0, sizeof(wm_tuple));
  }
  return 0;
}

/* Clear 384-388: tables emptied, tuples (and their order) kept */
void or_wm_clear(or_wm *wm) {
  for (int t = 0; t < wm->ntuples; t++) ck_clear(&wm->tuples[t].ht);
}

int or_wm_num_tuples(const or_wm *wm) { return wm->ntuples; }
void or_wm_tuple_mask(const or_wm *wm, int t, uint8_t mask_out[OR_KEY_BYTES]) {
  memcpy(mask_out, wm->tuples[t].mask, OR_KEY_BYTES);
}
size_t or_wm_tuple_count(const or_wm *wm, int t) {
  return wm->tuples[t].ht.num_entries;
}
int or_wm_iter(const or_wm *wm, int t, size_t *cursor,
               uint8_t key_out[OR_KEY_BYTES], int32_t *prio, uint16_t *gate) {
  const ck_entry *e = ck_iter(&wm->tuples[t].ht, cursor);
  if (!e) return 0;
  wm_data d;
  memcpy(&d, e->val, sizeof(d));
  memcpy(key_out, e->key, OR_KEY_BYTES);
  *prio = d.priority;
  *gate = d.ogate;
  return 1;
}

/* LookupEntry 136-157 */
static uint16_t wm_lookup(const or_wm *wm, const uint64_t *key,
                          uint16_t def_gate) {
  int32_t best_prio = INT32_MIN;
  uint16_t best_gate = def_gate;
  size_t nw = wm->total_key_size / 8;
  for (int t = 0; t < wm->ntuples; t++) {
    const wm_tuple *tp = &wm->tuples[t];
    uint64_t km[8];
    for (size_t i = 0; i < nw; i++) km[i] = key[i] & tp->mask[i];
    const ck_entry *e = ck_find(&tp->ht, km);
    if (e) {
      wm_data d;
      memcpy(&d, e->val, sizeof(d));
      if (d.priority >= best_prio) { /* '>=': later tuple wins a tie */
        best_prio = d.priority;
        best_gate = d.ogate;
      }
    }
  }
  return best_gate;
}

/* ProcessBatch 159-203 (offset fields: raw unmasked 8-byte loads) */
/* attr fields: ProcessBatch 177-195 reads buffer + mt_offset_to_databuf_
 * offset(attr_offset(attr_id)) -- the metadata attribute (packet.h:189-191) */
void or_wm_bind_attr(or_wm *wm, int idx, int mt_offset) {
  wm->fields[idx].attr_id = 0;
  wm->fields[idx].offset = mt_offset;
}

static void wm_process_batch_meta(const or_wm *wm, const uint8_t *const *heads,
                                  const uint8_t *const *metas, int cnt,
                                  uint16_t default_gate, uint16_t *gates) {
  uint64_t keys[OR_MAX_BURST][8];
  if (wm->total_key_size == 0) {
    for (int i = 0; i < cnt; i++) gates[i] = default_gate;
    return;
  }
  memset(keys, 0, sizeof(keys));
  for (int f = 0; f < wm->nfields; f++) {
    int off = wm->fields[f].offset, pos = wm->fields[f].pos;
    const int attr = wm->fields[f].attr_id >= 0;
    for (int j = 0; j < cnt; j++) {
      uint64_t v = ld64((attr ? metas[j] : heads[j]) + off);
      memcpy((uint8_t *)keys[j] + pos, &v, 8);
    }
  }
  for (int i = 0; i < cnt; i++) gates[i] = wm_lookup(wm, keys[i], default_gate);
}

void or_wm_process_batch(const or_wm *wm, const uint8_t *const *heads, int cnt,
                         uint16_t default_gate, uint16_t *gates) {
  wm_process_batch_meta(wm, heads, NULL, cnt, default_gate, gates);
}

void or_wm_process_meta(const or_wm *wm, const uint8_t *base, size_t stride,
                        const uint8_t *meta, size_t meta_stride, size_t n,
                        uint16_t default_gate, uint16_t *gates) {
  const uint8_t *heads[OR_MAX_BURST], *metas[OR_MAX_BURST];
  for (size_t i = 0; i < n; i += OR_MAX_BURST) {
    int cnt = (int)((n - i) < OR_MAX_BURST ? (n - i) : OR_MAX_BURST);
    for (int j = 0; j < cnt; j++) {
      heads[j] = base + (i + (size_t)j) * stride;
      metas[j] = meta ? meta + (i + (size_t)j) * meta_stride : NULL;
    }
    wm_process_batch_meta(wm, heads, metas, cnt, default_gate, gates + i);
  }
}

void or_wm_process(const or_wm *wm, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates) {
  or_wm_process_meta(wm, base, stride, NULL, 0, n, default_gate, gates);
}

/* ====================================================================== */
/* checksums (core/utils/checksum.h)                                       */
/* ====================================================================== */

/* CalculateSum 52-181: AVX2 two-stream unpack/accumulate for len >= 128,
 * then 8-word and 2-word add-with-carry loops, then u16 words, then the
 * trailing byte as a low byte; reduce to 32 bits with end-around carry. */
uint32_t or_calculate_sum(const void *buf, size_t len) {
  const uint8_t *p = (const uint8_t *)buf;
  uint64_t sum64 = 0;
  int odd = (int)(len & 1);
#ifdef __AVX2__
  if (len >= 128) {
    __m256i zero = _mm256_setzero_si256();
    __m256i a = _mm256_loadu_si256((const __m256i *)p);
    __m256i b = _mm256_loadu_si256((const __m256i *)(p + 32));
    __m256i sah = _mm256_unpackhi_epi32(a, zero);
    __m256i sal = _mm256_unpacklo_epi32(a, zero);
    __m256i sbh = _mm256_unpackhi_epi32(b, zero);
    __m256i sbl = _mm256_unpacklo_epi32(b, zero);
    len -= 64;
    p += 64;
    while (len >= 64) {
      a = _mm256_loadu_si256((const __m256i *)p);
      b = _mm256_loadu_si256((const __m256i *)(p + 32));
      sah = _mm256_add_epi64(sah, _mm256_unpackhi_epi32(a, zero));
      sal = _mm256_add_epi64(sal, _mm256_unpacklo_epi32(a, zero));
      sbh = _mm256_add_epi64(sbh, _mm256_unpackhi_epi32(b, zero));
      sbl = _mm256_add_epi64(sbl, _mm256_unpacklo_epi32(b, zero));
      len -= 64;
      p += 64;
    }
    __m256i s256 = _mm256_add_epi64(_mm256_add_epi64(sah, sal),
                                    _mm256_add_epi64(sbh, sbl));
    __m128i s128 = _mm_add_epi64(_mm256_extracti128_si256(s256, 0),
                                 _mm256_extracti128_si256(s256, 1));
    sum64 += (uint64_t)_mm_extract_epi64(s128, 0) +
             (uint64_t)_mm_extract_epi64(s128, 1);
  }
#endif
  while (len >= 64) { /* addq; adcq x7; adcq $0 (111-127) */
    unsigned long long s = sum64;
    unsigned char c = _addcarry_u64(0, s, ld64(p), &s);
    for (int k = 1; k < 8; k++) c = _addcarry_u64(c, s, ld64(p + 8 * k), &s);
    _addcarry_u64(c, s, 0, &s);
    sum64 = s;
    len -= 64;
    p += 64;
  }
  while (len >= 16) { /* 131-141 */
    unsigned long long s = sum64;
    unsigned char c = _addcarry_u64(0, s, ld64(p), &s);
    c = _addcarry_u64(c, s, ld64(p + 8), &s);
    _addcarry_u64(c, s, 0, &s);
    sum64 = s;
    len -= 16;
    p += 16;
  }
  sum64 = (sum64 >> 32) + (sum64 & 0xFFFFFFFF);
  while (len >= 2) { /* 165-169 */
    sum64 += ld16(p);
    p += 2;
    len -= 2;
  }
  if (odd) sum64 += *p; /* 172-174 */
  sum64 = (sum64 >> 32) + (sum64 & 0xFFFFFFFF);
  sum64 += (sum64 >> 32);
  return (uint32_t)sum64;
}

/* FoldChecksum 185-189 */
uint16_t or_fold_checksum(uint32_t cksum) {
  cksum = (cksum >> 16) + (cksum & 0xFFFF);
  cksum += (cksum >> 16);
  return (uint16_t)~cksum;
}

uint16_t or_generic_checksum(const void *buf, size_t len) {
  return or_fold_checksum(or_calculate_sum(buf, len));
}

/* 32-bit 'addl; adcl ...; adcl $0' chains used by the header helpers */
static inline uint32_t adc_chain32(uint32_t sum, const uint32_t *w, int n) {
  unsigned int s = sum;
  unsigned char c = _addcarry_u32(0, s, w[0], &s);
  for (int i = 1; i < n; i++) c = _addcarry_u32(c, s, w[i], &s);
  _addcarry_u32(c, s, 0, &s);
  return s;
}

/* CalculateIpv4NoOptChecksum 233-251 / CalculateIpv4Checksum 288-318 */
uint16_t or_ipv4_checksum(const uint8_t *ip) {
  size_t hl = (size_t)(ip[0] & 0x0F) << 2;
  uint32_t w[5];
  for (int i = 0; i < 5; i++) w[i] = ld32(ip + 4 * i);
  if (hl == 20) {
    uint32_t x[4] = {w[1], w[2] & 0xFFFF, w[3], w[4]};
    return or_fold_checksum(adc_chain32(w[0], x, 4));
  }
  if (hl < 20) return 0;
  uint32_t sum = or_calculate_sum(ip + 20, hl - 20);
  uint32_t x[5] = {w[0], w[1], w[2] & 0xFFFF, w[3], w[4]};
  return or_fold_checksum(adc_chain32(sum, x, 5));
}

/* VerifyIpv4NoOptChecksum 211-228 / VerifyIpv4Checksum 254-283 */
int or_ipv4_verify(const uint8_t *ip) {
  size_t hl = (size_t)(ip[0] & 0x0F) << 2;
  uint32_t w[5];
  for (int i = 0; i < 5; i++) w[i] = ld32(ip + 4 * i);
  if (hl == 20) return or_fold_checksum(adc_chain32(w[0], w + 1, 4)) == 0;
  if (hl < 20) return 0;
  uint32_t sum = or_calculate_sum(ip + 20, hl - 20);
  return or_fold_checksum(adc_chain32(sum, w, 5)) == 0;
}

static inline uint16_t bswap16(uint16_t v) { return (uint16_t)((v << 8) | (v >> 8)); }

/* CalculateIpv4UdpChecksum 371-393 + 398-407 */
uint16_t or_udp_checksum(const uint8_t *ip, const uint8_t *udp) {
  size_t udp_len = be16(udp + 4);
  if (udp_len < 8) return 0;
  uint32_t sum = or_calculate_sum(udp + 8, udp_len - 8);
  uint32_t len = bswap16((uint16_t)udp_len);
  uint32_t x[6] = {ld32(udp), ld32(udp + 4) & 0xFFFF, ld32(ip + 12),
                   ld32(ip + 16), len, 0x1100};
  uint16_t r = or_fold_checksum(adc_chain32(sum, x, 6));
  return r ? r : 0xFFFF;
}

/* VerifyIpv4UdpChecksum 324-362 */
int or_udp_verify(const uint8_t *ip, const uint8_t *udp) {
  size_t udp_len = be16(udp + 4);
  if (udp_len < 8) return 0;
  if (ld16(udp + 6) == 0) return 1;
  uint32_t sum = or_calculate_sum(udp + 8, udp_len - 8);
  uint32_t len = bswap16((uint16_t)udp_len);
  uint32_t x[6] = {ld32(udp), ld32(udp + 4), ld32(ip + 12), ld32(ip + 16), len,
                   0x1100};
  return or_fold_checksum(adc_chain32(sum, x, 6)) == 0;
}

/* CalculateIpv4TcpChecksum 461-487 + 492-504 */
uint16_t or_tcp_checksum(const uint8_t *ip, const uint8_t *tcp) {
  size_t ip_len = be16(ip + 2);
  size_t hl = (size_t)(ip[0] & 0x0F) << 2;
  if (ip_len < hl + 20) return 0;
  uint16_t tcp_len = (uint16_t)(ip_len - hl);
  uint32_t sum = or_calculate_sum(tcp + 20, (size_t)tcp_len - 20);
  uint32_t len = bswap16(tcp_len);
  uint32_t x[9] = {ld32(tcp),     ld32(tcp + 4),      ld32(tcp + 8),
                   ld32(tcp + 12), ld32(tcp + 16) >> 16, ld32(ip + 12),
                   ld32(ip + 16), len,                0x0600};
  return or_fold_checksum(adc_chain32(sum, x, 9));
}

/* VerifyIpv4TcpChecksum 413-452 */
int or_tcp_verify(const uint8_t *ip, const uint8_t *tcp) {
  size_t ip_len = be16(ip + 2);
  size_t hl = (size_t)(ip[0] & 0x0F) << 2;
  if (ip_len < hl + 20) return 0;
  uint16_t tcp_len = (uint16_t)(ip_len - hl);
  uint32_t sum = or_calculate_sum(tcp + 20, (size_t)tcp_len - 20);
  uint32_t len = bswap16(tcp_len);
  uint32_t x[9] = {ld32(tcp),      ld32(tcp + 4), ld32(tcp + 8),
                   ld32(tcp + 12), ld32(tcp + 16), ld32(ip + 12),
                   ld32(ip + 16),  len,           0x0600};
  return or_fold_checksum(adc_chain32(sum, x, 9)) == 0;
}

/* RFC 1624 incremental update, checksum.h:520-560 */
uint16_t or_update_checksum16(uint16_t old_ck, uint16_t old_v,
                              uint16_t new_v) {
  uint32_t inc = (uint32_t)(~old_v & 0xFFFF) + new_v;
  return or_fold_checksum((uint32_t)(~old_ck & 0xFFFF) + inc);
}
uint16_t or_update_checksum32(uint16_t old_ck, uint32_t old_v,
                              uint32_t new_v) {
  uint32_t inc = (~old_v >> 16) + (~old_v & 0xFFFF);
  inc += (new_v >> 16) + (new_v & 0xFFFF);
  return or_fold_checksum((uint32_t)(~old_ck & 0xFFFF) + inc);
}

static inline void st16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

/* IPChecksum::ProcessBatch ip_checksum.cc:39-84 */
void or_ip_checksum_batch(uint8_t *const *heads, int cnt, int verify,
                          uint16_t *gates) {
  for (int i = 0; i < cnt; i++) {
    uint8_t *eth = heads[i];
    uint8_t *data = eth + 14;
    uint16_t et = be16(eth + 12);
    if (et == 0x88a8) { /* kQinQ */
      uint8_t *qinq = data;
      data = qinq + 4;
      et = be16(qinq + 2);
      if (et != 0x8100) {
        gates[i] = 0;
        continue;
      }
    }
    if (et == 0x8100) { /* kVlan */
      uint8_t *vlan = data;
      data = vlan + 4;
      et = be16(vlan + 2);
    }
    if (et != 0x0800) {
      gates[i] = 0;
      continue;
    }
    uint8_t *ip = data;
    if (verify) {
      gates[i] = or_ipv4_verify(ip) ? 0 : 1;
    } else {
      st16(ip + 10, or_ipv4_checksum(ip));
      gates[i] = 0;
    }
  }
}

/* L4Checksum::ProcessBatch l4_checksum.cc:41-83 */
void or_l4_checksum_batch(uint8_t *const *heads, int cnt, int verify,
                          uint16_t *gates) {
  for (int i = 0; i < cnt; i++) {
    uint8_t *eth = heads[i];
    if (be16(eth + 12) != 0x0800) {
      gates[i] = 0;
      continue;
    }
    uint8_t *ip = eth + 14;
    size_t hl = (size_t)(ip[0] & 0x0F) << 2;
    if (ip[9] == 17) {
      uint8_t *udp = ip + hl;
      if (verify) {
        gates[i] = or_udp_verify(ip, udp) ? 0 : 1;
      } else {
        st16(udp + 6, or_udp_checksum(ip, udp));
        gates[i] = 0;
      }
    } else if (ip[9] == 6) {
      uint8_t *tcp = ip + hl;
      if (verify) {
        gates[i] = or_tcp_verify(ip, tcp) ? 0 : 1;
      } else {
        st16(tcp + 16, or_tcp_checksum(ip, tcp));
        gates[i] = OR_GATE_NONE; /* no EmitPacket (79-81) */
      }
    } else {
      gates[i] = OR_GATE_NONE; /* neither UDP nor TCP: never emitted */
    }
  }
}

static void cksum_batch(uint8_t *const *heads, int cnt, int mode, int verify,
                        uint16_t *ipg, uint16_t *l4g) {
  uint16_t g1[OR_MAX_BURST], g2[OR_MAX_BURST];
  if (mode & 1) {
    or_ip_checksum_batch(heads, cnt, verify, g1);
    if (ipg) memcpy(ipg, g1, (size_t)cnt * 2);
  }
  if (mode & 2) {
    if (mode & 1) {
      /* pipeline: only packets emitted on IPChecksum gate 0 reach L4 */
      uint8_t *sub[OR_MAX_BURST];
      int idx[OR_MAX_BURST], m = 0;
      for (int j = 0; j < cnt; j++)
        if (g1[j] == 0) {
          idx[m] = j;
          sub[m++] = heads[j];
        }
      uint16_t gs[OR_MAX_BURST];
      or_l4_checksum_batch(sub, m, verify, gs);
      for (int j = 0; j < cnt; j++) g2[j] = OR_GATE_NONE;
      for (int k = 0; k < m; k++) g2[idx[k]] = gs[k];
    } else {
      or_l4_checksum_batch(heads, cnt, verify, g2);
    }
    if (l4g) memcpy(l4g, g2, (size_t)cnt * 2);
  }
}

void or_cksum_process(uint8_t *base, size_t stride, size_t n, int mode,
                      int verify, uint16_t *ip_gates, uint16_t *l4_gates) {
  uint8_t *heads[OR_MAX_BURST];
  for (size_t i = 0; i < n; i += OR_MAX_BURST) {
    int cnt = (int)((n - i) < OR_MAX_BURST ? (n - i) : OR_MAX_BURST);
    for (int j = 0; j < cnt; j++) heads[j] = base + (i + (size_t)j) * stride;
    cksum_batch(heads, cnt, mode, verify, ip_gates ? ip_gates + i : NULL,
                l4_gates ? l4_gates + i : NULL);
  }
}

/* ====================================================================== */
/* threaded CPU-baseline drivers                                           */
/* ====================================================================== */

typedef struct {
  int kind; /* 0 em, 1 wm, 2 cksum */
  const void *obj;
  uint8_t *base;
  size_t stride, begin, end;
  uint16_t default_gate;
  uint16_t *gates;
  int mode, verify, reps, cpu;
  pthread_barrier_t *bar;
  uint64_t connected, sunk;  /* C1 pipeline */
} bench_arg;

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* Config C1 (bessctl/conf/samples/exactmatch.bess): Source -> ExactMatch
 * -> Sink on one worker. Per 32-packet batch (Source::RunTask,
 * source.cc:83-101, packets from the pool): ExactMatch::ProcessBatch
 * (exact_match.cc:224-244), then EmitPacket of each packet into its gate's
 * batch (core/module.h:543-594: a gate that is not connected drops; a full
 * batch of kMaxBurst goes to the next module), the Task running the
 * connected gates' batches into Sink (sink.cc:33-35, which frees them:
 * counted here) at the end of the call (ProcessOGates, 596-618). Returns
 * the packets the sink received. `connected`: gates 0..63 bitmap. */
static uint64_t c1_batches(const or_em *em, const uint8_t *base, size_t stride,
                           size_t n, uint16_t default_gate, uint64_t connected,
                           uint16_t *gates) {
  const uint8_t *heads[OR_MAX_BURST];
  uint64_t sunk = 0, dead = 0;
  int fill[64];
  for (size_t i = 0; i < n; i += OR_MAX_BURST) {
    int cnt = (int)((n - i) < OR_MAX_BURST ? (n - i) : OR_MAX_BURST);
    for (int j = 0; j < cnt; j++) heads[j] = base + (i + (size_t)j) * stride;
    uint16_t *g = gates + i;
    or_em_process_batch(em, heads, cnt, default_gate, g);
    memset(fill, 0, sizeof(fill));
    for (int j = 0; j < cnt; j++) {
      const uint16_t o = g[j];
      if (o >= 64 || !((connected >> o) & 1)) {  /* DropPacket */
        dead++;
        continue;
      }
      if (fill[o] >= OR_MAX_BURST) {  /* full: to the next module */
        sunk += (uint64_t)fill[o];
        fill[o] = 0;
      }
      fill[o]++;
    }
    for (int o = 0; o < 64; o++) sunk += (uint64_t)fill[o];  /* Sink */
  }
  (void)dead;
  return sunk;
}

static void *bench_thread(void *p) {
  bench_arg *a = (bench_arg *)p;
  if (a->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(a->cpu, &set);
    pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
  }
  pthread_barrier_wait(a->bar);
  size_t n = a->end - a->begin;
  for (int r = 0; r < a->reps; r++) {
    uint8_t *b = a->base + a->begin * a->stride;
    uint16_t *g = a->gates + a->begin;
    if (a->kind == 0)
      or_em_process((const or_em *)a->obj, b, a->stride, n, a->default_gate, g);
    else if (a->kind == 1)
      or_wm_process((const or_wm *)a->obj, b, a->stride, n, a->default_gate, g);
    else if (a->kind == 3)
      a->sunk += c1_batches((const or_em *)a->obj, b, a->stride, n,
                            a->default_gate, a->connected, g);
    else
      or_cksum_process(b, a->stride, n, a->mode, a->verify, NULL, g);
  }
  pthread_barrier_wait(a->bar);
  return NULL;
}

int or_num_cpus(void) {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return 1;
  return CPU_COUNT(&set);
}

static double run_bench_c1(int kind, const void *obj, uint8_t *base,
                           size_t stride, size_t n, uint16_t dg, uint16_t *gates,
                           int mode, int verify, int nthreads, int reps,
                           uint64_t connected, uint64_t *sunk) {
  if (nthreads < 1) nthreads = 1;
  cpu_set_t set;
  int cpus[1024], ncpu = 0;
  if (sched_getaffinity(0, sizeof(set), &set) == 0)
    for (int c = 0; c < CPU_SETSIZE && ncpu < 1024; c++)
      if (CPU_ISSET(c, &set)) cpus[ncpu++] = c;
  pthread_barrier_t bar;
  pthread_barrier_init(&bar, NULL, (unsigned)nthreads + 1);
  pthread_t *th = (pthread_t *)calloc((size_t)nthreads, sizeof(pthread_t));
  bench_arg *args = (bench_arg *)calloc((size_t)nthreads, sizeof(bench_arg));
  for (int t = 0; t < nthreads; t++) {
    bench_arg *a = &args[t];
    a->kind = kind;
    a->obj = obj;
    a->base = base;
    a->stride = stride;
    /* slices aligned to whole 32-packet batches */
    size_t nb = (n + OR_MAX_BURST - 1) / OR_MAX_BURST;
    size_t b0 = nb * (size_t)t / (size_t)nthreads,
           b1 = nb * (size_t)(t + 1) / (size_t)nthreads;
    a->begin = b0 * OR_MAX_BURST;
    a->end = b1 * OR_MAX_BURST < n ? b1 * OR_MAX_BURST : n;
    if (a->begin > a->end) a->begin = a->end;
    a->default_gate = dg;
    a->gates = gates;
    a->mode = mode;
    a->verify = verify;
    a->reps = reps;
    a->connected = connected;
    a->sunk = 0;
    a->cpu = ncpu ? cpus[t % ncpu] : -1;
    a->bar = &bar;
    pthread_create(&th[t], NULL, bench_thread, a);
  }
  pthread_barrier_wait(&bar);
  double t0 = now_s();
  pthread_barrier_wait(&bar);
  double t1 = now_s();
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  if (sunk) {
    *sunk = 0;
    for (int t = 0; t < nthreads; t++) *sunk += args[t].sunk;
  }
  pthread_barrier_destroy(&bar);
  free(th);
  free(args);
  return t1 - t0;
}

static double run_bench(int kind, const void *obj, uint8_t *base, size_t stride,
                        size_t n, uint16_t dg, uint16_t *gates, int mode,
                        int verify, int nthreads, int reps) {
  return run_bench_c1(kind, obj, base, stride, n, dg, gates, mode, verify,
                      nthreads, reps, 0, NULL);
}

double or_c1_bench(const or_em *em, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint64_t connected,
                   uint16_t *gates, int nthreads, int reps, uint64_t *sunk) {
  return run_bench_c1(3, em, (uint8_t *)base, stride, n, default_gate, gates, 0,
                      0, nthreads, reps, connected, sunk);
}

double or_em_bench(const or_em *em, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates,
                   int nthreads, int reps) {
  return run_bench(0, em, (uint8_t *)base, stride, n, default_gate, gates, 0, 0,
                   nthreads, reps);
}
double or_wm_bench(const or_wm *wm, const uint8_t *base, size_t stride,
                   size_t n, uint16_t default_gate, uint16_t *gates,
                   int nthreads, int reps) {
  return run_bench(1, wm, (uint8_t *)base, stride, n, default_gate, gates, 0, 0,
                   nthreads, reps);
}
double or_cksum_bench(uint8_t *base, size_t stride, size_t n, int mode,
                      int verify, uint16_t *l4_gates, int nthreads, int reps) {
  return run_bench(2, NULL, base, stride, n, 0, l4_gates, mode, verify,
                   nthreads, reps);
}
