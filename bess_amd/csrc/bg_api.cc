// bg_api.cc -- C ABI of libbessgpu.so (include/bessgpu.h): rule storage,
// device-table build/upload, kernel launch plumbing and host staging.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/bessgpu.h"
#include "bg_internal.h"
#include "bg_wm_jit.h"
#include "bg_kernels.h"
#include "bg_launch.h"
#include "bg_table.h"

namespace bg {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
  return -code;
}

int num_cus(int device) {
  // launch path: a lock-free per-device cache (the answer never changes)
  static std::atomic<int> cache[64];
  if (device < 0 || device >= 64) return 256;
  int v = cache[device].load(std::memory_order_relaxed);
  if (v > 0) return v;
  if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount,
                            device) != hipSuccess || v <= 0)
    v = 256;
  cache[device].store(v, std::memory_order_relaxed);
  return v;
}

int set_device(int device) {
  // launch path: one cached count (once positive) and a current-device check
  static std::atomic<int> cached{0};
  int n = cached.load(std::memory_order_relaxed);
  if (n <= 0) {
    int c = 0;
    const hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess || c <= 0)
      return fail(ENODEV, "no HIP device available (hipGetDeviceCount: %s, %d)",
                  hipGetErrorString(e), c);
    cached.store(c, std::memory_order_relaxed);
    n = c;
  }
  if (device < 0 || device >= n)
    return fail(ENODEV, "device %d out of range [0,%d)", device, n);
  int cur = -1;
  if (hipGetDevice(&cur) == hipSuccess && cur == device) return 0;
  HIP_TRY(hipSetDevice(device));
  return 0;
}

uint32_t round_kw(uint32_t key_bytes) {
  uint32_t w = (key_bytes + 7) / 8;
  if (w <= 1) return 1;
  if (w <= 2) return 2;
  if (w <= 4) return 4;
  return 8;
}

// Field plan for frames whose head_data() is at offset `base` of the
// buffer the kernel reads (base = 0 for slabs, -win_lo for staged windows).
// Byte-permute plan (FieldPlan::kd_*): for every key byte, the window byte
// it comes from and its mask byte; each key dword's sources are covered by
// dword pairs {w[d+1]:w[d]} of the window, one v_perm_b32 per pair (at most
// four: one per byte).
static void plan_perm(const std::vector<bg_field> &fields, int shift,
                      FieldPlan *p) {
  constexpr int kKeyBytes = 8 * kMaxKeyWords;
  int src[kKeyBytes];
  uint8_t mbyte[kKeyBytes] = {0};
  for (int b = 0; b < kKeyBytes; b++) src[b] = -1;
  for (int i = 0; i < p->nf; i++) {
    const bg_field &f = fields[i];
    for (int j = 0; j < f.size; j++) {
      const int kb = f.pos + j;
      if (kb < 0 || kb >= kKeyBytes) continue;
      src[kb] = f.offset + shift - p->win_lo + j;
      mbyte[kb] = (uint8_t)(p->fmask[i] >> (8 * j));
    }
  }
  int nkd = 0;
  for (int q = 0; q < 2 * kMaxKeyWords; q++) {
    uint32_t dw[4] = {0, 0, 0, 0}, mask = 0;
    uint32_t sel[4] = {kPermZero, kPermZero, kPermZero, kPermZero};
    int nops = 0;
    for (int b = 0; b < 4; b++) {
      const int s = src[4 * q + b];
      mask |= (uint32_t)mbyte[4 * q + b] << (8 * b);
      if (s < 0) continue;
      int op = -1;
      for (int o = 0; o < nops; o++)
        if (s >= (int)dw[o] * 4 && s < (int)dw[o] * 4 + 8) op = o;
      if (op < 0) {
        op = nops++;
        dw[op] = (uint32_t)(s / 4);
      }
      sel[op] = (sel[op] & ~(0xFFu << (8 * b))) |
                ((uint32_t)(s - 4 * (int)dw[op]) << (8 * b));
    }
    if (nops) nkd = q + 1;
    p->kd_nops[q >> 2] |= (uint32_t)nops << (8 * (q & 3));
    p->kd_dw[q] = dw[0] | (dw[1] << 8) | (dw[2] << 16) | (dw[3] << 24);
    for (int o = 0; o < 4; o++) p->kd_sel[o][q] = sel[o];
    p->kd_mask[q] = mask;
  }
  p->nkd = nkd;
}

// The device key of one frame, built on the host exactly as the kernels
// build it (window or direct mode) -- bg_debug_key.
static void host_key(const FieldPlan &p, const uint8_t *frame, int kw,
                     uint64_t *k) {
  for (int j = 0; j < kw; j++) k[j] = 0;
  if (!p.direct) {
    uint32_t w[kMaxWindowChunks * 4 + 2] = {0};
    memcpy(w, frame + p.win_lo, (size_t)p.nch * 16);
    for (int q = 0; q < 2 * kw && q < p.nkd; q++) {
      uint32_t x = 0;
      for (int o = 0; o < kd_nops_of(p, q); o++) {
        const uint32_t d = (p.kd_dw[q] >> (8 * o)) & 0xFF;
        x |= perm_host(w[d + 1], w[d], p.kd_sel[o][q]);
      }
      x &= p.kd_mask[q];
      k[q >> 1] |= (uint64_t)x << (32 * (q & 1));
    }
    return;
  }
  for (int f = 0; f < p.nf; f++) {
    const uint32_t spec = p.fspec[f];
    uint32_t d[3] = {0, 0, 0};
    memcpy(d, frame + 4 * fspec_d(spec), 4 * (size_t)fspec_nd(spec));
    const uint64_t lo = (uint64_t)d[0] | ((uint64_t)d[1] << 32);
    const int sh = fspec_shift_bits(spec);
    const uint64_t v =
        (sh ? ((lo >> sh) | ((uint64_t)d[2] << (64 - sh))) : lo) & p.fmask[f];
    const int pos = fspec_pos(spec), pw = pos >> 3, pb = (pos & 7) * 8;
    if (pw < kw) k[pw] |= v << pb;
    if (pb && pw + 1 < kw) k[pw + 1] |= v >> (64 - pb);
  }
}

FieldPlan make_plan(const std::vector<bg_field> &fields, bool em_masks,
                    int shift) {
  FieldPlan p;
  memset(&p, 0, sizeof(p));
  p.nf = (int)fields.size();
  if (p.nf == 0) return p;
  int lo = 1 << 30, hi = 0;
  for (auto &f : fields) {
    lo = std::min(lo, f.offset + shift);
    hi = std::max(hi, f.offset + shift + f.size);
  }
  p.win_lo = lo & ~15;
  p.nch = (hi - p.win_lo + 15) / 16;
  p.direct = p.nch > kMaxWindowChunks;
  if (p.direct) p.nch = 0;
  for (int i = 0; i < p.nf; i++) {
    const bg_field &f = fields[i];
    const int off = f.offset + shift;
    const int nd = ((off + f.size - 1) >> 2) - (off >> 2) + 1;
    const int d = p.direct ? (off >> 2) : ((off - p.win_lo) >> 2);
    p.fspec[i] = pack_fspec(d, off & 3, f.pos, nd);
    uint64_t size_mask = f.size >= 8 ? ~0ULL : ((1ULL << (8 * f.size)) - 1);
    p.fmask[i] = em_masks ? (f.mask & size_mask) : size_mask;
  }
  if (!p.direct) plan_perm(fields, shift, &p);  // window mode
  return p;
}

// --------------------------------------------------------------------------
// device table
// --------------------------------------------------------------------------
void relayout(TableLayout &L, uint32_t nbp) {
  L.nbp = nbp;
  L.keys_off = align256((uint64_t)nbp * 4);
  if (L.rec) {  // slot records (bg_table.h)
    L.vals_off = L.keys_off + (uint64_t)L.kw * 8;
    L.part_bytes = align256(L.keys_off + (uint64_t)nbp * kSlots * L.rec * 8);
    return;
  }
  L.vals_off = align256(L.keys_off + (uint64_t)nbp * kSlots * L.kw * 8);
  L.part_bytes =
      align256(L.vals_off + (L.vik ? 0 : (uint64_t)nbp * kSlots * L.val_bytes));
}

int DevTable::upload(int dev, const std::vector<uint8_t> &img,
                     const TableLayout &lay, hipStream_t s) {
  int r = set_device(dev);
  if (r) return r;
  if (d_image && owned && (device != dev || bytes < img.size())) {
    (void)hipFree(d_image);
    d_image = nullptr;
  }
  if (!d_image || !owned) {
    d_image = nullptr;
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_image),
                      std::max<size_t>(img.size(), 256)));
    owned = true;
  }
  HIP_TRY(hipMemcpyAsync(d_image, img.data(), img.size(),
                         hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  device = dev;
  bytes = img.size();
  L = lay;
  valid = true;
  return 0;
}

void DevTable::release() {
  if (d_image && owned) {
    int cur = 0;
    (void)hipGetDevice(&cur);
    (void)hipSetDevice(device);
    (void)hipFree(d_image);
    (void)hipSetDevice(cur);
  }
  d_image = nullptr;
  valid = false;
}

TableRef table_ref(const uint8_t *base, uint64_t bytes, const TableLayout &L,
                   uint64_t filt_off, uint32_t filt_words, bool tags_lds,
                   uint64_t aux_off) {
  TableRef t;
  memset(&t, 0, sizeof(t));
  t.base = base;
  t.part_bytes = L.part_bytes;
  t.keys_off = L.keys_off;
  t.vals_off = L.vals_off;
  t.seed = L.seed;
  t.nparts = L.nparts;
  t.nbp = L.nbp;
  t.kw = L.kw;
  const uint64_t tb = filt_words ? filt_off : aux_off ? aux_off : bytes;
  t.bytes_total = (uint32_t)std::min<uint64_t>(tb, 0xFFFFFFFFu);
  t.filt_words = filt_words;
  t.vik = L.vik;
  t.filt_off = filt_off;
  t.rec = L.rec;
  t.lds = tb <= kLdsTableMax ? kLdsTable
          : tags_lds       ? kLdsTags
          : filt_words     ? kLdsFilter
                           : kLdsNone;
  return t;
}

TableRef DevTable::ref() const {
  return table_ref(d_image, bytes, L, filt_off, filt_words, tags_lds, aux_off);
}

// Build a full single-device image (all partitions) from flat entries.
int build_image(uint32_t kw, uint32_t val_bytes, uint32_t nparts,
                const std::vector<uint64_t> &keys,
                const std::vector<uint8_t> &vals,
                const std::vector<uint64_t> &hashes, std::vector<uint8_t> *img,
                TableLayout *out_layout, double max_load, bool vik,
                uint32_t probe) {
  const size_t n = hashes.size();
  // count entries per partition to size the layout
  std::vector<std::vector<size_t>> members(nparts);
  for (size_t i = 0; i < n; i++)
    members[probe ? 0 : split_hash(hashes[i], nparts, 2).part].push_back(i);
  size_t maxc = 0;
  for (auto &m : members) maxc = std::max(maxc, m.size());
  TableLayout L = plan_layout(maxc, kw, val_bytes, nparts, kDefaultSeed, max_load, vik);
  L.probe = probe;
  // WildcardMatch (probe 1): key and value in one record per slot (a check
  // is one L2 request, not two); the bucket count the load asks for, not
  // the next power of two (wm_probe takes any count)
  if (probe) L.rec = val_bytes == 8 && !vik ? wm_rec_words(kw) : 0u;
  if (probe)
    relayout(L, std::max<uint32_t>(2, (uint32_t)((double)maxc / (kSlots * max_load)) + 1));
  for (int attempt = 0; attempt < 8; attempt++) {
    img->assign((size_t)L.part_bytes * nparts, 0);
    bool ok = true;
    for (uint32_t p = 0; p < nparts && ok; p++) {
      std::vector<uint64_t> pk, ps;
      std::vector<uint8_t> pv;
      for (size_t i : members[p]) {
        pk.insert(pk.end(), &keys[i * kw], &keys[i * kw] + kw);
        pv.insert(pv.end(), &vals[i * val_bytes], &vals[i * val_bytes] + val_bytes);
        ps.push_back(hashes[i]);
      }
      ok = build_partition(L, p, members[p].size(), pk.data(), pv.data(),
                           ps.data(), img->data() + (size_t)p * L.part_bytes);
    }
    if (ok) {
      *out_layout = L;
      return 0;
    }
    if (L.nbp >= kMaxBucketsPerPart) break;
    relayout(L, probe ? L.nbp + L.nbp / 8 + 1 : L.nbp * 2);
  }
  return fail(ENOSPC, "flow table build failed (%zu entries)", n);
}

// --------------------------------------------------------------------------
// host staging (pinned) + device scratch, grown on demand
// --------------------------------------------------------------------------
int Staging::ensure(int dev, size_t in_bytes, size_t out_bytes) {
  if (device != dev) {
    release();
    device = dev;
  }
  if (in_bytes > in_cap) {
    if (h_in) (void)hipHostFree(h_in);
    if (d_in) (void)hipFree(d_in);
    h_in = nullptr;
    d_in = nullptr;
    in_cap = std::max<size_t>(in_bytes, 1 << 16);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h_in), in_cap,
                          hipHostMallocDefault));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_in), in_cap));
  }
  if (out_bytes > out_cap) {
    if (h_out) (void)hipHostFree(h_out);
    if (d_out) (void)hipFree(d_out);
    h_out = nullptr;
    d_out = nullptr;
    out_cap = std::max<size_t>(out_bytes, 1 << 12);
    HIP_TRY(hipHostMalloc(reinterpret_cast<void **>(&h_out), out_cap,
                          hipHostMallocDefault));
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&d_out), out_cap));
  }
  return 0;
}

namespace {
struct ThreadStage {
  Staging st;
  hipStream_t streams[16] = {};
};
thread_local ThreadStage t_stage;
}  // namespace

Staging &thread_staging() { return t_stage.st; }

hipStream_t thread_stream(int device, hipStream_t given) {
  if (given) return given;
  if (device < 0 || device >= 16) return nullptr;
  hipStream_t &s = t_stage.streams[device];
  if (!s) {
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess)
      s = nullptr;  // fall back to the legacy stream
    else
      own_stream(s);  // (lives as long as the thread; never destroyed)
  }
  return s;
}

void Staging::release() {
  if (h_in) (void)hipHostFree(h_in);
  if (d_in) (void)hipFree(d_in);
  if (h_out) (void)hipHostFree(h_out);
  if (d_out) (void)hipFree(d_out);
  h_in = d_in = h_out = d_out = nullptr;
  in_cap = out_cap = 0;
}

}  // namespace bg

using namespace bg;

// ============================================================================
// ExactMatch
// ============================================================================
// one device's image of one rule-set version
struct EmImage : DevImage {
  TableRef t{};
};

struct bg_em {
  std::vector<bg_field> fields;
  bool has_attr = false;  // metadata-attribute fields (P15)
  // fields as the device reads them: attr fields resolved to slot offsets
  // by bg_em_bind_meta (meta_bound), otherwise = fields
  std::vector<bg_field> dfields;
  bool meta_bound = false;
  // attr_offset() of each attribute (bind_meta): where staged rows (pipes,
  // host paths) take each packet's attr field bytes from
  std::vector<int32_t> attr_offs;
  bool attrs_known = false;
  uint32_t key_size = 0;  // total_key_size_
  uint32_t raw_size = 0;  // raw_key_size_ (sum of field sizes)
  uint32_t kw = 1;        // device key words (1, 2, 4, 8)
  std::unordered_map<Key, uint16_t, KeyHash> rules;
  // Rule changes (THREAD_UNSAFE commands, workers paused) bump the version;
  // a device's image is rebuilt into a fresh allocation at the next launch
  // there, and the one it replaces is retired behind fences (bg_image.h).
  std::atomic<uint64_t> version{1};
  std::vector<uint8_t> host_img;  // the image of host_version (all devices)
  TableLayout host_L{};
  uint64_t host_version = 0;
  Published<EmImage> dev;  // per device
  TableLayout planned;  // sharded build
  bool planned_valid = false;
  std::mutex mu;  // serialises sync (lookups from many workers never lock)
};

static void em_changed(bg_em *em) { em->version.fetch_add(1, std::memory_order_acq_rel); }

static Key em_key(const bg_em *em, const uint8_t *key) {
  Key k;
  memset(&k, 0, sizeof(k));
  memcpy(k.w, key, em->key_size);
  return k;
}

static int check_fields(const bg_field *fields, int nfields) {
  if (nfields < 0 || nfields > BG_MAX_FIELDS)
    return fail(EINVAL, "nfields %d not in [0,%d]", nfields, BG_MAX_FIELDS);
  int acc = 0;
  for (int i = 0; i < nfields; i++) {
    const bg_field &f = fields[i];
    if (f.size < 1 || f.size > 8)
      return fail(EINVAL, "idx %d: 'size' must be in [1,8]", i);
    if (f.attr_id < 0 && (f.offset < 0 || f.offset > 1024))
      return fail(EINVAL, "idx %d: invalid 'offset'", i);
    if (f.pos != acc)
      return fail(EINVAL, "idx %d: pos %d != %d", i, f.pos, acc);
    acc += f.size;
  }
  return 0;
}

extern "C" {

const char *bg_version(void) { return "bessgpu 0.1 (gfx950)"; }
const char *bg_last_error(void) { return bg::g_err.c_str(); }

int bg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int bg_malloc(int device, size_t bytes, void **d_ptr) {
  int r = set_device(device);
  if (r) return r;
  HIP_TRY(hipMalloc(d_ptr, std::max<size_t>(bytes, 1)));
  return 0;
}
int bg_free(void *d_ptr) {
  HIP_TRY(hipFree(d_ptr));
  return 0;
}
int bg_memcpy_h2d(void *d_dst, const void *src, size_t bytes, bg_stream_t s) {
  HIP_TRY(hipMemcpyAsync(d_dst, src, bytes, hipMemcpyHostToDevice,
                         (hipStream_t)s));
  return 0;
}
int bg_memcpy_d2h(void *dst, const void *d_src, size_t bytes, bg_stream_t s) {
  HIP_TRY(hipMemcpyAsync(dst, d_src, bytes, hipMemcpyDeviceToHost,
                         (hipStream_t)s));
  return 0;
}
int bg_stream_sync(bg_stream_t s) {
  HIP_TRY(hipStreamSynchronize((hipStream_t)s));
  return 0;
}

int bg_em_create(const bg_field *fields, int nfields, bg_em **out) {
  int r = check_fields(fields, nfields);
  if (r) return r;
  bg_em *em = new bg_em();
  em->fields.assign(fields, fields + nfields);
  em->dfields = em->fields;
  for (int i = 0; i < nfields; i++) em->has_attr |= fields[i].attr_id >= 0;
  int acc = 0;
  for (int i = 0; i < nfields; i++) acc += fields[i].size;
  em->raw_size = (uint32_t)acc;
  em->key_size = (uint32_t)((acc + 7) / 8 * 8);
  em->kw = round_kw(em->key_size);
  *out = em;
  return 0;
}

void bg_em_destroy(bg_em *em) {
  if (!em) return;
  em->dev.release();  // retired behind the fences of its launches
  delete em;
}

size_t bg_em_key_size(const bg_em *em) { return em->key_size; }

int bg_em_add(bg_em *em, const uint8_t *key, uint16_t gate) {
  if (em->key_size == 0) return fail(EINVAL, "rule has no fields");
  em->rules[em_key(em, key)] = gate;
  em_changed(em);
  return 0;
}

int bg_em_delete(bg_em *em, const uint8_t *key) {
  if (em->key_size == 0) return fail(EINVAL, "rule has no fields");
  if (em->rules.erase(em_key(em, key)) == 0)
    return fail(ENOENT, "rule doesn't exist");
  em_changed(em);
  return 0;
}

void bg_em_clear(bg_em *em) {
  em->rules.clear();
  em_changed(em);
}

size_t bg_em_count(const bg_em *em) { return em->rules.size(); }

int bg_em_iter(const bg_em *em, size_t *cursor, uint8_t *key_out,
               uint16_t *gate_out) {
  // unordered_map iteration by position: O(n) per call is avoided by the
  // module layer, which snapshots once; here we walk from the start.
  size_t i = 0;
  for (auto &kv : em->rules) {
    if (i++ == *cursor) {
      memcpy(key_out, kv.first.w, em->key_size);
      *gate_out = kv.second;
      (*cursor)++;
      return 1;
    }
  }
  return 0;
}

static void em_entries(const bg_em *em, std::vector<uint64_t> *keys,
                       std::vector<uint8_t> *vals, std::vector<uint64_t> *seeds) {
  keys->clear();
  vals->clear();
  seeds->clear();
  keys->reserve(em->rules.size() * em->kw);
  for (auto &kv : em->rules) {
    keys->insert(keys->end(), kv.first.w, kv.first.w + em->kw);
    vals->push_back((uint8_t)kv.second);
    vals->push_back((uint8_t)(kv.second >> 8));
    seeds->push_back(hash_words(kv.first.w, (int)em->kw, kDefaultSeed));
  }
}

// the gate fits in the key's unused top bytes (value in the key)
static bool em_vik(const bg_em *em) {
  return em->raw_size + 2 <= em->kw * 8;
}

// the device's image if it is of the current rule-set version
static EmImage *em_fresh(bg_em *em, int device) {
  EmImage *v = em->dev.get(device);
  return v && v->version == em->version.load(std::memory_order_acquire) ? v : nullptr;
}

static int em_sync_locked(bg_em *em, int device, hipStream_t s) {
  if (em_fresh(em, device)) return 0;
  const uint64_t ver = em->version.load(std::memory_order_acquire);
  if (em->host_version != ver) {  // once per version, for every device
    std::vector<uint64_t> keys, seeds;
    std::vector<uint8_t> vals;
    em_entries(em, &keys, &vals, &seeds);
    TableLayout L;
    int r = build_image(em->kw, 2, 1, keys, vals, seeds, &em->host_img, &L, 0.75,
                        em_vik(em));
    if (r) return r;
    em->host_L = L;
    em->host_version = ver;
  }
  std::unique_ptr<EmImage> img(new EmImage());
  int r = upload_image(img.get(), device, em->host_img.data(), em->host_img.size(), s);
  if (r) return r;
  img->version = ver;
  img->t = table_ref(img->d, img->bytes, em->host_L, 0, 0, false, 0);
  em->dev.publish(device, img.release());
  return 0;
}

// The image launches on `device` read, rebuilt first if the rules changed
// (lock-free when it is current: the per-batch calls of many workers).
static int em_image(bg_em *em, int device, hipStream_t s, EmImage **out) {
  EmImage *v = em_fresh(em, device);
  if (!v) {
    std::lock_guard<std::mutex> lk(em->mu);
    if (int r = em_sync_locked(em, device, s)) return r;
    v = em->dev.get(device);
  }
  *out = v;
  return 0;
}

int bg_em_sync(bg_em *em, int device, bg_stream_t stream) {
  EmImage *img;
  return em_image(em, device, (hipStream_t)stream, &img);
}

static int em_launch(const std::vector<bg_field> &df, EmImage *img, const void *d_frames,
                     size_t stride,
                     size_t n, uint16_t default_gate, uint16_t *d_gates, int shift,
                     hipStream_t s) {
  EmArgs a;
  memset(&a, 0, sizeof(a));
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.gates = d_gates;
  a.default_gate = default_gate;
  a.fp = make_plan(df, true, shift);
  a.t = img->t;
  img->used_on(s);
  HIP_TRY(launch_em(a, num_cus(img->device), s));
  img->launched_on(s);
  return 0;
}

// the calling thread's current HIP device (classify calls run there)
static int current_device() {
  int d = 0;
  (void)hipGetDevice(&d);
  return d;
}

// Every byte a classify kernel reads for packet i lies in its slot, so the
// last packet's reads stay inside the slab: the staged window
// [win_lo, win_lo + 16 * nch), or in direct mode each field's dwords.
static int check_extent(const std::vector<bg_field> &fields, int shift,
                        size_t stride) {
  if (fields.empty()) return 0;
  const FieldPlan p = make_plan(fields, false, shift);
  int hi = 0;
  if (!p.direct) {
    hi = p.win_lo + 16 * p.nch;
  } else {
    for (int i = 0; i < p.nf; i++)
      hi = std::max(hi, (fspec_d(p.fspec[i]) + fspec_nd(p.fspec[i])) * 4);
  }
  if (hi > (int)stride || p.win_lo < 0)
    return fail(EINVAL, "fields read bytes up to %d, past the %zu-byte slot", hi,
                stride);
  return 0;
}

static int no_attr_datapath() {
  return fail(ENOTSUP, "metadata-attribute (attr_name) fields need the "
              "packets' metadata in the slot: bind its layout first "
              "(bg_em_bind_meta / bg_wm_bind_meta); host staging does not "
              "carry metadata");
}

// P15: attr fields read the packet's metadata area at the attribute's
// metadata offset (exact_match.cc:230-236 ptr_attr; wildcard_match.cc:
// 177-195 mt_offset_to_databuf_offset). The device slot carries the
// metadata area at meta_off, so an attr field becomes an offset field at
// meta_off + attr_offsets[attr_id].
static int resolve_attrs(const std::vector<bg_field> &fields, int meta_off,
                         const std::vector<int32_t> &offs, std::vector<bg_field> *out) {
  std::vector<bg_field> d = fields;
  for (auto &f : d) {
    if (f.attr_id < 0) continue;
    f.offset = meta_off + offs[f.attr_id];
    f.attr_id = -1;
  }
  out->swap(d);
  return 0;
}

// bg_*_bind_meta: the attribute offsets (kept for staged rows) and, with
// meta_off >= 0, the device slab's fields; meta_off -1: offsets only
static int bind_meta(const std::vector<bg_field> &fields, int meta_off,
                     const int32_t *attr_offsets, int nattrs,
                     std::vector<int32_t> *offs, std::vector<bg_field> *out,
                     bool *slab_bound) {
  if (meta_off < -1 || meta_off > 2048)
    return fail(EINVAL, "meta_off %d not in [-1,2048]", meta_off);
  if (nattrs < 0 || nattrs > 64) return fail(EINVAL, "nattrs %d", nattrs);
  std::vector<int32_t> o(attr_offsets ? attr_offsets : nullptr,
                         attr_offsets ? attr_offsets + nattrs : nullptr);
  for (auto &f : fields) {
    if (f.attr_id < 0) continue;
    if (f.attr_id >= nattrs || o[f.attr_id] < 0)
      return fail(EINVAL, "attribute %d has no metadata offset", f.attr_id);
    // (SNBUF_METADATA: a 128-byte area the attribute lies in)
    if (o[f.attr_id] + f.size > 128)
      return fail(EINVAL, "attribute %d at metadata offset %d: past the 128-byte area",
                  f.attr_id, o[f.attr_id]);
    if (meta_off >= 0 && meta_off + o[f.attr_id] + 8 > 2048)  // inside 2 KB
      return fail(EINVAL, "metadata field at slot offset %d: past 2040",
                  meta_off + o[f.attr_id]);
  }
  if (meta_off >= 0) {
    resolve_attrs(fields, meta_off, o, out);
    *slab_bound = true;
  } else {  // offsets only: the device-slab calls stay unbound until bound
    out->clear();
    *slab_bound = false;
  }
  offs->swap(o);
  return 0;
}

// The metadata bytes [lo, hi) the attr fields read (hi == lo: none)
static int meta_window(const std::vector<bg_field> &fields, bool has_attr, bool known,
                       const std::vector<int32_t> &offs, int *lo, int *hi) {
  *lo = *hi = 0;
  if (!has_attr) return 0;
  if (!known)
    return fail(ENOTSUP, "metadata-attribute (attr_name) fields: the attribute "
                "offsets are not bound yet (bg_module_bind_meta)");
  int l = 1 << 30, h = 0;
  for (auto &f : fields) {
    if (f.attr_id < 0) continue;
    l = std::min(l, offs[f.attr_id]);
    h = std::max(h, offs[f.attr_id] + f.size);
  }
  *lo = l;
  *hi = h;
  return 0;
}

}  // extern "C"

// The fields a launch reads, in frame coordinates: the device slab's
// (meta_row == kSlabMeta: attr fields at the bound meta_off) or a staged
// row's (byte 0 = frame byte win_off; metadata byte 0 at row offset
// meta_row, i.e. frame coordinate win_off + meta_row)
static int em_fields_for(const bg_em *em, int win_off, int meta_row,
                         std::vector<bg_field> *out) {
  if (!em->has_attr) {
    *out = em->fields;
    return 0;
  }
  if (meta_row == bg::kSlabMeta) {
    if (!em->meta_bound) return no_attr_datapath();
    *out = em->dfields;
    return 0;
  }
  if (!em->attrs_known) return no_attr_datapath();
  return resolve_attrs(em->fields, win_off + meta_row, em->attr_offs, out);
}

namespace bg {
// The device plan of a table for launches outside this file (the persistent
// ring, bg_ring.cc): table synced to `device`, field plan of the slot layout.
uint64_t em_version(const bg_em *em) { return em->version.load(std::memory_order_acquire); }

int em_device_plan(bg_em *em, int device, hipStream_t s, int win_off, int meta_row,
                   FieldPlan *fp, TableRef *t, int *read_end, uint64_t *version) {
  std::vector<bg_field> df;
  if (int r = em_fields_for(em, win_off, meta_row, &df)) return r;
  if (win_off < 0 || win_off > 1024) return fail(EINVAL, "win_off %d", win_off);
  if (int r = check_extent(df, -win_off, 0xFFFF)) return r;
  EmImage *img;
  if (int r = em_image(em, device, s, &img)) return r;
  *version = img->version;
  *fp = make_plan(df, true, -win_off);
  *t = img->t;
  int hi = 0;  // bytes of a slot the kernel reads (check_extent)
  if (!fp->direct) {
    hi = fp->nf ? fp->win_lo + 16 * fp->nch : 0;
  } else {
    for (int i = 0; i < fp->nf; i++)
      hi = std::max(hi, (fspec_d(fp->fspec[i]) + fspec_nd(fp->fspec[i])) * 4);
  }
  *read_end = hi;
  return 0;
}

int em_meta_window(const bg_em *em, int *lo, int *hi) {
  return meta_window(em->fields, em->has_attr, em->attrs_known, em->attr_offs, lo, hi);
}
}  // namespace bg

extern "C" {

int bg_em_bind_meta(bg_em *em, int meta_off, const int32_t *attr_offsets,
                    int nattrs) {
  std::lock_guard<std::mutex> lk(em->mu);
  int r = bind_meta(em->fields, meta_off, attr_offsets, nattrs, &em->attr_offs,
                    &em->dfields, &em->meta_bound);
  if (r) return r;
  em->attrs_known = true;
  // what was derived from the old offsets (a pipe's ring and its field
  // plan, PipeRingCurrent) is keyed on the version: a new layout is a new
  // version, even one whose metadata window [mlo, mhi) did not move
  em_changed(em);
  return 0;
}

int bg_em_classify(bg_em *em, const void *d_frames, size_t stride, size_t n,
                   uint16_t default_gate, uint16_t *d_gates,
                   bg_stream_t stream) {
  return bg_em_classify_window(em, d_frames, stride, n, 0, default_gate,
                               d_gates, stream);
}

int bg_em_classify_window(bg_em *em, const void *d_frames, size_t stride,
                          size_t n, int win_off, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream) {
  return bg_em_classify_staged(em, d_frames, stride, n, win_off, bg::kSlabMeta,
                               default_gate, d_gates, stream);
}

int bg_em_classify_staged(bg_em *em, const void *d_win, size_t stride, size_t n,
                          int win_off, int meta_row, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream) {
  if (win_off < 0 || win_off > 1024) return fail(EINVAL, "win_off %d", win_off);
  if (stride % 16 || ((uintptr_t)d_win & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned with stride %% 16 == 0");
  std::vector<bg_field> df;
  if (int r = em_fields_for(em, win_off, meta_row, &df)) return r;
  if (int r = check_extent(df, -win_off, stride)) return r;
  hipStream_t s = (hipStream_t)stream;
  const int dev = current_device();
  EmImage *img;
  if (int r = em_image(em, dev, s, &img)) return r;
  return em_launch(df, img, d_win, stride, n, default_gate, d_gates, -win_off, s);
}

int bg_em_meta_window(const bg_em *em, int *lo, int *hi) {
  return bg::em_meta_window(em, lo, hi);
}

// Stage [lo, hi) of every head (window covering all fields) at a fixed
// 16-byte-multiple stride, then classify on the device.
static int stage_windows(const std::vector<bg_field> &fields,
                         const uint8_t *const *heads, size_t n, Staging &st,
                         int dev, int *shift, size_t *wstride) {
  // +64 B: the last window's 16-byte loads may run past its slot
  int lo = 1 << 30, hi = 0;
  for (auto &f : fields) {
    lo = std::min(lo, f.offset);
    hi = std::max(hi, f.offset + f.size);
  }
  if (fields.empty()) lo = hi = 0;
  const size_t w = std::max<size_t>(16, (size_t)(hi - lo + 15) / 16 * 16);
  int r = st.ensure(dev, n * w + 64, n * 2);
  if (r) return r;
  for (size_t i = 0; i < n; i++)
    memcpy(st.h_in + i * w, heads[i] + lo, (size_t)(hi - lo));
  *shift = -lo;
  *wstride = w;
  return 0;
}

// Many workers may call this on one table at once (core/module.h:485,
// exact_match.h:55): each calling thread stages into its own pinned buffers
// and, unless it passes a stream, runs on its own HIP stream; the table lock
// is taken only when the device image must be (re)built.
int bg_em_process_host(bg_em *em, const uint8_t *const *heads, size_t n,
                       uint16_t default_gate, uint16_t *gates,
                       bg_stream_t stream) {
  if (em->has_attr) return no_attr_datapath();
  if (n == 0) return 0;
  const int dev = current_device();
  hipStream_t s = thread_stream(dev, (hipStream_t)stream);
  EmImage *img;
  int r = em_image(em, dev, s, &img);
  if (r) return r;
  Staging &st = thread_staging();
  int shift;
  size_t w;
  r = stage_windows(em->fields, heads, n, st, dev, &shift, &w);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.d_in, st.h_in, n * w, hipMemcpyHostToDevice, s));
  r = em_launch(em->fields, img, st.d_in, w, n, default_gate,
                reinterpret_cast<uint16_t *>(st.d_out), shift, s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.h_out, st.d_out, n * 2, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  memcpy(gates, st.h_out, n * 2);
  return 0;
}

// the frame bytes the offset fields cover (attr fields read the metadata
// area instead: bg_em_meta_window)
static void fields_window(const std::vector<bg_field> &fields, int *lo,
                          int *hi) {
  int l = 1 << 30, h = 0;
  for (auto &f : fields) {
    if (f.attr_id >= 0) continue;
    l = std::min(l, f.offset);
    h = std::max(h, f.offset + f.size);
  }
  if (h == 0) l = h = 0;
  *lo = l;
  *hi = h;
}

void bg_em_window(const bg_em *em, int *lo, int *hi) {
  fields_window(em->fields, lo, hi);
}

static int check_nparts(int nparts) {
  if (nparts < 1 || nparts > 8 || (nparts & (nparts - 1)))
    return fail(EINVAL, "nparts must be 1, 2, 4 or 8");
  return 0;
}

static uint32_t key_part(const bg_em *em, const uint64_t *w, int nparts) {
  return split_hash(hash_words(w, (int)em->kw, kDefaultSeed), (uint32_t)nparts, 2).part;
}

int bg_em_add_many(bg_em *em, const uint8_t *keys, size_t n, size_t key_stride,
                   const uint16_t *gates, int part, int nparts) {
  if (em->key_size == 0) return fail(EINVAL, "rule has no fields");
  if (part >= 0) {
    if (int r = check_nparts(nparts)) return r;
    if (part >= nparts) return fail(EINVAL, "part %d out of range", part);
  }
  em->rules.reserve(em->rules.size() + n);
  for (size_t i = 0; i < n; i++) {
    const Key k = em_key(em, keys + i * key_stride);
    if (part >= 0 && key_part(em, k.w, nparts) != (uint32_t)part) continue;
    em->rules[k] = gates[i];
  }
  em_changed(em);
  return 0;
}

int bg_em_plan(bg_em *em, int nparts, uint64_t *part_bytes) {
  if (int r = check_nparts(nparts)) return r;
  std::vector<size_t> cnt(nparts, 0);
  for (auto &kv : em->rules) cnt[key_part(em, kv.first.w, nparts)]++;
  size_t maxc = *std::max_element(cnt.begin(), cnt.end());
  return bg_em_plan_count(em, nparts, maxc, part_bytes);
}

int bg_em_part_count(const bg_em *em, int part, int nparts, uint64_t *count) {
  if (int r = check_nparts(nparts)) return r;
  uint64_t c = 0;
  for (auto &kv : em->rules) c += key_part(em, kv.first.w, nparts) == (uint32_t)part;
  *count = c;
  return 0;
}

int bg_em_plan_count(bg_em *em, int nparts, uint64_t max_part_entries,
                     uint64_t *part_bytes) {
  if (int r = check_nparts(nparts)) return r;
  em->planned = plan_layout(max_part_entries, em->kw, 2, (uint32_t)nparts,
                            kDefaultSeed, 0.75, em_vik(em));
  em->planned_valid = true;
  *part_bytes = em->planned.part_bytes;
  return 0;
}

// The partition's entries in (hash, key) order: the image depends only on
// the rule set, not on how (or on which rank) the rules were inserted.
int bg_em_build_part(bg_em *em, int part, void *host_dst) {
  if (!em->planned_valid) return fail(EINVAL, "bg_em_plan first");
  const TableLayout &L = em->planned;
  if (part < 0 || (uint32_t)part >= L.nparts)
    return fail(EINVAL, "part %d out of range", part);
  struct Ent {
    uint64_t h;
    const Key *k;
    uint16_t g;
  };
  std::vector<Ent> ents;
  for (auto &kv : em->rules) {
    uint64_t h = hash_words(kv.first.w, (int)em->kw, kDefaultSeed);
    if (split_hash(h, L.nparts, L.nbp).part != (uint32_t)part) continue;
    ents.push_back(Ent{h, &kv.first, kv.second});
  }
  std::sort(ents.begin(), ents.end(), [&](const Ent &a, const Ent &b) {
    if (a.h != b.h) return a.h < b.h;
    return memcmp(a.k->w, b.k->w, sizeof(a.k->w)) < 0;
  });
  std::vector<uint64_t> keys, seeds;
  std::vector<uint8_t> vals;
  keys.reserve(ents.size() * em->kw);
  for (const Ent &e : ents) {
    keys.insert(keys.end(), e.k->w, e.k->w + em->kw);
    vals.push_back((uint8_t)e.g);
    vals.push_back((uint8_t)(e.g >> 8));
    seeds.push_back(e.h);
  }
  if (!build_partition(L, (uint32_t)part, seeds.size(), keys.data(),
                       vals.data(), seeds.data(),
                       static_cast<uint8_t *>(host_dst)))
    return fail(ENOSPC, "partition %d build failed (%zu entries)", part,
                seeds.size());
  return 0;
}

// The assembled image becomes the device's image of the current rule set
// (the caller keeps the memory; a later rule change rebuilds from the rules
// this handle holds).
int bg_em_attach(bg_em *em, int device, const void *d_image) {
  if (!em->planned_valid) return fail(EINVAL, "bg_em_plan first");
  if (device < 0 || device >= kMaxDevices) return fail(ENODEV, "device %d", device);
  std::lock_guard<std::mutex> lk(em->mu);
  EmImage *img = new EmImage();
  img->device = device;
  img->d = static_cast<uint8_t *>(const_cast<void *>(d_image));
  img->owned = false;
  img->bytes = em->planned.part_bytes * em->planned.nparts;
  img->version = em->version.load(std::memory_order_acquire);
  img->t = table_ref(img->d, img->bytes, em->planned, 0, 0, false, 0);
  em->dev.publish(device, img);
  return 0;
}

}  // extern "C"

namespace bg {
int em_publish_owned(bg_em *em, int device, uint8_t *d_img, uint64_t bytes) {
  if (!em->planned_valid || device < 0 || device >= kMaxDevices) {
    DevImage tmp;  // frees d_img
    tmp.device = device;
    tmp.d = d_img;
    return fail(EINVAL, "no planned layout / bad device %d", device);
  }
  std::lock_guard<std::mutex> lk(em->mu);
  EmImage *img = new EmImage();
  img->device = device;
  img->d = d_img;
  img->owned = true;
  img->bytes = bytes;
  img->version = em->version.load(std::memory_order_acquire);
  img->t = table_ref(img->d, img->bytes, em->planned, 0, 0, false, 0);
  em->dev.publish(device, img);
  return 0;
}
}  // namespace bg

extern "C" {

int bg_em_table_info(const bg_em *em, uint64_t *bytes, int *in_lds) {
  const EmImage *img = const_cast<bg_em *>(em)->dev.get(current_device());
  if (!img) return fail(EINVAL, "no device table yet");
  *bytes = img->bytes;
  *in_lds = img->t.lds ? 1 : 0;
  return 0;
}

}  // extern "C"

// ============================================================================
// WildcardMatch
// ============================================================================
struct WmTupleH {
  Key mask;
  std::unordered_map<Key, WmVal, KeyHash> ht;
};

// one device's image of one rule-set version, with the launch arguments
// that go with it (tuple masks, seeds, direct tuples)
struct WmImage : DevImage {
  WmArgs a{};
  bool no_tags = false;  // BG_PATH_WM_NO_TAGS when it was built
  // the kernels compiled at run time for this image's shape (bg_wm_jit.cc;
  // shared with every image of the same shape), or null
  std::shared_ptr<WmJit> jit;
};

struct bg_wm {
  std::vector<bg_field> fields;
  bool has_attr = false;
  std::vector<bg_field> dfields;  // as in bg_em
  bool meta_bound = false;
  std::vector<int32_t> attr_offs;  // as in bg_em
  bool attrs_known = false;
  uint32_t key_size = 0;
  uint32_t kw = 1;
  std::vector<WmTupleH> tuples;
  std::atomic<uint64_t> version{1};  // as bg_em::version
  // the host image of (host_version, host_no_tags) and its launch arguments
  std::vector<uint8_t> host_img;
  WmArgs host_a{};
  uint64_t host_version = 0;
  bool host_no_tags = false;
  Published<WmImage> dev;
  // direct tuples of the image being built (WmArgs::ndirect ...)
  uint32_t ndirect = 0;
  uint32_t dtu[kMaxDirect] = {}, dspec[kMaxDirect] = {};
  uint64_t doff[kMaxDirect] = {};
  std::mutex mu;
};

static void wm_changed(bg_wm *wm) { wm->version.fetch_add(1, std::memory_order_acq_rel); }

static Key wm_key(const bg_wm *wm, const uint8_t *p) {
  Key k;
  memset(&k, 0, sizeof(k));
  memcpy(k.w, p, wm->key_size);
  return k;
}

static int wm_fields_for(const bg_wm *wm, int win_off, int meta_row,
                         std::vector<bg_field> *out) {  // as em_fields_for
  if (!wm->has_attr) {
    *out = wm->fields;
    return 0;
  }
  if (meta_row == bg::kSlabMeta) {
    if (!wm->meta_bound) return no_attr_datapath();
    *out = wm->dfields;
    return 0;
  }
  if (!wm->attrs_known) return no_attr_datapath();
  return resolve_attrs(wm->fields, win_off + meta_row, wm->attr_offs, out);
}

static int wm_find_tuple(const bg_wm *wm, const Key &mask) {
  for (size_t i = 0; i < wm->tuples.size(); i++)
    if (memcmp(wm->tuples[i].mask.w, mask.w, wm->key_size) == 0) return (int)i;
  return -ENOENT;
}

extern "C" {

int bg_wm_create(const bg_field *fields, int nfields, bg_wm **out) {
  int acc = 0;
  for (int i = 0; i < nfields; i++) acc += fields[i].size;
  if (acc > BG_KEY_BYTES) return fail(EINVAL, "key larger than 64 bytes");
  if (nfields > BG_MAX_FIELDS) {
    // the reference takes any number of fields whose sizes fit the key;
    // the device plan handles up to 8
    return fail(EINVAL, "more than %d fields", BG_MAX_FIELDS);
  }
  int r = check_fields(fields, nfields);
  if (r) return r;
  bg_wm *wm = new bg_wm();
  wm->fields.assign(fields, fields + nfields);
  wm->dfields = wm->fields;
  for (int i = 0; i < nfields; i++) wm->has_attr |= fields[i].attr_id >= 0;
  wm->key_size = (uint32_t)((acc + 7) / 8 * 8);
  wm->kw = round_kw(wm->key_size);
  *out = wm;
  return 0;
}

void bg_wm_destroy(bg_wm *wm) {
  if (!wm) return;
  wm->dev.release();  // retired behind the fences of its launches
  delete wm;
}

size_t bg_wm_key_size(const bg_wm *wm) { return wm->key_size; }

int bg_wm_add(bg_wm *wm, const uint8_t *key, const uint8_t *mask,
              int32_t priority, uint16_t gate) {
  Key m = wm_key(wm, mask);
  int idx = wm_find_tuple(wm, m);
  if (idx < 0) {
    if (wm->tuples.size() >= BG_MAX_TUPLES)
      return fail(ENOSPC, "failed to add a new wildcard pattern");
    wm->tuples.emplace_back();
    wm->tuples.back().mask = m;
    idx = (int)wm->tuples.size() - 1;
  }
  wm->tuples[idx].ht[wm_key(wm, key)] = WmVal{priority, gate};
  wm_changed(wm);
  return 0;
}

int bg_wm_delete(bg_wm *wm, const uint8_t *key, const uint8_t *mask) {
  Key m = wm_key(wm, mask);
  int idx = wm_find_tuple(wm, m);
  if (idx < 0) return fail(ENOENT, "failed to delete a rule");
  WmTupleH &t = wm->tuples[idx];
  if (t.ht.erase(wm_key(wm, key)) == 0 && t.ht.empty())
    wm->tuples.erase(wm->tuples.begin() + idx);  // DelEntry quirk (P6)
  wm_changed(wm);
  return 0;
}

void bg_wm_clear(bg_wm *wm) {
  for (auto &t : wm->tuples) t.ht.clear();
  wm_changed(wm);
}

int bg_wm_num_tuples(const bg_wm *wm) { return (int)wm->tuples.size(); }

int bg_wm_tuple_mask(const bg_wm *wm, int t, uint8_t *mask_out) {
  if (t < 0 || (size_t)t >= wm->tuples.size()) return fail(EINVAL, "bad tuple");
  memset(mask_out, 0, BG_KEY_BYTES);
  memcpy(mask_out, wm->tuples[t].mask.w, wm->key_size);
  return 0;
}

size_t bg_wm_tuple_count(const bg_wm *wm, int t) {
  if (t < 0 || (size_t)t >= wm->tuples.size()) return 0;
  return wm->tuples[t].ht.size();
}

int bg_wm_iter(const bg_wm *wm, int t, size_t *cursor, uint8_t *key_out,
               int32_t *priority, uint16_t *gate) {
  if (t < 0 || (size_t)t >= wm->tuples.size()) return 0;
  size_t i = 0;
  for (auto &kv : wm->tuples[t].ht) {
    if (i++ == *cursor) {
      memset(key_out, 0, BG_KEY_BYTES);
      memcpy(key_out, kv.first.w, wm->key_size);
      *priority = kv.second.priority;
      *gate = kv.second.gate;
      (*cursor)++;
      return 1;
    }
  }
  return 0;
}

static bool wm_want_no_tags() { return (path_flags() & kPathWmNoTags) != 0; }

// bit d: the tuple's mask has a nonzero dword d (wm_hash covers it)
static uint32_t wm_cover(const bg_wm *wm, size_t t) {
  uint32_t c = 0;
  for (uint32_t d = 0; d < 2 * wm->kw; d++) {
    uint32_t m;
    memcpy(&m, reinterpret_cast<const uint8_t *>(wm->tuples[t].mask.w) + 4 * d, 4);
    if (m) c |= 1u << d;
  }
  return c;
}

// A tuple whose mask covers one or two key bytes can be a direct tuple
// (WmArgs::ndirect): *spec = direct_index's byte positions and masks.
static bool wm_direct_spec(const bg_wm *wm, size_t t, uint32_t *spec) {
  const uint8_t *m = reinterpret_cast<const uint8_t *>(wm->tuples[t].mask.w);
  uint32_t pos[2] = {0, 0}, msk[2] = {0, 0}, nb = 0;
  for (uint32_t b = 0; b < 8 * wm->kw; b++) {
    if (!m[b]) continue;
    if (nb == 2) return false;
    pos[nb] = b;
    msk[nb++] = m[b];
  }
  if (nb == 0) return false;
  if (nb == 1) pos[1] = pos[0];
  *spec = pos[0] | pos[1] << 8 | msk[0] << 16 | msk[1] << 24;
  return true;
}

// The direct tuples of a tag-word image: up to kMaxDirect tuples of one or
// two mask bytes, one-byte masks first (their 2 KB tables stay in L2),
// then the tuples with the most entries (each saves a hash, two tag reads
// and its queue entries for every packet it matches). A direct tuple costs
// every packet one random L2 read; hashed, it costs an L2 read (one slot
// record) only for the packets whose fingerprint it holds -- about its
// density, entries / 65536, for a two-byte mask. The kernel's rate is
// bounded by its L2 requests in flight per CU (DESIGN §3, C4 counters), so
// a two-byte tuple goes direct only when at least half its 65536 keys are
// rules.
constexpr size_t kDirect2MinEntries = 32768;
static void wm_pick_direct(bg_wm *wm) {
  struct Cand {
    bool two;  // two mask bytes
    size_t n;  // entries
    uint32_t t;
  };
  std::vector<Cand> cand;
  for (size_t t = 0; t < wm->tuples.size(); t++) {
    uint32_t spec;
    if (!wm_direct_spec(wm, t, &spec) || wm->tuples[t].ht.empty()) continue;
    const bool two = (spec >> 24) != 0;
    if (two && wm->tuples[t].ht.size() < kDirect2MinEntries)
      continue;
    cand.push_back({two, wm->tuples[t].ht.size(), (uint32_t)t});
  }
  std::sort(cand.begin(), cand.end(), [](const Cand &a, const Cand &b) {
    if (a.two != b.two) return !a.two;
    if (a.n != b.n) return a.n > b.n;
    return a.t < b.t;
  });
  wm->ndirect = 0;
  for (auto &c : cand) {
    if (wm->ndirect == (uint32_t)kMaxDirect) break;
    uint32_t spec = 0;
    wm_direct_spec(wm, c.t, &spec);
    wm->dtu[wm->ndirect] = c.t;
    wm->dspec[wm->ndirect] = spec;
    wm->ndirect++;
  }
  std::sort(wm->dtu, wm->dtu + wm->ndirect);  // specs follow their tuples
  for (uint32_t d = 0; d < wm->ndirect; d++) wm_direct_spec(wm, wm->dtu[d], &wm->dspec[d]);
}

static bool wm_is_direct(const bg_wm *wm, size_t t) {
  for (uint32_t d = 0; d < wm->ndirect; d++)
    if (wm->dtu[d] == t) return true;
  return false;
}

// the hashed table's entries (all tuples but the direct ones)
static void wm_entries(const bg_wm *wm, std::vector<uint64_t> *keys,
                       std::vector<uint8_t> *vals, std::vector<uint64_t> *hashes) {
  keys->clear();
  vals->clear();
  hashes->clear();
  for (size_t t = 0; t < wm->tuples.size(); t++) {
    if (wm_is_direct(wm, t)) continue;
    const uint32_t cover = wm_cover(wm, t);
    const uint32_t seed = wm_seed32(tuple_seed(kDefaultSeed, (uint32_t)t));
    for (auto &kv : wm->tuples[t].ht) {
      keys->insert(keys->end(), kv.first.w, kv.first.w + wm->kw);
      uint64_t v = (uint64_t)(uint32_t)kv.second.priority |
                   ((uint64_t)kv.second.gate << 32) | ((uint64_t)t << 48);
      for (int b = 0; b < 8; b++) vals->push_back((uint8_t)(v >> (8 * b)));
      // the stored key is already masked: wm_hash of its dwords
      uint32_t kd[2 * kMaxKeyWords];
      memcpy(kd, kv.first.w, sizeof(kd));
      hashes->push_back(wm_hash(kd, cover, 2 * (int)wm->kw, seed));
    }
  }
}

// the host image of the current rules and the launch arguments that go with
// it (wm->host_img / host_a), built once per version for every device
static int wm_build_host(bg_wm *wm, bool no_tags) {
  std::vector<uint64_t> keys, hashes;
  std::vector<uint8_t> vals;
  std::vector<uint8_t> &img = wm->host_img;
  wm->ndirect = 0;
  wm_entries(wm, &keys, &vals, &hashes);
  TableLayout L;
  int r = build_image(wm->kw, 8, 1, keys, vals, hashes, &img, &L, 0.75, false, 1);
  if (r) return r;
  // Past the whole-table LDS size, a table whose tag words fit LDS (at a
  // higher load factor if need be: the bucketized 2x4 cuckoo table inserts
  // well past 0.9) keeps them there (bg_wm.hip) and needs no key filter;
  // its one- and two-byte tuples become direct tuples (WmArgs::ndirect).
  bool tags_lds = false;
  uint64_t aux_off = 0;
  if (img.size() > kLdsTableMax && !no_tags) {
    wm_pick_direct(wm);
    wm_entries(wm, &keys, &vals, &hashes);
    // the highest load that builds: the fewest tag words, the most LDS left
    // beside them (each packet checks the same 2 buckets per tuple; a fuller
    // bucket only adds fingerprint collisions, ~3 % per tuple at 0.95)
    for (double load : {0.95, 0.9, 0.75}) {
      std::vector<uint8_t> img2;
      TableLayout L2;
      if (build_image(wm->kw, 8, 1, keys, vals, hashes, &img2, &L2, load, false,
                      1) == 0 &&
          (uint64_t)L2.nbp * 4 <= kTagsLdsMax) {
        img.swap(img2);
        L = L2;
        tags_lds = true;
        break;
      }
    }
    if (!tags_lds && wm->ndirect) {  // back to the full table
      wm->ndirect = 0;
      wm_entries(wm, &keys, &vals, &hashes);
      r = build_image(wm->kw, 8, 1, keys, vals, hashes, &img, &L, 0.75, false, 1);
      if (r) return r;
    }
    if (wm->ndirect) {  // the direct tables after the hashed image
      aux_off = align256(img.size());
      uint64_t off = aux_off;
      for (uint32_t d = 0; d < wm->ndirect; d++) {
        const size_t nent = (wm->dspec[d] >> 24) ? 65536 : 256;
        wm->doff[d] = off;
        img.resize(off + nent * 8, 0xFF);  // empty: all ones (tuple 0xFFFF)
        uint64_t *tab = reinterpret_cast<uint64_t *>(img.data() + off);
        const uint32_t t = wm->dtu[d];
        for (auto &kv : wm->tuples[t].ht)
          tab[direct_index(kv.first.w, wm->dspec[d])] =
              (uint64_t)(uint32_t)kv.second.priority |
              ((uint64_t)kv.second.gate << 32) | ((uint64_t)t << 48);
        off = align256(off + nent * 8);
      }
    }
  }
  const size_t nkeys = hashes.size();
  // Tables too big for LDS get a blocked Bloom filter (up to 16 bits per
  // key, 64 KB by default so two workgroups fit a CU -- measured faster
  // than 128 KB at one workgroup per CU) that the kernel stages in LDS.
  uint32_t fw = 0;
  if (img.size() > kLdsTableMax && !tags_lds && nkeys > 0) {
    const uint32_t cap = std::min<uint32_t>(kFilterMaxWords, 64 * 256);
    fw = 1024;
    while (fw < cap && (uint64_t)fw * 32 < (uint64_t)nkeys * 16) fw *= 2;
    if ((uint64_t)fw * 32 < (uint64_t)nkeys * 4) fw = 0;  // < 4 bits/key
  }
  uint64_t foff = 0;
  if (fw) {
    foff = align256(img.size());
    img.resize(foff + (uint64_t)fw * 4, 0);
    uint32_t *f = reinterpret_cast<uint32_t *>(img.data() + foff);
    for (size_t i = 0; i < nkeys; i++) {
      const FilterProbe q = filter_probe(hashes[i], fw);
      f[q.word] |= q.bits;
    }
  }
  // the launch arguments of this image (base pointer filled per device)
  WmArgs &a = wm->host_a;
  memset(&a, 0, sizeof(a));
  a.t = table_ref(nullptr, img.size(), L, foff, fw, tags_lds, aux_off);
  a.ntuples = (uint32_t)wm->tuples.size();
  for (size_t t = 0; t < wm->tuples.size(); t++) {
    for (uint32_t j = 0; j < wm->kw; j++) a.tmask[t][j] = wm->tuples[t].mask.w[j];
    a.tcover[t] = wm_cover(wm, t);
    a.tseed[t] = wm_seed32(tuple_seed(a.t.seed, (uint32_t)t));
  }
  a.ndirect = wm->ndirect;
  for (uint32_t d = 0; d < wm->ndirect; d++) {
    a.dtu[d] = wm->dtu[d];
    a.dspec[d] = wm->dspec[d];
    a.doff[d] = wm->doff[d];
  }
  a.hmask = 0;
  for (size_t t = 0; t < wm->tuples.size(); t++)
    if (!wm_is_direct(wm, t)) a.hmask |= 1u << t;
  return 0;
}

// the device's image if it is of the current version and path flags
static WmImage *wm_fresh(bg_wm *wm, int device) {
  WmImage *v = wm->dev.get(device);
  return v && v->version == wm->version.load(std::memory_order_acquire) &&
                 v->no_tags == wm_want_no_tags()
             ? v
             : nullptr;
}

static int wm_sync_locked(bg_wm *wm, int device, hipStream_t s) {
  if (wm_fresh(wm, device)) return 0;
  const uint64_t ver = wm->version.load(std::memory_order_acquire);
  const bool no_tags = wm_want_no_tags();
  if (wm->host_version != ver || wm->host_no_tags != no_tags) {
    if (int r = wm_build_host(wm, no_tags)) return r;
    wm->host_version = ver;
    wm->host_no_tags = no_tags;
  }
  std::unique_ptr<WmImage> img(new WmImage());
  int r = upload_image(img.get(), device, wm->host_img.data(), wm->host_img.size(), s);
  if (r) return r;
  img->version = ver;
  img->no_tags = no_tags;
  img->a = wm->host_a;
  img->a.t.base = img->d;
  img->jit = wm_jit_request(img->a, make_plan(wm->dfields, false, 0), wm->kw, device);
  wm->dev.publish(device, img.release());
  return 0;
}

// as em_image
static int wm_image(bg_wm *wm, int device, hipStream_t s, WmImage **out) {
  WmImage *v = wm_fresh(wm, device);
  if (!v) {
    std::lock_guard<std::mutex> lk(wm->mu);
    if (int r = wm_sync_locked(wm, device, s)) return r;
    v = wm->dev.get(device);
  }
  *out = v;
  return 0;
}

}  // extern "C"

namespace bg {
uint64_t wm_version(const bg_wm *wm) { return wm->version.load(std::memory_order_acquire); }

// A WildcardMatch ring's plan (bg::wm_ring_create): the device image's
// arguments with the key plan of windows staged from win_off, the image's
// bytes and version, and the bytes of a slot the kernel reads
int wm_device_plan(bg_wm *wm, int device, hipStream_t s, int win_off, int meta_row,
                   WmArgs *a, uint64_t *bytes, int *read_end, uint64_t *version) {
  if (win_off < 0 || win_off > 1024) return fail(EINVAL, "win_off %d", win_off);
  std::vector<bg_field> df;
  if (int r = wm_fields_for(wm, win_off, meta_row, &df)) return r;
  if (int r = check_extent(df, -win_off, 0xFFFF)) return r;
  WmImage *img;
  if (int r = wm_image(wm, device, s, &img)) return r;
  *version = img->version;
  *a = img->a;
  a->fp = make_plan(df, false, -win_off);
  *bytes = img->bytes;
  const FieldPlan &fp = a->fp;
  int hi = 0;
  if (!fp.direct) {
    hi = fp.nf ? fp.win_lo + 16 * fp.nch : 0;
  } else {
    for (int i = 0; i < fp.nf; i++)
      hi = std::max(hi, (fspec_d(fp.fspec[i]) + fspec_nd(fp.fspec[i])) * 4);
  }
  *read_end = hi;
  return 0;
}
}  // namespace bg

extern "C" {

int bg_wm_sync(bg_wm *wm, int device, bg_stream_t stream) {
  WmImage *img;
  return wm_image(wm, device, (hipStream_t)stream, &img);
}

static int wm_launch(const std::vector<bg_field> &df, WmImage *img, const void *d_frames,
                     size_t stride,
                     size_t n, uint16_t default_gate, uint16_t *d_gates, int shift,
                     hipStream_t s) {
  WmArgs a = img->a;
  a.frames = static_cast<const uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.gates = d_gates;
  a.default_gate = default_gate;
  a.fp = make_plan(df, false, shift);
  img->used_on(s);
  hipError_t e;
  if (wm_jit_launch(img->jit.get(), a, img->device, num_cus(img->device), s, &e)) {
    HIP_TRY(e);
    img->launched_on(s);
    return 0;
  }
  HIP_TRY(launch_wm(a, num_cus(img->device), s));
  img->launched_on(s);
  return 0;
}

void bg_shutdown(void) { jit_shutdown(); }

int bg_wm_jit_wait(bg_wm *wm, int device, int timeout_ms) {
  int r = set_device(device);
  if (r) return r;
  WmImage *img;
  r = wm_image(wm, device, nullptr, &img);
  if (r) return r;
  return wm_jit_wait(img->jit.get(), timeout_ms);
}

int bg_wm_jit_check(bg_wm *wm, char *log, size_t len, size_t *code_bytes) {
  std::lock_guard<std::mutex> lk(wm->mu);
  const uint64_t ver = wm->version.load(std::memory_order_acquire);
  if (wm->host_version != ver || wm->host_no_tags) {
    if (int r = wm_build_host(wm, false)) return r;
    wm->host_version = ver;
    wm->host_no_tags = false;
  }
  std::string lg;
  size_t cb = 0;
  const int r = wm_jit_compile_now(wm->host_a, make_plan(wm->dfields, false, 0), wm->kw, &lg, &cb);
  if (code_bytes) *code_bytes = cb;
  if (log && len) {
    const size_t n = std::min(len - 1, lg.size());
    memcpy(log, lg.data(), n);
    log[n] = 0;
  }
  return r;
}

int bg_wm_jit_source(bg_wm *wm, int device, char *buf, size_t len, size_t *need) {
  std::string src;
  if (device < 0) {  // the host image's: no device
    std::lock_guard<std::mutex> lk(wm->mu);
    const uint64_t ver = wm->version.load(std::memory_order_acquire);
    if (wm->host_version != ver || wm->host_no_tags) {
      if (int r = wm_build_host(wm, false)) return r;
      wm->host_version = ver;
      wm->host_no_tags = false;
    }
    src = wm_jit_gen(wm->host_a, make_plan(wm->dfields, false, 0), wm->kw);
  } else {
    int r = set_device(device);
    if (r) return r;
    WmImage *img;
    r = wm_image(wm, device, nullptr, &img);
    if (r) return r;
    src = wm_jit_source(img->jit.get());
  }
  if (need) *need = src.size() + 1;
  if (src.empty()) return fail(ENOENT, "this table has no run-time compiled kernel");
  if (buf && len) {
    const size_t n = std::min(len - 1, src.size());
    memcpy(buf, src.data(), n);
    buf[n] = 0;
  }
  return 0;
}

int bg_wm_bind_meta(bg_wm *wm, int meta_off, const int32_t *attr_offsets,
                    int nattrs) {
  std::lock_guard<std::mutex> lk(wm->mu);
  int r = bind_meta(wm->fields, meta_off, attr_offsets, nattrs, &wm->attr_offs,
                    &wm->dfields, &wm->meta_bound);
  if (r) return r;
  wm->attrs_known = true;
  wm_changed(wm);  // as bg_em_bind_meta: rings of the old layout retire
  return 0;
}

int bg_wm_classify(bg_wm *wm, const void *d_frames, size_t stride, size_t n,
                   uint16_t default_gate, uint16_t *d_gates,
                   bg_stream_t stream) {
  return bg_wm_classify_window(wm, d_frames, stride, n, 0, default_gate,
                               d_gates, stream);
}

int bg_wm_classify_window(bg_wm *wm, const void *d_frames, size_t stride,
                          size_t n, int win_off, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream) {
  return bg_wm_classify_staged(wm, d_frames, stride, n, win_off, bg::kSlabMeta,
                               default_gate, d_gates, stream);
}

int bg_wm_classify_staged(bg_wm *wm, const void *d_win, size_t stride, size_t n,
                          int win_off, int meta_row, uint16_t default_gate,
                          uint16_t *d_gates, bg_stream_t stream) {
  if (win_off < 0 || win_off > 1024) return fail(EINVAL, "win_off %d", win_off);
  if (stride % 16 || ((uintptr_t)d_win & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned with stride %% 16 == 0");
  std::vector<bg_field> df;
  if (int r = wm_fields_for(wm, win_off, meta_row, &df)) return r;
  if (int r = check_extent(df, -win_off, stride)) return r;
  hipStream_t s = (hipStream_t)stream;
  WmImage *img;
  if (int r = wm_image(wm, current_device(), s, &img)) return r;
  return wm_launch(df, img, d_win, stride, n, default_gate, d_gates, -win_off, s);
}

int bg_wm_meta_window(const bg_wm *wm, int *lo, int *hi) {
  return meta_window(wm->fields, wm->has_attr, wm->attrs_known, wm->attr_offs, lo, hi);
}

int bg_wm_process_host(bg_wm *wm, const uint8_t *const *heads, size_t n,
                       uint16_t default_gate, uint16_t *gates,
                       bg_stream_t stream) {
  if (wm->has_attr) return no_attr_datapath();
  if (n == 0) return 0;
  const int dev = current_device();
  hipStream_t s = thread_stream(dev, (hipStream_t)stream);
  WmImage *img;
  int r = wm_image(wm, dev, s, &img);
  if (r) return r;
  Staging &st = thread_staging();
  int shift;
  size_t w;
  r = stage_windows(wm->fields, heads, n, st, dev, &shift, &w);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.d_in, st.h_in, n * w, hipMemcpyHostToDevice, s));
  r = wm_launch(wm->fields, img, st.d_in, w, n, default_gate,
                reinterpret_cast<uint16_t *>(st.d_out), shift, s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.h_out, st.d_out, n * 2, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  memcpy(gates, st.h_out, n * 2);
  return 0;
}

void bg_wm_window(const bg_wm *wm, int *lo, int *hi) {
  fields_window(wm->fields, lo, hi);
}

int bg_wm_table_info(const bg_wm *wm, uint64_t *bytes, int *in_lds) {
  const WmImage *img = const_cast<bg_wm *>(wm)->dev.get(current_device());
  if (!img) return fail(EINVAL, "no device table yet");
  *bytes = img->bytes;
  // 2: key filter in LDS, 3: tag words in LDS; bits 8+: direct tuples
  *in_lds = (int)img->a.t.lds | (int)(img->a.ndirect << 8);
  return 0;
}

// ============================================================================
// IPChecksum / L4Checksum
// ============================================================================
int bg_cksum(int device, void *d_frames, size_t stride, size_t n, int mode,
             int verify, uint16_t *d_ip_gates, uint16_t *d_l4_gates,
             bg_stream_t stream) {
  if (mode < 1 || mode > 3) return fail(EINVAL, "mode must be 1, 2 or 3");
  if (stride % 16 || ((uintptr_t)d_frames & 15) || stride > (1u << 30))
    return fail(EINVAL, "frame slab must be 16-byte aligned with stride %% 16 == 0");
  int r = set_device(device);
  if (r) return r;
  CkArgs a;
  a.frames = static_cast<uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.ptrs = nullptr;
  a.ip_gates = d_ip_gates;
  a.l4_gates = d_l4_gates;
  a.mode = mode;
  a.verify = verify ? 1 : 0;
  HIP_TRY(launch_cksum(a, num_cus(device), (hipStream_t)stream));
  return 0;
}

int bg_cksum_ptrs(int device, const uint64_t *d_ptrs, size_t span, size_t n, int mode,
                  int verify, uint16_t *d_ip_gates, uint16_t *d_l4_gates,
                  bg_stream_t stream) {
  if (mode < 1 || mode > 3) return fail(EINVAL, "mode must be 1, 2 or 3");
  if (span < 64 || span > 65535) return fail(EINVAL, "span %zu not in [64, 65535]", span);
  if (n && !d_ptrs) return fail(EINVAL, "bad arguments");
  int r = set_device(device);
  if (r) return r;
  CkArgs a;
  a.frames = nullptr;
  a.stride = span;
  a.n = n;
  a.ptrs = d_ptrs;
  a.ip_gates = d_ip_gates;
  a.l4_gates = d_l4_gates;
  a.mode = mode;
  a.verify = verify ? 1 : 0;
  HIP_TRY(launch_cksum(a, num_cus(device), (hipStream_t)stream));
  return 0;
}

int bg_cksum_process_host(int device, uint8_t *const *heads, size_t n,
                          size_t span, int mode, int verify,
                          uint16_t *ip_gates, uint16_t *l4_gates,
                          bg_stream_t stream) {
  if (n == 0) return 0;
  Staging &st = thread_staging();
  const size_t w = (span + 15) / 16 * 16;
  int r = set_device(device);
  if (r) return r;
  hipStream_t s = thread_stream(device, (hipStream_t)stream);
  r = st.ensure(device, n * w, n * 4);
  if (r) return r;
  for (size_t i = 0; i < n; i++) {
    memcpy(st.h_in + i * w, heads[i], span);
    if (w > span) memset(st.h_in + i * w + span, 0, w - span);
  }
  HIP_TRY(hipMemcpyAsync(st.d_in, st.h_in, n * w, hipMemcpyHostToDevice, s));
  uint16_t *dg = reinterpret_cast<uint16_t *>(st.d_out);
  r = bg_cksum(device, st.d_in, w, n, mode, verify, dg, dg + n, s);
  if (r) return r;
  HIP_TRY(hipMemcpyAsync(st.h_in, st.d_in, n * w, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipMemcpyAsync(st.h_out, st.d_out, n * 4, hipMemcpyDeviceToHost, s));
  HIP_TRY(hipStreamSynchronize(s));
  for (size_t i = 0; i < n; i++) memcpy(heads[i], st.h_in + i * w, span);
  const uint16_t *hg = reinterpret_cast<const uint16_t *>(st.h_out);
  if (ip_gates) memcpy(ip_gates, hg, n * 2);
  if (l4_gates) memcpy(l4_gates, hg + n, n * 2);
  return 0;
}

}  // extern "C"

extern "C" int bg_debug_key(const bg_field *fields, int nfields,
                            int em_masks, const uint8_t *frame,
                            uint8_t *key_out) {
  if (nfields < 0 || nfields > kMaxFields || (nfields && !fields) || !frame ||
      !key_out)
    return fail(EINVAL, "bad arguments");
  std::vector<bg_field> f(fields, fields + nfields);
  const FieldPlan p = make_plan(f, em_masks != 0, 0);
  uint64_t k[kMaxKeyWords];
  host_key(p, frame, kMaxKeyWords, k);
  memcpy(key_out, k, sizeof(k));
  return 0;
}
