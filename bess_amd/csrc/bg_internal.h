// bg_internal.h -- host-side helpers shared by the C ABI translation units.
#ifndef BESS_AMD_BG_INTERNAL_H_
#define BESS_AMD_BG_INTERNAL_H_

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../include/bessgpu.h"
#include "bg_image.h"
#include "bg_kernels.h"
#include "bg_table.h"

namespace bg {

constexpr uint64_t kDefaultSeed = 0x5EED5EED0B5E55ULL;

// A flow key as the reference stores it (ExactMatchKey / wm_hkey_t: eight
// u64 words, bytes past total_key_size zero).
struct Key {
  uint64_t w[8];
  bool operator==(const Key &o) const { return memcmp(w, o.w, sizeof(w)) == 0; }
};
struct KeyHash {
  size_t operator()(const Key &k) const {
    return (size_t)hash_words(k.w, 8, 0x1234567ULL);
  }
};

struct WmVal {  // WmData (wildcard_match.h:57-60)
  int32_t priority;
  uint16_t gate;
};

extern thread_local std::string g_err;
int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIP_TRY(expr)                                                  \
  do {                                                                 \
    hipError_t e_ = (expr);                                            \
    if (e_ != hipSuccess)                                              \
      return ::bg::fail(EIO, "%s: %s", #expr, hipGetErrorString(e_));  \
  } while (0)
int num_cus(int device);
int set_device(int device);
uint32_t round_kw(uint32_t key_bytes);
FieldPlan make_plan(const std::vector<bg_field> &fields, bool em_masks,
                    int shift);
void relayout(TableLayout &L, uint32_t nbp);
int build_image(uint32_t kw, uint32_t val_bytes, uint32_t nparts,
                const std::vector<uint64_t> &keys,
                const std::vector<uint8_t> &vals,
                const std::vector<uint64_t> &hashes, std::vector<uint8_t> *img,
                TableLayout *out_layout, double max_load = 0.75,
                bool vik = false, uint32_t probe = 0);

// The TableRef of a table image at `base` (bytes long, layout L; a key
// filter / direct-tuple tables appended at filt_off / aux_off).
TableRef table_ref(const uint8_t *base, uint64_t bytes, const TableLayout &L,
                   uint64_t filt_off, uint32_t filt_words, bool tags_lds,
                   uint64_t aux_off);

// A single-device table image updated in place in stream order (NAT's
// lookup copy, bg_dnat_api.cc: its batches run one at a time under the
// module's lock and are synchronous). Rule tables use bg_image.h instead.
struct DevTable {
  int device = -1;
  uint8_t *d_image = nullptr;
  bool owned = true;
  uint64_t bytes = 0;
  TableLayout L{};
  bool valid = false;
  uint64_t filt_off = 0;    // key filter appended to the image (WM)
  uint32_t filt_words = 0;
  bool tags_lds = false;    // tag words staged in LDS (WM, bg_wm.hip)
  uint64_t aux_off = 0;     // direct-tuple tables appended to the image (WM)
  int upload(int dev, const std::vector<uint8_t> &img, const TableLayout &lay,
             hipStream_t s);
  void release();
  TableRef ref() const;
};

struct Staging {
  int device = -1;
  uint8_t *h_in = nullptr, *d_in = nullptr, *h_out = nullptr, *d_out = nullptr;
  size_t in_cap = 0, out_cap = 0;
  int ensure(int dev, size_t in_bytes, size_t out_bytes);
  void release();
  ~Staging() { release(); }
};

// The synchronous host paths (bg_*_process_host, Module::ProcessPackets)
// may be entered by many worker threads on one table or module at once
// (core/module.h:485): each thread stages into its own pinned buffers and,
// when the caller passes no stream, runs on its own non-blocking stream per
// device (never the legacy stream, which would serialise the workers).
Staging &thread_staging();
// bg_api.cc: a table's field plan for slots that start at frame byte
// win_off, its synced device table, and the rule version that image holds
// meta_row: where a staged row carries the packet's metadata area (row
// offset of its byte 0; attr fields only), or kSlabMeta for a device slab
// laid out by bg_em_bind_meta
constexpr int kSlabMeta = -(1 << 30);
int em_device_plan(bg_em *em, int device, hipStream_t s, int win_off, int meta_row,
                   FieldPlan *fp, TableRef *t, int *read_end, uint64_t *version);
// the metadata bytes [lo, hi) the attr fields read (none: lo == hi == 0)
int em_meta_window(const bg_em *em, int *lo, int *hi);
// bg_ring.cc: bg_em_ring_create over staged rows with metadata at meta_row
int em_ring_create(bg_em *em, int device, int lanes, int slots, int blocks,
                   uint32_t idle_us, int win_off, int meta_row, bg_ring **out);
uint64_t em_version(const bg_em *em);  // bumped by every rule change
uint64_t wm_version(const bg_wm *wm);
int wm_device_plan(bg_wm *wm, int device, hipStream_t s, int win_off, int meta_row,
                   WmArgs *a, uint64_t *bytes, int *read_end, uint64_t *version);
// a persistent ring over a WildcardMatch table (bg_ring.cc; as em_ring_create)
int wm_ring_create(bg_wm *wm, int device, int lanes, int slots, int blocks,
                   uint32_t idle_us, int win_off, int meta_row, bg_ring **out);
// bg_ring.cc: the rule version a ring classifies with; whether a lane's
// ticket has finished (one host word, no lock)
uint64_t ring_version(const bg_ring *r);
bool ring_done(const bg_ring *r, int lane, int64_t ticket);
// the ring's grid is running (one host word read; no lock, no HIP call)
bool ring_live(const bg_ring *r);
hipStream_t thread_stream(int device, hipStream_t given);
// bg_comm.cc: an assembled image (d_img, bytes; hipMalloc'ed on `device`,
// laid out as bg_em_plan*) becomes the device's table image of the current
// rules, owned (and freed, behind fences) by the table
int em_publish_owned(bg_em *em, int device, uint8_t *d_img, uint64_t bytes);
// bg_host_register: the device address of host bytes [p, p + len) when they
// lie in one registered region (lock-free; false otherwise)
bool host_dev_addr(const void *p, size_t len, uint64_t *dev);

}  // namespace bg

#endif  // BESS_AMD_BG_INTERNAL_H_
