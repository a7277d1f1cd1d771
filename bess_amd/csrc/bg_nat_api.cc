// bg_nat_api.cc -- C ABI of the StaticNAT datapath (include/bessgpu.h
// bg_snat_*): the address-pair list, uploaded when it changes, per
// direction in the order the kernel scans it (bg_nat.hip).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <mutex>
#include <vector>

#include "bg_internal.h"

using namespace bg;

struct bg_snat {
  std::vector<uint32_t> int_addr, ext_addr, size;
  bool dirty = true;
  int device = -1;
  uint32_t *d_pairs = nullptr;  // [forward pairs][reverse pairs]
  size_t d_cap = 0;             // pairs per direction
  std::mutex mu;
  ~bg_snat() {
    if (d_pairs) (void)hipFree(d_pairs);
  }
};

static size_t padded(size_t n) { return std::max<size_t>((n + 3) / 4 * 4, 4); }

static int snat_sync_locked(bg_snat *h, int dev, hipStream_t s) {
  if (!h->dirty && h->device == dev && h->d_pairs) return 0;
  int r = set_device(dev);
  if (r) return r;
  const size_t n = h->size.size(), np = padded(n);
  std::vector<uint32_t> img(np * 8, 0);  // size 0: never matches
  for (size_t i = 0; i < n; i++) {
    uint32_t *fw = &img[i * 4], *rv = &img[np * 4 + i * 4];
    fw[0] = h->int_addr[i];
    fw[1] = h->ext_addr[i];
    fw[2] = h->size[i];
    rv[0] = h->ext_addr[i];
    rv[1] = h->int_addr[i];
    rv[2] = h->size[i];
  }
  if (!h->d_pairs || h->d_cap < np || h->device != dev) {
    if (h->d_pairs) (void)hipFree(h->d_pairs);
    h->d_pairs = nullptr;
    h->d_cap = std::max<size_t>(np, 64);
    HIP_TRY(hipMalloc(reinterpret_cast<void **>(&h->d_pairs), h->d_cap * 32));
  }
  HIP_TRY(hipMemcpyAsync(h->d_pairs, img.data(), img.size() * 4,
                         hipMemcpyHostToDevice, s));
  HIP_TRY(hipStreamSynchronize(s));
  h->device = dev;
  h->dirty = false;
  return 0;
}

extern "C" {

int bg_snat_create(bg_snat **out) {
  if (!out) return fail(EINVAL, "bad arguments");
  *out = new bg_snat();
  return 0;
}

void bg_snat_destroy(bg_snat *h) { delete h; }

int bg_snat_add(bg_snat *h, uint32_t int_addr, uint32_t ext_addr, uint32_t size) {
  std::lock_guard<std::mutex> lk(h->mu);
  h->int_addr.push_back(int_addr);
  h->ext_addr.push_back(ext_addr);
  h->size.push_back(size);
  h->dirty = true;
  return 0;
}

size_t bg_snat_count(const bg_snat *h) { return h->size.size(); }

int bg_snat_classify(bg_snat *h, void *d_frames, size_t stride, size_t n,
                     int dir, uint16_t *d_out, bg_stream_t stream) {
  if (stride % 16 || stride < 64 || ((uintptr_t)d_frames & 15))
    return fail(EINVAL, "frame slab must be 16-byte aligned, stride a 16-byte "
                "multiple >= 64");
  if (dir != 0 && dir != 1) return fail(EINVAL, "dir %d", dir);
  hipStream_t s = (hipStream_t)stream;
  int dev = 0;
  (void)hipGetDevice(&dev);
  NatArgs a;
  memset(&a, 0, sizeof(a));
  {
    std::lock_guard<std::mutex> lk(h->mu);
    if (h->device >= 0) dev = h->device;
    int r = snat_sync_locked(h, dev, s);
    if (r) return r;
    const size_t np = padded(h->size.size());
    a.pairs = h->d_pairs + (dir ? np * 4 : 0);
    a.npairs = (uint32_t)np;
  }
  int r = set_device(dev);
  if (r) return r;
  a.frames = static_cast<uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_out;
  a.dir = (uint32_t)dir;
  HIP_TRY(launch_nat(a, num_cus(dev), s));
  return 0;
}

}  // extern "C"
