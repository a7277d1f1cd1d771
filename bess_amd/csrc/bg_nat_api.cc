// bg_nat_api.cc -- C ABI of the StaticNAT datapath (include/bessgpu.h
// bg_snat_*): the address-pair list, uploaded when it changes, per
// direction in the order the kernel scans it (bg_nat.hip).
#include <errno.h>
#include <hip/hip_runtime.h>
#include <string.h>

#include <memory>
#include <mutex>
#include <vector>

#include "bg_internal.h"

using namespace bg;

// one device's pair list of one version: [forward pairs][reverse pairs]
struct SnatImage : DevImage {
  size_t np = 0;  // pairs per direction (padded)
};

struct bg_snat {
  std::vector<uint32_t> int_addr, ext_addr, size;
  std::atomic<uint64_t> version{1};  // bumped by add; images as bg_image.h
  Published<SnatImage> dev;
  std::mutex mu;
};

static size_t padded(size_t n) { return std::max<size_t>((n + 3) / 4 * 4, 4); }

static int snat_image(bg_snat *h, int dev, hipStream_t s, SnatImage **out) {
  SnatImage *v = h->dev.get(dev);
  const uint64_t ver = h->version.load(std::memory_order_acquire);
  if (v && v->version == ver) {
    *out = v;
    return 0;
  }
  std::lock_guard<std::mutex> lk(h->mu);
  v = h->dev.get(dev);
  if (v && v->version == ver) {
    *out = v;
    return 0;
  }
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
  std::unique_ptr<SnatImage> p(new SnatImage());
  int r = upload_image(p.get(), dev, img.data(), img.size() * 4, s);
  if (r) return r;
  p->version = ver;
  p->np = np;
  *out = p.get();
  h->dev.publish(dev, p.release());
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
  h->version.fetch_add(1, std::memory_order_acq_rel);
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
  SnatImage *img;
  if (int r = snat_image(h, dev, s, &img)) return r;
  NatArgs a;
  memset(&a, 0, sizeof(a));
  a.pairs = reinterpret_cast<const uint32_t *>(img->d) + (dir ? img->np * 4 : 0);
  a.npairs = (uint32_t)img->np;
  img->used_on(s);
  a.frames = static_cast<uint8_t *>(d_frames);
  a.stride = stride;
  a.n = n;
  a.out = d_out;
  a.dir = (uint32_t)dir;
  HIP_TRY(launch_nat(a, num_cus(dev), s));
  img->launched_on(s);
  return 0;
}

}  // extern "C"
