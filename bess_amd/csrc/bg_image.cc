// bg_image.cc -- fenced retirement of device table images (bg_image.h).
#include "bg_image.h"

#include <errno.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <shared_mutex>
#include <unordered_set>
#include <vector>

#include "bg_internal.h"

namespace bg {

namespace {

// a stream as a users[] word: never 0 (the null stream is 1)
inline uintptr_t enc(hipStream_t s) { return reinterpret_cast<uintptr_t>(s) ^ 1u; }
inline hipStream_t dec(uintptr_t e) { return reinterpret_cast<hipStream_t>(e ^ 1u); }

struct Dead {
  DevImage *img;
  std::vector<hipEvent_t> evs;
  bool sync_device;  // more streams than users[] slots: wait for the device
};

struct Registry {
  std::mutex mu;
  std::unordered_set<DevImage *> live;  // for stream_gone
  std::vector<Dead> dead;
  std::shared_mutex own_mu;
  std::unordered_set<uintptr_t> own;  // the library's streams (own_stream)
};

Registry &reg() {
  static Registry *r = new Registry();  // never destroyed: images outlive statics
  return *r;
}

// the calling thread's device is restored when this goes out of scope
struct DeviceGuard {
  int cur = -1;
  DeviceGuard() { (void)hipGetDevice(&cur); }
  ~DeviceGuard() {
    if (cur >= 0) (void)hipSetDevice(cur);
  }
};

bool done(Dead &x, bool wait) {
  for (hipEvent_t &e : x.evs) {
    if (!e) continue;
    hipError_t q = wait ? hipEventSynchronize(e) : hipEventQuery(e);
    if (q == hipErrorNotReady) return false;
    (void)hipEventDestroy(e);  // completed (or failed: the stream is gone)
    e = nullptr;
  }
  if (x.sync_device) {
    if (!wait) return false;
    (void)hipSetDevice(x.img->device);
    (void)hipDeviceSynchronize();
  }
  return true;
}

// the null stream or one the library created: fenced by recording on it
bool library_stream(hipStream_t s) {
  if (!s) return true;
  std::shared_lock<std::shared_mutex> lk(reg().own_mu);
  return reg().own.count(reinterpret_cast<uintptr_t>(s)) != 0;
}

}  // namespace

void own_stream(hipStream_t s) {
  if (!s) return;
  std::unique_lock<std::shared_mutex> lk(reg().own_mu);
  reg().own.insert(reinterpret_cast<uintptr_t>(s));
}

DevImage::DevImage() {
  for (auto &u : users) u.store(0, std::memory_order_relaxed);
  for (auto &u : ext) u.store(0, std::memory_order_relaxed);
  std::lock_guard<std::mutex> lk(reg().mu);
  reg().live.insert(this);
}

DevImage::~DevImage() {
  {
    std::lock_guard<std::mutex> lk(reg().mu);
    reg().live.erase(this);
  }
  if (d && owned && device >= 0) {
    DeviceGuard g;
    (void)hipSetDevice(device);
    (void)hipFree(d);
  }
  d = nullptr;
  for (hipEvent_t &e : ext_ev)
    if (e) (void)hipEventDestroy(e);  // (retire handed the recorded ones on)
}

void DevImage::used_on(hipStream_t s) {
  if (!library_stream(s)) return;  // launched_on fences it
  const uintptr_t e = enc(s);
  for (auto &u : users) {
    uintptr_t v = u.load(std::memory_order_acquire);
    if (v == e) return;
    if (v == 0) {
      if (u.compare_exchange_strong(v, e, std::memory_order_acq_rel)) return;
      if (v == e) return;
    }
  }
  overflow.store(true, std::memory_order_release);
}

void DevImage::launched_on(hipStream_t s) {
  if (library_stream(s)) return;
  const uintptr_t e = enc(s);
  int z = 0;
  while (!ext_lock.compare_exchange_weak(z, 1, std::memory_order_acquire)) z = 0;
  int slot = -1;
  for (int i = 0; i < kMaxImageExtUsers && slot < 0; i++) {
    const uintptr_t v = ext[i].load(std::memory_order_relaxed);
    if (v == e) slot = i;
  }
  for (int i = 0; i < kMaxImageExtUsers && slot < 0; i++)
    if (ext[i].load(std::memory_order_relaxed) == 0) {
      ext[i].store(e, std::memory_order_relaxed);
      slot = i;
    }
  bool ok = slot >= 0;
  if (ok && !ext_ev[slot] &&
      hipEventCreateWithFlags(&ext_ev[slot], hipEventDisableTiming) != hipSuccess) {
    ext_ev[slot] = nullptr;
    ok = false;
  }
  if (ok && hipEventRecord(ext_ev[slot], s) != hipSuccess) ok = false;
  ext_lock.store(0, std::memory_order_release);
  if (!ok) overflow.store(true, std::memory_order_release);
}

int upload_image(DevImage *img, int dev, const void *host, uint64_t bytes,
                 hipStream_t s) {
  reap_images(false);
  int r = set_device(dev);
  if (r) return r;
  img->device = dev;
  img->owned = true;
  img->bytes = bytes;
  HIP_TRY(hipMalloc(reinterpret_cast<void **>(&img->d), std::max<uint64_t>(bytes, 256)));
  if (bytes) {
    HIP_TRY(hipMemcpyAsync(img->d, host, bytes, hipMemcpyHostToDevice, s));
    HIP_TRY(hipStreamSynchronize(s));
  }
  return 0;
}

void retire_image(DevImage *img) {
  if (!img) return;
  Dead x{img, {}, img->overflow.load(std::memory_order_acquire)};
  {
    DeviceGuard g;
    if (img->device >= 0 && hipSetDevice(img->device) == hipSuccess) {
      for (auto &u : img->users) {
        const uintptr_t v = u.load(std::memory_order_acquire);
        if (!v) continue;
        hipEvent_t ev = nullptr;
        if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
          x.sync_device = true;
          continue;
        }
        // a stream that no longer exists has nothing left in flight
        if (hipEventRecord(ev, dec(v)) != hipSuccess) {
          (void)hipEventDestroy(ev);
          continue;
        }
        x.evs.push_back(ev);
      }
      // callers' streams: the events their launches recorded
      for (int i = 0; i < kMaxImageExtUsers; i++)
        if (img->ext[i].load(std::memory_order_acquire) && img->ext_ev[i]) {
          x.evs.push_back(img->ext_ev[i]);
          img->ext_ev[i] = nullptr;
        }
    }
  }
  {
    std::lock_guard<std::mutex> lk(reg().mu);
    reg().dead.push_back(std::move(x));
  }
  reap_images(false);
}

void reap_images(bool wait) {
  std::vector<DevImage *> free_now;
  {
    std::lock_guard<std::mutex> lk(reg().mu);
    DeviceGuard g;
    auto &dl = reg().dead;
    for (size_t i = 0; i < dl.size();) {
      if (done(dl[i], wait)) {
        free_now.push_back(dl[i].img);
        dl[i] = std::move(dl.back());
        dl.pop_back();
      } else {
        i++;
      }
    }
  }
  for (DevImage *p : free_now) delete p;
}

void stream_gone(hipStream_t s) {
  const uintptr_t e = enc(s);
  {
    std::unique_lock<std::shared_mutex> lk(reg().own_mu);
    reg().own.erase(reinterpret_cast<uintptr_t>(s));
  }
  std::lock_guard<std::mutex> lk(reg().mu);
  for (DevImage *img : reg().live)
    for (auto &u : img->users) {
      uintptr_t v = e;
      u.compare_exchange_strong(v, 0, std::memory_order_acq_rel);
    }
}

}  // namespace bg

extern "C" {

int bg_stream_attach(bg_stream_t stream) {
  if (!stream) return 0;  // the null stream is always fenced lazily
  bg::own_stream(reinterpret_cast<hipStream_t>(stream));
  return 0;
}

int bg_stream_detach(bg_stream_t stream) {
  if (!stream) return 0;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // its launches done, it drops out of the images' lazily fenced streams
  const hipError_t e = hipStreamSynchronize(s);
  bg::stream_gone(s);
  if (e != hipSuccess) return bg::fail(EIO, "hipStreamSynchronize: %s", hipGetErrorString(e));
  return 0;
}

}  // extern "C"
