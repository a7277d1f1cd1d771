// bg_image.h -- device images of rule tables: one immutable upload per table
// version and device, published per device, retired behind fences.
//
// BESS changes rules only from THREAD_UNSAFE commands, which bessd runs with
// the workers paused (core/module.cc:97-101), but a GPU module keeps work in
// flight across that pause: a bg_pipe holds launched batches, an async
// classify on a caller's stream may still be queued. Such a batch must see
// the rules as they were when it was submitted. So a table never writes a
// device image a kernel may read:
//   * a rule change bumps the table's version;
//   * the next launch on a device whose image is older builds a NEW image
//     (fresh allocation), uploads it and publishes it for that device;
//   * the image it replaces is retired: an event is recorded on every stream
//     of the library's own that launched against it (DevImage::used_on),
//     and a caller's stream -- whose handle the library must not keep, as
//     the caller may destroy it -- is fenced by an event the launch itself
//     recorded after it (DevImage::launched_on); the image is freed only
//     when all those events have completed (reap_images).
// Each device has its own published image (a replica), so one module can be
// driven from workers on several GPUs of one process (core/worker.h:77).
#ifndef BESS_AMD_BG_IMAGE_H_
#define BESS_AMD_BG_IMAGE_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>

namespace bg {

constexpr int kMaxDevices = 16;
constexpr int kMaxImageUsers = 256;
constexpr int kMaxImageExtUsers = 64;

// One device copy of one table version (subclassed by each table for the
// launch arguments that go with the image).
struct DevImage {
  int device = -1;
  uint64_t version = 0;
  uint8_t *d = nullptr;  // the image (device memory on `device`)
  uint64_t bytes = 0;
  bool owned = true;     // false: an externally assembled image (attach)

  DevImage();
  virtual ~DevImage();
  // A launch against this image is about to be queued on `s` (lock-free
  // for the library's own streams and the null stream, which retirement
  // fences by recording on them).
  void used_on(hipStream_t s);
  // ... and was queued: a stream the library does not own gets an event
  // recorded behind the launch (the image's event for that stream).
  void launched_on(hipStream_t s);

  std::atomic<uintptr_t> users[kMaxImageUsers];
  std::atomic<bool> overflow{false};  // more streams than slots: device sync
  // callers' streams: the handle (identity only, never recorded on at
  // retirement) and the event its launches re-record
  std::atomic<uintptr_t> ext[kMaxImageExtUsers];
  hipEvent_t ext_ev[kMaxImageExtUsers] = {};
  std::atomic<int> ext_lock{0};
};

// The library created `s` (pipe slots, worker threads' streams): images
// fence it by recording on it at retirement; stream_gone() before it is
// destroyed.
void own_stream(hipStream_t s);

// Allocate img->d (bytes, at least 256) on `dev` and copy `host` into it on
// stream s, synchronously (control path). Returns 0 or -errno.
int upload_image(DevImage *img, int dev, const void *host, uint64_t bytes,
                 hipStream_t s);
// Hand an image over to the fence list (nullptr: nothing). Never blocks.
void retire_image(DevImage *img);
// Free the retired images whose fences have passed (wait: block for all).
void reap_images(bool wait);
// A stream is about to be destroyed (after it was synchronized): drop it
// from every live image's users.
void stream_gone(hipStream_t s);

// The published image of each device.
template <class T>
class Published {
 public:
  Published() {
    for (auto &c : cur_) c.store(nullptr, std::memory_order_relaxed);
  }
  ~Published() { release(); }
  T *get(int dev) const {
    return (unsigned)dev < (unsigned)kMaxDevices ? cur_[dev].load(std::memory_order_acquire)
                                                 : nullptr;
  }
  // publish img for dev (control path, the table's lock held); the image it
  // replaces is retired
  void publish(int dev, T *img) {
    T *old = cur_[dev].exchange(img, std::memory_order_acq_rel);
    retire_image(old);
  }
  void release() {
    for (int d = 0; d < kMaxDevices; d++) publish(d, nullptr);
  }

 private:
  std::atomic<T *> cur_[kMaxDevices];
};

}  // namespace bg

#endif  // BESS_AMD_BG_IMAGE_H_
