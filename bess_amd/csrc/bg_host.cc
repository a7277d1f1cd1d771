// bg_host.cc -- host memory the device reads and writes in place
// (bg_host_register): BESS's packet pool (core/packet_pool.h, DPDK mempool
// memory) registered once, so that a module whose device datapath works on
// whole frames (the checksum modules) takes each packet's head pointer
// instead of a copy of its bytes: the kernel reads the frame over PCIe and
// writes the checksum words back into the packet buffer (bg_pipe's
// zero-copy slots, bg_cksum_ptrs).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <atomic>
#include <mutex>

#include "../../include/bessgpu.h"
#include "bg_internal.h"

namespace bg {
namespace {

constexpr int kMaxRegions = 64;

// Regions are published once filled (count after the entry) and never
// moved; an unregistered entry keeps its slot with 0 bytes. The datapath's
// lookups take no lock.
struct Region {
  std::atomic<uintptr_t> base{0};
  std::atomic<uint64_t> bytes{0};
  std::atomic<uintptr_t> dev{0};
};
Region g_regions[kMaxRegions];
std::atomic<int> g_count{0};
std::mutex g_mu;  // registrations

}  // namespace

bool host_dev_addr(const void *p, size_t len, uint64_t *dev) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(p);
  const int n = g_count.load(std::memory_order_acquire);
  for (int i = 0; i < n; i++) {
    const Region &r = g_regions[i];
    const uint64_t z = r.bytes.load(std::memory_order_acquire);
    const uintptr_t b = r.base.load(std::memory_order_relaxed);
    if (a - b < z && len <= z - (a - b)) {
      *dev = r.dev.load(std::memory_order_relaxed) + (a - b);
      return true;
    }
  }
  return false;
}

}  // namespace bg

using bg::fail;

extern "C" {

int bg_host_register(void *base, size_t bytes) {
  if (!base || !bytes) return fail(EINVAL, "bad arguments");
  std::lock_guard<std::mutex> lk(bg::g_mu);
  const int n = bg::g_count.load(std::memory_order_relaxed);
  const uintptr_t a = reinterpret_cast<uintptr_t>(base);
  for (int i = 0; i < n; i++) {
    const bg::Region &r = bg::g_regions[i];
    const uint64_t z = r.bytes.load(std::memory_order_relaxed);
    const uintptr_t b = r.base.load(std::memory_order_relaxed);
    if (z && a < b + z && b < a + bytes)
      return fail(EEXIST, "host memory %p+%zu overlaps a registered region", base, bytes);
  }
  int slot = n;
  for (int i = 0; i < n; i++)
    if (!bg::g_regions[i].bytes.load(std::memory_order_relaxed)) slot = i;
  if (slot == bg::kMaxRegions) return fail(ENOSPC, "%d host regions registered", slot);
  // mapped into every device's address space (portable), coherent: the
  // device reads what the host wrote before a launch, and its writes reach
  // the host by the launch's end
  hipError_t e = hipHostRegister(base, bytes, hipHostRegisterMapped | hipHostRegisterPortable);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return fail(EIO, "hipHostRegister(%p, %zu): %s", base, bytes, hipGetErrorString(e));
  }
  void *d = nullptr;
  e = hipHostGetDevicePointer(&d, base, 0);
  if (e != hipSuccess) {
    (void)hipHostUnregister(base);
    return fail(EIO, "hipHostGetDevicePointer: %s", hipGetErrorString(e));
  }
  bg::Region &r = bg::g_regions[slot];
  r.base.store(a, std::memory_order_relaxed);
  r.dev.store(reinterpret_cast<uintptr_t>(d), std::memory_order_relaxed);
  r.bytes.store(bytes, std::memory_order_release);
  if (slot == n) bg::g_count.store(n + 1, std::memory_order_release);
  return 0;
}

int bg_host_unregister(void *base) {
  std::lock_guard<std::mutex> lk(bg::g_mu);
  const int n = bg::g_count.load(std::memory_order_relaxed);
  for (int i = 0; i < n; i++) {
    bg::Region &r = bg::g_regions[i];
    if (r.bytes.load(std::memory_order_relaxed) &&
        r.base.load(std::memory_order_relaxed) == reinterpret_cast<uintptr_t>(base)) {
      // lookups stop finding the region before it is unpinned; if the
      // runtime refuses, the region stays pinned and is tracked again
      const uint64_t bytes = r.bytes.exchange(0, std::memory_order_acq_rel);
      hipError_t e = hipHostUnregister(base);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        r.bytes.store(bytes, std::memory_order_release);
        return fail(EIO, "hipHostUnregister: %s", hipGetErrorString(e));
      }
      return 0;
    }
  }
  return fail(ENOENT, "%p is not a registered region", base);
}

int bg_host_dev_addr(const void *p, size_t len, uint64_t *dev) {
  if (!dev) return fail(EINVAL, "bad arguments");
  if (!bg::host_dev_addr(p, len, dev))
    return fail(ENOENT, "%p+%zu is not in a registered region", p, len);
  return 0;
}

}  // extern "C"
