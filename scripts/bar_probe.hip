// Can the host write device memory directly (through the PCIe BAR)?
// For each allocation kind: does the pointer dereference on the CPU (a
// SIGSEGV is caught, the probe goes on), does a kernel see what the host
// wrote, and what does a host 32-byte descriptor write cost.
// Build: hipcc --offload-arch=gfx950 -O2 -o scripts/bin/bar_probe scripts/bar_probe.hip -lpthread
#include <hip/hip_runtime.h>
#include <setjmp.h>
#include <signal.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <time.h>
#include <x86intrin.h>

#include <thread>
#include <vector>

static sigjmp_buf jb;
static void on_segv(int) { siglongjmp(jb, 1); }

__global__ void read_back(const uint64_t *p, uint64_t *out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = __hip_atomic_load(p + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

static void probe(const char *name, void *d, size_t bytes) {
  hipPointerAttribute_t at;
  memset(&at, 0, sizeof at);
  hipError_t e = hipPointerGetAttributes(&at, d);
  printf("{\"kind\": \"%s\", \"attr_rc\": %d, \"type\": %d, \"host_ptr\": %s",
         name, (int)e, (int)at.type, at.hostPointer ? "true" : "false");
  uint64_t *h = static_cast<uint64_t *>(at.hostPointer ? at.hostPointer : d);
  struct sigaction sa, old;
  memset(&sa, 0, sizeof sa);
  sa.sa_handler = on_segv;
  sigaction(SIGSEGV, &sa, &old);
  sigaction(SIGBUS, &sa, nullptr);
  int ok = 0;
  if (sigsetjmp(jb, 1) == 0) {
    volatile uint64_t *v = h;
    v[0] = 0x1234;
    ok = v[0] == 0x1234 ? 1 : 2;
  }
  sigaction(SIGSEGV, &old, nullptr);
  sigaction(SIGBUS, &old, nullptr);
  printf(", \"cpu_rw\": %d", ok);
  if (ok) {
    const int n = 4096;  // 32 KB
    for (int i = 0; i < n; i++) __atomic_store_n(h + i, (uint64_t)i * 7 + 1, __ATOMIC_RELAXED);
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    uint64_t *dout = nullptr;
    (void)hipMalloc(&dout, n * 8);
    read_back<<<n / 256, 256>>>(static_cast<uint64_t *>(d), dout, n);
    uint64_t back[n];
    (void)hipMemcpy(back, dout, n * 8, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < n; i++) bad += back[i] != (uint64_t)i * 7 + 1;
    printf(", \"gpu_sees_host_writes\": %s", bad ? "false" : "true");
    // host write cost: 32-byte descriptors (4 words) + a count word
    const int reps = 1 << 16;
    const double t0 = now();
    for (int i = 0; i < reps; i++) {
      uint64_t *q = h + (i % 1024) * 4;
      for (int k = 0; k < 4; k++) __atomic_store_n(q + k, (uint64_t)i, __ATOMIC_RELAXED);
      __atomic_store_n(h + 4096 - 8, (uint64_t)i, __ATOMIC_RELEASE);
    }
    const double t1 = now();
    // the same with an sfence per descriptor (out of the write-combining
    // buffers before the count)
    for (int i = 0; i < reps; i++) {
      uint64_t *q = h + (i % 1024) * 4;
      for (int k = 0; k < 4; k++) __atomic_store_n(q + k, (uint64_t)i, __ATOMIC_RELAXED);
      _mm_sfence();
      __atomic_store_n(h + 4096 - 8, (uint64_t)i, __ATOMIC_RELEASE);
    }
    const double t1s = now();
    printf(", \"host_desc_write_sfence_ns\": %.1f", (t1s - t1) / reps * 1e9);
    // 16 threads, each its own 32 KB, sfence per descriptor
    {
      std::vector<std::thread> th;
      const double a0 = now();
      for (int w = 0; w < 16; w++)
        th.emplace_back([h, w, reps] {
          uint64_t *b = h + 8192 + w * 4096;
          for (int i = 0; i < reps; i++) {
            uint64_t *q = b + (i % 1000) * 4;
            for (int k = 0; k < 4; k++) __atomic_store_n(q + k, (uint64_t)i, __ATOMIC_RELAXED);
            _mm_sfence();
            __atomic_store_n(b + 4096 - 8, (uint64_t)i, __ATOMIC_RELEASE);
          }
        });
      for (auto &x : th) x.join();
      const double a1 = now();
      th.clear();
      for (int w = 0; w < 16; w++)
        th.emplace_back([h, w, reps] {
          uint64_t *b = h + 8192 + w * 4096;
          for (int i = 0; i < reps; i++) {
            uint64_t *q = b + (i % 1000) * 4;
            for (int k = 0; k < 4; k++) __atomic_store_n(q + k, (uint64_t)i, __ATOMIC_RELAXED);
            __atomic_store_n(b + 4096 - 8, (uint64_t)i, __ATOMIC_RELEASE);
          }
        });
      for (auto &x : th) x.join();
      const double a2 = now();
      printf(", \"t16_desc_per_us_sfence\": %.1f, \"t16_desc_per_us\": %.1f",
             16.0 * reps / ((a1 - a0) * 1e6), 16.0 * reps / ((a2 - a1) * 1e6));
    }
    const double t1b = now();
    volatile uint64_t sink = 0;
    for (int i = 0; i < 1024; i++) sink += __atomic_load_n(h + i, __ATOMIC_ACQUIRE);
    const double t2 = now();
    printf(", \"host_desc_write_ns\": %.1f, \"host_read_ns\": %.1f", (t1 - t0) / reps * 1e9,
           (t2 - t1b) / 1024 * 1e9);
    (void)hipFree(dout);
  }
  printf("}\n");
  fflush(stdout);
}

int main() {
  const size_t bytes = 1 << 20;  // (16 threads x 32 KB past the first 64 KB)
  void *d = nullptr;
  if (hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained) == hipSuccess) {
    probe("device_finegrained", d, bytes);
    (void)hipFree(d);
  } else {
    printf("{\"kind\": \"device_finegrained\", \"alloc\": false}\n");
  }
  d = nullptr;
  if (hipExtMallocWithFlags(&d, bytes, hipDeviceMallocUncached) == hipSuccess) {
    probe("device_uncached", d, bytes);
    (void)hipFree(d);
  } else {
    printf("{\"kind\": \"device_uncached\", \"alloc\": false}\n");
  }
  d = nullptr;
  if (hipMalloc(&d, bytes) == hipSuccess) {
    probe("device_plain", d, bytes);
    (void)hipFree(d);
  }
  d = nullptr;
  if (hipHostMalloc(&d, bytes, hipHostMallocMapped | hipHostMallocCoherent) == hipSuccess) {
    probe("host_coherent", d, bytes);
    (void)hipHostFree(d);
  }
  return 0;
}
