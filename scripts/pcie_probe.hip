// pcie_probe.hip -- what the host link carries on this box: the practical
// ceiling the host end-to-end legs are placed against, beside
// the 63 GB/s PCIe Gen5 x16 spec figure. Not part of libbessgpu.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/pcie_probe scripts/pcie_probe.hip
//   ./pcie_probe [MiB]      (256 MiB by default)
//
// Shapes, each the best of 5 timed repetitions (HIP events):
//   h2d_copy      hipMemcpyAsync host (pinned) -> device, the DMA engines
//   d2h_copy      hipMemcpyAsync device -> host (pinned)
//   zc_read16     a kernel reading pinned host memory in place with
//                 lane-contiguous 16 B loads (the zero-copy checksum pipes'
//                 access), one sum per lane written to device memory
//   zc_read1500   the same over 1504 B of every 2048 B slot (the pooled
//                 L4Checksum's frames)
//   zc_read1500r  1504 B of every 2624 B snbuf at +512 (the pool's layout)
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// slot s covers bytes [s * stride + off, + len) of src; a wave per slot,
// 16 B per lane per step
__global__ __launch_bounds__(256) void zc_read(const u32x4 *src, size_t nslots, size_t stride,
                                               size_t off, size_t len, uint32_t *out) {
  const int lane = threadIdx.x & 63;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint32_t acc = 0;
  for (size_t s = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; s < nslots; s += nw) {
    const u32x4 *p = src + (s * stride + off) / 16;
    for (size_t u = lane; u < len / 16; u += 64) {
      const u32x4 v = __builtin_nontemporal_load(p + u);
      acc += v.x ^ v.y ^ v.z ^ v.w;
    }
  }
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

int main(int argc, char **argv) {
  const size_t mib = argc > 1 ? (size_t)atoi(argv[1]) : 256;
  const size_t bytes = mib << 20;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  void *h = nullptr, *d = nullptr;
  CK(hipHostMalloc(&h, bytes, hipHostMallocDefault));
  memset(h, 0x5a, bytes);
  CK(hipMalloc(&d, bytes));
  uint32_t *out = nullptr;
  const int blocks = cus * 8;
  CK(hipMalloc(&out, (size_t)blocks * 256 * 4));
  void *hd = nullptr;  // the device address of the pinned buffer
  CK(hipHostGetDevicePointer(&hd, h, 0));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto best_ms = [&](auto launch) {
    launch();
    CK(hipDeviceSynchronize());
    std::vector<float> ms;
    for (int r = 0; r < 5; r++) {
      CK(hipEventRecord(e0, 0));
      launch();
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms.push_back(t);
    }
    return *std::min_element(ms.begin(), ms.end());
  };
  auto report = [&](const char *name, double moved, float ms) {
    printf("{\"shape\": \"%s\", \"bytes\": %.0f, \"ms\": %.4f, \"GBps\": %.2f, "
           "\"frac_of_63GBps\": %.3f}\n",
           name, moved, ms, moved / (ms * 1e-3) / 1e9, moved / (ms * 1e-3) / 1e9 / 63.0);
    fflush(stdout);
  };
  float ms = best_ms([&] { CK(hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, 0)); });
  report("h2d_copy", (double)bytes, ms);
  ms = best_ms([&] { CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0)); });
  report("d2h_copy", (double)bytes, ms);
  struct Z {
    const char *name;
    size_t stride, off, len;
  } zs[] = {{"zc_read16", 1024, 0, 1024}, {"zc_read1500", 2048, 0, 1504},
            {"zc_read1500r", 2624, 512, 1504}};
  for (auto &z : zs) {
    const size_t nslots = bytes / z.stride;
    ms = best_ms([&] {
      hipLaunchKernelGGL(zc_read, dim3(blocks), dim3(256), 0, 0,
                         reinterpret_cast<const u32x4 *>(hd), nslots, z.stride, z.off, z.len,
                         out);
    });
    report(z.name, (double)nslots * z.len, ms);
  }
  CK(hipGetLastError());
  return 0;
}
