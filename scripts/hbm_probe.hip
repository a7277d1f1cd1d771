// hbm_probe.hip -- calibration of the HBM read roofline on the box, for the
// access shapes the classify kernels use (not part of libbessgpu).
//
//   hipcc --offload-arch=gfx950 -O3 -o hbm_probe scripts/hbm_probe.hip
//   ./hbm_probe [GiB]
//
// Shapes over one resident slab of 64-byte packet slots:
//   full16  : every byte, 16 B per lane per load, lanes contiguous
//   em32    : bytes 16..47 of every 64 B slot (two 16 B loads per lane, lane
//             = slot) + one 2-byte store per slot -- the C2 ExactMatch shape
//   slot64  : all 64 B of every slot (four 16 B loads per lane, lane = slot)
//   half32  : bytes 16..47 of every slot, two lanes per slot, lanes contiguous
// Write shapes (`./hbm_probe GiB w`; TB/s of bytes written):
//   wfull16 : every byte, 16 B per lane per store, lanes contiguous
//   w64s192 : 64 B at +128 of every 192 B slot, 4 lanes per slot (the
//             Rewrite bench's shape: a 60 B template in 32 B blocks)
//   w64s128 : 64 B at +64 of every 128 B slot (one half line per slot)
// Prints one JSON line per (shape, blocks/CU) with sustained TB/s of slab
// bytes read (median of 5 rounds of 20 back-to-back launches).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldnt(const u32x4 *p) {
  return __builtin_nontemporal_load(p);
}

__global__ __launch_bounds__(512) void full16(const u32x4 *src, size_t n16,
                                              uint32_t *sink) {
  uint32_t acc = 0;
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += step) {
    u32x4 v = ldnt(src + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

__global__ __launch_bounds__(512) void em32(const u32x4 *src, size_t nslots,
                                            uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots;
       i += step) {
    u32x4 a = ldnt(src + 4 * i + 1), b = ldnt(src + 4 * i + 2);
    gates[i] = (uint16_t)(a.x ^ a.w ^ b.y ^ b.z);
  }
}

__global__ __launch_bounds__(512) void slot64(const u32x4 *src, size_t nslots,
                                              uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots;
       i += step) {
    u32x4 a = ldnt(src + 4 * i), b = ldnt(src + 4 * i + 1),
          c = ldnt(src + 4 * i + 2), d = ldnt(src + 4 * i + 3);
    gates[i] = (uint16_t)(a.x ^ b.w ^ c.y ^ d.z);
  }
}

// bytes 16..47 of every slot with lane-paired loads: lanes 2j, 2j+1 read
// chunks 1 and 2 of slot j (32 contiguous bytes per slot, the other 32
// skipped) -- the ExactMatch 5-tuple window only
__global__ __launch_bounds__(512) void half32(const u32x4 *src, size_t nslots,
                                              uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < nslots * 2;
       u += step) {
    const size_t slot = u >> 1;
    u32x4 a = ldnt(src + 4 * slot + 1 + (u & 1));
    const uint32_t x = a.x ^ a.w;
    if ((u & 1) == 0) gates[slot] = (uint16_t)x;
  }
}

__global__ __launch_bounds__(512) void wfull16(u32x4 *dst, size_t n16) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += step)
    dst[i] = u32x4{(uint32_t)i, 1u, 2u, 3u};
}

// 64 B of every `slot`-byte slot at offset `off`: lane u writes chunk u & 3
// of slot u >> 2
__global__ __launch_bounds__(512) void w64(u32x4 *dst, size_t nslots, uint32_t slot,
                                           uint32_t off) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t u = (size_t)blockIdx.x * blockDim.x + threadIdx.x; u < nslots * 4;
       u += step)
    dst[((u >> 2) * slot + off) / 16 + (u & 3)] = u32x4{(uint32_t)u, 1u, 2u, 3u};
}

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));             \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 1.0;
  const size_t bytes = (size_t)(gib * (1 << 30)) & ~(size_t)63;
  const size_t nslots = bytes / 64;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *src;
  uint16_t *gates;
  uint32_t *sink;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&gates, nslots * 2));
  CK(hipMalloc(&sink, 4096));
  CK(hipMemset(src, 0x5a, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const bool wr = argc > 2 && argv[2][0] == 'w';
  const char *names[7] = {"full16", "em32", "slot64", "half32",
                          "wfull16", "w64s192", "w64s128"};
  for (int shape = wr ? 4 : 0; shape < (wr ? 7 : 4); shape++) {
    for (int bpc : {1, 2, 4, 8}) {
      const int blocks = cus * bpc;
      double moved = (double)bytes;  // bytes read or written per launch
      if (shape == 5) moved = (double)(bytes / 192) * 64;
      if (shape == 6) moved = (double)(bytes / 128) * 64;
      auto launch = [&]() {
        if (shape == 0)
          hipLaunchKernelGGL(full16, dim3(blocks), dim3(512), 0, 0, src,
                             bytes / 16, sink);
        else if (shape == 1)
          hipLaunchKernelGGL(em32, dim3(blocks), dim3(512), 0, 0, src, nslots,
                             gates);
        else if (shape == 2)
          hipLaunchKernelGGL(slot64, dim3(blocks), dim3(512), 0, 0, src,
                             nslots, gates);
        else if (shape == 3)
          hipLaunchKernelGGL(half32, dim3(blocks), dim3(512), 0, 0, src,
                             nslots, gates);
        else if (shape == 4)
          hipLaunchKernelGGL(wfull16, dim3(blocks), dim3(512), 0, 0, src, bytes / 16);
        else if (shape == 5)
          hipLaunchKernelGGL(w64, dim3(blocks), dim3(512), 0, 0, src, bytes / 192,
                             192u, 128u);
        else
          hipLaunchKernelGGL(w64, dim3(blocks), dim3(512), 0, 0, src, bytes / 128,
                             128u, 64u);
      };
      for (int w = 0; w < 20; w++) launch();
      CK(hipDeviceSynchronize());
      std::vector<float> ms;
      for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < 20; k++) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t / 20);
      }
      std::sort(ms.begin(), ms.end());
      const double t = ms[2] * 1e-3;
      printf("{\"shape\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, "
             "\"TBps\": %.3f}\n",
             names[shape], bpc, ms[2], moved / t / 1e12);
      fflush(stdout);
    }
  }
  return 0;
}
