// gate_probe.hip -- C2's access shape (a wave reads its tile of 64 slots,
// 4 KB, with four lane-contiguous 16 B loads; each slot's 2-byte gate is
// stored) with the gate stores placed differently, over three separately
// allocated slabs. Does writing the gates apart from the reads (in bursts
// or at the end) close the gap between the read-only stream and the
// kernel? Not part of libbessgpu.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/gate_probe scripts/gate_probe.hip
//   ./gate_probe [GiB]          (1 GiB: C2's 16 M slots)
//
// Shapes:
//   read64    the tiles' loads only (a result kept per lane, stored once)
//   slab66    + each tile's 64 gates, normal stores (hbm_probe slab66)
//   slab66nt  + each tile's 64 gates, streaming stores (the kernel's)
//   hold16    the gates of 16 consecutive grid-stride tiles held in
//             registers, stored after them (streaming)
//   hold64    the same over 64 tiles: with 4096 waves and 16 M slots every
//             wave's gates leave after its last read
//   hold32 / hold128   the same over 32 / 128 tiles
//   lds64 / lds128     the gates of 64 / 128 tiles held in LDS (a loop that is
//             not unrolled: the classifier's tile body is too large to
//             unroll 64 times), then stored from LDS 16 B per lane
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ u32x4 ldnt(const u32x4 *p) { return __builtin_nontemporal_load(p); }

__device__ __forceinline__ uint16_t tile_x(const u32x4 *src, size_t t, int lane) {
  const u32x4 *g = src + t * 256;
  const u32x4 a = ldnt(g + lane), b = ldnt(g + 64 + lane), c = ldnt(g + 128 + lane),
              d = ldnt(g + 192 + lane);
  return (uint16_t)(a.x ^ b.y ^ c.z ^ d.w);
}

// MODE 0: no gates (one value per lane at the end), 1: normal, 2: streaming
template <int MODE>
__global__ __launch_bounds__(512) void per_tile(const u32x4 *src, size_t ntiles,
                                                uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  const size_t w0 = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  uint32_t acc = 0;
  for (size_t t = w0; t < ntiles; t += nw) {
    const uint16_t x = tile_x(src, t, lane);
    if (MODE == 0)
      acc ^= x;
    else if (MODE == 1)
      gates[t * 64 + lane] = x;
    else
      __builtin_nontemporal_store(x, gates + t * 64 + lane);
  }
  if (MODE == 0) __builtin_nontemporal_store((uint16_t)acc, gates + w0 * 64 + lane);
}

template <int R>
__global__ __launch_bounds__(512) void hold(const u32x4 *src, size_t ntiles, uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t b = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; b < ntiles;
       b += nw * R) {
    uint16_t g[R];
#pragma unroll
    for (int k = 0; k < R; k++) {
      const size_t t = b + (size_t)k * nw;
      g[k] = t < ntiles ? tile_x(src, t, lane) : 0;
    }
#pragma unroll
    for (int k = 0; k < R; k++) {
      const size_t t = b + (size_t)k * nw;
      if (t < ntiles) __builtin_nontemporal_store(g[k], gates + t * 64 + lane);
    }
  }
}

template <int R>
__global__ __launch_bounds__(512) void ldshold(const u32x4 *src, size_t ntiles,
                                               uint16_t *gates) {
  __shared__ __attribute__((aligned(16))) uint16_t held[8][R * 64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const size_t nw = ((size_t)gridDim.x * blockDim.x) >> 6;
  uint16_t *h = held[wid];
  for (size_t b = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; b < ntiles;
       b += nw * R) {
#pragma unroll 1
    for (int k = 0; k < R; k++) {
      const size_t t = b + (size_t)k * nw;
      if (t >= ntiles) break;
      h[k * 64 + lane] = tile_x(src, t, lane);
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave's LDS writes done
    // 16 B per lane: 8 lanes per tile, 8 tiles per store instruction
#pragma unroll
    for (int i = 0; i < R / 8; i++) {
      const int k = i * 8 + (lane >> 3);
      const size_t t = b + (size_t)k * nw;
      if (t < ntiles)
        __builtin_nontemporal_store(reinterpret_cast<const u32x4 *>(h + k * 64)[lane & 7],
                                    reinterpret_cast<u32x4 *>(gates + t * 64) + (lane & 7));
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                  \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

typedef void (*Kern)(const u32x4 *, size_t, uint16_t *);

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 1.0;
  const size_t bytes = ((size_t)(gib * (1 << 30)) / 4096) * 4096;
  const size_t nslots = bytes / 64, ntiles = nslots / 64;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  constexpr int kSlabs = 3;
  u32x4 *slabs[kSlabs];
  for (int i = 0; i < kSlabs; i++) {
    CK(hipMalloc(&slabs[i], bytes));
    CK(hipMemset(slabs[i], 0x5a, bytes));
  }
  uint16_t *gates;
  CK(hipMalloc(&gates, nslots * 2));
  struct V {
    const char *name;
    Kern k;
  } vars[] = {{"read64", per_tile<0>}, {"slab66", per_tile<1>}, {"slab66nt", per_tile<2>},
              {"hold16", hold<16>},     {"hold32", hold<32>},
              {"hold64", hold<64>},     {"hold128", hold<128>},
              {"lds64", ldshold<64>},   {"lds128", ldshold<128>}};
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (auto &v : vars) {
    for (int bpc : {1, 2}) {
      const int blocks = cus * bpc;
      float per[kSlabs];
      for (int sl = 0; sl < kSlabs; sl++) {
        auto launch = [&]() {
          hipLaunchKernelGGL(v.k, dim3(blocks), dim3(512), 0, 0, slabs[sl], ntiles, gates);
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
        per[sl] = ms[2];
      }
      const float best = *std::min_element(per, per + kSlabs);
      printf("{\"shape\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"TBps_66B\": %.3f, "
             "\"ms_by_slab\": [%.4f, %.4f, %.4f], \"pkts\": %zu}\n",
             v.name, bpc, best, nslots * 66.0 / (best * 1e-3) / 1e12, per[0], per[1], per[2],
             nslots);
      fflush(stdout);
    }
  }
  CK(hipGetLastError());
  return 0;
}
