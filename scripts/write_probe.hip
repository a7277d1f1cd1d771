// write_probe.hip -- Rewrite's store shape alone (the 64 B template written
// into every 192 B slot at +128, plus 2 B data_off and 4 B length per
// packet), against plain streaming writes, over 16 M slots: the ceiling
// bench.py's Rewrite leg is placed against. Not part of
// libbessgpu.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/write_probe scripts/write_probe.hip
//   ./write_probe [Mslots]       (16 by default)
//
// Shapes (4 lanes per packet, 16 B per lane, grid-strided as rewrite_kernel):
//   tmpl      the 64 B at +128 of each 192 B slot (one full line in three)
//   tmpl_hl   + the 2 B data_off and 4 B length arrays (Rewrite's stores)
//   dense64   64 B per packet, contiguous (a plain streaming write)
//   dense192  the whole 192 B slot (contiguous; 3x the bytes)
//   tile      tmpl_hl with a wave per 64 consecutive packets: 4 rounds of 16
//             packets' 64 B, then data_off / length of all 64 as whole lines
//   split     tmpl's grid-strided template stores first, then data_off /
//             length grid-strided a lane per packet (whole lines), in one launch
//   kernel    rewrite_kernel's body itself: 4 templates of 60 B read from a
//             4 x 1536 B buffer, sizes from an array, the round-robin turn
// Each: best of 5 x 10 launches per blocks-per-CU setting, GB/s of the
// bytes the shape writes.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

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

// MODE 0 tmpl, 1 tmpl_hl, 2 dense64, 3 dense192
template <int MODE>
__global__ __launch_bounds__(256) void wr(uint4 *slots, uint16_t *head, uint32_t *len,
                                          size_t n) {
  constexpr int kChunks = MODE == 3 ? 12 : 4;  // 16 B chunks per packet
  constexpr int kStride = MODE == 2 ? 4 : 12;  // 16 B units per slot
  constexpr int kOff = MODE <= 1 ? 8 : 0;      // +128 B
  const size_t lane_g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  const uint4 v = make_uint4((uint32_t)lane_g, 1, 2, 3);
  for (size_t u = lane_g; u < n * kChunks; u += lanes) {
    const size_t i = u / kChunks, c = u % kChunks;
    slots[i * kStride + kOff + c] = v;
    if (MODE == 1 && c == 0) {
      head[i] = 128;
      len[i] = 60;
    }
  }
}

__global__ __launch_bounds__(256) void wr_tile(uint4 *slots, uint16_t *head, uint32_t *len,
                                               size_t n) {
  const int lane = threadIdx.x & 63;
  const size_t wave = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const size_t waves = ((size_t)gridDim.x * blockDim.x) >> 6;
  const uint4 v = make_uint4((uint32_t)lane, 1, 2, 3);
  for (size_t tile = wave; tile * 64 < n; tile += waves) {
    const size_t p0 = tile * 64;
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const size_t i = p0 + r * 16 + (lane >> 2);
      if (i < n) slots[i * 12 + 8 + (lane & 3)] = v;
    }
    if (p0 + lane < n) {
      head[p0 + lane] = 128;
      len[p0 + lane] = 60;
    }
  }
}

__global__ __launch_bounds__(256) void wr_split(uint4 *slots, uint16_t *head, uint32_t *len,
                                                size_t n) {
  const size_t lane_g = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  const size_t lanes = (size_t)gridDim.x * blockDim.x;
  const uint4 v = make_uint4((uint32_t)lane_g, 1, 2, 3);
  for (size_t u = lane_g; u < n * 4; u += lanes) slots[(u >> 2) * 12 + 8 + (u & 3)] = v;
  for (size_t i = lane_g; i < n; i += lanes) {
    head[i] = 128;
    len[i] = 60;
  }
}

// rewrite_kernel's loop (bess_amd/csrc/bg_rewrite.hip) on the probe's slab
__global__ __launch_bounds__(256) void wr_kernel(uint4 *slots, uint16_t *head, uint32_t *len,
                                                 size_t n, const uint8_t *tmpl,
                                                 const uint16_t *tsize) {
  constexpr uint32_t ntempl = 4, lpp_log2 = 2, headroom = 128, stride = 192;
  const uint32_t lpp = 1u << lpp_log2;
  const uint64_t lane_g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  const uint64_t step = ((uint64_t)gridDim.x * 256) >> lpp_log2;
  const uint32_t sub = (uint32_t)lane_g & (lpp - 1);
  uint64_t i = lane_g >> lpp_log2;
  uint32_t t = (uint32_t)(i % ntempl);
  const uint32_t tstep = (uint32_t)(step % ntempl);
  uint8_t *base = reinterpret_cast<uint8_t *>(slots);
  for (; i < n; i += step, t = t + tstep >= ntempl ? t + tstep - ntempl : t + tstep) {
    const uint32_t size = tsize[t];
    const uint32_t chunks = ((size + 31) & ~31u) / 16;
    const uint4 *src = reinterpret_cast<const uint4 *>(tmpl + (uint64_t)t * 1536);
    uint4 *dst = reinterpret_cast<uint4 *>(base + i * stride + headroom);
    for (uint32_t c = sub; c < chunks; c += lpp) dst[c] = src[c];
    if (sub == 0) {
      head[i] = (uint16_t)headroom;
      len[i] = size;
    }
  }
}

int main(int argc, char **argv) {
  const size_t n = (size_t)(argc > 1 ? atoi(argv[1]) : 16) << 20;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint4 *slots = nullptr;
  uint16_t *head = nullptr;
  uint32_t *len = nullptr;
  CK(hipMalloc(&slots, n * 192));
  CK(hipMalloc(&head, n * 2));
  CK(hipMalloc(&len, n * 4));
  CK(hipMemset(slots, 0, n * 192));
  uint8_t *tmpl = nullptr;
  uint16_t *tsize = nullptr;
  CK(hipMalloc(&tmpl, 4 * 1536));
  CK(hipMalloc(&tsize, 4 * 2));
  {
    std::vector<uint8_t> h(4 * 1536, 0);
    for (int t = 0; t < 4; t++)
      for (int b = 0; b < 60; b++) h[t * 1536 + b] = (uint8_t)(t * 61 + b);
    const uint16_t sz[4] = {60, 60, 60, 60};
    CK(hipMemcpy(tmpl, h.data(), h.size(), hipMemcpyHostToDevice));
    CK(hipMemcpy(tsize, sz, sizeof sz, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct S {
    const char *name;
    void (*k)(uint4 *, uint16_t *, uint32_t *, size_t);
    double bytes_per_pkt;
  } shapes[] = {{"tmpl", wr<0>, 64}, {"tmpl_hl", wr<1>, 70}, {"dense64", wr<2>, 64},
                {"dense192", wr<3>, 192},
                {"tile", wr_tile, 70}, {"split", wr_split, 70}, {"kernel", nullptr, 70}};
  for (auto &sh : shapes) {
    for (int bpc : {2, 4, 8}) {
      const int blocks = cus * bpc;
      auto launch = [&] {
        if (sh.k)
          hipLaunchKernelGGL(sh.k, dim3(blocks), dim3(256), 0, 0, slots, head, len, n);
        else
          hipLaunchKernelGGL(wr_kernel, dim3(blocks), dim3(256), 0, 0, slots, head, len, n,
                             (const uint8_t *)tmpl, (const uint16_t *)tsize);
      };
      for (int w = 0; w < 10; w++) launch();
      CK(hipDeviceSynchronize());
      std::vector<float> ms;
      for (int r = 0; r < 5; r++) {
        CK(hipEventRecord(e0, 0));
        for (int k = 0; k < 10; k++) launch();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float t = 0;
        CK(hipEventElapsedTime(&t, e0, e1));
        ms.push_back(t / 10);
      }
      const float best = *std::min_element(ms.begin(), ms.end());
      printf("{\"shape\": \"%s\", \"blocks_per_cu\": %d, \"ms\": %.4f, \"GBps\": %.1f, "
             "\"Gpkts_per_s\": %.2f, \"pkts\": %zu}\n",
             sh.name, bpc, best, n * sh.bytes_per_pkt / (best * 1e-3) / 1e9,
             n / (best * 1e-3) / 1e9, n);
      fflush(stdout);
    }
  }
  CK(hipGetLastError());
  return 0;
}
