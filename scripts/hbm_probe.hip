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
// Scattered read shapes (`./hbm_probe GiB s`; TB/s of the 66 B/packet
// algorithmic basis, and Gpkts/s):
//   s2k32   : bytes 16..47 of every 2048 B slot (two 16 B loads per lane,
//             lane = slot) + a 2-byte store -- C4's header window in 2 KB
//             IMIX slots
//   s2k64   : bytes 0..63 of every 2048 B slot (four 16 B loads)
//   rnd36   : the em32 stream over 64 B slots + per packet one random 4 B
//             read from a 4 MiB tag region and, for half the packets, one
//             random 16 B read from a 32 MiB key region -- C5's 1 M-rule
//             ExactMatch probe shape (36 MB table)
//   rnd36s  : the same random reads behind the C5 kernel's own stream: a
//             wave reads its 64 slots (4 KB) with four lane-contiguous 16 B
//             loads (em_slab_kernel's shape), lane l then makes slot l's
//             random reads with a hash of the data it loaded
// Line-op shapes (`./hbm_probe GiB c`; TB/s of the 66 / 130 B/packet basis):
//   slab66  : em_slab_kernel's / line_slab_kernel's memory traffic alone --
//             a wave reads its 64 slots (4 KB) with four lane-contiguous
//             16 B loads and lane l stores slot l's 2-byte gate (no LDS, no
//             lookup): the ceiling of C2 and the header-line ops
//   slab130 : the same tile read, every line stored back in place (lane-
//             contiguous 16 B stores) and the gates: UpdateTTL's / StaticNAT's
//             traffic (130 B/packet basis)
//   ck1502  : the 94 16 B chunks of each 2048 B slot's 1496 B frame as one
//             lane-contiguous stream, two 2-byte words stored in place per
//             slot: C3's checksum traffic (1502 B basis)
//   slab66c : slab66 with each wave taking runs of 8 consecutive tiles
//   slab66g : slab66c with the run's 512 gates gathered in LDS and stored as
//             one 1 KB block (16 B per lane)
// `./hbm_probe GiB only SHAPE BLOCKS_PER_CU LAUNCHES` runs one shape (for
// rocprofv3 --pmc passes: FETCH_SIZE per launch against a known shape).
// Prints one JSON line per (shape, blocks/CU) with sustained TB/s of slab
// bytes read (median of 5 rounds of 20 back-to-back launches).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

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

// bytes [off, off + 16 * nch) of every 2048 B slot, lane = slot
template <int NCH, int OFF>
__global__ __launch_bounds__(512) void s2k(const u32x4 *src, size_t nslots,
                                           uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots;
       i += step) {
    uint32_t x = 0;
#pragma unroll
    for (int c = 0; c < NCH; c++) {
      const u32x4 a = ldnt(src + 128 * i + OFF / 16 + c);
      x ^= a.x ^ a.w;
    }
    gates[i] = (uint16_t)x;
  }
}

__device__ __forceinline__ uint32_t mix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  return h ^ (h >> 16);
}

// em32 + a random tag word (4 MiB) + for half the packets a random 16 B key
// (32 MiB): the C5 probe shape. tab: 36 MiB.
__global__ __launch_bounds__(512) void rnd36(const u32x4 *src, size_t nslots,
                                             const uint32_t *tab, uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  const u32x4 *keys = reinterpret_cast<const u32x4 *>(tab + (1u << 20));
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots;
       i += step) {
    const u32x4 a = ldnt(src + 4 * i + 1), b = ldnt(src + 4 * i + 2);
    const uint32_t h = mix32((uint32_t)i ^ a.x ^ b.z);
    uint32_t x = tab[h & ((1u << 20) - 1)];
    if (h >> 31) {
      const u32x4 k = keys[(h >> 8) & ((1u << 21) - 1)];
      x ^= k.x ^ k.w;
    }
    gates[i] = (uint16_t)x;
  }
}

// rnd36 with em_slab_kernel's load shape (nslots: a multiple of 64)
__global__ __launch_bounds__(512) void rnd36s(const u32x4 *src, size_t nslots,
                                              const uint32_t *tab, uint16_t *gates) {
  const u32x4 *keys = reinterpret_cast<const u32x4 *>(tab + (1u << 20));
  const int lane = threadIdx.x & 63;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t * 64 < nslots;
       t += nwaves) {
    const u32x4 *g = src + t * 256;
    const u32x4 a = ldnt(g + lane), b = ldnt(g + 64 + lane), c = ldnt(g + 128 + lane),
                d = ldnt(g + 192 + lane);
    const uint32_t h = mix32((uint32_t)(t * 64 + lane) ^ a.x ^ b.y ^ c.z ^ d.w);
    uint32_t x = tab[h & ((1u << 20) - 1)];
    if (h >> 31) {
      const u32x4 k = keys[(h >> 8) & ((1u << 21) - 1)];
      x ^= k.x ^ k.w;
    }
    gates[t * 64 + lane] = (uint16_t)x;
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

// rnd36s's stream without the random reads (nslots: a multiple of 64)
__global__ __launch_bounds__(512) void slab66(const u32x4 *src, size_t nslots,
                                              uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t * 64 < nslots;
       t += nwaves) {
    const u32x4 *g = src + t * 256;
    const u32x4 a = ldnt(g + lane), b = ldnt(g + 64 + lane), c = ldnt(g + 128 + lane),
                d = ldnt(g + 192 + lane);
    gates[t * 64 + lane] = (uint16_t)(a.x ^ b.y ^ c.z ^ d.w);
  }
}

// slab66 with each wave taking runs of 8 consecutive tiles (512 slots,
// 32 KB); GW = 1: the 8 tiles' gates gathered in LDS and stored as one
// 1 KB block (16 B per lane), GW = 0: stored per tile as slab66 does
template <int GW>
__global__ __launch_bounds__(512) void slab66g(const u32x4 *src, size_t nslots,
                                               uint16_t *gates) {
  __shared__ uint16_t gl[8][512];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t r = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; r * 512 < nslots;
       r += nwaves) {
#pragma unroll 1
    for (int k = 0; k < 8; k++) {
      const size_t t = r * 8 + k;
      const u32x4 *g = src + t * 256;
      const u32x4 a = ldnt(g + lane), b = ldnt(g + 64 + lane), c = ldnt(g + 128 + lane),
                  d = ldnt(g + 192 + lane);
      const uint16_t x = (uint16_t)(a.x ^ b.y ^ c.z ^ d.w);
      if (GW)
        gl[wid][k * 64 + lane] = x;
      else
        gates[t * 64 + lane] = x;
    }
    if (GW) {
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's LDS writes
      reinterpret_cast<u32x4 *>(gates + r * 512)[lane] =
          reinterpret_cast<const u32x4 *>(gl[wid])[lane];
    }
  }
}

// slab66 with every line written back (in place)
__global__ __launch_bounds__(512) void slab130(u32x4 *src, size_t nslots, uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nwaves = ((size_t)gridDim.x * blockDim.x) >> 6;
  for (size_t t = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; t * 64 < nslots;
       t += nwaves) {
    u32x4 *g = src + t * 256;
    u32x4 a = ldnt(g + lane), b = ldnt(g + 64 + lane), c = ldnt(g + 128 + lane),
          d = ldnt(g + 192 + lane);
    a.x ^= 1u; b.y ^= 1u; c.z ^= 1u; d.w ^= 1u;
    g[lane] = a;
    g[64 + lane] = b;
    g[128 + lane] = c;
    g[192 + lane] = d;
    gates[t * 64 + lane] = (uint16_t)(a.y ^ b.x);
  }
}

// C3's checksum traffic alone: the 94 16-byte chunks covering each 2048 B
// slot's 1496-byte frame, read as one lane-contiguous stream (chunk u of the
// grid = chunk u % 94 of slot u / 94), and two 2-byte words stored in place
// per slot (the IPv4 and UDP checksum fields, offsets 24 and 40)
__global__ __launch_bounds__(512) void ck1502(u32x4 *src, size_t nslots) {
  const uint32_t step = gridDim.x * blockDim.x, total = (uint32_t)(nslots * 94);
  for (uint32_t u = blockIdx.x * blockDim.x + threadIdx.x; u < total; u += step) {
    const uint32_t slot = u / 94u, c = u - slot * 94u;  // (32-bit: a multiply-high)
    const u32x4 a = ldnt(src + (size_t)slot * 128 + c);
    const uint32_t x = a.x ^ a.y ^ a.z ^ a.w;
    uint16_t *f = reinterpret_cast<uint16_t *>(src + (size_t)slot * 128);
    if (c == 1) f[12] = (uint16_t)x;  // bytes 24..25 (chunk 1)
    if (c == 2) f[20] = (uint16_t)x;  // bytes 40..41 (chunk 2)
  }
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
  const bool sc = argc > 2 && argv[2][0] == 's';
  const bool only = argc > 5 && !strcmp(argv[2], "only");
  const bool cs = argc > 2 && argv[2][0] == 'c';
  const char *names[16] = {"full16", "em32",  "slot64", "half32", "wfull16", "w64s192", "w64s128",
                           "s2k32",  "s2k64", "rnd36",  "rnd36s", "slab66",  "slab130", "ck1502",
                           "slab66c", "slab66g"};
  uint32_t *tab = nullptr;
  CK(hipMalloc(&tab, 36u << 20));
  CK(hipMemset(tab, 0x33, 36u << 20));
  int s0 = wr ? 4 : sc ? 7 : cs ? 11 : 0, s1 = wr ? 7 : sc ? 11 : cs ? 16 : 4;
  int only_bpc = 0, only_launches = 0;
  if (only) {
    for (int k = 0; k < 16; k++)
      if (!strcmp(argv[3], names[k])) s0 = k, s1 = k + 1;
    only_bpc = atoi(argv[4]);
    only_launches = atoi(argv[5]);
  }
  for (int shape = s0; shape < s1; shape++) {
    for (int bpc : {1, 2, 4, 8}) {
      if (only && bpc != only_bpc) continue;
      const int blocks = cus * bpc;
      double moved = (double)bytes;  // bytes read or written per launch
      double pkts = (double)nslots;
      if (shape == 5) moved = (double)(bytes / 192) * 64;
      if (shape == 6) moved = (double)(bytes / 128) * 64;
      if (shape == 7 || shape == 8) pkts = (double)(bytes / 2048);
      if (shape == 13) pkts = (double)(bytes / 2048);
      if (shape >= 7) moved = pkts * (shape == 13 ? 1502 : shape == 12 ? 130 : 66);  // the algorithmic basis
      if (shape >= 14 && nslots % 512) continue;  // (whole 512-slot runs only)
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
        else if (shape == 6)
          hipLaunchKernelGGL(w64, dim3(blocks), dim3(512), 0, 0, src, bytes / 128,
                             128u, 64u);
        else if (shape == 7)
          hipLaunchKernelGGL((s2k<2, 16>), dim3(blocks), dim3(512), 0, 0, src,
                             bytes / 2048, gates);
        else if (shape == 8)
          hipLaunchKernelGGL((s2k<4, 0>), dim3(blocks), dim3(512), 0, 0, src,
                             bytes / 2048, gates);
        else if (shape == 9)
          hipLaunchKernelGGL(rnd36, dim3(blocks), dim3(512), 0, 0, src, nslots, tab,
                             gates);
        else if (shape == 10)
          hipLaunchKernelGGL(rnd36s, dim3(blocks), dim3(512), 0, 0, src, nslots, tab,
                             gates);
        else if (shape == 11)
          hipLaunchKernelGGL(slab66, dim3(blocks), dim3(512), 0, 0, src, nslots, gates);
        else if (shape == 12)
          hipLaunchKernelGGL(slab130, dim3(blocks), dim3(512), 0, 0, src, nslots, gates);
        else if (shape == 13)
          hipLaunchKernelGGL(ck1502, dim3(blocks), dim3(512), 0, 0, src, bytes / 2048);
        else if (shape == 14)
          hipLaunchKernelGGL(slab66g<0>, dim3(blocks), dim3(512), 0, 0, src, nslots, gates);
        else
          hipLaunchKernelGGL(slab66g<1>, dim3(blocks), dim3(512), 0, 0, src, nslots, gates);
      };
      if (only) {  // a fixed number of launches, no timing (rocprofv3 passes)
        for (int w = 0; w < only_launches; w++) launch();
        CK(hipDeviceSynchronize());
        printf("{\"shape\": \"%s\", \"launches\": %d, \"pkts\": %.0f}\n", names[shape],
               only_launches, pkts);
        continue;
      }
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
             "\"TBps\": %.3f, \"Gpkts\": %.2f}\n",
             names[shape], bpc, ms[2], moved / t / 1e12, pkts / t / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
