// scatter_probe.hip -- can a 32 B window per 2 KB slot be read faster than
// the s2k32 shape's 48.5 G slots/s (profiles/r04_calibration.json)? The
// shape of C4 on 2 KB slots and of ExactMatch on 1500 B frames: per slot,
// bytes 16..47 of its first line, a 2-byte result stored. Not part of
// libbessgpu.
//
//   hipcc --offload-arch=gfx950 -O3 -o scripts/bin/scatter_probe scripts/scatter_probe.hip
//   ./scatter_probe GiB [variant block bpc launches]
//
// Variants (all read the same 32 bytes of every slot, XOR them, store a gate):
//   vec2    lane = slot, two 16 B loads (the r04 s2k32 shape)
//   pair    lanes 2m / 2m+1 load slot m's two chunks: one 32 B request per slot
//           (em_pair_kernel, wm_tags_body PAIR 1)
//   quad64  lanes 4m..4m+3 load slot m's whole first 64 B line: one 64 B
//           request per slot, twice the bytes
//   pairU4  pair, each wave issuing the loads of 4 tiles (256 slots) before
//           it uses any (issue order: all loads first)
//   vec2U4  vec2 over 4 slots per lane, all 8 loads issued first
//   scalar  the wave's 64 slots read with scalar loads (one 32 B scalar load
//           per slot, uniform address, through the scalar cache, not the
//           vector L1), the result moved to the slot's lane
//   mixS8 / mixS16 / mixS32  pair loads for 56 / 48 / 32 slots of each tile,
//           scalar loads for the other 8 / 16 / 32 (the two request paths
//           side by side)
// Without arguments: every variant at 256-, 512- and 1024-thread blocks and
// 1, 2, 4, 8 workgroups per CU (whole-residency grids beyond fall back to
// the grid-stride loop), one JSON line each: median ms of 5 rounds of 20
// launches on each of three separately allocated slabs (ms_by_slab; ms and
// G slots/s from the fastest). With `variant block bpc launches`: that many
// launches of one configuration on the first slab, untimed (rocprofv3 --pmc
// passes).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));
typedef const __attribute__((address_space(4))) u32x8 *cptr8;

constexpr uint32_t kSlot = 2048, kOff = 16;

__device__ __forceinline__ u32x4 ldnt(const u32x4 *p) { return __builtin_nontemporal_load(p); }

// slot s's two chunks (u32x4 index of chunk 0)
__device__ __forceinline__ size_t chunk0(size_t s) { return s * (kSlot / 16) + kOff / 16; }

__global__ void vec2(const u32x4 *src, size_t nslots, uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += step) {
    const u32x4 a = ldnt(src + chunk0(i)), b = ldnt(src + chunk0(i) + 1);
    __builtin_nontemporal_store((uint16_t)(a.x ^ a.w ^ b.y ^ b.z), gates + i);
  }
}

template <int U>
__global__ void vec2u(const u32x4 *src, size_t nslots, uint16_t *gates) {
  const size_t step = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += step * U) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t s = i + u * step;
      a[u] = b[u] = u32x4{0, 0, 0, 0};
      if (s < nslots) a[u] = ldnt(src + chunk0(s)), b[u] = ldnt(src + chunk0(s) + 1);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t s = i + u * step;
      if (s < nslots)
        __builtin_nontemporal_store((uint16_t)(a[u].x ^ a[u].w ^ b[u].y ^ b[u].z), gates + s);
    }
  }
}

// tiles of 64 slots per wave; lane l loads chunk (l & 1) of slot (l >> 1)
// (+32 for the second load): one 32 B request per slot. U tiles' loads are
// issued before any is used. The gate of slot m is stored by lane 2m, m < 32
// (first load) and by lane 2(m - 32) + ... : lanes 2m' store slots m' and
// m' + 32.
template <int U>
__global__ void pair(const u32x4 *src, size_t nslots, uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  const size_t ntiles = nslots / 64;
  for (size_t t = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles;
       t += nw * U) {
    u32x4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t tt = t + u * nw;
      a[u] = b[u] = u32x4{0, 0, 0, 0};
      if (tt < ntiles) {
        const size_t s0 = tt * 64 + (lane >> 1);
        a[u] = ldnt(src + chunk0(s0) + (lane & 1));
        b[u] = ldnt(src + chunk0(s0 + 32) + (lane & 1));
      }
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t tt = t + u * nw;
      // the partner lane's half of the window
      const uint32_t xa = a[u].x ^ a[u].w, xb = b[u].y ^ b[u].z;
      const uint32_t ya = __shfl_xor(xa, 1), yb = __shfl_xor(xb, 1);
      if (tt < ntiles && (lane & 1) == 0) {
        const size_t s0 = tt * 64 + (lane >> 1);
        __builtin_nontemporal_store((uint16_t)(xa ^ ya), gates + s0);
        __builtin_nontemporal_store((uint16_t)(xb ^ yb), gates + s0 + 32);
      }
    }
  }
}

// lanes 4m..4m+3 load slot m's first 64 B (16 slots per load, 4 loads per tile)
__global__ void quad64(const u32x4 *src, size_t nslots, uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  const size_t ntiles = nslots / 64;
  for (size_t t = (size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); t < ntiles;
       t += nw) {
    u32x4 v[4];
#pragma unroll
    for (int c = 0; c < 4; c++)
      v[c] = ldnt(src + (t * 64 + c * 16 + (lane >> 2)) * (kSlot / 16) + (lane & 3));
#pragma unroll
    for (int c = 0; c < 4; c++) {
      uint32_t x = v[c].x ^ v[c].w;
      x ^= __shfl_xor(x, 1);
      x ^= __shfl_xor(x, 2);
      if ((lane & 3) == 0)
        __builtin_nontemporal_store((uint16_t)x, gates + t * 64 + c * 16 + (lane >> 2));
    }
  }
}

// S of each tile's 64 slots by scalar loads (slots 64 - S .. 63), the rest
// by pair loads. S = 64: scalar only.
template <int S>
__global__ void mix(const u32x4 *src, size_t nslots, uint16_t *gates) {
  const int lane = threadIdx.x & 63;
  const size_t nw = (size_t)gridDim.x * (blockDim.x >> 6);
  const size_t ntiles = nslots / 64;
  const uint8_t *bytes = reinterpret_cast<const uint8_t *>(src);
  for (size_t t = (size_t)__builtin_amdgcn_readfirstlane(
           (uint32_t)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
       t < ntiles; t += nw) {
    constexpr int V = 64 - S;  // vector slots
    u32x4 a = u32x4{0, 0, 0, 0}, b = a;
    const int m = lane >> 1;
    if (V > 0 && m < V) a = ldnt(src + chunk0(t * 64 + m) + (lane & 1));
    if (V > 32 && m + 32 < V) b = ldnt(src + chunk0(t * 64 + m + 32) + (lane & 1));
    uint32_t mine = 0;  // this lane's scalar slot's result (lane 64 - S + j)
#pragma unroll
    for (int g = 0; g < S; g += 8) {  // 8 scalar loads in flight (64 SGPRs)
      u32x8 w[8];
#pragma unroll
      for (int j = 0; j < 8; j++)
        w[j] = *(cptr8)(bytes + (t * 64 + V + g + j) * kSlot + kOff);
#pragma unroll
      for (int j = 0; j < 8; j++) {
        const uint32_t x = w[j][0] ^ w[j][3] ^ w[j][5] ^ w[j][6];
        mine = lane == V + g + j ? x : mine;
      }
    }
    if (S > 0 && lane >= V) __builtin_nontemporal_store((uint16_t)mine, gates + t * 64 + lane);
    const uint32_t xa = a.x ^ a.w, xb = b.y ^ b.z;
    const uint32_t ya = __shfl_xor(xa, 1), yb = __shfl_xor(xb, 1);
    if ((lane & 1) == 0) {
      if (m < V) __builtin_nontemporal_store((uint16_t)(xa ^ ya), gates + t * 64 + m);
      if (m + 32 < V) __builtin_nontemporal_store((uint16_t)(xb ^ yb), gates + t * 64 + m + 32);
    }
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
struct Var {
  const char *name;
  Kern k;
};

int main(int argc, char **argv) {
  const double gib = argc > 1 ? atof(argv[1]) : 16.0;
  const size_t bytes = ((size_t)(gib * (1 << 30)) / (64 * kSlot)) * (64 * kSlot);
  const size_t nslots = bytes / kSlot;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  // three slabs: a scattered read's rate depends on the physical pages an
  // allocation gets, so every shape is timed on each
  constexpr int kSlabs = 3;
  u32x4 *slabs[kSlabs];
  uint16_t *gates;
  for (int i = 0; i < kSlabs; i++) {
    CK(hipMalloc(&slabs[i], bytes));
    CK(hipMemset(slabs[i], 0x5a, bytes));
  }
  CK(hipMalloc(&gates, nslots * 2));
  u32x4 *src = slabs[0];
  const Var vars[] = {{"vec2", vec2},          {"pair", pair<1>},         {"quad64", quad64},
                      {"pairU4", pair<4>},      {"vec2U4", vec2u<4>},      {"scalar", mix<64>},
                      {"mixS8", mix<8>},        {"mixS16", mix<16>},       {"mixS32", mix<32>}};
  const int nv = sizeof(vars) / sizeof(vars[0]);
  const bool one = argc > 5;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int v = 0; v < nv; v++) {
    if (one && strcmp(argv[2], vars[v].name)) continue;
    for (int block : {256, 512, 1024}) {
      if (one && block != atoi(argv[3])) continue;
      int occ = 0;
      CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, vars[v].k, block, 0));
      for (int bpc : {1, 2, 4, 8}) {
        if (one && bpc != atoi(argv[4])) continue;
        if (!one && bpc > occ && bpc > 1) continue;
        const int blocks = cus * bpc;
        auto launch = [&]() {
          hipLaunchKernelGGL(vars[v].k, dim3(blocks), dim3(block), 0, 0, src, nslots, gates);
        };
        if (one) {
          for (int w = 0; w < atoi(argv[5]); w++) launch();
          CK(hipDeviceSynchronize());
          printf("{\"variant\": \"%s\", \"block\": %d, \"bpc\": %d, \"launches\": %s}\n",
                 vars[v].name, block, bpc, argv[5]);
          continue;
        }
        float per[kSlabs];
        for (int sl = 0; sl < kSlabs; sl++) {
          src = slabs[sl];
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
        src = slabs[0];
        const float best = *std::min_element(per, per + kSlabs);
        printf("{\"variant\": \"%s\", \"block\": %d, \"bpc\": %d, \"occupancy\": %d, "
               "\"ms\": %.4f, \"Gslots\": %.2f, \"slots\": %zu, \"ms_by_slab\": [%.4f, %.4f, %.4f]}\n",
               vars[v].name, block, bpc, occ, best, nslots / (best * 1e-3) / 1e9, nslots,
               per[0], per[1], per[2]);
        fflush(stdout);
      }
    }
  }
  CK(hipGetLastError());
  return 0;
}
