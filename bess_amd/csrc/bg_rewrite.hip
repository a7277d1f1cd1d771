// bg_rewrite.hip -- gfx950 kernel for Rewrite::ProcessBatch
// (core/modules/rewrite.cc:72-113): every packet's data becomes a template,
// round robin from the module's turn. Pure HBM writes: a packet takes
// 2^lpp_log2 lanes (the next power of two of its largest template's 16-byte
// chunks, <= 64; larger templates loop), each lane storing whole 16-byte
// chunks read from the templates (48 KB at most, L2-resident), so a wave
// writes 64 contiguous chunks of one or several packets per store.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "bg_kernels.h"
#include "bg_launch.h"

namespace bg {
namespace {

constexpr int kRwBlock = 256;

typedef unsigned int rw_u32x4 __attribute__((ext_vector_type(4)));

// NT: streaming (nontemporal) stores for the templates and the metadata
// (A/B build: BG_RW_NT)
template <int NT>
__global__ __launch_bounds__(kRwBlock) void rewrite_kernel(RewriteArgs a) {
  const uint32_t lpp = 1u << a.lpp_log2;
  const uint64_t lane_g = (uint64_t)blockIdx.x * kRwBlock + threadIdx.x;
  const uint64_t step = ((uint64_t)gridDim.x * kRwBlock) >> a.lpp_log2;  // packets
  const uint32_t sub = (uint32_t)lane_g & (lpp - 1);
  uint64_t i = lane_g >> a.lpp_log2;
  // the template index advances by step % ntempl per iteration: one 64-bit
  // modulo per thread, not per packet
  uint32_t t = (uint32_t)((a.start + i) % a.ntempl);
  const uint32_t tstep = (uint32_t)(step % a.ntempl);
  for (; i < a.n; i += step, t = t + tstep >= a.ntempl ? t + tstep - a.ntempl : t + tstep) {
    const uint32_t size = a.tsize[t];
    const uint32_t chunks = ((size + 31) & ~31u) / 16;
    const uint4 *src = reinterpret_cast<const uint4 *>(a.tmpl + (uint64_t)t * kRwMaxSize);
    uint4 *dst = reinterpret_cast<uint4 *>(a.slots + i * a.stride + a.headroom);
    for (uint32_t c = sub; c < chunks; c += lpp) {
      if (NT) {
        const uint4 v = src[c];
        const rw_u32x4 x = {v.x, v.y, v.z, v.w};
        __builtin_nontemporal_store(x, reinterpret_cast<rw_u32x4 *>(dst + c));
      } else {
        dst[c] = src[c];
      }
    }
    if (sub == 0) {
      if (NT) {
        __builtin_nontemporal_store((uint16_t)a.headroom, a.head + i);
        __builtin_nontemporal_store(size, a.len + i);
      } else {
        a.head[i] = (uint16_t)a.headroom;
        a.len[i] = size;
      }
    }
  }
}

}  // namespace

hipError_t launch_rewrite(const RewriteArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0 || a.ntempl == 0) return hipSuccess;
  const uint64_t lanes = a.n << a.lpp_log2;
  uint64_t blocks = (lanes + kRwBlock - 1) / kRwBlock;
  const uint64_t cap = (uint64_t)num_cus * std::max(1, knob("BG_RW_BPC", 8));
  if (blocks > cap) blocks = cap;
  auto kern = knob("BG_RW_NT", 0) ? rewrite_kernel<1> : rewrite_kernel<0>;
  hipLaunchKernelGGL(kern, dim3((unsigned)blocks), dim3(kRwBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bg
