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
    // (streaming stores measured slower: 0.391 against 0.372 ms,
    // profiles/r05/rewrite_nt_r05o.json)
    for (uint32_t c = sub; c < chunks; c += lpp) dst[c] = src[c];
    if (sub == 0) {
      a.head[i] = (uint16_t)a.headroom;
      a.len[i] = size;
    }
  }
}

}  // namespace

hipError_t launch_rewrite(const RewriteArgs &a, int num_cus, hipStream_t s) {
  if (a.n == 0 || a.ntempl == 0) return hipSuccess;
  const uint64_t lanes = a.n << a.lpp_log2;
  uint64_t blocks = (lanes + kRwBlock - 1) / kRwBlock;
  const uint64_t cap = (uint64_t)num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(rewrite_kernel, dim3((unsigned)blocks), dim3(kRwBlock), 0, s, a);
  return hipGetLastError();
}

}  // namespace bg
