# Rewrite: the templates (ntempl x units 16 B chunks) and their sizes staged
# in LDS once per workgroup, so a packet's size and chunks are LDS reads
# instead of two dependent L2 reads. RW_BPC (8) caps workgroups per CU.
import os
BPC = int(os.environ.get("RW_BPC", "8"))
U = int(os.environ.get("RW_UNROLL", "1"))  # packets per thread per pass, loads first
p = 'bess_amd/csrc/bg_rewrite.hip'
s = open(p).read()
a = s[s.index("__global__ __launch_bounds__(kRwBlock) void rewrite_kernel(RewriteArgs a) {"):
      s.index("}  // namespace\n")]
b = """__global__ __launch_bounds__(kRwBlock) void rewrite_kernel(RewriteArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint4 lt[];  // ntempl x units
  uint32_t *lsz = reinterpret_cast<uint32_t *>(lt + (size_t)a.ntempl * a.units);
  for (uint32_t u = threadIdx.x; u < a.ntempl * a.units; u += kRwBlock) {
    const uint32_t tt = u / a.units, c = u % a.units;
    lt[u] = reinterpret_cast<const uint4 *>(a.tmpl + (uint64_t)tt * kRwMaxSize)[c];
  }
  for (uint32_t tt = threadIdx.x; tt < a.ntempl; tt += kRwBlock) lsz[tt] = a.tsize[tt];
  __syncthreads();
  const uint32_t lpp = 1u << a.lpp_log2;
  const uint64_t lane_g = (uint64_t)blockIdx.x * kRwBlock + threadIdx.x;
  const uint64_t step = ((uint64_t)gridDim.x * kRwBlock) >> a.lpp_log2;  // packets
  const uint32_t sub = (uint32_t)lane_g & (lpp - 1);
  uint64_t i = lane_g >> a.lpp_log2;
  uint32_t t = (uint32_t)((a.start + i) % a.ntempl);
  const uint32_t tstep = (uint32_t)(step % a.ntempl);
  auto adv = [&](uint32_t x) { return x + tstep >= a.ntempl ? x + tstep - a.ntempl : x + tstep; };
  if (a.units <= lpp) {  // one chunk per lane per packet: U packets per pass, loads first
    constexpr int U = @U@;
    for (; i < a.n; i += step * U) {
      uint32_t sz[U];
      uint4 x[U];
#pragma unroll
      for (int k = 0; k < U; k++) {
        sz[k] = lsz[t];
        x[k] = lt[(size_t)t * a.units + (sub < a.units ? sub : 0)];
        t = adv(t);
      }
#pragma unroll
      for (int k = 0; k < U; k++) {
        const uint64_t ii = i + (uint64_t)k * step;
        if (ii >= a.n) break;
        const uint32_t chunks = ((sz[k] + 31) & ~31u) / 16;
        uint4 *dst = reinterpret_cast<uint4 *>(a.slots + ii * a.stride + a.headroom);
        if (sub < chunks) dst[sub] = x[k];
        if (sub == 0) {
          a.head[ii] = (uint16_t)a.headroom;
          a.len[ii] = sz[k];
        }
      }
    }
    return;
  }
  for (; i < a.n; i += step, t = adv(t)) {
    const uint32_t size = lsz[t];
    const uint32_t chunks = ((size + 31) & ~31u) / 16;
    const uint4 *src = lt + (size_t)t * a.units;
    uint4 *dst = reinterpret_cast<uint4 *>(a.slots + i * a.stride + a.headroom);
    for (uint32_t c = sub; c < chunks; c += lpp) dst[c] = src[c];
    if (sub == 0) {
      a.head[i] = (uint16_t)a.headroom;
      a.len[i] = size;
    }
  }
}

""".replace("@U@", str(U))
s = s.replace(a, b)
a = """  const uint64_t cap = (uint64_t)num_cus * 8;
  if (blocks > cap) blocks = cap;
  hipLaunchKernelGGL(rewrite_kernel, dim3((unsigned)blocks), dim3(kRwBlock), 0, s, a);"""
b = """  const uint64_t cap = (uint64_t)num_cus * %d;
  if (blocks > cap) blocks = cap;
  const size_t lds = (size_t)a.ntempl * a.units * 16 + (size_t)a.ntempl * 4;
  hipLaunchKernelGGL(rewrite_kernel, dim3((unsigned)blocks), dim3(kRwBlock), lds, s, a);""" % BPC
assert s.count(a) == 1
s = s.replace(a, b)
open(p, 'w').write(s)
