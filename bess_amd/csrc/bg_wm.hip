// bg_wm.hip -- WildcardMatch::ProcessBatch (core/modules/wildcard_match.cc:
// 159-203, LookupEntry 136-157) for tables whose tag words fit in LDS: the
// ahead-of-time kernels over any table (bg_wm_body.h with WmRuntimeSpec,
// the tuple data read from the kernel arguments). bg_wm_jit.cc compiles the
// same body per rule-set shape with the tuple data as constants.
#include <hip/hip_runtime.h>

#include "bg_launch.h"
#include "bg_wm_body.h"

namespace bg {
namespace {

template <int KW, int NCH, int PAIR>
__global__ __launch_bounds__(kWmBlock) void wm_tags_kernel(WmArgs a) {
  wm_tags_body<WmRuntimeSpec, KW, NCH, PAIR>(a);
}

template <int KW, int NCH, int PAIR>
hipError_t launch_tags(const WmArgs &a, int num_cus, hipStream_t s) {
  const size_t lds = wm_tags_lds_bytes(a.t.nbp, KW);
  const uint64_t ntiles = (a.n + 63) / 64;
  uint64_t blocks = (ntiles + kWaves - 1) / kWaves;
  if (blocks > (uint64_t)num_cus) blocks = (uint64_t)num_cus;
  if (blocks == 0) return hipSuccess;
  hipLaunchKernelGGL((wm_tags_kernel<KW, NCH, PAIR>), dim3((unsigned)blocks),
                     dim3(kWmBlock), lds, s, a);
  return hipGetLastError();
}

}  // namespace

hipError_t launch_wm_tags(const WmArgs &a, int num_cus, hipStream_t s) {
  const bool n2 = fits_nch2(a.fp);
  if (a.fp.direct || a.fp.nch > 4 || a.t.nbp > (1u << 15)) return hipErrorInvalidValue;
  // the pair loads: a window of two chunks inside the slot's first line,
  // lanes 2m / 2m+1 loading slot m's two (one 32 B request per slot per
  // load instead of two 16 B ones): on the dense 64 B slab and, since round
  // 4, on any stride (C4's 2 KB slots 0.319 -> 0.262 ms, same gates,
  // profiles/r04_wm_pair_2k_ab.jsonl)
  // (both chunks inside the slot: no read past a staged row or the slab)
  const bool pair = n2 && a.fp.win_lo % 16 == 0 && a.fp.win_lo + 32 <= 64 &&
                    a.fp.win_lo + 32 <= a.stride && a.stride <= 65536;
  // (measured and not kept, round 5: a streamed form -- producer waves
  // loading the windows into an LDS ring -- and a line form staging whole
  // 64 B slots through LDS; both slower on C4)
#define BG_WT(KW)                                                          \
  if (a.t.kw == KW)                                                        \
    return pair ? launch_tags<KW, 2, 1>(a, num_cus, s)                     \
           : n2 ? launch_tags<KW, 2, 0>(a, num_cus, s)                     \
                : launch_tags<KW, 4, 0>(a, num_cus, s);
  BG_WT(1) BG_WT(2) BG_WT(4) BG_WT(8)
#undef BG_WT
  return hipErrorInvalidValue;
}

}  // namespace bg
