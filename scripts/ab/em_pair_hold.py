# em_pair_kernel (ExactMatch on 1500 B frames in 2 KB slots): each tile's
# gates held in registers for H grid-stride tiles, then stored. H from
# PAIR_HOLD; PAIR_PC (if set) caps the workgroups per CU of its launch.
import os
H = int(os.environ.get("PAIR_HOLD", "16"))
p = 'bess_amd/csrc/bg_kernels.hip'
s = open(p).read()
a = """  if (t < ntiles) load_pair(a.frames, a.n, t * 64, lane, a.fp.win_lo, stride, wn);
  for (; t < ntiles; t += nw) {
    uint32_t w[10];"""
b = """  if (t < ntiles) load_pair(a.frames, a.n, t * 64, lane, a.fp.win_lo, stride, wn);
  for (uint64_t t0 = t; t0 < ntiles; t0 += nw * %d) {
  uint16_t held[%d];
#pragma unroll
  for (int h = 0; h < %d; h++) {
    const uint64_t t = t0 + (uint64_t)h * nw;
    held[h] = 0;
    if (t >= ntiles) break;
    uint32_t w[10];""" % (H, H, H)
assert s.count(a) == 1
s = s.replace(a, b)
a = """    const uint64_t idx = t * 64 + pair_slot(lane);
    if (idx < a.n) __builtin_nontemporal_store((uint16_t)g, a.gates + idx);
  }
}"""
b = """    held[h] = (uint16_t)g;
  }
#pragma unroll
  for (int h = 0; h < %d; h++) {
    const uint64_t idx = (t0 + (uint64_t)h * nw) * 64 + pair_slot(lane);
    if (idx < a.n) __builtin_nontemporal_store(held[h], a.gates + idx);
  }
  }
}""" % H
assert s.count(a) == 1
s = s.replace(a, b)
open(p, 'w').write(s)
