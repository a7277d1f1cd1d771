# em_slab_kernel: each tile's gates held in registers for H tiles (the grid-
# stride tiles t, t + nwaves, ...), then stored, so the gate stores leave in
# bursts between the tile reads (scripts/gate_probe.hip hold16). H from the
# EM_HOLD environment variable of the patch run; EM_OCC1=1 also launches the
# LDS-table slab kernel at one workgroup per CU.
import os
H = int(os.environ.get("EM_HOLD", "8"))
p = 'bess_amd/csrc/bg_kernels.hip'
s = open(p).read()
a = """  if (t < ntiles) load_tile(t, v);
  for (; t < ntiles; t += nwaves) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[stage_unit(u >> 2, u & 3)] = v[c];
    }
    lds_fence();
    if (t + nwaves < ntiles) load_tile(t + nwaves, v);"""
b = """  if (t < ntiles) load_tile(t, v);
  for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * %d) {
  uint16_t held[%d];
#pragma unroll
  for (int hh = 0; hh < %d; hh++) {
    const uint64_t t = t0 + (uint64_t)hh * nwaves;
    held[hh] = 0;
    if (t >= ntiles) break;
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[stage_unit(u >> 2, u & 3)] = v[c];
    }
    lds_fence();
    if (t + nwaves < ntiles) load_tile(t + nwaves, v);""" % (H, H, H)
assert s.count(a) == 1
s = s.replace(a, b)
a = """    const uint64_t idx = t * 64 + lane;
    if (idx < a.n)  // a streaming store
      __builtin_nontemporal_store((uint16_t)g, a.gates + idx);
    lds_fence();  // this tile's stage reads retire before the next writes
  }
}
"""
b = """    held[hh] = (uint16_t)g;
    lds_fence();  // this tile's stage reads retire before the next writes
  }
#pragma unroll
  for (int hh = 0; hh < %d; hh++) {
    const uint64_t idx = (t0 + (uint64_t)hh * nwaves) * 64 + lane;
    if (idx < a.n) __builtin_nontemporal_store(held[hh], a.gates + idx);
  }
  }
}
""" % H
assert s.count(a) == 1
s = s.replace(a, b)
if os.environ.get("EM_OCC1") == "1":
    a = """    if (a.t.lds == kLdsNone) pc = std::min(pc, 2);"""
    b = """    if (a.t.lds == kLdsNone) pc = std::min(pc, 2);
    else pc = 1;"""
    assert s.count(a) == 1
    s = s.replace(a, b)
open(p, 'w').write(s)
