# line_slab_kernel: each tile's gate held in registers for H grid-stride
# tiles, then stored (as em_slab_kernel's hold variants); LINE_OCC1=1 also
# launches it at one workgroup per CU. H from LINE_HOLD.
import os
H = int(os.environ.get("LINE_HOLD", "16"))
p = 'bess_amd/csrc/bg_line_dev.h'
s = open(p).read()
a = """  if (t < ntiles) load_tile(t);
  for (; t < ntiles; t += nwaves) {
#pragma unroll
    for (int c = 0; c < 4; c++) {
      const uint32_t u = c * 64 + lane;
      stage[line_stage_unit(u >> 2, u & 3)] = v[c];
    }"""
b = """  if (t < ntiles) load_tile(t);
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
      stage[line_stage_unit(u >> 2, u & 3)] = v[c];
    }""" % (H, H, H)
assert s.count(a) == 1
s = s.replace(a, b)
a = """    if (idx < a.n) {
      uint8_t *f = const_cast<uint8_t *>(a.frames) + idx * 64;
      // (a streaming store, as em_slab_kernel's gates: measured faster)
      __builtin_nontemporal_store((uint16_t)Op::decide(a, lds, d, f), a.out + idx);
    }"""
b = """    if (idx < a.n) {
      uint8_t *f = const_cast<uint8_t *>(a.frames) + idx * 64;
      held[hh] = (uint16_t)Op::decide(a, lds, d, f);
    }"""
assert s.count(a) == 1
s = s.replace(a, b)
a = """    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}

// The 4 bytes at l4"""
b = """    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
#pragma unroll
  for (int hh = 0; hh < %d; hh++) {
    const uint64_t idx = (t0 + (uint64_t)hh * nwaves) * 64 + lane;
    if (idx < a.n) __builtin_nontemporal_store(held[hh], a.out + idx);
  }
  }
}

// The 4 bytes at l4""" % H
assert s.count(a) == 1
s = s.replace(a, b)
if os.environ.get("LINE_OCC1") == "1":
    a = "    occ = std::min(occ, 2);"
    assert s.count(a) == 1
    s = s.replace(a, "    occ = 1;")
open(p, 'w').write(s)
