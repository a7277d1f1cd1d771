# em_slab_kernel: the gates of H grid-stride tiles held in LDS (a per-wave
# region after the stage, H x 128 B) instead of registers, the tile loop
# unrolled only U times (the register hold unrolls the tile body kGateHold
# times and spills past 32), then stored from LDS with 16 B per lane (8 lanes
# per tile). H from EMH_H (64), U from EMH_U (4).
import os
H = int(os.environ.get("EMH_H", "64"))
U = int(os.environ.get("EMH_U", "4"))
p = 'bess_amd/csrc/bg_kernels.hip'
s = open(p).read()
a = """  if (t < ntiles) load_tile(t, v);
  for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * kGateHold) {
  uint16_t held[kGateHold];
#pragma unroll
  for (int h = 0; h < kGateHold; h++) {
    const uint64_t t = t0 + (uint64_t)h * nwaves;
    held[h] = 0;
    if (t >= ntiles) break;"""
b = """  constexpr int H = %d;
  uint16_t *hold = reinterpret_cast<uint16_t *>(lds + stage_off + kWaves * 4096) + wid * (H * 64);
  const bool al16 = ((uintptr_t)a.gates & 15) == 0;
  if (t < ntiles) load_tile(t, v);
  for (uint64_t t0 = t; t0 < ntiles; t0 += nwaves * H) {
#pragma unroll %d
  for (int h = 0; h < H; h++) {
    const uint64_t t = t0 + (uint64_t)h * nwaves;
    if (t >= ntiles) break;""" % (H, U)
assert s.count(a) == 1
s = s.replace(a, b)
a = """    held[h] = (uint16_t)g;
    lds_fence();  // this tile's stage reads retire before the next writes
  }
#pragma unroll
  for (int h = 0; h < kGateHold; h++) {  // the held gates, streaming stores
    const uint64_t idx = (t0 + (uint64_t)h * nwaves) * 64 + lane;
    if (idx < a.n) __builtin_nontemporal_store(held[h], a.gates + idx);
  }
  }
}"""
b = """    hold[h * 64 + lane] = (uint16_t)g;
    lds_fence();  // this tile's stage reads retire before the next writes
  }
  lds_fence();
#pragma unroll
  for (int i = 0; i < H / 8; i++) {  // 8 lanes per tile, 16 B each
    const int k = i * 8 + (lane >> 3);
    const uint64_t idx = (t0 + (uint64_t)k * nwaves) * 64 + (lane & 7) * 8;
    if (idx >= a.n) continue;
    const uint4 x = reinterpret_cast<const uint4 *>(hold + k * 64)[lane & 7];
    if (al16 && idx + 8 <= a.n) {
      st_stream(reinterpret_cast<uint4 *>(a.gates + idx), x);
    } else {
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
      for (int j = 0; j < 8 && idx + j < a.n; j++)
        a.gates[idx + j] = (uint16_t)(xs[j >> 1] >> (16 * (j & 1)));
    }
  }
  lds_fence();  // the region is rewritten by the next round
  }
}"""
assert s.count(a) == 1
s = s.replace(a, b)
a = """  constexpr size_t kStage = (size_t)(kEmBlock / 64) * 4096;
  return launch_slab(em_slab_kernel<KW, NCH>, a, num_cus, s, kEmBlock, kStage);"""
b = """  constexpr size_t kStage = (size_t)(kEmBlock / 64) * (4096 + %d * 128);
  return launch_slab(em_slab_kernel<KW, NCH>, a, num_cus, s, kEmBlock, kStage);""" % H
assert s.count(a) == 1
s = s.replace(a, b)
open(p, 'w').write(s)
