# WildcardMatch tag-word kernels (wm_tags_body, ahead-of-time and run-time
# compiled): each tile's gates held in LDS for H grid-stride tiles (a per-
# wave region after the kernel's other LDS, H x 128 B), then stored 16 B per
# lane, as the ExactMatch slab kernel does. H from WMH (16).
import os
H = int(os.environ.get("WMH", "16"))
p = 'bess_amd/csrc/bg_kernels.h'
s = open(p).read()
a = """  return ((uint64_t)nbp * 4 + 15) / 16 * 16 + (uint64_t)kMaxTuples * kw * 8 + kWmDirLds +
         (uint64_t)kWmWaves * kWmWaveLds;"""
b = """  return ((uint64_t)nbp * 4 + 15) / 16 * 16 + (uint64_t)kMaxTuples * kw * 8 + kWmDirLds +
         (uint64_t)kWmWaves * kWmWaveLds + (uint64_t)kWmWaves * %d * 128;""" % H
assert s.count(a) == 1
s = s.replace(a, b)
open(p, 'w').write(s)

p = 'bess_amd/csrc/bg_wm_body.h'
s = open(p).read()
a = """__device__ __forceinline__ void wm_tile(const WmArgs &a, const uint32_t *tags,"""
b = """__device__ __forceinline__ uint32_t wm_tile(const WmArgs &a, const uint32_t *tags,"""
assert s.count(a) == 1
s = s.replace(a, b)
a = """  if (live)  // (a streaming store)
    __builtin_nontemporal_store(bb ? (uint16_t)bb : (uint16_t)a.default_gate, a.gates + idx);
}"""
b = """  return bb ? (uint32_t)(uint16_t)bb : a.default_gate;
}"""
assert s.count(a) == 1
s = s.replace(a, b)
a = """  for (; t < ntiles; t += nw) {
    const uint64_t idx = t * 64 + (PAIR ? pair_slot(lane) : (uint64_t)lane);"""
b = """  constexpr uint32_t HL = %d;
  uint16_t *hold = reinterpret_cast<uint16_t *>(
      lds + wm_tags_lds_bytes(nbp, a.t.kw) - (uint64_t)kWaves * HL * 128) + wid * HL * 64;
  for (uint64_t t0 = t; t0 < ntiles; t0 += nw * HL) {
  for (uint32_t hh = 0; hh < HL; hh++) {
    t = t0 + (uint64_t)hh * nw;
    if (t >= ntiles) break;
    const uint64_t idx = t * 64 + (PAIR ? pair_slot(lane) : (uint64_t)lane);""" % H
assert s.count(a) == 1
s = s.replace(a, b)
a = """    wm_tile<Spec, KW, NCH>(a, tags, mlds, best, q, nbp, lane, idx, live, w, [&]() {"""
b = """    const uint32_t g = wm_tile<Spec, KW, NCH>(a, tags, mlds, best, q, nbp, lane, idx, live, w, [&]() {"""
assert s.count(a) == 1
s = s.replace(a, b)
a = """          load_window<NCH>(a.frames + nidx * a.stride, a.fp, wn);
      }
    });
  }
}"""
b = """          load_window<NCH>(a.frames + nidx * a.stride, a.fp, wn);
      }
    });
    // slot of this lane's packet within the tile (pair loads: pair_slot)
    hold[hh * 64 + (uint32_t)(idx - t * 64)] = (uint16_t)g;
  }
  lds_fence();
  const bool al16 = ((unsigned long long)a.gates & 15) == 0;
  for (uint32_t i = 0; i < HL; i += 8) {
    const uint32_t h = i + (lane >> 3);
    const uint64_t gi = (t0 + (uint64_t)h * nw) * 64 + (lane & 7) * 8;
    if (gi >= a.n) continue;
    const uint4 x = reinterpret_cast<const uint4 *>(hold + h * 64)[lane & 7];
    if (al16 && gi + 8 <= a.n) {
      st_stream(reinterpret_cast<uint4 *>(a.gates + gi), x);
    } else {
      const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
      for (int j = 0; j < 8 && gi + j < a.n; j++)
        a.gates[gi + j] = (uint16_t)(xs[j >> 1] >> (16 * (j & 1)));
    }
  }
  lds_fence();
  }
}"""
assert s.count(a) == 1
s = s.replace(a, b)
open(p, 'w').write(s)
